"""HIP 2:4 sparse-MFMA unpool conv-down (csrc/conv_sparse.hip) vs the fp32 PyTorch reference
ReLU(conv_transpose(ReLU(unpool(v, code)), W)) -- app/deepdream.py:78-89,191-209."""
import pytest
import torch
import torch.nn.functional as F

from deconv_api_amd.ops import sparse_unpool as su
from deconv_api_amd.ops.conv import unpool_ref

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(4, 7, 7, 64, 128, 2), (3, 5, 9, 32, 256, 1), (8, 14, 14, 512, 512, 4),
                                   (2, 28, 28, 256, 128, 2)])
def test_sparse_unpool_conv_matches_fp32(shape):
    NB, PH, PW, C, Ci, cdiv = shape
    g = torch.Generator().manual_seed(sum(shape))
    v = torch.randn(NB, PH, PW, C, generator=g).to(torch.bfloat16)
    code = torch.randint(0, 4, (NB // cdiv, PH, PW, C), generator=g, dtype=torch.uint8)
    w = (torch.randn(C, Ci, 3, 3, generator=g) / (3 * C ** 0.5)).to(torch.bfloat16)
    dev = torch.device("cuda", 0)
    wt = su.pack_for_kernel(w, dev)
    got = su.sparse_unpool_conv(v.to(dev), code.to(dev), wt, cdiv).float().cpu()
    u = unpool_ref(v.float().clamp_min(0), code, cdiv)
    ref = F.conv_transpose2d(u.permute(0, 3, 1, 2), w.float(), padding=1).permute(0, 2, 3, 1).clamp_min(0)
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= 1e-2 * scale + 1e-3, (err, scale)
