"""2:4 sparse re-grouping of unpool-fed conv-downs (ops/sparse_unpool.py) vs the dense reference:
ReLU(conv_transpose(ReLU(unpool(v, code)), W)) -- app/deepdream.py:78-89,191-209."""
import pytest
import torch
import torch.nn.functional as F

from deconv_api_amd.ops import sparse_unpool as su
from deconv_api_amd.ops.conv import unpool_ref


def _dense(v, code, w):
    u = unpool_ref(v.float().clamp_min(0), code)
    y = F.conv_transpose2d(u.permute(0, 3, 1, 2), w.float(), padding=1)
    return y.permute(0, 2, 3, 1).clamp_min(0)


@pytest.mark.parametrize("shape", [(2, 4, 5, 32, 24), (1, 3, 3, 16, 8), (1, 7, 7, 48, 16)])
def test_sparse_phase_equals_dense(shape):
    N, PH, PW, Co, Ci = shape
    g = torch.Generator().manual_seed(sum(shape))
    v = torch.randn(N, PH, PW, Co, generator=g)
    code = torch.randint(0, 4, (N, PH, PW, Co), generator=g, dtype=torch.uint8)
    w = torch.randn(Co, Ci, 3, 3, generator=g)
    packed = su.pack_phase_weights(w)
    assert packed.shape == (4, Co // 16, 160, Ci)
    got = su.sparse_unpool_conv_ref(v, code, packed)
    ref = _dense(v, code, w)
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4)


def test_two_four_contract():
    """Every group of 4 logical rows carries <= 2 nonzeros in ascending, distinct slots."""
    g = torch.Generator().manual_seed(3)
    v = torch.randn(2, 6, 6, 32, generator=g)
    code = torch.randint(0, 4, (2, 6, 6, 32), generator=g, dtype=torch.uint8)
    for a in range(2):
        for b in range(2):
            val, idx = su.compress_operand(v, code, a, b)
            assert val.shape[-3:] == (5, 8, 2)
            assert bool((idx[..., 0] < idx[..., 1]).all())
            assert int(idx.min()) >= 0 and int(idx.max()) <= 3


def test_mfma_count_ratio():
    dense, sparse = su.smfmac_counts(802816, 512, 256)   # block4_conv3.down-shaped (B*K=1024)
    assert abs(dense / sparse - 1.8) < 1e-6
