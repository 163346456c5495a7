"""GPU race detection by schedule perturbation: the full deconvnet step (forward
with fused pools, top-k, B x K backward, fused deprocess statistics, mosaic) is run in a child
process with every kernel launch serialized (AMD_SERIALIZE_KERNEL=3, HIP_LAUNCH_BLOCKING=1) and
compared with the normal asynchronous run in this process, and two back-to-back asynchronous runs
are compared with each other. A missing dependency between kernels, a stream race or an
uninitialized read shows up as a difference. The only legitimately order-dependent values are the
fp64 atomic deprocess sums (rounding at ~1e-16), so mosaics may differ by at most 1 level."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import sys, torch
sys.path.insert(0, {root!r})
from deconv_api_amd import ops
from deconv_api_amd.engine.deconvnet import DeconvNet
from deconv_api_amd.models.vgg16 import VGG16
ops.native.load()
dev = torch.device("cuda", 0)
eng = DeconvNet(VGG16.random(0, include_top=False).build(dev, torch.bfloat16))
g = torch.Generator().manual_seed(5)
img = torch.randint(0, 256, (3, 224, 224, 3), dtype=torch.uint8, generator=g).to(dev)
x = torch.empty(3, 224, 224, 8, dtype=torch.bfloat16, device=dev)
ops.resize_preprocess(img, x)
res = eng.run(x, {layer!r}, k=4)
torch.cuda.synchronize()
torch.save({{"mosaic": res.mosaic.cpu(), "filters": res.filters.cpu(), "recon": res.recon.cpu()}}, {out!r})
"""


def _run(tmp_path, name, layer, env_extra):
    out = str(tmp_path / f"{name}.pt")
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, "-c", SCRIPT.format(root=ROOT, layer=layer, out=out)], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return torch.load(out, weights_only=True)


@pytest.mark.parametrize("layer", ["block5_conv3", "block3_pool"])
def test_serialized_launches_match_async(native_lib, tmp_path, layer):
    a = _run(tmp_path, "async", layer, {})
    b = _run(tmp_path, "async2", layer, {})
    s = _run(tmp_path, "serial", layer, {"AMD_SERIALIZE_KERNEL": "3", "HIP_LAUNCH_BLOCKING": "1"})
    for other in (b, s):
        assert torch.equal(a["filters"], other["filters"])
        assert torch.equal(a["recon"], other["recon"])  # every kernel but the atomics is deterministic
        assert (a["mosaic"].int() - other["mosaic"].int()).abs().max() <= 1
