"""The DV_DEBUG device bounds checks (common.h DV_BOUNDS) compile: the conv kernels are built with
-DDV_DEBUG=1 into a scratch directory (CPU-only cross compile for gfx950; the production .so is
not touched). In a debug build an out-of-range conv load/store prints its site and is skipped."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "deconv_api_amd", "csrc")


@pytest.mark.parametrize("src", ["conv_halo_stream.hip", "conv_smalln.hip"])
def test_debug_bounds_checks_compile(tmp_path, src):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    obj = tmp_path / (src + ".o")
    cmd = [hipcc, "-O1", "-DDV_DEBUG=1", "--offload-arch=gfx950", "-fPIC", "-std=c++17", "-Wno-unused-result",
           f"-I{CSRC}", "-c", os.path.join(CSRC, src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-4000:]
    assert obj.stat().st_size > 0


def test_debug_macro_is_a_constant_in_release():
    """Release builds must not pay for the checks: DV_BOUNDS is the literal `true` there."""
    src = open(os.path.join(CSRC, "common.h")).read()
    assert "#define DV_BOUNDS(off, n, extent, what) true" in src
    assert src.count("DV_BOUNDS") >= 3
    for f in ("conv_dma_impl.h", "conv_halo_stream.hip", "conv_smalln.hip"):
        assert "DV_BOUNDS" in open(os.path.join(CSRC, f)).read(), f
