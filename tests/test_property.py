"""Property tests (hypothesis): generated NHWC shapes and tie-heavy post-ReLU values for the
integer-valued paths of the deconvnet - max-pool switches (first max in row-major window order), max-unpool,
and the stable positive top-k of find_top_filters (app/deepdream.py:369-380) - compared EXACTLY.

CPU: the vectorized oracle (ops.maxpool_switch_ref / unpool_ref / topk_positive) vs the naive loops written
from the spec (oracle/naive.py). GPU (@gpu): the HIP kernels (maxpool2x2, unpool2x2, topk_pos, channel_sum)
vs that oracle."""
from __future__ import annotations

import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from deconv_api_amd import ops
from deconv_api_amd.oracle import naive

# a handful of distinct levels, zero-heavy (post-ReLU) so that windows tie often
LEVELS = np.array([0.0, 0.0, 0.0, 0.5, 1.0, 1.5, 2.0], dtype=np.float32)


@st.composite
def nhwc(draw, max_n=3, max_hw=12, chans=(1, 3, 8, 16, 24)):
    n = draw(st.integers(1, max_n))
    h = 2 * draw(st.integers(1, max_hw // 2))
    w = 2 * draw(st.integers(1, max_hw // 2))
    c = draw(st.sampled_from(chans))
    seed = draw(st.integers(0, 2 ** 31 - 1))
    rng = np.random.default_rng(seed)
    return LEVELS[rng.integers(0, len(LEVELS), (n, h, w, c))]


CPU = settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.too_slow])
GPU = settings(max_examples=30, deadline=None, suppress_health_check=[HealthCheck.too_slow,
                                                                     HealthCheck.function_scoped_fixture])


@CPU
@given(x=nhwc())
def test_pool_switch_oracle_vs_naive(x):
    val, code = ops.maxpool_switch_ref(torch.from_numpy(x))
    pooled, onehot = naive.maxpool_with_switch(x)
    assert np.array_equal(val.numpy(), pooled.astype(np.float32))
    # the naive switch is a one-hot map at the first maximum; code 2 dy + dx names the same position
    n, ph, pw, c = code.shape
    got = onehot.reshape(n, ph, 2, pw, 2, c).transpose(0, 1, 3, 2, 4, 5).reshape(n, ph, pw, 4, c).argmax(axis=3)
    assert np.array_equal(code.numpy(), got.astype(np.uint8))
    # unpool(pool(x)) puts every pooled value back at its switch position, zeros elsewhere
    up = ops.unpool_ref(val, code).numpy()
    assert np.array_equal(up, naive.unpool(pooled, onehot).astype(np.float32))


@CPU
@given(sums=st.lists(st.sampled_from([-1.0, 0.0, 0.25, 0.5, 0.5, 1.0, 2.0, 2.0]), min_size=1, max_size=40),
       k=st.integers(1, 8))
def test_topk_positive_oracle_vs_naive(sums, k):
    v = torch.tensor([sums], dtype=torch.float32)
    idx, val = ops.topk_positive(v, k)
    want = naive.top_filters(np.array(sums, dtype=np.float64).reshape(1, 1, 1, -1), top=k)
    got = [(int(i), float(s)) for i, s in zip(idx[0].tolist(), val[0].tolist()) if i >= 0]
    assert got == [(f, s) for f, s in want]


def _dev16(x: np.ndarray, dtype=torch.bfloat16) -> torch.Tensor:
    return torch.from_numpy(x).to(dtype).cuda()


@pytest.mark.gpu
@GPU
@given(x=nhwc(max_n=3, max_hw=40, chans=(8, 16, 64, 72, 3, 5)), fp16=st.booleans())
def test_gpu_maxpool_switch_exact(native_lib, x, fp16):
    """maxpool2x2 (vectorized kernel for C % 8 == 0, scalar otherwise): values and first-max codes."""
    xd = _dev16(x, torch.float16 if fp16 else torch.bfloat16)
    val, code = ops.maxpool2x2(xd)
    rv, rc = ops.maxpool_switch_ref(xd.float().cpu())
    assert torch.equal(val.float().cpu(), rv) and torch.equal(code.cpu(), rc)


@pytest.mark.gpu
@GPU
@given(x=nhwc(max_n=4, max_hw=24, chans=(8, 16, 64)), div=st.sampled_from([1, 2]), relu=st.booleans())
def test_gpu_unpool_exact(native_lib, x, div, relu):
    """unpool2x2 with per-image codes shared by `div` consecutive signals (the B x K layout)."""
    _, code = ops.maxpool_switch_ref(torch.from_numpy(x))         # [n, ...]: one code map per image
    p = torch.from_numpy(np.repeat(x, div, axis=0)[:, ::2, ::2] - 1.0).to(torch.bfloat16)  # n * div signals, signed
    got = ops.unpool2x2(p.cuda(), code.cuda(), div, relu).float().cpu()
    want = ops.unpool_ref(p.float(), code, div)
    if relu:
        want = want.clamp_min(0)
    assert torch.equal(got, want)


@pytest.mark.gpu
@GPU
@given(rows=st.integers(1, 6), c=st.sampled_from([1, 7, 64, 130, 512]), k=st.integers(1, 8),
       seed=st.integers(0, 2 ** 31 - 1))
def test_gpu_topk_positive_exact(native_lib, rows, c, k, seed):
    """topk_pos kernel: value-descending, index-ascending among ties, strictly positive only, -1 padded."""
    rng = np.random.default_rng(seed)
    v = torch.from_numpy(rng.choice(np.array([-1.0, 0.0, 0.5, 1.0, 3.0], np.float32), size=(rows, c)))
    gi, gv = ops.topk_positive(v.cuda(), k)
    ri, rv = ops.topk_positive(v, k)
    assert torch.equal(gi.cpu(), ri) and torch.equal(gv.cpu(), rv)


@pytest.mark.gpu
@GPU
@given(x=nhwc(max_n=3, max_hw=40, chans=(8, 64, 512)))
def test_gpu_channel_sum(native_lib, x):
    """Per-image channel sums (fp32 accumulation of bf16 maps) against an fp64 sum; the order of the
    positive sums - what find_top_filters consumes - is the same."""
    xd = _dev16(x)
    got = ops.channel_sum(xd).cpu().double()
    want = torch.from_numpy(x).double().sum(dim=(1, 2))
    assert torch.allclose(got, want, rtol=1e-6, atol=1e-6)
    assert torch.equal(ops.topk_positive(got.float(), 8)[0], ops.topk_positive(want.float(), 8)[0])
