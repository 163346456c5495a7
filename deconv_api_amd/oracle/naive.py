"""Deliberately naive loop implementations (written from the spec) used to
cross-check the vectorized oracle on small shapes: explicit per-window first-max pooling,
per-channel summation with a stable sort, and a direct 3x3 'same' convolution."""
from __future__ import annotations

import numpy as np


def maxpool_with_switch(x: np.ndarray):
    """x [N, H, W, C] -> (pooled [N, H/2, W/2, C], switch one-hot [N, H, W, C])."""
    N, H, W, C = x.shape
    pooled = np.zeros((N, H // 2, W // 2, C), dtype=np.float64)
    switch = np.zeros(x.shape, dtype=np.float64)
    for n in range(N):
        for c in range(C):
            for r in range(H // 2):
                for q in range(W // 2):
                    best, br, bq = None, 0, 0
                    for dy in range(2):
                        for dx in range(2):
                            v = x[n, 2 * r + dy, 2 * q + dx, c]
                            if best is None or v > best:
                                best, br, bq = v, dy, dx
                    pooled[n, r, q, c] = best
                    switch[n, 2 * r + br, 2 * q + bq, c] = 1.0
    return pooled, switch


def unpool(y: np.ndarray, switch: np.ndarray) -> np.ndarray:
    N, PH, PW, C = y.shape
    out = np.zeros(switch.shape, dtype=np.float64)
    for n in range(N):
        for c in range(C):
            for h in range(2 * PH):
                for w in range(2 * PW):
                    out[n, h, w, c] = y[n, h // 2, w // 2, c] * switch[n, h, w, c]
    return out


def top_filters(output: np.ndarray, top: int = 8):
    sums = []
    for f in range(output.shape[-1]):
        s = 0.0
        for v in output[..., f].ravel():
            s += float(v)
        if s > 0:
            sums.append((f, s))
    # insertion sort, stable (ties keep ascending index)
    ordered = []
    for item in sums:
        k = len(ordered)
        while k > 0 and ordered[k - 1][1] < item[1]:
            k -= 1
        ordered.insert(k, item)
    return ordered[:top]


def conv3x3_same(x: np.ndarray, w_hwio: np.ndarray, b=None) -> np.ndarray:
    N, H, W, C = x.shape
    O = w_hwio.shape[3]
    xp = np.zeros((N, H + 2, W + 2, C))
    xp[:, 1:-1, 1:-1] = x
    out = np.zeros((N, H, W, O))
    for kh in range(3):
        for kw in range(3):
            out += np.einsum("nhwc,co->nhwo", xp[:, kh:kh + H, kw:kw + W], w_hwio[kh, kw])
    if b is not None:
        out += b
    return out
