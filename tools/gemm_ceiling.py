"""hipBLASLt (torch.matmul) TFLOP/s on the plain-GEMM equivalents of the deconvnet's conv shapes:
a practical ceiling for the implicit-GEMM conv kernels (same M x N x K, no im2col gather).

    python tools/gemm_ceiling.py
"""
import time

import torch

SHAPES = [(200704, 512, 4608), (802816, 512, 4608), (802816, 256, 2304), (3211264, 128, 1152),
          (3211264, 256, 2304), (12845056, 64, 1152), (12845056, 128, 1152)]


def main():
    dev = torch.device("cuda", 0)
    for M, N, K in SHAPES:
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
        c = a @ b
        torch.cuda.synchronize()
        reps = 5
        t = time.perf_counter()
        for _ in range(reps):
            c = a @ b
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / reps
        print(f"M={M} N={N} K={K}: {dt * 1e3:.3f} ms {2.0 * M * N * K / dt / 1e12:.1f} TF/s", flush=True)
        del a, b, c


if __name__ == "__main__":
    main()
