#!/usr/bin/env python
"""Does a device -> host copy slow concurrent compute? Times a bf16 GEMM loop alone and with a
154 MB D2H copy (the config-2 mosaic copy-back) on a side stream, for a hipHostMalloc'd (torch
pinned) and a hipHostRegister'd destination; run it under different runtime copy settings.

  python tools/copy_overlap_probe.py
"""
import time

import torch


def main():
    dev = torch.device("cuda")
    x = torch.randint(0, 255, (256, 448, 448, 3), dtype=torch.uint8, device=dev)
    a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    pinned = torch.empty(x.shape, dtype=torch.uint8, pin_memory=True)
    reg = torch.empty(x.shape, dtype=torch.uint8)
    rc = torch.cuda.cudart().cudaHostRegister(reg.data_ptr(), reg.numel(), 0)
    s = torch.cuda.Stream(dev)
    for _ in range(3):
        a @ a
    torch.cuda.synchronize()

    def gemms(n=10):
        for _ in range(n):
            a @ a

    for name, host in (("pinned", pinned), ("registered", reg if int(rc) == 0 else None)):
        if host is None:
            print(f"{name}: hostRegister failed ({rc})")
            continue
        res = {}
        for rep in range(2):
            torch.cuda.synchronize()
            t = time.perf_counter()
            gemms()
            torch.cuda.synchronize()
            res["gemm_alone_ms"] = (time.perf_counter() - t) * 1e3
            t = time.perf_counter()
            with torch.cuda.stream(s):
                host.copy_(x, non_blocking=True)
            s.synchronize()
            res["copy_alone_ms"] = (time.perf_counter() - t) * 1e3
            torch.cuda.synchronize()
            t = time.perf_counter()
            with torch.cuda.stream(s):
                host.copy_(x, non_blocking=True)
            gemms()
            torch.cuda.synchronize()
            res["both_ms"] = (time.perf_counter() - t) * 1e3
        ok = bool(torch.equal(host[:2].to(dev), x[:2]))
        print(name, {k: round(v, 3) for k, v in res.items()}, "exact", ok, flush=True)


if __name__ == "__main__":
    main()
