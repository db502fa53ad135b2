"""Calibrate achievable HBM rates on the box (dev tool): fill (write-only), copy, and read (sum)."""
import time

import torch

dev = torch.device("cuda", 0)


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


for gb in (4, 16):
    n = gb * (1 << 30) // 8
    x = torch.empty(n, dtype=torch.int64, device=dev)
    y = torch.empty(n, dtype=torch.int64, device=dev)
    t = timeit(lambda: x.fill_(7))
    print(f"fill   {gb:3d} GiB: {n * 8 / t / 1e12:.2f} TB/s")
    t = timeit(lambda: y.copy_(x))
    print(f"copy   {gb:3d} GiB: {2 * n * 8 / t / 1e12:.2f} TB/s (read+write)")
    t = timeit(lambda: x.sum())
    print(f"read   {gb:3d} GiB: {n * 8 / t / 1e12:.2f} TB/s")
    del x, y
    torch.cuda.empty_cache()
