"""fp64 GEMM ceiling of the vendor library on this GPU (torch.matmul -> hipBLASLt / rocBLAS), as a
reference point for the hand-written tile GEMM's fraction of the datasheet peak.
Square GEMMs and the batched 128 x K x 128 products the left-looking Cholesky update performs."""
import json
import time

import torch


def rate(f, flops, reps=10):
    f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    return flops * reps / (time.perf_counter() - t) / 1e12


out = {}
for n in (4096, 8192, 16384):
    a = torch.randn(n, n, dtype=torch.float64, device="cuda")
    b = torch.randn(n, n, dtype=torch.float64, device="cuda")
    c = torch.empty_like(a)
    out[f"square_{n}"] = rate(lambda: torch.matmul(a, b, out=c), 2.0 * n ** 3, reps=5 if n == 16384 else 10)
    del a, b, c
for k in (256, 1024, 1920):
    batch = 250 * 8           # one update launch's tiles at 250 subsets, mid factorisation
    a = torch.randn(batch, 128, k, dtype=torch.float64, device="cuda")
    b = torch.randn(batch, k, 128, dtype=torch.float64, device="cuda")
    out[f"batched_128x{k}x128_x{batch}"] = rate(lambda: torch.bmm(a, b), 2.0 * batch * 128 * 128 * k)
    del a, b
print(json.dumps({"unit": "TFLOP/s", "peak": 78.6, **out}), flush=True)
