#!/usr/bin/env python3
"""Library-GEMM calibration (torch.matmul -> hipBLASLt) on the wide-kernel layer shapes:
what a tuned dense GEMM of the same M x N x K reaches on this box (random fp16 data)."""
import torch

dev = torch.device("cuda", 0)
for name, M, N, K in (("bneck 3x3", 131072, 256, 2304), ("dec3 3x3", 524288, 128, 1152),
                      ("aspp", 131072, 256, 2304), ("square 8k", 8192, 8192, 8192)):
    a = torch.randn(M, K, device=dev, dtype=torch.float16)
    b = torch.randn(K, N, device=dev, dtype=torch.float16)
    for _ in range(3):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 20
    e0.record()
    for _ in range(it):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / it
    print(f"{name:10s} M {M} N {N} K {K}: {ms:.3f} ms  {2 * M * N * K / ms / 1e9:.1f} TF/s")
