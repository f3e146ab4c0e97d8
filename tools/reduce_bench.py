"""Microbenchmark of the training step's per-channel reductions (upr_t_bn_stats,
upr_t_chan_sum, upr_t_bn_bwd_fused) on the training shapes: achieved GB/s.
Run on the GPU box: python tools/reduce_bench.py"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "retinex-image-enhancement_amd"), REPO]

import torch  # noqa: E402

from upr import _lib as L  # noqa: E402


def p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    lib = L.lib()
    dev = torch.device("cuda", 0)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for (B, HW, C) in ((8, 512 * 512, 32), (8, 256 * 256, 64), (8, 128 * 128, 128), (8, 64 * 64, 256)):
        M = B * HW
        x = torch.randn(M, C, device=dev)
        g = torch.randn(M, C, device=dev)
        dx = torch.empty_like(x)
        acc = torch.zeros(2 * C, dtype=torch.float64, device=dev)
        out = torch.zeros(C, device=dev)
        mean = torch.zeros(C, device=dev)
        inv = torch.ones(C, device=dev)
        gam = torch.ones(C, device=dev)
        bet = torch.zeros(C, device=dev)
        dg = torch.zeros(C, device=dev)
        db = torch.zeros(C, device=dev)
        t_stats = timeit(lambda: lib.upr_t_bn_stats(p(x), M, C, C, 0, p(acc), st))
        t_sum = timeit(lambda: lib.upr_t_chan_sum(p(g), M, C, C, 0, p(out), 1, st))
        t_bwd = timeit(lambda: lib.upr_t_bn_bwd_fused(p(g), C, 0, p(x), C, p(mean), p(inv), p(gam), p(bet), 1, M, C,
                                                       p(acc), p(dg), p(db), p(dx), C, 0, 0, 1, None, st))
        nb = M * C * 4
        print(f"M={M:8d} C={C:4d}: bn_stats {t_stats * 1e3:7.1f} us {nb / t_stats / 1e6:7.0f} GB/s | "
              f"chan_sum {t_sum * 1e3:7.1f} us {nb / t_sum / 1e6:7.0f} GB/s | "
              f"bn_bwd_fused {t_bwd * 1e3:7.1f} us {5 * nb / t_bwd / 1e6:7.0f} GB/s (5 passes of bytes)")


if __name__ == "__main__":
    main()
