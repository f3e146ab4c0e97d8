"""Measured ceilings of the device (csrc/calib.hip via upr_calib_run), for the
bench's roofline report: what an fp16 MFMA loop on random register operands
and a streaming HBM copy actually reach on this chip, next to the nominal
2516.6 TF/s / 8.0 TB/s peaks (MI355X_MICROARCH.md: the fp16 MFMA clock drops
under load on random data; a float4 copy reaches ~79% of the HBM spec)."""
import ctypes
import time

import torch

from upr import _lib as L


def _run(lib, which, blocks, iters, src, dst, nbytes, reps, stream):
    ms = ctypes.c_float(0.0)
    rc = lib.upr_calib_run(which, blocks, iters, ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()),
                           nbytes, reps, ctypes.byref(ms), stream)
    L.check(rc, "upr_calib_run")
    return ms.value


def measure(dev, warm_s=2.0, copy_bytes=1 << 30):
    """-> dict: mfma_f16_TF (best of 1 and 2 waves per SIMD, after warm_s of
    back-to-back launches so the clock has settled), hbm_copy_TBps (read +
    write bytes / time, best of two grid sizes), and the per-variant numbers."""
    lib = L.lib()
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    g = torch.Generator(device=dev).manual_seed(7)
    src = torch.randn(1024 * 4 * 64 * 8, generator=g, device=dev).half()
    out = {"mfma_f16": {}, "hbm_copy": {}}
    iters = 100000
    for blocks in (256, 512):
        sink = torch.empty(blocks * 256 * 4, device=dev)
        flop = blocks * 4 * iters * 8 * 16384.0
        ms = _run(lib, L.UPR_CALIB_MFMA_F16, blocks, iters, src, sink, src.numel() * 2, 1, stream)
        t_end = time.perf_counter() + warm_s
        while time.perf_counter() < t_end:
            _run(lib, L.UPR_CALIB_MFMA_F16, blocks, iters, src, sink, src.numel() * 2,
                 max(1, int(200.0 / max(ms, 1e-3))), stream)
        ms = _run(lib, L.UPR_CALIB_MFMA_F16, blocks, iters, src, sink, src.numel() * 2,
                  max(1, int(500.0 / max(ms, 1e-3))), stream)
        out["mfma_f16"][f"{blocks // 256}_wave_per_simd"] = flop / (ms * 1e-3) / 1e12
        del sink
    a = torch.empty(copy_bytes, dtype=torch.uint8, device=dev).random_(0, 255, generator=g)
    b = torch.empty_like(a)
    for mode, name in ((0, "stride"), (1, "stride_nt"), (2, "slice")):
        for blocks in (1024, 2048, 4096):
            _run(lib, L.UPR_CALIB_HBM_COPY, blocks, mode, a, b, copy_bytes, 5, stream)
            ms = _run(lib, L.UPR_CALIB_HBM_COPY, blocks, mode, a, b, copy_bytes, 50, stream)
            out["hbm_copy"][f"{name}_grid_{blocks}"] = 2.0 * copy_bytes / (ms * 1e-3) / 1e12
    assert torch.equal(a[-4096:], b[-4096:])
    del a, b
    out["mfma_f16_TF"] = max(out["mfma_f16"].values())
    out["hbm_copy_TBps"] = max(out["hbm_copy"].values())
    return out


if __name__ == "__main__":
    import json
    print(json.dumps(measure(torch.device("cuda:0"))))
