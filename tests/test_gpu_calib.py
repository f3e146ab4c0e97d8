"""The bench's measured-ceiling kernels (csrc/calib.hip, upr_calib_run): the
copy forms move every byte, the MFMA loop leaves the accumulator sum it is
expected to (8 accumulators of iters x A.B products, checked in fp64), and bad
arguments are rejected before any launch."""
import ctypes

import pytest
import torch

from conftest import has_gpu

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs a ROCm device")]


def _run(which, blocks, iters, src, dst, nbytes, reps=1):
    from upr import _lib as L
    ms = ctypes.c_float(0.0)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rc = L.lib().upr_calib_run(which, blocks, iters, ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()),
                               nbytes, reps, ctypes.byref(ms), st)
    return rc, ms.value


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_calib_copy_exact(mode):
    from upr import _lib as L
    n = (3 << 20) + 16 * 37  # not a multiple of the grid's step
    a = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    b = torch.zeros_like(a)
    rc, ms = _run(L.UPR_CALIB_HBM_COPY, 64, mode, a, b, n)
    torch.cuda.synchronize()
    assert rc == 0 and ms > 0
    assert torch.equal(a, b)


def test_calib_mfma_sum():
    from upr import _lib as L
    torch.manual_seed(0)
    src = (torch.randint(-2, 3, (1024 * 4 * 64 * 8,), device="cuda").half()) / 4  # exact in fp16 / fp32 sums
    blocks, iters = 2, 3
    sink = torch.empty(blocks * 256 * 4, device="cuda")
    rc, _ = _run(L.UPR_CALIB_MFMA_F16, blocks, iters, src, sink, src.numel() * 2)
    torch.cuda.synchronize()
    assert rc == 0
    # fragments of wave w: A0, A1, B0, B1 = 16x32 operand tiles (lane l holds row l % 16, k 8(l/16)..+7)
    frag = src.double().cpu().view(1024, 4, 64, 8)

    def tile(f):  # [64 lanes, 8] -> [16 rows, 32 k]
        return f.view(4, 16, 8).permute(1, 0, 2).reshape(16, 32)

    got = sink.double().cpu().view(blocks * 4, 64, 4)
    for w in range(blocks * 4):
        a0, a1, b0, b1 = (tile(frag[w, i]) for i in range(4))
        # acc = A_tile @ B_tile^T (16x16); 8 products per iteration, summed
        prods = [(a0, b0), (a1, b0), (a0, b1), (a1, b1), (b0, a0), (b1, a0), (b0, a1), (b1, a1)]
        ref = sum(x @ y.T for x, y in prods) * iters  # [row i (A side), col j (B side)]
        # lane l holds column l % 16, rows 4(l/16)..4(l/16)+3
        out = got[w].view(4, 16, 4).permute(0, 2, 1).reshape(16, 16)
        assert torch.allclose(out, ref, atol=1e-9), w


def test_calib_rejects_bad_args():
    from upr import _lib as L
    a = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    assert _run(L.UPR_CALIB_HBM_COPY, 16, 3, a, a, 4096)[0] != 0     # unknown copy form
    assert _run(L.UPR_CALIB_HBM_COPY, 16, 0, a, a, 4095)[0] != 0     # not a multiple of 16
    assert _run(L.UPR_CALIB_MFMA_F16, 16, 10, a, a, 4096)[0] != 0    # source smaller than 1024 waves' operands
    assert _run(7, 16, 10, a, a, 4096)[0] != 0
