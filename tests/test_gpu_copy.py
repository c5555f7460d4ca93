"""ctn_copy_bytes, bench.py's bandwidth-calibration copy: every byte copied, for sizes
that leave a partial last round of the 4-deep grid-stride loop."""
import pytest
import torch


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, 1, 2, 3])
@pytest.mark.parametrize("n16,wgs", [(1, 1), (1000, 3), (256 * 8 * 7 + 5, 7), (1 << 20, 1024)])
def test_copy_bytes(n16, wgs, flags):
    import ctn_lib as L
    lib = L.load()
    dev = torch.device("cuda")
    a = torch.randint(-2**31, 2**31 - 1, (n16 * 4,), dtype=torch.int32, device=dev)
    b = torch.zeros_like(a)
    s = torch.cuda.current_stream(dev).cuda_stream
    L.check(lib.ctn_copy_bytes(b.data_ptr(), a.data_ptr(), n16 * 16, wgs, flags, s), "ctn_copy_bytes")
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [0, 1])
def test_mfma_peak(shape):
    """ctn_mfma_peak, bench.py's matrix-peak calibration: the reported FLOP count and a
    finite output, at a rate between a tenth of and the 2.5 PF/s dense datasheet peak."""
    import ctypes
    import ctn_lib as L
    lib = L.load()
    dev = torch.device("cuda")
    wgs, iters = 512, 4000
    out = torch.full((wgs * 256,), float("nan"), device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    flops = ctypes.c_double(0.0)
    L.check(lib.ctn_mfma_peak(shape, wgs, iters, out.data_ptr(), ctypes.byref(flops), s), "ctn_mfma_peak")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    L.check(lib.ctn_mfma_peak(shape, wgs, iters, out.data_ptr(), None, s), "ctn_mfma_peak")
    e1.record()
    e1.synchronize()
    assert flops.value == wgs * 4 * iters * (8 * 16384 if shape == 0 else 4 * 32768)
    assert torch.isfinite(out).all()
    tflops = flops.value / (e0.elapsed_time(e1) * 1e-3) / 1e12
    print("shape", shape, "TFLOP/s", tflops)
    assert 250 < tflops < 2600
