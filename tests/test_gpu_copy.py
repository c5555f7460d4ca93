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
