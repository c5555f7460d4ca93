"""The kernel timer bench.py reads its roofline from (ctn_timer_*): every launch of an
enabled kind bracketed at stride 1, every n-th at ctn_timer_set_stride(n) (ABI v11, the
timed region's sampling), counted from the enable, with positive durations."""
import ctypes

import pytest
import torch

TIMER_GEMM1 = 1   # include/ctn.h CTN_TIMER_GEMM1: the forward B -> H 1x1 GEMM, one per block


def _forward(model, mix):
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        model(mix)
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_timer_stride_samples_every_nth_launch():
    import conv_tasnet as ct
    import ctn_lib as L
    lib = L.load()
    torch.manual_seed(0)
    X, R = 2, 2
    model = ct.ConvTasNet(64, 20, 64, 128, 3, X, R, 2, norm_type="gLN").cuda()
    mix = torch.randn(2, 8000, device="cuda")
    _forward(model, mix)                                   # weights packed, plans cached
    counts = {}
    try:
        for stride, passes in ((1, 1), (3, 3)):
            L.check(lib.ctn_timer_set_stride(stride), "ctn_timer_set_stride")
            L.check(lib.ctn_timer_enable(TIMER_GEMM1, 64), "ctn_timer_enable")
            for _ in range(passes):
                _forward(model, mix)
            tot, n = ctypes.c_double(0.0), ctypes.c_int(0)
            L.check(lib.ctn_timer_read_kind(TIMER_GEMM1, ctypes.byref(tot), ctypes.byref(n)), "ctn_timer_read_kind")
            counts[stride] = n.value
            assert tot.value > 0.0
    finally:
        lib.ctn_timer_enable(0, 0)
        lib.ctn_timer_set_stride(1)
    assert counts[1] == X * R                              # one bracket per block
    assert counts[3] == (3 * X * R + 2) // 3               # launches 0, 3, 6, 9 of 12
