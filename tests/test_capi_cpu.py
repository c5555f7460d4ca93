"""C-ABI library checks that need no GPU: it loads, reports its ABI, exports
every symbol include/ctn.h declares, and validates arguments (error codes and
messages) before touching the device."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "ctn.h")


@pytest.fixture(scope="module")
def lib():
    import ctn_lib as L
    if not os.path.exists(L.LIB_PATH):
        pytest.fail(f"{L.LIB_PATH} not built (run make / __graft_entry__.build())")
    return L.load()


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ctn_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = declared_functions()
    for must in ("ctn_tblock_forward", "ctn_tblock_backward", "ctn_encoder_forward", "ctn_encoder_backward",
                 "ctn_decoder_forward", "ctn_decoder_backward", "ctn_pit_forward", "ctn_pit_backward"):
        assert must in names


def test_every_declared_symbol_exported(lib):
    import ctn_lib as L
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert set(declared_functions()) == set(L.EXPORTED_SYMBOLS), "ctypes signature table out of sync with ctn.h"


def test_abi_and_padding(lib):
    import ctn_lib as L
    assert lib.ctn_abi_version() == L.ABI_VERSION
    assert lib.ctn_padded_frames(3199) == 3200
    assert lib.ctn_padded_frames(128) == 128
    assert lib.ctn_padded_frames(7999) == 8064


def _desc(**kw):
    import ctn_lib as L
    d = dict(M=2, K=3199, Kp=3200, B=256, H=512, P=3, dilation=4, causal=0, norm_type=0, dtype=1)
    d.update(kw)
    return L.TBlockDesc(**d)


def test_tblock_validation(lib):
    import ctn_lib as L
    ok = _desc()
    assert lib.ctn_tblock_workspace_bytes(ctypes.byref(ok), 0) > 0
    assert lib.ctn_tblock_workspace_bytes(ctypes.byref(ok), 1) > lib.ctn_tblock_workspace_bytes(ctypes.byref(ok), 0)
    assert lib.ctn_tblock_stats_floats(ctypes.byref(ok)) == 4 * 2
    assert lib.ctn_tblock_stats_floats(ctypes.byref(_desc(norm_type=1))) == 4 * 2 * 3200
    bn = _desc(norm_type=2)                         # BatchNorm: per-channel statistics
    assert lib.ctn_tblock_stats_floats(ctypes.byref(bn)) == 4 * bn.H
    assert lib.ctn_tblock_workspace_bytes(ctypes.byref(bn), 1) > 0
    assert lib.ctn_tblock_workspace_bytes(ctypes.byref(_desc(norm_type=3)), 0) == 0
    cases = [(_desc(Kp=3199), L.CtnLibraryError, "multiple of 128"),
             (_desc(P=2), None, "odd P"),
             (_desc(B=100), None, "multiples of 8")]
    for d, _, msg in cases:
        assert lib.ctn_tblock_workspace_bytes(ctypes.byref(d), 0) == 0
        rc = lib.ctn_tblock_forward(ctypes.byref(d), None, None, None, None, None, 0, None)
        assert rc in (1, 2)
        assert msg in lib.ctn_last_error().decode()


def test_forward_rejects_null_and_small_workspace(lib):
    import ctn_lib as L
    d = _desc()
    p = L.TBlockParams()
    sv = L.TBlockSaved()
    assert lib.ctn_tblock_forward(ctypes.byref(d), ctypes.byref(p), None, None, ctypes.byref(sv), None, 0, None) == 1
    assert lib.ctn_pit_forward(None, None, None, None, None, None, None, None, None, None, 0, None) == 1
    pd = L.PitDesc(2, 17, 100)
    assert lib.ctn_pit_workspace_bytes(ctypes.byref(pd)) == 0          # C > 16 unsupported
    pd = L.PitDesc(2, 8, 100)
    assert lib.ctn_pit_workspace_bytes(ctypes.byref(pd)) > 0           # C! = 40,320 permutations


def test_codec_validation(lib):
    import ctn_lib as L
    good = L.CodecDesc(M=2, T=32000, K=3199, Kp=3200, N=256, L=20, B=256, C=2, mask_type=0, dtype=1)
    assert lib.ctn_encoder_workspace_bytes(ctypes.byref(good), 1) > 0
    assert lib.ctn_decoder_workspace_bytes(ctypes.byref(good), 1) > 0
    bad = L.CodecDesc(M=2, T=32000, K=3000, Kp=3072, N=256, L=20, B=256, C=2, mask_type=0, dtype=1)
    assert lib.ctn_encoder_workspace_bytes(ctypes.byref(bad), 0) == 0
    rc = lib.ctn_encoder_forward(ctypes.byref(bad), *([None] * 8), None, 0, None)
    assert rc == 1 and "K=3000" in lib.ctn_last_error().decode()


def test_timer_off_by_default(lib):
    tot, n = ctypes.c_double(1.0), ctypes.c_int(7)
    assert lib.ctn_timer_read(ctypes.byref(tot), ctypes.byref(n)) == 0
    assert n.value == 0 and tot.value == 0.0


def test_timer_stride_validation(lib):
    assert lib.ctn_timer_set_stride(0) != 0
    assert "stride" in lib.ctn_last_error().decode()
    assert lib.ctn_timer_set_stride(8) == 0
    assert lib.ctn_timer_set_stride(1) == 0


def test_copy_validation(lib):
    """ctn_copy_bytes (bench calibration copy) checks sizes and alignment before launching."""
    buf = ctypes.create_string_buffer(64)
    p = ctypes.addressof(buf)
    assert lib.ctn_copy_bytes(None, None, 16, 1, 0, None) == 1
    assert lib.ctn_copy_bytes(p, p, 20, 1, 0, None) == 1       # not a multiple of 16
    assert "16-byte" in lib.ctn_last_error().decode()
    assert lib.ctn_copy_bytes(p, p, 16, 0, 0, None) == 1       # no workgroups
    assert lib.ctn_copy_bytes(p, p, 16, 1, 4, None) == 1       # unknown flag


def test_pack_weights_validation(lib):
    """ctn_pack_weights checks its table before launching anything: an entry needs a
    destination, and the fragment-order copies need rows and cols in multiples of 32."""
    import ctn_lib as L
    assert lib.ctn_pack_weights(None, 0, None) == 0
    empty = (L.WeightPack * 1)(L.WeightPack(16, 64, 64, None, None, None, None))
    assert lib.ctn_pack_weights(empty, 1, None) == 1
    assert "no destination" in lib.ctn_last_error().decode()
    ragged = (L.WeightPack * 1)(L.WeightPack(16, 40, 64, None, None, 256, None))
    assert lib.ctn_pack_weights(ragged, 1, None) == 1
    assert "multiples of 32" in lib.ctn_last_error().decode()
    ragged_t = (L.WeightPack * 1)(L.WeightPack(16, 64, 72, None, None, None, 256))
    assert lib.ctn_pack_weights(ragged_t, 1, None) == 1


def test_device_code_has_no_packed_fp32(tmp_path):
    """The library's gfx950 code objects contain no packed-FP32 VALU instructions
    (v_pk_fma/mul/add_f32): on gfx950 a packed instruction that takes a source half through
    op_sel/op_sel_hi right after the VALU that wrote that register occasionally reads the
    stale value when another wave on the SIMD is busy, and the compiler inserts no wait
    state for it (tools/microbench/pk_hazard.hip).  The Makefile builds with
    the packed-fp32-ops target feature off; this guards against a build without it."""
    import re
    import shutil
    import subprocess
    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    if not os.path.exists(objdump):
        pytest.skip("llvm-objdump not available")
    lib = os.path.join(ROOT, "conv-tasnet_amd", "libctn_hip.so")
    if not os.path.exists(lib):
        pytest.skip("libctn_hip.so not built")
    shutil.copy(lib, tmp_path / "lib.so")
    subprocess.run([objdump, "--offloading", "lib.so"], cwd=tmp_path, check=True, capture_output=True)
    objs = [p for p in os.listdir(tmp_path) if "gfx950" in p]
    assert objs, "no gfx950 code object in the library"
    pk = re.compile(r"\bv_pk_(fma|mul|add)_f32\b")
    n_pk = n_mfma = 0
    for o in objs:
        txt = subprocess.run([objdump, "-d", o], cwd=tmp_path, check=True, capture_output=True, text=True).stdout
        n_pk += len(pk.findall(txt))
        n_mfma += txt.count("v_mfma_")
    assert n_mfma > 0, "disassembly found no MFMA: the check itself is broken"
    assert n_pk == 0, f"{n_pk} packed-FP32 instructions in the device code"


def _plan(lib, backward, **kw):
    buf = ctypes.create_string_buffer(256)
    assert lib.ctn_tblock_plan(ctypes.byref(_desc(**kw)), backward, buf, 256) == 0
    return dict(kv.split("=") for kv in buf.value.decode().split(","))


def test_tblock_plan_bench_shape_and_2gb_fallback(lib):
    """The persistent kernels (weight-stationary GEMMs, wave-specialised dual GEMM,
    wave-item depthwise kernels) address their tiles with 32-bit offsets: at 2^21 frame
    rows (M*Kp*512*2 bytes = 2 GiB) the launch must fall back to the tiled kernels
    (ADVICE r04), while the bench shape takes the persistent ones."""
    fwd, bwd = _plan(lib, 0, M=32), _plan(lib, 1, M=32)
    assert fwd == {"gemm1": "ws", "dw_fwd": "wave", "gemm2": "ws"}, fwd
    assert bwd["pairA"] == "dual_ws" and bwd["dw_bwd"] == "wave" and bwd["gx"] == "ws_n1bwd", bwd
    big = dict(M=656, K=3199, Kp=3200)        # 656 * 3200 = 2,099,200 rows >= 2^21
    fwd, bwd = _plan(lib, 0, **big), _plan(lib, 1, **big)
    assert fwd == {"gemm1": "rows", "dw_fwd": "lane", "gemm2": "rows"}, fwd
    assert bwd["pairA"] not in ("dual_ws", "dual", "ws+cols") and bwd["dw_bwd"] == "lane", bwd
    assert "gx" not in bwd or bwd["gx"] != "ws_n1bwd", bwd
    just_below = dict(M=655, K=3199, Kp=3200)  # 2,096,000 rows
    assert _plan(lib, 1, **just_below)["pairA"] == "dual_ws"


def test_pit_speaker_range(lib):
    """ctn_pit_workspace_bytes: 1..16 speakers (C <= 10 enumerated, 11..16 by assignment),
    0 bytes (unsupported) beyond."""
    import ctn_lib as L
    for C, ok in ((1, True), (8, True), (9, True), (16, True), (17, False)):
        n = lib.ctn_pit_workspace_bytes(ctypes.byref(L.PitDesc(4, C, 1000)))
        assert (n > 0) == ok, (C, n)


def test_mfma_peak_validation(lib):
    """ctn_mfma_peak (bench calibration microbenchmark) checks its arguments before launching."""
    buf = ctypes.create_string_buffer(64)
    p = ctypes.addressof(buf)
    assert lib.ctn_mfma_peak(0, 1, 1, None, None, None) == 1          # no output
    assert lib.ctn_mfma_peak(2, 1, 1, p, None, None) == 1             # unknown shape
    assert "shape" in lib.ctn_last_error().decode()
    assert lib.ctn_mfma_peak(0, 0, 1, p, None, None) == 1             # no workgroups
    assert lib.ctn_mfma_peak(1, 1, 0, p, None, None) == 1             # no iterations
