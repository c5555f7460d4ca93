"""ctypes binding of libctn_hip.so (include/ctn.h).

The shared library is the product: every forward/backward of the drop-in
modules runs through it.  Loading is lazy; a missing or unloadable library
raises ``CtnLibraryError`` — there is no fallback path.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CTN_HIP_LIB", os.path.join(_HERE, "libctn_hip.so"))
ABI_VERSION = 12

DTYPE_F32, DTYPE_BF16 = 0, 1
NORM_GLN, NORM_CLN, NORM_BN = 0, 1, 2
MASK_RELU, MASK_SOFTMAX = 0, 1
ROW_TILE = 128

c_int32, c_void_p, c_size_t = ctypes.c_int32, ctypes.c_void_p, ctypes.c_size_t


class CtnLibraryError(RuntimeError):
    """libctn_hip.so is missing, stale or failed a call."""


# ----------------------------------------------------------------------------
# C structs (mirror include/ctn.h)
# ----------------------------------------------------------------------------
class TBlockDesc(ctypes.Structure):
    _fields_ = [(n, c_int32) for n in
                ("M", "K", "Kp", "B", "H", "P", "dilation", "causal", "norm_type", "dtype")]


_TB_PARAM_NAMES = ("w1", "alpha1", "gamma1", "beta1", "wd", "alpha2", "gamma2", "beta2", "w2")


class TBlockParams(ctypes.Structure):
    _fields_ = ([(n, c_void_p) for n in _TB_PARAM_NAMES + ("w1_bf16", "w2_bf16", "w1t_bf16", "w2t_bf16",
                                                           "bn_mean1", "bn_var1", "bn_mean2", "bn_var2")] +
                [("bn_training", c_int32), ("bn_momentum1", ctypes.c_float), ("bn_momentum2", ctypes.c_float),
                 ("bn_eps1", ctypes.c_float), ("bn_eps2", ctypes.c_float)] +
                [(n, c_void_p) for n in ("w1_frag", "w2_frag", "w1t_frag", "w2t_frag")])


class WeightPack(ctypes.Structure):
    _fields_ = [("src", c_void_p), ("rows", c_int32), ("cols", c_int32), ("dst", c_void_p), ("dst_t", c_void_p),
                ("dst_frag", c_void_p), ("dst_t_frag", c_void_p)]


class TBlockGrads(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in _TB_PARAM_NAMES]


class TBlockSaved(ctypes.Structure):
    _fields_ = [("h1", c_void_p), ("d", c_void_p), ("stats", c_void_p)]


class CodecDesc(ctypes.Structure):
    _fields_ = [(n, c_int32) for n in ("M", "T", "K", "Kp", "N", "L", "B", "C", "mask_type", "dtype")]


class PitDesc(ctypes.Structure):
    _fields_ = [(n, c_int32) for n in ("M", "C", "T")]


MASK_IDENTITY = 2


class RowsDesc(ctypes.Structure):
    _fields_ = [(n, c_int32) for n in ("M", "K", "Kp", "C", "dtype")]


class StreamDesc(ctypes.Structure):
    _fields_ = [(n, c_int32) for n in ("M", "K", "N", "L", "B", "H", "P", "C", "norm", "mask_type")]


class StreamBlockParams(ctypes.Structure):
    """ctn_stream_block_params (include/ctn.h, ABI v7)."""
    _fields_ = [("dilation", c_int32), ("ring_frames", c_int32)] + [
        (n, c_void_p) for n in ("w1_t", "alpha1", "norm1_a", "norm1_b", "wd", "alpha2", "norm2_a", "norm2_b", "w2_t",
                                "ring")]


class StreamModel(ctypes.Structure):
    """ctn_stream_model (include/ctn.h, ABI v7): `blocks` points to a host array."""
    _fields_ = [(n, c_void_p) for n in ("U", "gamma0", "beta0", "wb_t", "wm_t", "V", "blocks")] + [
        ("nblocks", c_int32)]


class OptSegment(ctypes.Structure):
    _fields_ = [("param", c_void_p), ("grad", c_void_p), ("exp_avg", c_void_p), ("exp_avg_sq", c_void_p),
                ("numel", ctypes.c_int64)]


class OptChunk(ctypes.Structure):
    _fields_ = [("seg", c_int32), ("len", ctypes.c_uint32), ("off", ctypes.c_int64)]


class AdamHParams(ctypes.Structure):
    _fields_ = [("lr", ctypes.c_float), ("beta1", ctypes.c_float), ("beta2", ctypes.c_float),
                ("eps", ctypes.c_float), ("weight_decay", ctypes.c_float), ("step", c_int32)]


# ----------------------------------------------------------------------------
_lib = None
_lock = threading.Lock()

_SIGS = {
    "ctn_abi_version": (ctypes.c_int, []),
    "ctn_last_error": (ctypes.c_char_p, []),
    "ctn_padded_frames": (ctypes.c_int, [ctypes.c_int]),
    "ctn_tblock_stats_floats": (ctypes.c_int, [c_void_p]),
    "ctn_tblock_workspace_bytes": (c_size_t, [c_void_p, ctypes.c_int]),
    "ctn_tblock_forward": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                          c_void_p, c_size_t, c_void_p]),
    "ctn_tblock_backward": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                           c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "ctn_tblock_backward_split": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                                 c_void_p, c_void_p, c_void_p, c_size_t, c_void_p, c_void_p]),
    "ctn_tblock_partials_bytes": (c_size_t, [c_void_p]),
    "ctn_tblock_deferred_workspace_bytes": (c_size_t, [c_void_p]),
    "ctn_tblock_backward_deferred": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                                    c_void_p, c_void_p, c_void_p, c_size_t, c_void_p, c_size_t,
                                                    c_void_p]),
    "ctn_tblock_reduce_grads": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, ctypes.c_int, c_void_p]),
    "ctn_encoder_workspace_bytes": (c_size_t, [c_void_p, ctypes.c_int]),
    "ctn_encoder_forward": (ctypes.c_int, [c_void_p] + [c_void_p] * 8 + [c_void_p, c_size_t, c_void_p]),
    "ctn_encoder_backward": (ctypes.c_int, [c_void_p] + [c_void_p] * 13 + [c_void_p, c_size_t, c_void_p]),
    "ctn_decoder_workspace_bytes": (c_size_t, [c_void_p, ctypes.c_int]),
    "ctn_decoder_forward": (ctypes.c_int, [c_void_p] + [c_void_p] * 6 + [c_void_p, c_size_t, c_void_p]),
    "ctn_decoder_backward": (ctypes.c_int, [c_void_p] + [c_void_p] * 10 + [c_void_p, c_size_t, c_void_p]),
    "ctn_pit_workspace_bytes": (c_size_t, [c_void_p]),
    "ctn_pit_forward": (ctypes.c_int, [c_void_p] + [c_void_p] * 8 + [c_void_p, c_size_t, c_void_p]),
    "ctn_pit_backward": (ctypes.c_int, [c_void_p] + [c_void_p] * 7 + [c_void_p]),
    "ctn_pack_weights": (ctypes.c_int, [c_void_p, ctypes.c_int, c_void_p]),
    "ctn_opt_plan": (ctypes.c_int, [c_void_p, ctypes.c_int, c_void_p, ctypes.c_int]),
    "ctn_grad_clip_norm": (ctypes.c_int, [c_void_p, c_void_p, ctypes.c_int, ctypes.c_float, c_void_p, c_void_p,
                                          c_void_p]),
    "ctn_adam_step": (ctypes.c_int, [c_void_p, c_void_p, ctypes.c_int, c_void_p, c_void_p]),
    "ctn_opt_write_segments": (ctypes.c_int, [c_void_p, c_void_p, ctypes.c_int, c_void_p]),
    "ctn_adam_step_dev": (ctypes.c_int, [c_void_p, c_void_p, ctypes.c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "ctn_layernorm_workspace_bytes": (c_size_t, [c_void_p, ctypes.c_int, ctypes.c_int]),
    "ctn_layernorm_forward": (ctypes.c_int, [c_void_p, ctypes.c_int] + [c_void_p] * 5 + [c_void_p, c_size_t,
                                                                                       c_void_p]),
    "ctn_layernorm_backward": (ctypes.c_int, [c_void_p, ctypes.c_int] + [c_void_p] * 7 + [c_void_p, c_size_t,
                                                                                        c_void_p]),
    "ctn_prelu_workspace_bytes": (c_size_t, [c_void_p]),
    "ctn_prelu_forward": (ctypes.c_int, [c_void_p] * 5),
    "ctn_prelu_backward": (ctypes.c_int, [c_void_p] * 6 + [c_void_p, c_size_t, c_void_p]),
    "ctn_depthwise_workspace_bytes": (c_size_t, [c_void_p, ctypes.c_int]),
    "ctn_depthwise_forward": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int] + [c_void_p] * 4),
    "ctn_depthwise_backward": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int] + [c_void_p] * 5 +
                               [c_void_p, c_size_t, c_void_p]),
    "ctn_conv1x1_workspace_bytes": (c_size_t, [c_void_p, ctypes.c_int, ctypes.c_int]),
    "ctn_conv1x1_forward": (ctypes.c_int, [c_void_p, ctypes.c_int] + [c_void_p] * 3 + [c_void_p, c_size_t, c_void_p]),
    "ctn_conv1x1_backward": (ctypes.c_int, [c_void_p, ctypes.c_int] + [c_void_p] * 5 + [c_void_p, c_size_t,
                                                                                      c_void_p]),
    "ctn_mask_forward": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, c_void_p, c_void_p, c_void_p]),
    "ctn_mask_backward": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int, c_void_p, c_void_p, c_void_p,
                                         c_void_p]),
    "ctn_stream_encode": (ctypes.c_int, [c_void_p, c_void_p, ctypes.c_int64] + [c_void_p] * 6 + [c_void_p]),
    "ctn_stream_block": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int] + [c_void_p] * 12 +
                         [c_void_p]),
    "ctn_stream_decode": (ctypes.c_int, [c_void_p] + [c_void_p] * 8 + [c_void_p]),
    "ctn_stream_workspace_bytes": (c_size_t, [c_void_p]),
    "ctn_stream_call": (ctypes.c_int, [c_void_p, c_void_p, ctypes.c_int64, c_void_p, ctypes.c_int64] + [c_void_p] * 4 +
                        [c_size_t, c_void_p]),
    "ctn_timer_enable": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "ctn_timer_set_stride": (ctypes.c_int, [ctypes.c_int]),
    "ctn_copy_bytes": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_void_p]),
    "ctn_mfma_peak": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p]),
    "ctn_timer_read": (ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]),
    "ctn_timer_enable_mask": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_int]),
    "ctn_timer_read_kind": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_int)]),
    "ctn_device_status": (ctypes.c_int, [c_void_p, ctypes.POINTER(ctypes.c_uint32), ctypes.c_int]),
    "ctn_tblock_plan": (ctypes.c_int, [c_void_p, ctypes.c_int, ctypes.c_char_p, c_size_t]),
}

EXPORTED_SYMBOLS = tuple(_SIGS)


def load(path: str = LIB_PATH):
    """Load (once) and return the CDLL; raises CtnLibraryError if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise CtnLibraryError(
                f"HIP extension not built: {path} is missing (run `make` or "
                f"`python -c 'import __graft_entry__ as g; g.build()'`)")
        try:
            lib = ctypes.CDLL(path)
        except OSError as e:
            raise CtnLibraryError(f"cannot load {path}: {e}") from e
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        v = lib.ctn_abi_version()
        if v != ABI_VERSION:
            raise CtnLibraryError(f"{path} has ABI {v}, expected {ABI_VERSION}; rebuild")
        _lib = lib
        return lib


def check(rc: int, what: str):
    if rc != 0:
        msg = load().ctn_last_error().decode(errors="replace")
        raise CtnLibraryError(f"{what} failed (status {rc}): {msg}")


def padded_frames(K: int) -> int:
    return ((K + ROW_TILE - 1) // ROW_TILE) * ROW_TILE


def ptr(t):
    return None if t is None else t.data_ptr()


def stream_handle(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.float32:
        return DTYPE_F32
    if dt == torch.bfloat16:
        return DTYPE_BF16
    raise CtnLibraryError(f"unsupported activation dtype {dt} (float32 or bfloat16)")


def workspace(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)


def require_device(t: torch.Tensor, what: str):
    if not t.is_cuda:
        raise CtnLibraryError(
            f"{what}: the MI355X build runs on a ROCm device only (got a {t.device} tensor); "
            f"the CPU restatement in oracle/ is test infrastructure, not a fallback")
