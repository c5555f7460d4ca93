"""WAV file I/O for the data pipeline, without
librosa / soundfile (neither is installed in this image).

``read_wav(path, sr)`` returns what ``librosa.load(path, sr=sr)`` returns for
the PCM and IEEE-float WAV files of the wsj0-2mix corpus the reference reads
(src/data.py:254-256,287; src/preprocess.py:20): float32 samples, integer PCM
scaled by 2^-(bits-1) (libsndfile's read convention, which librosa uses through
soundfile), channels averaged to mono.  A file whose rate differs from ``sr``
is resampled with a polyphase filter (scipy.signal.resample_poly, same output
length ceil(n * sr / rate) as librosa); librosa's own resampler is not
reproduced sample for sample — the 8 kHz wsj0-2mix corpus needs none.

``write_wav(path, x, sr)`` writes mono PCM_16 like
``soundfile.write(path, x, sr, 'PCM_16')`` (src/separate.py:55-57): x * 32767
rounded to nearest (libsndfile's write convention), clipped to int16 (libsndfile
without clipping enabled wraps values beyond +-1 instead).
"""
from __future__ import annotations

import struct
from math import gcd

import numpy as np

WAVE_FORMAT_PCM, WAVE_FORMAT_IEEE_FLOAT, WAVE_FORMAT_EXTENSIBLE = 1, 3, 0xFFFE


class WavFormatError(ValueError):
    """Not a RIFF/WAVE file, or an encoding this reader does not decode."""


def _chunks(blob: bytes, path):
    if len(blob) < 12 or blob[:4] != b"RIFF" or blob[8:12] != b"WAVE":
        raise WavFormatError(f"{path}: not a RIFF/WAVE file")
    pos, fmt, payload = 12, None, None
    while pos + 8 <= len(blob):
        cid = blob[pos:pos + 4]
        size = struct.unpack_from("<I", blob, pos + 4)[0]
        body = blob[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            fmt = body
        elif cid == b"data":
            payload = body
        pos += 8 + size + (size & 1)
    if fmt is None or payload is None or len(fmt) < 16:
        raise WavFormatError(f"{path}: missing fmt or data chunk")
    return fmt, payload


def _format(fmt: bytes, path):
    tag, ch, rate, _, align, bits = struct.unpack_from("<HHIIHH", fmt, 0)
    if tag == WAVE_FORMAT_EXTENSIBLE and len(fmt) >= 26:
        tag = struct.unpack_from("<H", fmt, 24)[0]   # leading code of the SubFormat GUID
    if ch < 1 or align != ch * ((bits + 7) // 8):
        raise WavFormatError(f"{path}: inconsistent fmt chunk (channels={ch} align={align} bits={bits})")
    return tag, ch, rate, align, bits


def _decode(payload: bytes, tag, ch, align, bits, path) -> np.ndarray:
    n = len(payload) // align
    payload = payload[:n * align]
    if tag == WAVE_FORMAT_PCM:
        if bits == 8:
            x = (np.frombuffer(payload, np.uint8).astype(np.float32) - 128.0) / 128.0
        elif bits == 16:
            x = np.frombuffer(payload, "<i2").astype(np.float32) / 32768.0
        elif bits == 24:
            b = np.frombuffer(payload, np.uint8).reshape(-1, 3).astype(np.int32)
            v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
            v = np.where(v >= 1 << 23, v - (1 << 24), v)
            x = (v.astype(np.float64) / float(1 << 23)).astype(np.float32)
        elif bits == 32:
            x = (np.frombuffer(payload, "<i4").astype(np.float64) / 2147483648.0).astype(np.float32)
        else:
            raise WavFormatError(f"{path}: {bits}-bit PCM is not decoded")
    elif tag == WAVE_FORMAT_IEEE_FLOAT and bits in (32, 64):
        x = np.frombuffer(payload, "<f4" if bits == 32 else "<f8").astype(np.float32)
    else:
        raise WavFormatError(f"{path}: WAVE format tag {tag:#x} ({bits} bits) is not decoded")
    return x.reshape(n, ch)


def _read(path):
    with open(path, "rb") as f:
        blob = f.read()
    fmt, payload = _chunks(blob, path)
    return _format(fmt, path), payload


def read_wav_info(path):
    """-> (frames, rate, channels) of a WAV file."""
    (_, ch, rate, align, _), payload = _read(path)
    return len(payload) // align, rate, ch


def read_wav(path, sr=None):
    """-> (float32 mono samples [T], rate), as librosa.load(path, sr=sr)."""
    (tag, ch, rate, align, bits), payload = _read(path)
    x = _decode(payload, tag, ch, align, bits, path)
    x = x[:, 0].copy() if ch == 1 else x.mean(axis=1, dtype=np.float32)
    if sr is not None and int(sr) != rate:
        from scipy.signal import resample_poly
        g = gcd(int(sr), int(rate))
        x = resample_poly(x, int(sr) // g, int(rate) // g).astype(np.float32)
        rate = int(sr)
    return x, rate


def write_wav(path, x, sr):
    """Mono PCM_16 WAV, as soundfile.write(path, x, sr, 'PCM_16') (separate.py:55-57)."""
    x = np.asarray(x, dtype=np.float64).reshape(-1)
    data = np.clip(np.rint(x * 32767.0), -32768, 32767).astype("<i2").tobytes()
    sr = int(sr)
    hdr = (b"RIFF" + struct.pack("<I", 36 + len(data)) + b"WAVE" + b"fmt " +
           struct.pack("<IHHIIHH", 16, WAVE_FORMAT_PCM, 1, sr, sr * 2, 2, 16) + b"data" + struct.pack("<I", len(data)))
    with open(path, "wb") as f:
        f.write(hdr + data)
