"""BSS Eval v3 source metrics (SDR / SIR / SAR) without mir_eval.

The reference's evaluate.py computes SDRi with ``mir_eval.separation.
bss_eval_sources`` (evaluate.py:10,90-105), a dependency this image does not
have.  This is a from-scratch restatement of that published
algorithm — E. Vincent, R. Gribonval, C. Fevotte, "Performance measurement in
blind audio source separation", IEEE TASLP 14(4), 2006, as implemented by
mir_eval 0.6/0.7 (``bss_eval_sources`` with ``compute_permutation=True``):

* each estimate is decomposed against the references with time-invariant
  distortion filters of ``flen`` = 512 taps: s_true (the reference, zero-padded
  by flen-1), e_spat (its filtered version minus itself), e_interf (what the
  other references' filters add), e_artif (the rest of the estimate);
* the projections solve the normal equations G c = D, where G holds the inner
  products of all delayed references and D those with the estimate, both taken
  from FFT cross-correlations;
* SDR = 10 log10(|s_true+e_spat|^2 / |e_interf+e_artif|^2),
  SIR = 10 log10(|s_true+e_spat|^2 / |e_interf|^2),
  SAR = 10 log10(|s_true+e_spat+e_interf|^2 / |e_artif|^2);
* the estimate-to-source assignment is the permutation with the largest mean SIR.

Parity with mir_eval is UNPINNED (mir_eval is not installed and no fixture of
its output exists in the reference); tests/test_pipeline.py checks the
metric's defining properties instead (exact estimates, filtered estimates,
additive noise at a known SNR, permutation recovery).
"""
from __future__ import annotations

import itertools

import numpy as np
from scipy.linalg import toeplitz
from scipy.signal import fftconvolve

FLEN = 512


def _project(refs: np.ndarray, est: np.ndarray, flen: int) -> np.ndarray:
    """Least-squares projection of est onto all flen-tap filtered versions of refs
    [nsrc, T] -> [T + flen - 1]."""
    nsrc, T = refs.shape
    refs_p = np.hstack((refs, np.zeros((nsrc, flen - 1))))
    est_p = np.hstack((est, np.zeros(flen - 1)))
    n_fft = int(2 ** np.ceil(np.log2(T + flen - 1.0)))
    sf = np.fft.fft(refs_p, n=n_fft, axis=1)
    sef = np.fft.fft(est_p, n=n_fft)
    G = np.zeros((nsrc * flen, nsrc * flen))
    for i in range(nsrc):
        for j in range(i, nsrc):
            ssf = np.real(np.fft.ifft(sf[i] * np.conj(sf[j])))
            ss = toeplitz(np.hstack((ssf[0], ssf[-1:-flen:-1])), r=ssf[:flen])
            G[i * flen:(i + 1) * flen, j * flen:(j + 1) * flen] = ss
            G[j * flen:(j + 1) * flen, i * flen:(i + 1) * flen] = ss.T
    D = np.zeros(nsrc * flen)
    for i in range(nsrc):
        ssef = np.real(np.fft.ifft(sf[i] * np.conj(sef)))
        D[i * flen:(i + 1) * flen] = np.hstack((ssef[0], ssef[-1:-flen:-1]))
    try:
        C = np.linalg.solve(G, D).reshape(flen, nsrc, order="F")
    except np.linalg.LinAlgError:
        C = np.linalg.lstsq(G, D, rcond=None)[0].reshape(flen, nsrc, order="F")
    sproj = np.zeros(T + flen - 1)
    for i in range(nsrc):
        sproj += fftconvolve(C[:, i], refs_p[i])[:T + flen - 1]
    return sproj


def _decompose(refs: np.ndarray, est: np.ndarray, j: int, flen: int):
    """(s_true, e_spat, e_interf, e_artif) of estimate `est` against reference j."""
    T = est.size
    s_true = np.hstack((refs[j], np.zeros(flen - 1)))
    e_spat = _project(refs[j:j + 1], est, flen) - s_true
    e_interf = _project(refs, est, flen) - s_true - e_spat
    e_artif = -s_true - e_spat - e_interf
    e_artif[:T] += est
    return s_true, e_spat, e_interf, e_artif


def _db(num: float, den: float) -> float:
    return np.inf if den == 0 else 10.0 * np.log10(num / den)


def _criteria(s_true, e_spat, e_interf, e_artif):
    s_filt = s_true + e_spat
    sdr = _db(np.sum(s_filt ** 2), np.sum((e_interf + e_artif) ** 2))
    sir = _db(np.sum(s_filt ** 2), np.sum(e_interf ** 2))
    sar = _db(np.sum((s_filt + e_interf) ** 2), np.sum(e_artif ** 2))
    return sdr, sir, sar


def bss_eval_sources(reference_sources, estimated_sources, compute_permutation=True, flen=FLEN):
    """reference_sources, estimated_sources [nsrc, T] (or [T]) -> (sdr, sir, sar, perm),
    each [nsrc]; perm[j] = the estimate assigned to reference j (mir_eval's popt)."""
    refs = np.atleast_2d(np.asarray(reference_sources, dtype=np.float64))
    ests = np.atleast_2d(np.asarray(estimated_sources, dtype=np.float64))
    if refs.shape != ests.shape:
        raise ValueError(f"shape mismatch: references {refs.shape}, estimates {ests.shape}")
    if refs.shape[1] < flen:
        raise ValueError(f"signals of {refs.shape[1]} samples are shorter than the {flen}-tap filters")
    if np.any(np.all(refs == 0, axis=1)):
        raise ValueError("a reference source is all zeros (undefined SDR)")
    n = refs.shape[0]
    if not compute_permutation:
        out = np.array([_criteria(*_decompose(refs, ests[j], j, flen)) for j in range(n)])
        return out[:, 0], out[:, 1], out[:, 2], np.arange(n)
    sdr, sir, sar = (np.empty((n, n)) for _ in range(3))
    for je in range(n):
        for jt in range(n):
            sdr[je, jt], sir[je, jt], sar[je, jt] = _criteria(*_decompose(refs, ests[je], jt, flen))
    perms = list(itertools.permutations(range(n)))
    dum = np.arange(n)
    best = perms[int(np.argmax([np.mean(sir[list(p), dum]) for p in perms]))]
    idx = (list(best), dum)
    return sdr[idx], sir[idx], sar[idx], np.asarray(best)
