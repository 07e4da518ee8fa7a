"""Seeded synthetic signals shared by the golden generator (oracle/gen_goldens.py) and the tests.

TEST INFRASTRUCTURE ONLY.  Nothing here touches the reference; the generator feeds these to the
reference, the tests regenerate them instead of storing megabytes of audio in tests/golden/.
"""
from __future__ import annotations

import numpy as np


def reference_audio(n: int, seed: int) -> np.ndarray:
    """Voice-like test tone: two partials, a 3 Hz amplitude envelope and a little noise (fp32)."""
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 44100.0
    x = 0.4 * np.sin(2 * np.pi * 220 * t) + 0.2 * np.sin(2 * np.pi * 1375 * t + 0.3)
    x = x * (0.6 + 0.4 * np.sin(2 * np.pi * 3 * t)) + 0.05 * rng.standard_normal(n)
    return x.astype(np.float32)


def codec_codes(n_codebooks: int, semantic_codebook_size: int, codebook_size: int, T: int,
                seed: int) -> np.ndarray:
    """(1, n_codebooks + 1, T) int64 codes: row 0 semantic, rows 1.. residual."""
    rng = np.random.default_rng(seed)
    c = np.zeros((1, n_codebooks + 1, T), dtype=np.int64)
    c[0, 0] = rng.integers(0, semantic_codebook_size, T)
    c[0, 1:] = rng.integers(0, codebook_size, (n_codebooks, T))
    return c


def stft_logmag_error_db(x: np.ndarray, ref: np.ndarray, ffts=(512, 1024, 2048), floor_db=-60.0):
    """Multi-resolution STFT log-magnitude error: for each FFT size (Hann window,
    hop n/4), the mean over time-frequency bins of |20 log10 |X| - 20 log10 |R||, counting only bins
    whose reference magnitude is within `floor_db` of the reference's peak at that resolution;
    returns the mean over resolutions in dB."""
    x = np.asarray(x, np.float64).ravel()
    ref = np.asarray(ref, np.float64).ravel()
    errs = []
    for n in ffts:
        hop = n // 4
        if ref.size < n:
            continue
        w = np.hanning(n)
        idx = np.arange(0, ref.size - n + 1, hop)[:, None] + np.arange(n)[None]
        X = np.abs(np.fft.rfft(x[idx] * w, axis=1))
        R = np.abs(np.fft.rfft(ref[idx] * w, axis=1))
        floor = R.max() * 10 ** (floor_db / 20)
        keep = R > floor
        d = np.abs(20 * np.log10(np.maximum(X, floor)) - 20 * np.log10(np.maximum(R, floor)))
        errs.append(float(d[keep].mean()))
    return float(np.mean(errs))
