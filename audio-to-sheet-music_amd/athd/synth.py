"""Synthetic 44.1 kHz stereo mixtures (SURVEY.md §8(d) "Synthetic inputs").

MUSDB18 is not available offline, so benches and parity tests use seeded signals with non-degenerate spectra:
a sum of 8 harmonic tones (random f0 in 55-880 Hz, decaying partial amplitudes, per-channel gain/phase) plus
pink-ish noise (white noise through a one-pole low-pass mix), scaled to RMS 0.1 and clipped to +-1.
"""
from __future__ import annotations

import numpy as np
from scipy.signal import lfilter

SAMPLE_RATE = 44100


def synthetic_mixture(length: int, seed: int = 1234, sr: int = SAMPLE_RATE) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    t = np.arange(length, dtype=np.float64) / sr
    out = np.zeros((2, length), dtype=np.float64)
    for _ in range(8):
        f0 = rng.uniform(55.0, 880.0)
        amp = rng.uniform(0.2, 1.0)
        for h in range(1, 6):
            if f0 * h >= sr / 2:
                break
            ph = rng.uniform(0, 2 * np.pi, size=2)
            g = rng.uniform(0.5, 1.0, size=2)
            out += (amp / h) * g[:, None] * np.sin(2 * np.pi * f0 * h * t[None, :] + ph[:, None])
    white = rng.standard_normal(size=(2, length))
    pink = lfilter([0.02], [1.0, -0.98], white, axis=1)     # one-pole low-pass
    noise = 0.5 * white + 5.0 * pink
    out = out / (np.sqrt(np.mean(out ** 2)) + 1e-12) + 0.3 * noise / (np.sqrt(np.mean(noise ** 2)) + 1e-12)
    out = 0.1 * out / (np.sqrt(np.mean(out ** 2)) + 1e-12)
    return np.clip(out, -1.0, 1.0).astype(np.float32)


def synthetic_batch(B: int, length: int, seed0: int = 1234) -> np.ndarray:
    return np.stack([synthetic_mixture(length, seed0 + i) for i in range(B)])
