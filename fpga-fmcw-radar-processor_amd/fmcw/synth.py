"""Synthetic chirp cubes shaped like the reference's testbench stimuli.

x[c, n] = sum_k A_k exp(2 pi i (r_k n / Ns + d_k c / Nc)) + uniform noise, rounded and
saturated to the int16 ADC range, then stored as complex64 / f16 / int16 pairs.

  recipe "two_targets"  rtl/old/tb_radar_core.vhd:37-44, :106-129: targets (r = 100 Ns/1024,
                        d = +5, A = 8000) and (r = 500 Ns/1024, d = -10, A = 5000), noise +-20.
                        (Per-frame RNG: numpy PCG64, seed = seed + frame.)
  recipe "random_target" rtl/src/tb_radar_core.vhd:88-107: one target per frame at
                        r = U*0.88 Ns + 0.05 Ns, d = U*(100/128) Nc, A = 20000, noise +-100.
  phase offset per rx   2 pi rx 0.25.

Used by bench.py and the tests; the product path never generates data itself.
"""
from __future__ import annotations

import numpy as np


def _targets(recipe: str, ns: int, nc: int, rng: np.random.Generator):
    if recipe == "two_targets":
        return [(100.0 * ns / 1024, 5.0, 8000.0), (500.0 * ns / 1024, -10.0, 5000.0)], 20.0
    if recipe == "random_target":
        r = rng.uniform() * 0.88 * ns + 0.05 * ns
        d = rng.uniform() * (100.0 / 128.0) * nc
        return [(r, d, 20000.0)], 100.0
    raise ValueError(recipe)


def frame(ns: int, nc: int, n_rx: int = 1, recipe: str = "two_targets", seed: int = 1234,
          dtype: str = "f32") -> np.ndarray:
    """One frame [rx][chirp][sample] as complex64 (f32), or [rx][chirp][sample][2] f16/int16."""
    rng = np.random.Generator(np.random.PCG64(seed))
    tg, noise = _targets(recipe, ns, nc, rng)
    n = np.arange(ns)[None, :]
    c = np.arange(nc)[:, None]
    out = np.empty((n_rx, nc, ns), np.complex128)
    for rx in range(n_rx):
        x = np.zeros((nc, ns), np.complex128)
        for (r, d, a) in tg:
            x += a * np.exp(2j * np.pi * (r * n / ns + d * c / nc + 0.25 * rx))
        x += noise * (rng.uniform(-1, 1, (nc, ns)) + 1j * rng.uniform(-1, 1, (nc, ns)))
        out[rx] = x
    i = np.clip(np.rint(out.real), -32768, 32767)
    q = np.clip(np.rint(out.imag), -32768, 32767)
    if dtype == "f32":
        return (i + 1j * q).astype(np.complex64)
    if dtype == "i16":
        return np.stack([i, q], axis=-1).astype(np.int16)
    if dtype == "f16":
        return (np.stack([i, q], axis=-1) / 32768.0).astype(np.float16)
    raise ValueError(dtype)


def frames(n_frames: int, ns: int, nc: int, n_rx: int = 1, recipe: str = "two_targets",
           seed: int = 1234, dtype: str = "f32") -> np.ndarray:
    return np.stack([frame(ns, nc, n_rx, recipe, seed + f, dtype) for f in range(n_frames)])


def golden_chirp_frame(samples: np.ndarray, n_chirps: int = 128, n_samples: int = 256) -> np.ndarray:
    """BASELINE config 1 framing: data/golden_input_chirp.txt holds 2000 I/Q
    samples of one tone; a frame is n_chirps identical chirps = samples[0:n_samples]
    (a stationary target: all energy in Doppler bin 0)."""
    s = np.asarray(samples)
    z = (s[:n_samples, 0] + 1j * s[:n_samples, 1]).astype(np.complex64)
    return np.broadcast_to(z, (1, n_chirps, n_samples)).copy()
