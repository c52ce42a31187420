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


def ieee_uniform(seed1: int, seed2: int, n: int):
    """IEEE 1076.2 MATH_REAL.UNIFORM (L'Ecuyer's combined multiplicative LCG, the RNG of every
    reference testbench): n draws from (seed1, seed2); returns (draws float64, seed1, seed2)."""
    out = np.empty(n, np.float64)
    s1, s2 = int(seed1), int(seed2)
    for k in range(n):
        s1 = (40014 * s1) % 2147483563     # = Schrage's form K := S/53668; 40014 (S - 53668 K) - 12211 K
        s2 = (40692 * s2) % 2147483399
        z = s1 - s2
        if z < 1:
            z += 2147483562
        out[k] = z * 4.656613e-10
    return out, s1, s2


def tb_radar_core_v3_cpis(n_cpi: int = 2, ns: int = 1024, nc: int = 128) -> np.ndarray:
    """The stimulus of rtl/old/tb_radar_core.vhd:86-141 (the testbench of radar_core_v3, the
    likely producer of data/radar_output.txt): targets (range 100, Doppler +5.0,
    amplitude 8000) and (500, -10.0, 5000) (:37-44), noise +-20 from UNIFORM with seeds (1, 1)
    drawn I then Q per sample (:121-124), VHDL integer() rounding (nearest, halves away from
    zero) and int16 saturation (:126-129), chirp-major, n_cpi CPIs.  Returns int16
    [cpi][chirp][sample][2] = (I, Q), the 32-bit AXI word {Q, I} (:131)."""
    n = np.arange(ns, dtype=np.float64)[None, :]
    c = np.arange(nc, dtype=np.float64)[:, None]
    ph1 = 2.0 * np.pi * (100.0 * n / ns + 5.0 * c / nc)
    ph2 = 2.0 * np.pi * (500.0 * n / ns + -10.0 * c / nc)
    i_t = 8000.0 * np.cos(ph1) + 5000.0 * np.cos(ph2)
    q_t = 8000.0 * np.sin(ph1) + 5000.0 * np.sin(ph2)
    draws, _, _ = ieee_uniform(1, 1, 2 * n_cpi * nc * ns)
    draws = draws.reshape(n_cpi, nc, ns, 2)
    i_acc = i_t[None] + 20.0 * (draws[..., 0] - 0.5) * 2.0
    q_acc = q_t[None] + 20.0 * (draws[..., 1] - 0.5) * 2.0

    def vhdl_int(x):
        return np.sign(x) * np.floor(np.abs(x) + 0.5)
    i = np.clip(vhdl_int(i_acc), -32768, 32767)
    q = np.clip(vhdl_int(q_acc), -32768, 32767)
    return np.stack([i, q], axis=-1).astype(np.int16)


def golden_chirp_frame(samples: np.ndarray, n_chirps: int = 128, n_samples: int = 256) -> np.ndarray:
    """BASELINE config 1 framing: data/golden_input_chirp.txt holds 2000 I/Q
    samples of one tone; a frame is n_chirps identical chirps = samples[0:n_samples]
    (a stationary target: all energy in Doppler bin 0)."""
    s = np.asarray(samples)
    z = (s[:n_samples, 0] + 1j * s[:n_samples, 1]).astype(np.complex64)
    return np.broadcast_to(z, (1, n_chirps, n_samples)).copy()
