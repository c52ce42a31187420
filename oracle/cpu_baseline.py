"""CPU baseline: the oracle's algorithm as a throughput-oriented fp32 NumPy/SciPy port.

TEST/BENCH INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).  Same stages and arithmetic
as fmcw_oracle.process (window -> range FFT -> corner turn -> Doppler window -> Doppler FFT
-> |X| -> 1-D OS-CFAR 16/4 in its counting form), but fp32 and vectorised over frames, with
scipy.fft's pocketfft using `workers` threads.  The reference itself has no software path
(VHDL + Xilinx FFT IP), so this "port" is the CPU number the GPU is
reported beside.
"""
from __future__ import annotations

import os
import time

import numpy as np
import scipy.fft as sfft

import fmcw_oracle as O


def process_frames(cube: np.ndarray, workers: int, cfar=O.Cfar1D()):
    """cube [F][chirp][sample] complex64 -> (map [F][range][doppler] f32, n_dets)."""
    f, nc, ns = cube.shape
    wr = O.window_f32(ns)
    wd = O.window_f32(nc)
    x = cube * wr[None, None, :]
    x = sfft.fft(x, axis=-1, workers=workers, overwrite_x=True)          # range FFT
    x = np.ascontiguousarray(np.swapaxes(x, -1, -2))                     # corner turn
    x *= wd[None, None, :]
    x = sfft.fft(x, axis=-1, workers=workers, overwrite_x=True)          # Doppler FFT
    mag = np.abs(x).astype(np.float32)
    offs = [-(cfar.guard + 1 + i) for i in range(cfar.ref)] + [cfar.guard + 1 + i for i in range(cfar.ref)]
    cnt = np.zeros(mag.shape, np.int8)
    a = np.float32(cfar.alpha)
    for o in offs:
        cnt += (a * np.roll(mag, -o, axis=-1)) >= mag
    det = cnt < (2 * cfar.ref - cfar.rank)
    return mag, int(det.sum())


def measure(ns: int, nc: int, make_frames, target_s: float = 12.0, max_frames: int = 2048,
            batch: int = 8, workers: int | None = None):
    """Time process_frames on batches of `batch` frames until ~target_s of CPU work."""
    workers = workers or min(16, os.cpu_count() or 1)
    frames = make_frames(batch)
    process_frames(frames[:1], workers)  # warm-up (plans, pages)
    done, t0 = 0, time.perf_counter()
    while done < max_frames:
        process_frames(frames, workers)
        done += batch
        if time.perf_counter() - t0 >= target_s:
            break
    dt = time.perf_counter() - t0
    return {"frames": done, "seconds": dt, "frames_per_s": done / dt, "workers": workers}
