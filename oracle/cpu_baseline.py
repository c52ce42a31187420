"""CPU baseline of bench.py: the oracle's algorithm timed on the host cores.

TEST/BENCH INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).  The reference has no software
path (VHDL + Xilinx FFT IP), so the CPU number the GPU is reported beside is
the build's own restatement (SURVEY.md 8d "CPU baseline"):

  C backend   oracle/fmcw_cpu.c (OpenMP, fp32 Stockham FFT, the oracle's CFAR definitions):
              single-core and all-core frames/s, median of >= 20 timed runs after a warm-up.
  NumPy port  process_frames below (scipy.fft with `workers` threads, 1-D CFAR in counting
              form): reported beside it for continuity with round 1.

Thread count: every CPU this process may run on (os.sched_getaffinity), capped by
OMP_NUM_THREADS when the environment sets it (the GPU box grants a job 16 CPUs and sets
OMP_NUM_THREADS=16; nproc there counts the whole machine).  All of it is reported.
"""
from __future__ import annotations

import os
import statistics
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


def threads_allowed() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return max(1, n)


def _median_runs(fn, runs: int, budget_s: float):
    fn()                                   # warm-up (pages, plans, thread pool)
    times = []
    t_end = time.perf_counter() + budget_s
    while len(times) < runs or (time.perf_counter() < t_end and len(times) < 4 * runs):
        t0 = time.perf_counter()
        fn()
        times.append(time.perf_counter() - t0)
        if len(times) >= runs and time.perf_counter() > t_end:
            break
    return statistics.median(times), len(times)


def measure_c(cube: np.ndarray, cfar, runs: int = 20, budget_s: float = 8.0) -> dict:
    """C backend on `cube` [F][rx][chirp][sample]: median seconds per run -> frames/s, at one
    thread and at threads_allowed() threads."""
    import cpu_backend as CB
    F = cube.shape[0]
    info = CB.host_info()
    nt = threads_allowed()
    out = {"frames_per_run": F, "threads_all": nt, **info}
    for key, th in (("single_core", 1), ("all_core", nt)):
        med, n = _median_runs(lambda: CB.process(cube, cfar, threads=th, want_map=False), runs, budget_s)
        out[key] = {"frames_per_s": F / med, "median_s": med, "runs": n, "threads": th}
    return out


def measure(ns: int, nc: int, make_frames, target_s: float = 12.0, max_frames: int = 2048,
            batch: int = 8, workers: int | None = None):
    """NumPy port: time process_frames on batches of `batch` frames until ~target_s."""
    workers = workers or threads_allowed()
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
