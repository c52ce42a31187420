"""ctypes wrapper of oracle/lib/libfmcw_cpu.so (oracle/fmcw_cpu.c).

TEST/BENCH INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg and tests/test_cpu_backend.py.
The product path never imports this.  Build: ``make -C oracle`` (or __graft_entry__.build()).
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

import fmcw_oracle as O

LIB = Path(__file__).resolve().parent / "lib" / "libfmcw_cpu.so"


class _Cfar(C.Structure):
    _fields_ = [("kind", C.c_int), ("ref1", C.c_int), ("guard1", C.c_int), ("rank1", C.c_int),
                ("alpha", C.c_float), ("ref_r", C.c_int), ("guard_r", C.c_int), ("ref_d", C.c_int),
                ("guard_d", C.c_int), ("rank_pct", C.c_int), ("smin", C.c_int), ("snom", C.c_int),
                ("smax", C.c_int), ("override_", C.c_int)]


_lib = None


def load():
    global _lib
    if _lib is None:
        if not LIB.exists():
            raise FileNotFoundError(f"{LIB} not built: make -C {LIB.parent.parent}")
        lib = C.CDLL(str(LIB))
        lib.fmcw_cpu_process.restype = C.c_size_t
        lib.fmcw_cpu_process.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(_Cfar),
                                         C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        lib.fmcw_cpu_cfar.restype = C.c_size_t
        lib.fmcw_cpu_cfar.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(_Cfar), C.c_void_p,
                                      C.c_size_t, C.c_int]
        lib.fmcw_cpu_max_threads.restype = C.c_int
        _lib = lib
    return _lib


def _cfar(cfar) -> _Cfar:
    c = _Cfar()
    if isinstance(cfar, O.Cfar1D):
        c.kind, c.ref1, c.guard1, c.rank1, c.alpha = 1, cfar.ref, cfar.guard, cfar.rank, cfar.alpha
    elif isinstance(cfar, O.Cfar2D):
        c.kind = 2
        c.ref_r, c.guard_r, c.ref_d, c.guard_d = (cfar.ref_range, cfar.guard_range, cfar.ref_doppler,
                                                  cfar.guard_doppler)
        c.rank_pct, c.smin, c.snom, c.smax = cfar.rank_pct, cfar.scale_min, cfar.scale_nom, cfar.scale_max
        c.override_ = cfar.scale_override
    return c


def process(cube: np.ndarray, cfar=None, threads: int = 0, want_map: bool = True, cap: int = 1 << 20):
    """cube complex64 [F][rx][chirp][sample] (or [F][chirp][sample]) -> (map [F][range][doppler]
    float32 or None, detections O.DET_DTYPE, n found)."""
    x = np.ascontiguousarray(cube, np.complex64)
    if x.ndim == 3:
        x = x[:, None]
    F, nrx, nc, ns = x.shape
    m = np.empty((F, ns, nc), np.float32) if want_map else None
    dets = np.empty(cap, O.DET_DTYPE)
    c = _cfar(cfar)
    n = load().fmcw_cpu_process(x.ctypes.data, F, ns, nc, nrx, C.byref(c),
                                m.ctypes.data if m is not None else None, dets.ctypes.data, cap, threads)
    return m, dets[: min(n, cap)].copy(), int(n)


def cfar(maps: np.ndarray, cfar, threads: int = 0, cap: int = 1 << 22):
    """The oracle's CFAR (cfar_os1d / cfar_os2d semantics, bit-exact) on float32 maps
    [F][range][doppler] -> detections O.DET_DTYPE (frame = index in maps)."""
    m = np.ascontiguousarray(maps, np.float32)
    if m.ndim == 2:
        m = m[None]
    F, ns, nc = m.shape
    dets = np.empty(cap, O.DET_DTYPE)
    c = _cfar(cfar)
    n = load().fmcw_cpu_cfar(m.ctypes.data, F, ns, nc, C.byref(c), dets.ctypes.data, cap, threads)
    if n > cap:
        raise RuntimeError(f"{n} detections > cap {cap}")
    return dets[:n].copy()


def max_threads() -> int:
    return int(load().fmcw_cpu_max_threads())


def host_info() -> dict:
    """nproc, the CPUs this process may run on, OMP_NUM_THREADS and the CPU model string."""
    model = ""
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    return {"nproc": os.cpu_count() or 1, "affinity": affinity,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "cpu_model": model}
