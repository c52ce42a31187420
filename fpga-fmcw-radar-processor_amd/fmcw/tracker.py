"""Track-while-scan tracker over detection lists (ctypes over fmcw_tws_*, include/fmcw.h).

Mirrors the tws_tracker entity (rtl/src/tws_tracker.vhd:9-40): the constructor takes its
generics by name, ``scan`` plays one COLLECT .. OUTPUT cycle over one frame's detections and
returns what the trk_* ports stream (firm and coasting tracks, track-file order) plus
active_tracks.  The library implements it in C++ on the host (csrc/tws_tracker.cpp).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L

TRACK_DTYPE = np.dtype([("id", np.uint16), ("status", np.uint8), ("quality", np.uint8),
                        ("range_q2", np.int32), ("doppler_q2", np.int32), ("vel_r", np.int32),
                        ("vel_d", np.int32), ("last_mag", np.uint32), ("age", np.uint32)])
STATUS_NAMES = {0: "FREE", 1: "TENT", 2: "FIRM", 3: "COAST"}


class TwsTracker:
    def __init__(self, MAX_TRACKS: int = 32, INIT_HITS: int = 2, COAST_MAX: int = 5,
                 ASSOC_GATE_R: int = 10, ASSOC_GATE_D: int = 5, ALPHA_GAIN: int = 128,
                 BETA_GAIN: int = 64, MAX_DETS: int = 64, rtl_compat: bool = False):
        self._lib = L.load()
        cfg = L.FmcwTwsConfig()
        self._lib.fmcw_tws_config_default(C.byref(cfg))
        cfg.max_tracks, cfg.max_dets, cfg.init_hits, cfg.coast_max = MAX_TRACKS, MAX_DETS, INIT_HITS, COAST_MAX
        cfg.gate_r, cfg.gate_d, cfg.alpha_q8, cfg.beta_q8 = ASSOC_GATE_R, ASSOC_GATE_D, ALPHA_GAIN, BETA_GAIN
        cfg.rtl_compat = int(bool(rtl_compat))
        self.cfg = cfg
        h = C.c_void_p()
        L.check(self._lib.fmcw_tws_create(C.byref(cfg), C.byref(h)))
        self._h = h
        self._out = (L.FmcwTrack * MAX_TRACKS)()
        self.active_tracks = 0

    def scan(self, dets) -> np.ndarray:
        """dets: structured array with fields range, doppler, mag (DET_DTYPE), or an (n, 3)
        array of (range, doppler, mag).  Returns TRACK_DTYPE records; sets active_tracks."""
        d = np.asarray(dets)
        n = len(d)
        buf = (L.FmcwDet * max(n, 1))()
        if n:
            if d.dtype.names:
                r, dd, m = d["range"], d["doppler"], d["mag"]
                fr = d["frame"] if "frame" in d.dtype.names else np.zeros(n, np.int64)
            else:
                r, dd, m, fr = d[:, 0], d[:, 1], d[:, 2], np.zeros(n, np.int64)
            for i in range(n):
                buf[i].frame, buf[i].range, buf[i].doppler = int(fr[i]), int(r[i]), int(dd[i])
                buf[i].mag, buf[i].threshold = float(m[i]), 0.0
        n_out, n_act = C.c_size_t(0), C.c_uint32(0)
        L.check(self._lib.fmcw_tws_scan(self._h, buf, n, self._out, len(self._out), C.byref(n_out),
                                         C.byref(n_act)))
        self.active_tracks = int(n_act.value)
        raw = C.string_at(C.addressof(self._out), n_out.value * C.sizeof(L.FmcwTrack))
        return np.frombuffer(raw, TRACK_DTYPE).copy()

    def close(self):
        if self._h:
            self._lib.fmcw_tws_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
