"""Host-side mirror of the reference's radar_core entity, backed by libfmcw.so on MI355X.

Reference interface (Aurellia-Beam/fpga-fmcw-radar-processor, rtl/src/radar_core.vhd):

  generics  N_RANGE, N_DOPPLER, CFAR_REF_R, CFAR_REF_D, CFAR_GUARD_R, CFAR_GUARD_D   (:12-19)
  in        s_axis_tdata {Q[31:16], I[15:0]}, tlast at sample N_RANGE-1 of each chirp (:25-29)
  control   mti_bypass, cfar_scale_ovr                                           (:47-49)
  out       det_tdata[16:0], det_range_bin[9:0], det_doppler_bin[6:0]             (:31-35)
  status    status_overflow (sticky)                                             (:51-55)

``RadarCore`` keeps those names and meanings: the CFAR generics are the os_cfar_2d
generics *as the RTL applies them* (os_cfar_2d.vhd:41-47, :119-146): CFAR_REF_R and
CFAR_GUARD_R size the window along the stream axis, which is Doppler, and CFAR_REF_D /
CFAR_GUARD_D along the line-buffer rows, which are range bins.  ``cfar="os1d"`` selects the
earlier 1-D core (rtl/old/radar_core_v3.vhd:373-381, os_cfar REF 8 / GUARD 2 / RANK 12 / x4).

Frames are whole CPIs: ``cube[frame][rx][chirp][sample]`` (the AXI stream with its tlast
framing, reshaped).  Outputs are per frame, range-major like the RTL's idx_proc counters
(radar_core.vhd:396-418); Doppler bin 0 is zero Doppler.

Errors are raised (FmcwError) with the library's status name; nothing falls back to CPU.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _lib as L

DET_DTYPE = np.dtype([("frame", "<u4"), ("range", "<u2"), ("doppler", "<u2"),
                      ("mag", "<f4"), ("threshold", "<f4")])
assert DET_DTYPE.itemsize == C.sizeof(L.FmcwDet) == 16

_IN_DTYPES = {"f32": (L.IN_F32, np.complex64), "f16": (L.IN_F16, np.float16),
              "i16": (L.IN_I16, np.int16)}


@dataclass
class RadarOutput:
    """What radar_core emits for a batch of frames."""
    dets: np.ndarray                 # structured DET_DTYPE, sorted by (frame, range, doppler)
    rd_map: Optional[np.ndarray]     # [frame][range][doppler] float32 (linear or dB), or None
    n_dets: int

    @property
    def det_tdata(self):            # radar_core.vhd:32 (CUT magnitude of each detection)
        return self.dets["mag"]

    @property
    def det_range_bin(self):        # :34
        return self.dets["range"]

    @property
    def det_doppler_bin(self):      # :35
        return self.dets["doppler"]

    # status words 2 / 3 (fmcw.h): samples saturated by the RTL-compat integer windows, and int16
    # spectrum words / canceller outputs clipped
    window_saturations: int = 0
    word_saturations: int = 0

    @property
    def status_overflow(self) -> bool:
        """The RTL's sticky flag (radar_core.vhd:447-456): set by the window multipliers'
        saturation (win1_saturation / win2_saturation, :451) only.  The canceller's output
        saturates silently in the RTL (doppler_notch.vhd:75-93), and this build's int16 word
        clipping is counted separately in `word_saturations`, an extension outside the flag."""
        return bool(self.window_saturations)


def pack_adc_words(i: np.ndarray, q: np.ndarray) -> np.ndarray:
    """32-bit AXI words {Q[31:16], I[15:0]} (rtl/src/tb_radar_core.vhd:115-118)."""
    i16 = np.asarray(i).astype(np.int16).view(np.uint16).astype(np.uint32)
    q16 = np.asarray(q).astype(np.int16).view(np.uint16).astype(np.uint32)
    return (q16 << 16) | i16


def adc_words_to_cube(words: np.ndarray, n_chirps: int, n_samples: int) -> np.ndarray:
    """AXI words -> int16 cube [..., chirp, sample, 2] (I, Q): the layout FMCW_IN_I16 reads."""
    w = np.asarray(words, dtype=np.uint32)
    iq = np.stack([(w & 0xFFFF).astype(np.uint16).view(np.int16),
                   (w >> 16).astype(np.uint16).view(np.int16)], axis=-1)
    return iq.reshape(iq.shape[:-2] + (n_chirps, n_samples, 2)) if iq.ndim > 2 else \
        iq.reshape(n_chirps, n_samples, 2)


class DeviceBuffer:
    """A device allocation owned through the C-ABI (no torch needed)."""

    def __init__(self, nbytes: int, device: int = 0):
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        L.check(L.load().fmcw_device_alloc(self.nbytes, C.byref(p), device))
        self.ptr = p.value

    def upload(self, arr: np.ndarray, offset: int = 0):
        a = np.ascontiguousarray(arr)
        assert offset + a.nbytes <= self.nbytes
        L.check(L.load().fmcw_memcpy(self.ptr + offset, a.ctypes.data, a.nbytes, 0))

    def download(self, dtype, shape, offset: int = 0) -> np.ndarray:
        out = np.empty(shape, dtype=dtype)
        assert offset + out.nbytes <= self.nbytes
        L.check(L.load().fmcw_memcpy(out.ctypes.data, self.ptr + offset, out.nbytes, 1))
        return out

    def copy_from(self, src: "DeviceBuffer", nbytes: int, src_offset: int = 0, dst_offset: int = 0):
        """Device-to-device copy (e.g. tiling a few frames into a large batch)."""
        assert src_offset + nbytes <= src.nbytes and dst_offset + nbytes <= self.nbytes
        L.check(L.load().fmcw_memcpy(self.ptr + dst_offset, src.ptr + src_offset, nbytes, 2))

    def free(self):
        if self.ptr:
            L.load().fmcw_device_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def _ptr(x):
    """(pointer, is_device) for numpy arrays, DeviceBuffers and torch CUDA tensors."""
    if x is None:
        return None, False
    if isinstance(x, DeviceBuffer):
        return x.ptr, True
    if hasattr(x, "data_ptr") and hasattr(x, "is_cuda"):
        if not x.is_contiguous():
            raise ValueError("tensor must be contiguous")
        return x.data_ptr(), bool(x.is_cuda)
    if isinstance(x, np.ndarray):
        if not x.flags["C_CONTIGUOUS"]:
            raise ValueError("array must be C-contiguous")
        return x.ctypes.data, False
    raise TypeError(f"unsupported buffer type {type(x)}")


class RadarCore:
    """MI355X radar_core: window -> range FFT -> corner turn -> Doppler window -> Doppler FFT ->
    magnitude (|X|, NCI over rx, or AMBM) -> OS-CFAR (1-D or 2-D) -> detection list."""

    def __init__(self, N_RANGE: int = 1024, N_DOPPLER: int = 128, N_RX: int = 1,
                 CFAR_REF_R: int = 4, CFAR_REF_D: int = 4, CFAR_GUARD_R: int = 2,
                 CFAR_GUARD_D: int = 1, cfar_scale_ovr: int = 0, cfar: str = "os2d",
                 cfar_rank_pct: int = 75, cfar_scales=(2, 4, 6),
                 cfar1d=(8, 2, 12, 4.0), in_dtype: str = "f32", window: str = "hamming",
                 magnitude: str = "abs", map_kind: str = "linear", max_frames: int = 1,
                 chunk_frames: int = 0, device: int = 0, mti_bypass: bool = True,
                 NOTCH_MODE: int = 2, compat_rtl=(), range_shift: int = 0, spectrum: str = "f32",
                 det_capacity: int = 0):
        """mti_bypass / NOTCH_MODE mirror radar_core's u_mti (radar_core.vhd:329-338, port
        :48).  The RTL port defaults to '0' (MTI on); this mirror defaults to bypass because
        the north-star path and BASELINE configs exclude MTI and tb_radar_core bypasses it
        (rtl/src/tb_radar_core.vhd:66).

        compat_rtl: RTL-compat arithmetic (fmcw.h fmcw_compat): any of "cfar" (17-bit integer
        CFAR, os_cfar.vhd:132 / os_cfar_2d.vhd:189-199) and "mti" (int16 saturating canceller,
        doppler_notch.vhd:73-93).  range_shift: range spectrum scaled by 2^-range_shift (the
        FFT IP's fixed scaling schedule), so that the 16-bit spectrum words of the compat MTI and
        of window="q15_rtl" (integer windows on both axes) are meaningful.
        spectrum: "f32", "f16" or "s48", the element type of the internal corner-turned spectrum
        (fmcw.h fmcw_spectrum_dtype): "f16" halves its HBM traffic, map within 2e-3; "s48" takes 6
        bytes per point, map within the 1e-4 of "f32" -- a chirp group of a range bin shares one
        8-bit exponent: quads of 23-bit significands at n_range <= 1024 (adjacent chirps up to
        n_range 512, chirps n_doppler / 16 apart at 1024), pairs of 22-bit significands n_doppler /
        16 apart above; needs n_doppler >= 64 and MTI off.
        det_capacity: detection records one call can hold (fmcw.h fmcw_config.det_capacity); 0 =
        every cell of max_frames frames, so no call loses a detection its det_cap has room for."""
        lib = L.load()
        cfg = L.default_config()
        cfg.mti_mode = L.MTI_OFF if mti_bypass else {2: L.MTI_2PULSE, 3: L.MTI_3PULSE}[NOTCH_MODE]
        cfg.n_range, cfg.n_doppler, cfg.n_rx = N_RANGE, N_DOPPLER, N_RX
        cfg.in_dtype = _IN_DTYPES[in_dtype][0]
        cfg.window = {"hamming": L.WIN_HAMMING, "none": L.WIN_NONE, "q15_rtl": L.WIN_Q15_RTL}[window]
        cfg.mag_mode = {"abs": L.MAG_ABS, "ambm": L.MAG_AMBM}[magnitude]
        cfg.map_kind = {"linear": L.MAP_LINEAR, "db": L.MAP_DB}[map_kind]
        cfg.cfar_kind = {"none": L.CFAR_NONE, "os1d": L.CFAR_OS1D, "os2d": L.CFAR_OS2D}[cfar]
        cfg.cfar1d_ref, cfg.cfar1d_guard, cfg.cfar1d_rank, cfg.cfar1d_alpha = cfar1d
        # os_cfar_2d generics as the RTL applies them (see module docstring)
        cfg.cfar2d_ref_doppler, cfg.cfar2d_guard_doppler = CFAR_REF_R, CFAR_GUARD_R
        cfg.cfar2d_ref_range, cfg.cfar2d_guard_range = CFAR_REF_D, CFAR_GUARD_D
        cfg.cfar2d_rank_pct = cfar_rank_pct
        cfg.cfar2d_scale_min, cfg.cfar2d_scale_nom, cfg.cfar2d_scale_max = cfar_scales
        cfg.cfar2d_scale_override = cfar_scale_ovr
        cfg.max_frames, cfg.chunk_frames, cfg.device_id = max_frames, chunk_frames, device
        flags = {"cfar": L.COMPAT_CFAR, "mti": L.COMPAT_MTI}
        cfg.compat_rtl = compat_rtl if isinstance(compat_rtl, int) else \
            sum(flags[k] for k in set(compat_rtl))
        cfg.range_shift = range_shift
        cfg.spectrum_dtype = {"f32": L.SPEC_F32, "f16": L.SPEC_F16, "s48": L.SPEC_S48}[spectrum]
        cfg.det_capacity = det_capacity
        self.cfg = cfg
        self.in_dtype = in_dtype
        self.device = device
        h = C.c_void_p()
        L.check(lib.fmcw_create(C.byref(cfg), C.byref(h)))
        self._h = h
        self._lib = lib

    # -- sizes ---------------------------------------------------------------------------
    @property
    def frame_shape(self):
        c = self.cfg
        return (c.n_rx, c.n_doppler, c.n_range)

    def frame_input_bytes(self) -> int:
        c = self.cfg
        return c.n_rx * c.n_doppler * c.n_range * (8 if self.in_dtype == "f32" else 4)

    def _n_frames(self, cube) -> int:
        nbytes = cube.nbytes if isinstance(cube, (np.ndarray, DeviceBuffer)) else \
            cube.numel() * cube.element_size()
        n, rem = divmod(nbytes, self.frame_input_bytes())
        if rem or n < 1:
            raise ValueError(f"cube of {nbytes} B is not a whole number of frames "
                             f"({self.frame_input_bytes()} B each)")
        return n

    # -- whole path ----------------------------------------------------------------------
    def process(self, cube, want_map: bool = True, det_cap: Optional[int] = None) -> RadarOutput:
        """Synchronous: host numpy (or device) cube -> detections (+ map) on the host."""
        nf = self._n_frames(cube)
        c = self.cfg
        rd_map = np.empty((nf, c.n_range, c.n_doppler), np.float32) if want_map else None
        cap = det_cap if det_cap is not None else nf * 4096
        dets = np.empty(cap, DET_DTYPE)
        n = C.c_size_t(0)
        cp, _ = _ptr(cube)
        rc = self._lib.fmcw_process(self._h, cp, nf, _ptr(rd_map)[0], dets.ctypes.data if cap else None,
                                    cap, C.byref(n), None)
        if rc == L.FMCW_EDETCAP and det_cap is None:
            return self.process(cube, want_map, det_cap=int(n.value))
        L.check(rc)
        return RadarOutput(dets=dets[: n.value].copy(), rd_map=rd_map, n_dets=int(n.value),
                           window_saturations=self.info("window_saturations"),
                           word_saturations=self.info("word_saturations"))

    def enqueue(self, cube, n_frames: int, rd_map=None, dets=None, det_cap: int = 0,
                n_dets=None, stream: int = 0):
        """Asynchronous, device pointers only (DeviceBuffer / torch CUDA tensors / ints).  n_dets:
        FMCW_STATUS_WORDS (4) uint32 device words: found, lost, window / word saturations."""
        def p(x):
            return x if isinstance(x, int) or x is None else _ptr(x)[0]
        L.check(self._lib.fmcw_enqueue(self._h, p(cube), n_frames, p(rd_map), p(dets), det_cap,
                                       p(n_dets), stream or None))

    # -- stages --------------------------------------------------------------------------
    def range_ct(self, cube_dev, spec_dev, n_frames: int, stream: int = 0):
        """window + range FFT + corner turn -> spec[frame][rx][range][chirp] complex64."""
        L.check(self._lib.fmcw_range_ct(self._h, _ptr(cube_dev)[0] if not isinstance(cube_dev, int) else cube_dev,
                                        n_frames, _ptr(spec_dev)[0] if not isinstance(spec_dev, int) else spec_dev,
                                        stream or None))

    def cfar(self, map_dev, n_frames: int, dets_dev, det_cap: int, n_dets_dev, stream: int = 0):
        """OS-CFAR of this core's kind on a caller-supplied [frame][range][doppler] map."""
        p = lambda x: x if isinstance(x, int) else _ptr(x)[0]  # noqa: E731
        L.check(self._lib.fmcw_cfar(self._h, p(map_dev), n_frames, p(dets_dev), det_cap,
                                    p(n_dets_dev), stream or None))

    # -- profiling -----------------------------------------------------------------------
    def set_profiling(self, on: bool):
        L.check(self._lib.fmcw_set_profiling(self._h, 1 if on else 0))

    def kernel_times(self):
        ms = (C.c_double * L.K_COUNT)()
        n = (C.c_uint64 * L.K_COUNT)()
        L.check(self._lib.fmcw_kernel_times(self._h, ms, n))
        return {L.KERNEL_NAMES[k]: (ms[k], n[k]) for k in range(L.K_COUNT)}

    def set_param(self, key: str, value: int) -> None:
        """fmcw_set_param (tuning; results never depend on it): "cfar2d_steps" = 2-D CFAR steps
        per strip, 0 = the library's cost model."""
        k = {"cfar2d_steps": L.PARAM_CFAR2D_STEPS}[key]
        L.check(self._lib.fmcw_set_param(self._h, k, int(value)))

    def info(self, key: str) -> int:
        """fmcw_get_info: "chunk" (frames per K1 -> K2 chunk), "range_kernel" (0 k_range,
        2 k_range_sq, 3 k_range_px; 1 retired), "window_saturations" / "word_saturations" (status
        words 2 / 3 of the last process() call; window_saturations is the sticky status_overflow
        of radar_core.vhd:447-456 as a count), "cfar2d_steps" (strip length of the last 2-D CFAR
        launch)."""
        k = {"chunk": L.INFO_CHUNK, "range_kernel": L.INFO_RANGE_KERNEL,
             "window_saturations": L.INFO_WINDOW_SATURATIONS,
             "word_saturations": L.INFO_WORD_SATURATIONS, "cfar2d_steps": L.INFO_CFAR2D_STEPS}[key]
        v = C.c_int64(0)
        L.check(self._lib.fmcw_get_info(self._h, k, C.byref(v)))
        return int(v.value)

    def reset_kernel_times(self):
        L.check(self._lib.fmcw_reset_kernel_times(self._h))

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            self._lib.fmcw_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def magnitude(iq_dev, out_dev, n: int, mode: str = "abs", stream: int = 0):
    """magnitude_calc stage (rtl/src/magnitude_calc.vhd): |X| or AMBM on n complex64 values."""
    p = lambda x: x if isinstance(x, int) else _ptr(x)[0]  # noqa: E731
    L.check(L.load().fmcw_magnitude(p(iq_dev), p(out_dev), n,
                                    {"abs": L.MAG_ABS, "ambm": L.MAG_AMBM}[mode], stream or None))
