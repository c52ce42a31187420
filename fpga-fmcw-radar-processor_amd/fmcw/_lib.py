"""ctypes binding of libfmcw.so (include/fmcw.h).

This is the binding a maintainer of the reference's Python tooling (model/) would add:
plain ctypes over the C-ABI, no compiled Python extension.  The library is built in-tree
(``make -C fpga-fmcw-radar-processor_amd``) and loaded from ``lib/libfmcw.so`` next to this
package; it never falls back to anything else -- a missing library is an error.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parent.parent          # fpga-fmcw-radar-processor_amd/
LIB_PATH = Path(os.environ.get("FMCW_LIB", PKG_ROOT / "lib" / "libfmcw.so"))
HEADER_PATH = PKG_ROOT.parent / "include" / "fmcw.h"

# enums (fmcw.h)
FMCW_OK, FMCW_EINVAL, FMCW_ENOMEM, FMCW_EHIP, FMCW_EDETCAP, FMCW_ENODEV = 0, -1, -2, -3, -4, -5
IN_F32, IN_F16, IN_I16 = 0, 1, 2
WIN_NONE, WIN_HAMMING, WIN_Q15_RTL = 0, 1, 2
MAG_ABS, MAG_AMBM = 0, 1
MAP_LINEAR, MAP_DB = 1, 2
CFAR_NONE, CFAR_OS1D, CFAR_OS2D = 0, 1, 2
MTI_OFF, MTI_2PULSE, MTI_3PULSE = 0, 2, 3
COMPAT_CFAR, COMPAT_MTI = 1, 2
SPEC_F32, SPEC_F16, SPEC_S48 = 0, 1, 2
COMM_ID_BYTES = 128
K_RANGE, K_DOPPLER, K_CFAR2D, K_COMPACT, K_COUNT = 0, 1, 2, 3, 4
KERNEL_NAMES = ("k_range", "k_doppler", "k_cfar", "k_compact")
INFO_CHUNK, INFO_RANGE_KERNEL, INFO_WINDOW_SATURATIONS, INFO_WORD_SATURATIONS = 4, 6, 7, 8
INFO_CFAR2D_STEPS = 9
PARAM_CFAR2D_STEPS = 1   # fmcw_set_param keys
# FMCW_INFO_RANGE_KERNEL 0..3 (1 = round 2's k_range2, retired in ABI 6)
RANGE_KERNELS = ("k_range", "k_range2 (retired)", "k_range_sq", "k_range_px")
STATUS_WORDS = 4      # FMCW_STATUS_WORDS: n_dets_dev = found, lost, window / word saturations

STATUS_NAMES = {0: "FMCW_OK", -1: "FMCW_EINVAL", -2: "FMCW_ENOMEM", -3: "FMCW_EHIP",
                -4: "FMCW_EDETCAP", -5: "FMCW_ENODEV"}


class FmcwConfig(C.Structure):
    _fields_ = [
        ("n_range", C.c_uint32), ("n_doppler", C.c_uint32), ("n_rx", C.c_uint32),
        ("in_dtype", C.c_int32), ("window", C.c_int32), ("mag_mode", C.c_int32),
        ("map_kind", C.c_int32), ("cfar_kind", C.c_int32), ("mti_mode", C.c_int32),
        ("cfar1d_ref", C.c_uint32), ("cfar1d_guard", C.c_uint32), ("cfar1d_rank", C.c_uint32),
        ("cfar1d_alpha", C.c_float),
        ("cfar2d_ref_range", C.c_uint32), ("cfar2d_guard_range", C.c_uint32),
        ("cfar2d_ref_doppler", C.c_uint32), ("cfar2d_guard_doppler", C.c_uint32),
        ("cfar2d_rank_pct", C.c_uint32), ("cfar2d_scale_min", C.c_uint32),
        ("cfar2d_scale_nom", C.c_uint32), ("cfar2d_scale_max", C.c_uint32),
        ("cfar2d_scale_override", C.c_uint32),
        ("max_frames", C.c_uint32), ("chunk_frames", C.c_uint32), ("device_id", C.c_int32),
        ("compat_rtl", C.c_uint32), ("range_shift", C.c_uint32), ("spectrum_dtype", C.c_int32),
        ("det_capacity", C.c_uint32),
    ]


class FmcwDet(C.Structure):
    _fields_ = [("frame", C.c_uint32), ("range", C.c_uint16), ("doppler", C.c_uint16),
                ("mag", C.c_float), ("threshold", C.c_float)]


class FmcwTwsConfig(C.Structure):
    _fields_ = [("max_tracks", C.c_uint32), ("max_dets", C.c_uint32), ("init_hits", C.c_uint32),
                ("coast_max", C.c_uint32), ("gate_r", C.c_uint32), ("gate_d", C.c_uint32),
                ("alpha_q8", C.c_uint32), ("beta_q8", C.c_uint32), ("rtl_compat", C.c_int32)]


class FmcwTrack(C.Structure):
    _fields_ = [("id", C.c_uint16), ("status", C.c_uint8), ("quality", C.c_uint8),
                ("range_q2", C.c_int32), ("doppler_q2", C.c_int32), ("vel_r", C.c_int32),
                ("vel_d", C.c_int32), ("last_mag", C.c_uint32), ("age", C.c_uint32)]


# every symbol include/fmcw.h declares, with its ctypes signature
_VP, _SZ, _I, _U32P = C.c_void_p, C.c_size_t, C.c_int, C.POINTER(C.c_uint32)
SIGNATURES = {
    "fmcw_version": (C.c_char_p, []),
    "fmcw_abi_version": (_I, []),
    "fmcw_last_error": (C.c_char_p, []),
    "fmcw_config_default": (None, [C.POINTER(FmcwConfig)]),
    "fmcw_create": (_I, [C.POINTER(FmcwConfig), C.POINTER(_VP)]),
    "fmcw_destroy": (_I, [_VP]),
    "fmcw_enqueue": (_I, [_VP, _VP, _SZ, _VP, _VP, _SZ, _VP, _VP]),
    "fmcw_process": (_I, [_VP, _VP, _SZ, _VP, _VP, _SZ, C.POINTER(_SZ), _VP]),
    "fmcw_range_ct": (_I, [_VP, _VP, _SZ, _VP, _VP]),
    "fmcw_magnitude": (_I, [_VP, _VP, _SZ, _I, _VP]),
    "fmcw_cfar": (_I, [_VP, _VP, _SZ, _VP, _SZ, _VP, _VP]),
    "fmcw_set_profiling": (_I, [_VP, _I]),
    "fmcw_get_info": (_I, [_VP, _I, C.POINTER(C.c_int64)]),
    "fmcw_set_param": (_I, [_VP, _I, C.c_int64]),
    "fmcw_kernel_times": (_I, [_VP, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]),
    "fmcw_reset_kernel_times": (_I, [_VP]),
    "fmcw_device_alloc": (_I, [_SZ, C.POINTER(_VP), _I]),
    "fmcw_device_free": (_I, [_VP]),
    "fmcw_memcpy": (_I, [_VP, _VP, _SZ, _I]),
    "fmcw_device_count": (_I, [C.POINTER(_I)]),
    "fmcw_comm_unique_id": (_I, [_VP]),
    "fmcw_comm_create": (_I, [_VP, _I, _I, _I, _SZ, C.POINTER(_VP)]),
    "fmcw_comm_destroy": (_I, [_VP]),
    "fmcw_comm_info": (_I, [_VP, C.POINTER(_I), C.POINTER(_I), C.POINTER(_I), C.POINTER(_SZ)]),
    "fmcw_gather_dets": (_I, [_VP, _VP, _SZ, _VP, C.c_uint32, _VP, _VP, _I, _VP]),
    "fmcw_comm_fail_next_alloc_for_test": (_I, [_I]),
    "fmcw_comm_check_decide_for_test": (_I, [C.POINTER(C.c_uint64), _I, _SZ]),
    "fmcw_gather_pack_for_test": (_I, [_VP, _SZ, _VP, _SZ, C.c_uint32, _VP, _VP]),
    "fmcw_gather_compact_for_test": (_I, [_VP, _I, _SZ, _VP, _VP, _VP]),
    "fmcw_tws_config_default": (None, [C.POINTER(FmcwTwsConfig)]),
    "fmcw_tws_create": (_I, [C.POINTER(FmcwTwsConfig), C.POINTER(_VP)]),
    "fmcw_tws_destroy": (_I, [_VP]),
    "fmcw_tws_scan": (_I, [_VP, _VP, _SZ, C.POINTER(FmcwTrack), _SZ, C.POINTER(_SZ), _U32P]),
}

_lib = None


class FmcwError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{STATUS_NAMES.get(code, code)}: {msg}")
        self.code = code


def load() -> C.CDLL:
    """Load libfmcw.so (once).  Raises if it has not been built -- no fallback exists."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise FileNotFoundError(
                f"{LIB_PATH} not built: run `make -C {PKG_ROOT}` or __graft_entry__.build()")
        lib = C.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def check(code: int) -> int:
    if code != FMCW_OK:
        raise FmcwError(code, load().fmcw_last_error().decode(errors="replace"))
    return code


def default_config() -> FmcwConfig:
    cfg = FmcwConfig()
    load().fmcw_config_default(C.byref(cfg))
    return cfg


def device_count() -> int:
    n = C.c_int(0)
    load().fmcw_device_count(C.byref(n))
    return n.value
