"""fmcw -- MI355X-native FMCW range-Doppler + OS-CFAR hot path (host side).

The compute runs in libfmcw.so (hand-written HIP for gfx950, include/fmcw.h); this package
is the thin host shim the reference's Python tooling (model/) would call, mirroring the
reference's radar_core interface (rtl/src/radar_core.vhd:11-57).
"""
from ._lib import FmcwError, load, device_count, LIB_PATH, HEADER_PATH  # noqa: F401
from .radar_core import RadarCore, RadarOutput, DeviceBuffer, DET_DTYPE, magnitude  # noqa: F401
from .radar_core import pack_adc_words, adc_words_to_cube  # noqa: F401
from .tracker import TwsTracker, TRACK_DTYPE  # noqa: F401
from . import synth, formats  # noqa: F401

__all__ = ["RadarCore", "RadarOutput", "DeviceBuffer", "DET_DTYPE", "FmcwError", "load",
           "device_count", "magnitude", "TwsTracker", "TRACK_DTYPE", "synth", "formats", "pack_adc_words", "adc_words_to_cube"]
