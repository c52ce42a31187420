"""CPU oracle for the FMCW range-Doppler + OS-CFAR hot path.

TEST INFRASTRUCTURE ONLY.  This module is the *checker*: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.
The product path (``fpga-fmcw-radar-processor_amd/``) never imports, links or
falls back to anything in ``oracle/``.

What it restates (reference = Aurellia-Beam/fpga-fmcw-radar-processor, VHDL RTL):

  stage                     reference (file:line)                         here
  ------------------------  --------------------------------------------  -----------------------
  ADC word {Q[31:16],I}     rtl/src/tb_radar_core.vhd:115-118             cube[..., chirp, sample]
  Hamming window (half ROM) rtl/src/window_multiplier.vhd:34-49, 97-102   hamming_table()
  Q15 window (compat)       rtl/src/window_multiplier.vhd:126-158         window_q15_rtl()
  range FFT (fwd, natural)  rtl/src/radar_core.vhd:247, 303-316           range_ct()
  corner turn               rtl/src/corner_turner.vhd:79-80               range_ct() (transpose)
  Doppler window + FFT      rtl/src/radar_core.vhd:340-364                doppler_fft()
  magnitude (AMBM compat)   rtl/src/magnitude_calc.vhd:57-81              ambm()
  |X|, NCI, log-mag         SURVEY.md 8a-R7; model/visualize_radar_targets.py:468   magnitude(), log_mag()
  1-D OS-CFAR 16/4          rtl/old/os_cfar.vhd:98-144, radar_core_v3.vhd:373-381   cfar_os1d()
  2-D OS-CFAR 128 refs      rtl/src/os_cfar_2d.vhd:140-217, radar_core.vhd:376-382  cfar_os2d()
  detection emission        rtl/src/radar_core.vhd:396-418                detections()

Parity status (see DESIGN.md "Oracle"):
  * The reference's FFT is the Xilinx LogiCORE FFT v9.1 (16-bit block floating
    point, block exponent discarded at radar_core.vhd:310).  Its bit-accurate C
    model may not be executed here (recorded denial), and no VHDL
    simulator exists, so FFT *values* are pinned against the fp64 DFT definition
    (numpy.fft) and the golden chirp's spectral peak, not against the IP:
    "parity unpinned" at the IP boundary.
  * Pinned by the reference's own known-answer tests / fixtures:
    magnitude KAT (rtl/src/tb_magnitude_calc.vhd:49-73), corner-turn encode/decode
    (rtl/src/tb_corner_turner.vhd:36-49,146-186), window endpoint/centre/symmetry
    checks (rtl/src/tb_window_multiplier.vhd:182-240), the CFAR map
    (rtl/src/tb_os_cfar_2d.vhd:52-75, ">= 2 detections"), the golden chirp
    (data/golden_input_chirp.txt) and coarse invariants of data/radar_output.txt.

The CFAR restatements here *sort* the reference cells literally, like the RTL
bubble sort; the HIP kernels use an equivalent counting formulation, so the
oracle is an independent check of that reformulation.  All CFAR arithmetic is
float32 with a fixed, documented order so detections compare bit-exactly.
"""
from __future__ import annotations

from dataclasses import dataclass
import numpy as np

# ---------------------------------------------------------------------------
# Window
# ---------------------------------------------------------------------------


def hamming_table(n: int) -> np.ndarray:
    """Hamming coefficients w[n] = 0.54 - 0.46 cos(2 pi i / (N-1)), fp64.

    The RTL keeps only the first N/2 coefficients in a ROM and mirrors the
    address for the second half (window_multiplier.vhd:40-42, :97-102), so the
    table is exactly symmetric; for even N that equals the closed formula.
    """
    half = n // 2
    idx = np.arange(n)
    addr = np.where(idx < half, idx, n - 1 - idx)
    addr = np.minimum(addr, max(half - 1, 0))  # :102 clamp (only matters for odd N)
    return 0.54 - 0.46 * np.cos(2.0 * np.pi * addr / (n - 1))


def hamming_q15(n: int) -> np.ndarray:
    """Integer ROM contents c[i] = integer(w * 32767) (window_multiplier.vhd:43-46)."""
    half = n // 2
    w = 0.54 - 0.46 * np.cos(2.0 * np.pi * np.arange(half) / (n - 1))
    c = np.floor(w * 32767.0 + 0.5).astype(np.int64)  # VHDL integer(real): round to nearest
    return np.clip(c, 0, 32767)


def window_q15_rtl(x: np.ndarray, n: int) -> np.ndarray:
    """RTL-compat int16 window: y = sat16((x*c + 2^14) >> 14)  (window_multiplier.vhd:146-158).

    Note the reference quirk: this is a 2x gain with a +1 LSB
    bias, so a zero input yields 1.  Provenance only; the build's product path
    is the fp32 window.
    """
    rom = hamming_q15(n)
    half = n // 2
    idx = np.arange(n)
    addr = np.minimum(np.where(idx < half, idx, n - 1 - idx), half - 1)
    c = rom[addr]
    y = (x.astype(np.int64) * c + (1 << 14)) >> 14
    return np.clip(y, -32768, 32767).astype(np.int64)


def window_q15_cube(cube_i16: np.ndarray) -> np.ndarray:
    """RTL-compat windowed ADC words of a cube [..., chirp, sample, 2] (I, Q int16) as complex
    integers: window_q15_rtl on I and on Q (both lanes of window_multiplier.vhd:146-158)."""
    x = np.asarray(cube_i16)
    ns = x.shape[-2]
    return window_q15_rtl(x[..., 0], ns) + 1j * window_q15_rtl(x[..., 1], ns)


# ---------------------------------------------------------------------------
# FFT stages (fp64 reference; unscaled forward DFT, natural order)
# ---------------------------------------------------------------------------


def window_f32(n: int) -> np.ndarray:
    """The exact fp32 window table the HIP path multiplies by."""
    return hamming_table(n).astype(np.float32)


def range_ct(cube: np.ndarray, window: bool = True) -> np.ndarray:
    """Window + range FFT + corner turn.

    cube: [..., chirp, sample] complex.  Returns [..., range, chirp] complex128:
    X[r, c] = sum_n w[n] x[c, n] exp(-2 pi i r n / Ns) (forward, FWD_INV=1 at
    radar_core.vhd:247; natural order, xfft_0.xci output ordering), then the
    corner turn out[r][c] = in[c][r] (corner_turner.vhd:79-80).
    """
    x = cube.astype(np.complex128)
    ns = x.shape[-1]
    if window:
        x = x * window_f32(ns).astype(np.float64)
    return np.swapaxes(np.fft.fft(x, axis=-1), -1, -2)


def mti(spec_rc: np.ndarray, mode: int) -> np.ndarray:
    """MTI / Doppler notch (rtl/src/doppler_notch.vhd:72-102) along slow time (last axis) of
    the corner-turned spectrum, one delay line per range bin zeroed at its first chirp (the
    reset on tlast, :99-102).  2-pulse y[c] = x[c] - x[c-1]; 3-pulse x[c] - 2x[c-1] + x[c-2].
    mode 0 = bypass.  Build spec: complex fp arithmetic, no int16 saturation (:76-93)."""
    x = np.asarray(spec_rc)
    if mode == 0:
        return x
    x1 = np.zeros_like(x)
    x1[..., 1:] = x[..., :-1]
    if mode == 2:
        return x - x1
    if mode == 3:
        x2 = np.zeros_like(x)
        x2[..., 2:] = x[..., :-2]
        return x - 2 * x1 + x2
    raise ValueError(mode)


def mti_rtl_int16(i: np.ndarray, q: np.ndarray, mode: int):
    """RTL-compat MTI on int16 I/Q streams (one range bin's slow-time sequence): the same
    difference with saturation to [-32768, 32767] (doppler_notch.vhd:76-93)."""
    def one(x):
        x = np.asarray(x, np.int64)
        x1 = np.concatenate([[0], x[:-1]])
        y = x - x1 if mode == 2 else x - 2 * x1 + np.concatenate([[0, 0], x[:-2]])
        return np.clip(y, -32768, 32767)
    if mode == 0:
        return np.asarray(i, np.int64), np.asarray(q, np.int64)
    return one(i), one(q)


def doppler_fft(spec_rc: np.ndarray, window: bool = True) -> np.ndarray:
    """Doppler window over slow time + forward Nc-point FFT per range bin (radar_core.vhd:340-364).

    spec_rc: [..., range, chirp].  Returns [..., range, doppler]; bin 0 = zero
    Doppler (natural order, no fftshift).
    """
    x = spec_rc.astype(np.complex128)
    nc = x.shape[-1]
    if window:
        x = x * window_f32(nc).astype(np.float64)
    return np.fft.fft(x, axis=-1)


def magnitude(rd: np.ndarray, rx_axis: int | None = None) -> np.ndarray:
    """|X| (fp64).  With rx_axis: non-coherent integration sqrt(sum_rx |X_rx|^2)."""
    p = rd.real ** 2 + rd.imag ** 2
    if rx_axis is not None:
        p = p.sum(axis=rx_axis)
    return np.sqrt(p)


def log_mag(mag: np.ndarray) -> np.ndarray:
    """20 log10(mag + 1), the visualizer's display transform (visualize_radar_targets.py:468)."""
    return 20.0 * np.log10(mag + 1.0)


def ambm(i, q):
    """Alpha-max-beta-min |z| ~ max + floor(min/4) + floor(min/8) (magnitude_calc.vhd:57-81)."""
    ai = np.abs(np.asarray(i, dtype=np.int64))
    aq = np.abs(np.asarray(q, dtype=np.int64))
    mx = np.maximum(ai, aq)
    mn = np.minimum(ai, aq)
    return mx + (mn >> 2) + (mn >> 3)


# ---------------------------------------------------------------------------
# OS-CFAR (float32, literal sort)
# ---------------------------------------------------------------------------


@dataclass
class Cfar1D:
    """1-D OS-CFAR along Doppler: rtl/old/os_cfar.vhd generics as instantiated at
    rtl/old/radar_core_v3.vhd:373-381 (REF 8, GUARD 2, RANK 12, alpha 4/1)."""
    ref: int = 8
    guard: int = 2
    rank: int = 12
    alpha: float = 4.0


@dataclass
class Cfar2D:
    """2-D OS-CFAR: rtl/src/os_cfar_2d.vhd as instantiated at radar_core.vhd:376-382.

    Axis naming follows what each generic *does* in the RTL:
    the line-buffer rows are range bins, the shift positions Doppler bins, so
    the reference's GUARD_RANGE=2 acts along Doppler and GUARD_DOPPLER=1 along
    range.  Defaults reproduce the reference window: 11 range rows x 13 Doppler
    cells, guard 3 x 5, 128 reference cells, rank floor(128*75/100) = 96.
    """
    ref_range: int = 4
    guard_range: int = 1
    ref_doppler: int = 4
    guard_doppler: int = 2
    rank_pct: int = 75
    scale_min: int = 2
    scale_nom: int = 4
    scale_max: int = 6
    scale_override: int = 0

    @property
    def n_ref(self) -> int:
        wr = 2 * (self.ref_range + self.guard_range) + 1
        wd = 2 * (self.ref_doppler + self.guard_doppler) + 1
        return wr * wd - (2 * self.guard_range + 1) * (2 * self.guard_doppler + 1)

    @property
    def rank(self) -> int:
        k = (self.n_ref * self.rank_pct) // 100  # os_cfar_2d.vhd:181-182
        return min(k, self.n_ref - 1)


def cfar_os1d(mag: np.ndarray, p: Cfar1D = Cfar1D()):
    """1-D OS-CFAR along the last (Doppler) axis, circular.

    Refs: p.ref cells each side beyond p.guard guard cells (rtl/old/os_cfar.vhd:98-109),
    sorted ascending (:117-125), T = alpha * refs[rank] (:132), detect CUT > T
    (:137).  Build spec differences: circular in Doppler, no
    17-bit truncation of T, fp32 arithmetic.

    Returns (det mask bool, threshold float32) with mag's shape.
    """
    m = np.asarray(mag, dtype=np.float32)
    offs = [-(p.guard + 1 + i) for i in range(p.ref)] + [p.guard + 1 + i for i in range(p.ref)]
    refs = np.stack([np.roll(m, -o, axis=-1) for o in offs])  # refs[j][..., d] = m[..., d+o_j]
    refs.sort(axis=0)
    thr = (np.float32(p.alpha) * refs[p.rank]).astype(np.float32)
    return m > thr, thr


def cfar2d_offsets(p: Cfar2D):
    """Reference-cell offsets (dr, dd) in the fixed summation order: dr ascending
    (outer), dd ascending (inner), guard block skipped (os_cfar_2d.vhd:155-167)."""
    hr = p.ref_range + p.guard_range
    hd = p.ref_doppler + p.guard_doppler
    out = []
    for dr in range(-hr, hr + 1):
        for dd in range(-hd, hd + 1):
            if abs(dr) <= p.guard_range and abs(dd) <= p.guard_doppler:
                continue
            out.append((dr, dd))
    return out


def tree_sum_f32(refs: np.ndarray) -> np.ndarray:
    """Sum over axis 0 in the build's fixed fp32 order: pad with zeros to 128 (adding 0
    is exact), then halve: s[i] = x[i] + x[i + n/2] until one term remains.  The RTL
    sums exact integers (os_cfar_2d.vhd:163); fp32 needs *an* order, and this one is
    what a wave computes with one add per lane followed by xor-shuffles 32..1."""
    x = np.asarray(refs, dtype=np.float32)
    n = x.shape[0]
    assert n <= 128
    if n < 128:
        x = np.concatenate([x, np.zeros((128 - n,) + x.shape[1:], np.float32)])
    while x.shape[0] > 1:
        h = x.shape[0] // 2
        x = (x[:h] + x[h:]).astype(np.float32)
    return x[0]


def cfar_os2d(mag: np.ndarray, p: Cfar2D = Cfar2D()):
    """2-D OS-CFAR over a [range, doppler] map (fp32), Doppler circular.

    Per CUT (os_cfar_2d.vhd:152-217): the n_ref reference cells are sorted
    ascending and ranked = refs[rank]; mean = tree_sum_f32(refs in cfar2d_offsets()
    order) / n_ref; scale = override if nonzero, else scale_max
    if ranked > mean + mean/2, scale_min if ranked < mean/2, else scale_nom;
    detect if CUT > fl32(ranked * scale).  Range edges: a CUT is tested only when
    its whole range extent lies inside the map (build spec).

    Returns (det mask bool, threshold float32); threshold is 0 on untested rows.
    """
    m = np.asarray(mag, dtype=np.float32)
    nr, nd = m.shape
    hr = p.ref_range + p.guard_range
    offs = cfar2d_offsets(p)
    det = np.zeros((nr, nd), dtype=bool)
    thr_out = np.zeros((nr, nd), dtype=np.float32)
    if nr < 2 * hr + 1:
        return det, thr_out
    rows = np.arange(hr, nr - hr)
    refs = np.empty((len(offs), rows.size, nd), dtype=np.float32)
    for j, (dr, dd) in enumerate(offs):
        refs[j] = np.roll(m[rows + dr], -dd, axis=-1)
    mean = (tree_sum_f32(refs) / np.float32(len(offs))).astype(np.float32)
    refs.sort(axis=0)
    ranked = refs[p.rank]
    if p.scale_override:
        scale = np.full(ranked.shape, p.scale_override, dtype=np.float32)
    else:
        half = (mean * np.float32(0.5)).astype(np.float32)
        hi = (mean + half).astype(np.float32)
        scale = np.where(ranked > hi, np.float32(p.scale_max),
                         np.where(ranked < half, np.float32(p.scale_min), np.float32(p.scale_nom)))
    thr = (ranked * scale.astype(np.float32)).astype(np.float32)
    det[rows] = m[rows] > thr
    thr_out[rows] = thr
    return det, thr_out


# ---------------------------------------------------------------------------
# RTL-compat CFAR arithmetic (integer).  Cells are the 17-bit unsigned
# CFAR input words (DATA_WIDTH 17, os_cfar.vhd:13, os_cfar_2d.vhd:11).
# ---------------------------------------------------------------------------
Q17_MAX = (1 << 17) - 1


def q17(mag: np.ndarray) -> np.ndarray:
    """Map cells -> the 17-bit CFAR word: min(floor(max(x, 0)), 2^17 - 1), int64."""
    m = np.floor(np.maximum(np.asarray(mag, np.float64), 0.0))
    return np.minimum(m, Q17_MAX).astype(np.int64)


def cfar_os1d_rtl(mag: np.ndarray, p: Cfar1D = Cfar1D()):
    """rtl/old/os_cfar.vhd:98-144 in integers: refs sorted (bubble sort :117-125),
    threshold = resize(refs[RANK] * SCALING_MULT / SCALING_DIV, DATA_WIDTH) (:132), i.e. the
    product taken mod 2^17, detect cut > threshold (:137).  alpha = SCALING_MULT (DIV = 1).
    Circular along Doppler (build spec).  Returns (det, threshold int64)."""
    assert float(p.alpha).is_integer()
    m = q17(mag)
    offs = [-(p.guard + 1 + i) for i in range(p.ref)] + [p.guard + 1 + i for i in range(p.ref)]
    refs = np.sort(np.stack([np.roll(m, -o, axis=-1) for o in offs]), axis=0)
    thr = (refs[p.rank] * int(p.alpha)) % (1 << 17)
    return m > thr, thr


def cfar_os2d_rtl(mag: np.ndarray, p: Cfar2D = Cfar2D()):
    """rtl/src/os_cfar_2d.vhd:152-217 in integers: exact sum of the refs (:163), mean =
    floor(sum / N_REF) (:189), brackets with the 17-bit add mean + (mean >> 1) (:193, wraps mod
    2^17) and mean >> 1 (:195), threshold = ranked * scale at full width (:204), detect
    cut > threshold (:213).  Doppler circular, range edges as cfar_os2d."""
    m = q17(mag)
    nr, nd = m.shape
    hr = p.ref_range + p.guard_range
    offs = cfar2d_offsets(p)
    det = np.zeros((nr, nd), bool)
    thr_out = np.zeros((nr, nd), np.int64)
    if nr < 2 * hr + 1:
        return det, thr_out
    rows = np.arange(hr, nr - hr)
    refs = np.stack([np.roll(m[rows + dr], -dd, axis=-1) for (dr, dd) in offs])
    mean = refs.sum(axis=0) // len(offs)
    ranked = np.sort(refs, axis=0)[p.rank]
    if p.scale_override:
        scale = np.full(ranked.shape, p.scale_override, np.int64)
    else:
        hi = (mean + (mean >> 1)) % (1 << 17)
        lo = mean >> 1
        scale = np.where(ranked > hi, p.scale_max, np.where(ranked < lo, p.scale_min, p.scale_nom))
    thr = ranked * scale
    det[rows] = m[rows] > thr
    thr_out[rows] = thr
    return det, thr_out


def detections_rtl(det: np.ndarray, mag: np.ndarray, thr: np.ndarray, frame: int = 0) -> np.ndarray:
    """Detection records of the compat CFAR: mag = the 17-bit cut word, threshold = T."""
    return detections(det, q17(mag).astype(np.float32), np.asarray(thr).astype(np.float32), frame)


def mti_spectrum_rtl(spec_rc: np.ndarray, mode: int) -> np.ndarray:
    """FMCW_COMPAT_MTI on a (scaled) corner-turned spectrum [..., range, chirp]: each
    component rounded half-to-even and saturated to int16 (the FFT IP's 16-bit output word),
    then mti_rtl_int16 along slow time per range bin (doppler_notch.vhd:67-102)."""
    x = np.asarray(spec_rc)

    def one(v):  # mti_rtl_int16 along the last axis, all range bins at once
        v = np.clip(np.rint(v), -32768, 32767).astype(np.int64)
        v1 = np.zeros_like(v)
        v1[..., 1:] = v[..., :-1]
        if mode == 2:
            y = v - v1
        else:
            v2 = np.zeros_like(v)
            v2[..., 2:] = v[..., :-2]
            y = v - 2 * v1 + v2
        return np.clip(y, -32768, 32767)
    return one(x.real) + 1j * one(x.imag)


def spectrum_words(spec_rc: np.ndarray) -> np.ndarray:
    """The FFT IP's 16-bit output words as the corner turner hands them on: each component of the
    (scaled) spectrum rounded half-to-even and saturated to int16 (xfft_0.xci: convergent
    rounding, 16-bit output)."""
    x = np.asarray(spec_rc)
    return np.clip(np.rint(x.real), -32768, 32767) + 1j * np.clip(np.rint(x.imag), -32768, 32767)


def saturation_counts(cube_i16: np.ndarray, range_shift: int, mti_mode: int = 0, q15_rtl: bool = True,
                      mti_rtl: bool = False):
    """RTL-compat status as counts (fmcw.h status words 2, 3 -- the sticky status_overflow of
    radar_core.vhd:447-456 counted per sample): (window saturations, word saturations) of one
    frame [rx, chirp, sample, 2].  A sample counts once when its I or Q clips:
      window: window_multiplier's sat_flag (:152-158) in u_range_window (ADC words) and, with
              q15_rtl, in u_doppler_window (spectrum words after the canceller);
      word:   the spectrum rounded to int16 (spectrum_words) and the canceller's saturating
              output (doppler_notch.vhd:76-93), when the path carries 16-bit words."""
    x = np.asarray(cube_i16, np.int64)
    if x.ndim == 3:
        x = x[None]
    ns, nc = x.shape[-2], x.shape[-3]

    def win_clips(v, n):            # v [..., n] integers, window along the last axis
        rom = hamming_q15(n)
        half = n // 2
        idx = np.arange(n)
        c = rom[np.minimum(np.where(idx < half, idx, n - 1 - idx), half - 1)]
        y = (v * c + (1 << 14)) >> 14
        return (y < -32768) | (y > 32767)

    wsat = 0
    words = None
    if q15_rtl:
        wsat += int((win_clips(x[..., 0], ns) | win_clips(x[..., 1], ns)).sum())
        c = window_q15_cube(x)
        spec = range_ct(c, window=False)
    else:
        spec = range_ct(x[..., 0] + 1j * x[..., 1], window=False)
    spec = spec * 2.0 ** -range_shift
    nsat = 0
    if q15_rtl or mti_rtl:
        r = np.rint(spec.real), np.rint(spec.imag)
        nsat += int(((np.abs(r[0] + 0.5) > 32767.5) | (np.abs(r[1] + 0.5) > 32767.5)).sum())
        words = [np.clip(r[0], -32768, 32767).astype(np.int64), np.clip(r[1], -32768, 32767).astype(np.int64)]
        if mti_mode:
            out = []
            clip = np.zeros(words[0].shape, bool)
            for v in words:
                v1 = np.zeros_like(v)
                v1[..., 1:] = v[..., :-1]
                if mti_mode == 2:
                    y = v - v1
                else:
                    v2 = np.zeros_like(v)
                    v2[..., 2:] = v[..., :-2]
                    y = v - 2 * v1 + v2
                clip |= (y < -32768) | (y > 32767)
                out.append(np.clip(y, -32768, 32767))
            nsat += int(clip.sum())
            words = out
        if q15_rtl:
            wsat += int((win_clips(words[0], nc) | win_clips(words[1], nc)).sum())
    return wsat, nsat


DET_DTYPE = np.dtype([("frame", "<u4"), ("range", "<u2"), ("doppler", "<u2"),
                      ("mag", "<f4"), ("threshold", "<f4")])


def detections(det: np.ndarray, mag: np.ndarray, thr: np.ndarray, frame: int = 0) -> np.ndarray:
    """Detection list in range-major scan order (radar_core.vhd:396-418: index
    counters walk range-major, emit only non-zero CFAR outputs)."""
    r, d = np.nonzero(det)
    out = np.empty(r.size, dtype=DET_DTYPE)
    out["frame"] = frame
    out["range"] = r
    out["doppler"] = d
    out["mag"] = np.asarray(mag, dtype=np.float32)[r, d]
    out["threshold"] = thr[r, d]
    return out


# ---------------------------------------------------------------------------
# Whole pipeline
# ---------------------------------------------------------------------------


def doppler_stage(spec: np.ndarray, window: bool = True, mti_mode: int = 0, q15_rtl: bool = False,
                  mti_rtl: bool = False) -> np.ndarray:
    """From the (scaled) corner-turned spectrum [..., range, chirp] to the range-Doppler
    spectrum: MTI canceller (radar_core.vhd:329-338), Doppler window, Doppler FFT (:340-364).
    mti_rtl / q15_rtl: the canceller on the IP's 16-bit words (mti_spectrum_rtl); q15_rtl also
    windows those words in the RTL's integer arithmetic (window_q15_rtl along slow time)."""
    if mti_rtl or q15_rtl:
        words = spectrum_words(spec)
        spec = mti_spectrum_rtl(words, mti_mode) if mti_mode else words
    else:
        spec = mti(spec, mti_mode)
    if q15_rtl:
        nc = spec.shape[-1]
        spec = window_q15_rtl(spec.real.astype(np.int64), nc) + 1j * window_q15_rtl(spec.imag.astype(np.int64), nc)
        return doppler_fft(spec, window=False)
    return doppler_fft(spec, window)


def process(cube: np.ndarray, cfar=None, window: bool = True, mti_mode: int = 0,
            q15_rtl: bool = False, range_shift: int = 0, mti_rtl: bool = False):
    """Full hot path for one frame.

    cube: [rx, chirp, sample] (or [chirp, sample]) complex.  Returns dict with the
    fp64 map 'mag' [range, doppler], the float32 map used by the CFAR, the
    detection mask and the detection list.  With several rx channels the map is
    the non-coherent integration sqrt(sum_rx |X|^2).
    q15_rtl: cube is int16 [rx, chirp, sample, 2] and both windows are the RTL's integer Q15
    arithmetic: the range window on the ADC words (window_q15_cube, u_range_window), the
    Doppler window on the corner-turned spectrum's 16-bit words (spectrum_words, after the MTI
    canceller; u_doppler_window, radar_core.vhd:340-349).
    """
    if q15_rtl:
        c = window_q15_cube(cube)
        if c.ndim == 2:
            c = c[None]
        spec = range_ct(c, window=False)
    else:
        c = np.asarray(cube)
        if c.ndim == 2:
            c = c[None]
        spec = range_ct(c, window)
    spec = spec * 2.0 ** -range_shift            # the IP's fixed scaling schedule (exact)
    rd = doppler_stage(spec, window, mti_mode, q15_rtl, mti_rtl)  # [rx, range, doppler]
    mag = magnitude(rd, rx_axis=0)
    mag32 = mag.astype(np.float32)
    if cfar is None:
        det = np.zeros(mag.shape, bool)
        thr = np.zeros(mag.shape, np.float32)
    elif isinstance(cfar, Cfar1D):
        det, thr = cfar_os1d(mag32, cfar)
    else:
        det, thr = cfar_os2d(mag32, cfar)
    return {"rd": rd, "mag": mag, "mag32": mag32, "det": det, "thr": thr,
            "dets": detections(det, mag32, thr)}
