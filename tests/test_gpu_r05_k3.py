"""Round 5, second half: the reworked 2-D CFAR at NC = 1024 (k_cfar2d_lv with nibble prefix rows,
upper bounds for levels C / D and compat as a template switch; K3b's pipelined fetches and DPP
halving tree; K3c's lane-per-tile pass).  The bench maps reach only the default scales on
Rayleigh clutter; these maps reach the other paths -- RTL-compat integer cells, a scale override,
other scale sets (the rules' s2 / rule-A conditions), bright patches full of C / D cells, targets
on the Doppler wrap, and lattices dense enough that K3a's strip buffer overflows into per-tile
reservations and K3c's whole-wave path runs for most tiles.  Bit-exact vs the oracles
(oracle/fmcw_cpu.c via cpu_backend.cfar; fmcw_oracle.cfar_os2d_rtl for compat)."""
import numpy as np
import pytest

import cpu_backend as CB
import fmcw_oracle as O
from fmcw import RadarCore
from test_gpu_parity import run_cfar_stage
from test_gpu_r02 import _rtl_dets

pytestmark = pytest.mark.gpu

NS, NC = 256, 1024


def _clutter(seed, nf=2, ns=NS):
    rng = np.random.default_rng(seed)
    m = rng.rayleigh(10.0, (nf, ns, NC)).astype(np.float32)
    m[:, 100:120, 200:260] = rng.rayleigh(150.0, (nf, 20, 60))  # bright patch: C / D cells, long runs
    m[:, 200:230, 600:700] = 0.02                                # quiet patch
    m[0, 50, 7] = 900.0
    m[0, 51, 1023] = 800.0                                       # on the Doppler wrap
    m[1, 180, 0] = 700.0
    m[1, 10:12, 512] = 800.0
    m[1, 5, 300] = 1e30                                          # far above every level window
    return m


@pytest.mark.parametrize("scales,ovr", [((2, 4, 6), 0), ((2, 4, 6), 3), ((3, 5, 7), 0), ((1, 2, 2), 0)])
def test_lv_scales_and_override(scales, ovr):
    m = _clutter(61 + scales[0] + ovr)
    p = O.Cfar2D(scale_min=scales[0], scale_nom=scales[1], scale_max=scales[2], scale_override=ovr)
    with RadarCore(N_RANGE=NS, N_DOPPLER=NC, cfar="os2d", cfar_scales=scales, cfar_scale_ovr=ovr,
                   max_frames=2) as core:
        got = run_cfar_stage(core, m, cap=1 << 20)
    want = CB.cfar(m, p, threads=16)
    assert len(want) >= 4
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("steps", [0, 1, 3])
def test_lv_strips(steps):
    """Strip lengths 1 (every step a strip's first: the whole ring staged, prefixes from zero) and
    3 (upward strips end on a partial step at the frame's end), 3 frames of 512 rows."""
    m = _clutter(71, nf=3, ns=512)
    with RadarCore(N_RANGE=512, N_DOPPLER=NC, cfar="os2d", max_frames=3) as core:
        core.set_param("cfar2d_steps", steps)
        got = run_cfar_stage(core, m, cap=1 << 20)
    np.testing.assert_array_equal(got, CB.cfar(m, O.Cfar2D(), threads=16))


def test_lv_dense_lattice():
    """Every third cell of every third row detects: ~450 survivors per 4096-cell step (past the
    192-cell strip buffer), runs far longer than K3c's per-lane check."""
    rng = np.random.default_rng(73)
    m = rng.rayleigh(1.0, (2, NS, NC)).astype(np.float32)
    m[:, ::3, ::3] = 50.0
    with RadarCore(N_RANGE=NS, N_DOPPLER=NC, cfar="os2d", max_frames=2) as core:
        got = run_cfar_stage(core, m, cap=1 << 21)
    want = CB.cfar(m, O.Cfar2D(), threads=16)
    assert len(want) > 2 * NS * NC // 12
    np.testing.assert_array_equal(got, want)


def test_lv_compat():
    """FMCW_COMPAT_CFAR at NC = 1024 (the CMP instantiation): cells across the 17-bit range,
    saturating cells, fractions and a negative cell; bit-exact vs cfar_os2d_rtl."""
    rng = np.random.default_rng(79)
    m = rng.uniform(5000, 15000, (2, NS, NC)).astype(np.float32)
    m[0, 50, 60], m[1, 60, 1000], m[1, 90, 3] = 131000.0, 120000.0, 70000.5
    m[0, 10:12, :] = 150000.0                                  # saturates at 2^17 - 1
    m[0, 100, 5:9] = 2.0 ** 17 - 1.5
    m[1, 20:40, 10:30] = rng.uniform(90000, 131000, (20, 20))  # the 17-bit bracket add wraps
    m[1, 30, 20] = 131071.0
    m[1, 50, 50] = -5.0
    with RadarCore(N_RANGE=NS, N_DOPPLER=NC, cfar="os2d", compat_rtl=("cfar",), max_frames=2) as core:
        got = run_cfar_stage(core, m, cap=1 << 20)
    want = _rtl_dets(m, O.Cfar2D())
    assert len(want) > 0
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("dist", ["exponential", "lognormal", "uniform", "sparse"])
def test_lv_clutter_shapes(dist):
    """Clutter whose level spacing differs from the bench's Rayleigh magnitudes: exponential (power
    maps: ~10 % of cells at the C level, so the C bound often fails), lognormal (wide: B clamped to
    1.5 A), uniform (narrow), and a sparse map (mostly zeros: levels at the bottom of the key range).
    The screen only ever keeps more cells; the detections must not change."""
    rng = np.random.default_rng({"exponential": 81, "lognormal": 83, "uniform": 85, "sparse": 87}[dist])
    shape = (2, NS, NC)
    if dist == "exponential":
        m = rng.exponential(5.0, shape)
    elif dist == "lognormal":
        m = rng.lognormal(1.0, 1.2, shape)
    elif dist == "uniform":
        m = rng.uniform(9.0, 11.0, shape)
    else:
        m = np.where(rng.random(shape) < 0.02, rng.rayleigh(10.0, shape), 0.0)
    m = m.astype(np.float32)
    m[0, 60, 100] = 4000.0
    m[1, 200, 1020] = 3000.0
    m[:, 120:124, 400:460] *= 30.0
    with RadarCore(N_RANGE=NS, N_DOPPLER=NC, cfar="os2d", max_frames=2) as core:
        got = run_cfar_stage(core, m, cap=1 << 21)
    want = CB.cfar(m, O.Cfar2D(), threads=16)
    assert len(want) >= 2
    np.testing.assert_array_equal(got, want)
