"""Round-4 GPU tests (libfmcw.so on gfx950 vs the CPU oracle, through the C-ABI).

  * BASELINE configs 3 and 5 at the bench's OWN shape (bench.py WORKLOADS): 16 frames per call,
    the library's auto chunk (3 frames per K1 -> K2 launch pair) and one 2-D CFAR launch over all
    16 frames with the cost model's strip length -- exactly the composition whose time the driver
    credits.  Maps of the first and last frame within 1e-4 of the fp64 oracle (the fp16-dequantised
    input at config 5), every frame's detections bit-exact against the C oracle's 2-D OS-CFAR on
    the GPU's map (oracle/fmcw_cpu.c, pinned to the NumPy oracle by tests/test_cpu_backend.py).
    Semantics: rtl/src/radar_core.vhd:303-390, rtl/src/os_cfar_2d.vhd:152-217.
"""
import sys

import numpy as np
import pytest

import cpu_backend as CB
import fmcw_oracle as O
from conftest import REPO
from fmcw import RadarCore, synth
from test_gpu_parity import check_map, run_cfar_stage, to_complex

pytestmark = pytest.mark.gpu

if str(REPO) not in sys.path:
    sys.path.insert(0, str(REPO))


@pytest.mark.parametrize("wl", ["c3", "c5"])
def test_bench_shape_parity(wl):
    import bench  # the workload table the bench times (imports nothing heavy at module level)
    w = bench.WORKLOADS[wl]
    F, ns, nc, nrx, dtype = w["frames"], w["ns"], w["nc"], w["nrx"], w["dtype"]
    assert F == 16
    # bench.run_workload at rank 0: 16 distinct frames, seed 1234 + first global frame
    cube = synth.frames(F, ns, nc, nrx, w["recipe"], seed=1234, dtype=dtype)
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, N_RX=nrx, in_dtype=dtype, cfar=w["cfar"], max_frames=F) as core:
        assert core.info("chunk") == 3
        out = core.process(cube)
        steps = core.info("cfar2d_steps")
    # the cost model's strip length for 16 frames (config 5: 32 steps of 16 rows; config 3 ~11)
    assert steps >= 8, steps
    for f in (0, F - 1):
        ref = O.process(to_complex(cube[f], dtype), None)["mag"]
        check_map(out.rd_map[f:f + 1], ref[None])
    want = CB.cfar(out.rd_map, O.Cfar2D(), threads=16)
    np.testing.assert_array_equal(out.dets, want)
    assert set(out.dets["frame"].tolist()) == set(range(F))
    hit = set(zip(out.dets["frame"].tolist(), out.dets["range"].tolist(), out.dets["doppler"].tolist()))
    assert (0, round(100 * ns / 1024), 5) in hit and (F - 1, round(100 * ns / 1024), 5) in hit


@pytest.mark.parametrize("want_map,map_kind", [(False, "linear"), (True, "db")])
def test_cfar2d_on_chunk_scratch(want_map, map_kind):
    """No linear map from the caller (map-less call, or a dB map): the 2-D CFAR runs per K1/K2
    chunk on the handle's scratch map, one K3 launch (and candidate-counter slot) per chunk --
    7 chunks of 3 frames here.  Detections bit-exact vs the C oracle on the linear map of the
    same frames (from a linear-map handle, itself checked against the oracle elsewhere)."""
    ns, nc, nf = 1024, 256, 20
    cube = synth.frames(nf, ns, nc, 1, "random_target", seed=41)
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, cfar="os2d", max_frames=nf, chunk_frames=3) as core:
        lin = core.process(cube).rd_map
    want = CB.cfar(lin, O.Cfar2D(), threads=16)
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, cfar="os2d", max_frames=nf, chunk_frames=3,
                   map_kind=map_kind) as core:
        out = core.process(cube, want_map=want_map)
    np.testing.assert_array_equal(out.dets, want)
    assert out.n_dets >= nf


def test_cfar2d_stage_in_pieces():
    """fmcw_cfar on more frames than one K3 launch's candidate list holds (16 + chunk): the stage
    runs in pieces, each with its own counters; the list is the oracle's, in order."""
    ns, nc, nf = 256, 128, 45
    rng = np.random.default_rng(43)
    m = rng.rayleigh(10.0, (nf, ns, nc)).astype(np.float32)
    m[:, 60, 17] = 800.0
    m[::3, 150:153, 90] = 400.0
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, cfar="os2d", max_frames=nf, chunk_frames=2) as core:
        got = run_cfar_stage(core, m, cap=1 << 18)
    want = CB.cfar(m, O.Cfar2D(), threads=16)
    np.testing.assert_array_equal(got, want)
    assert set(got["frame"].tolist()) == set(range(nf))


def test_cfar2d_dense_candidates_exact_count():
    """A lattice where ~1/9 of all cells detect (every candidate run is long, many tiles spill into
    the overflow region): the candidate list (room for every cell) keeps the count exact, and the
    records equal the oracle's."""
    ns, nc, nf = 512, 256, 2
    rng = np.random.default_rng(47)
    m = rng.rayleigh(1.0, (nf, ns, nc)).astype(np.float32)
    m[:, ::3, ::3] = 50.0
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, cfar="os2d", max_frames=nf) as core:
        got = run_cfar_stage(core, m, cap=1 << 20)
    want = CB.cfar(m, O.Cfar2D(), threads=16)
    assert len(want) > nf * ns * nc // 12
    np.testing.assert_array_equal(got, want)


def test_counters_rearmed_across_calls():
    """The per-call device counters (overflow use, drops, saturations, the 2-D CFAR launches'
    candidate counters) are re-armed by each call's last kernel (k_det_list), not zeroed at the
    next call's start: alternate fmcw_cfar stage calls on a map that fills the overflow region
    (every third cell detects) with whole-path calls on a cube, on one handle, and check every
    call against the oracle."""
    ns, nc, nf = 512, 256, 2
    rng = np.random.default_rng(53)
    m = rng.rayleigh(1.0, (nf, ns, nc)).astype(np.float32)
    m[:, ::3, ::3] = 50.0
    want_m = CB.cfar(m, O.Cfar2D(), threads=16)
    cube = synth.frames(nf, ns, nc, 1, "random_target", seed=54)
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, cfar="os2d", max_frames=nf) as core:
        for _ in range(3):
            got = run_cfar_stage(core, m, cap=1 << 20)
            np.testing.assert_array_equal(got, want_m)
            out = core.process(cube)
            np.testing.assert_array_equal(out.dets, CB.cfar(out.rd_map, O.Cfar2D(), threads=16))
            assert out.n_dets >= nf and out.window_saturations == 0 and out.word_saturations == 0


def test_detection_list_many_blocks():
    """The one-pass ordered list (k_det_list, decoupled look-back over 1024-tile blocks) at config
    2's bench shape -- 1024 frames in one call, ten K1 -> K2 chunks, far more than 64 look-back
    blocks, so a workgroup may sum several windows of predecessors -- equals the same frames run as
    16 calls of 64 frames (a few blocks each), frame ids shifted; two whole calls agree (the
    look-back words are reused under the next call's epoch)."""
    ns, nc, F, part = 1024, 256, 1024, 64
    base = synth.frames(part, ns, nc, 1, "two_targets", seed=61, dtype="i16")
    cube = np.concatenate([base] * (F // part))
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, cfar="os1d", in_dtype="i16", max_frames=F) as core:
        whole = core.process(cube, want_map=False)
        again = core.process(cube, want_map=False)
        parts = [core.process(cube[k * part:(k + 1) * part], want_map=False) for k in range(F // part)]
    np.testing.assert_array_equal(whole.dets, again.dets)
    cat = []
    for k, p in enumerate(parts):
        d = p.dets.copy()
        d["frame"] += k * part
        cat.append(d)
    np.testing.assert_array_equal(whole.dets, np.concatenate(cat))
    assert whole.n_dets == sum(p.n_dets for p in parts) >= F
