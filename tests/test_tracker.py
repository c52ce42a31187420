"""Track-while-scan tracker: the library's host-side fmcw_tws_* against
oracle/tws_oracle.py (a literal restatement of rtl/src/tws_tracker.vhd), pinned by the
scenario and assertions of rtl/src/tb_tws_tracker.vhd:100-180.  CPU only (no device)."""
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "fpga-fmcw-radar-processor_amd"))
sys.path.insert(0, str(REPO / "oracle"))

import tws_oracle as T  # noqa: E402
from fmcw import TwsTracker, formats  # noqa: E402


def run_both(scans, rtl, **gen):
    p = T.TwsParams(rtl=rtl, **{k.lower(): v for k, v in gen.items()})
    o = T.TwsOracle(p)
    names = dict(max_tracks="MAX_TRACKS", coast_max="COAST_MAX", init_hits="INIT_HITS",
                 gate_r="ASSOC_GATE_R", gate_d="ASSOC_GATE_D", alpha_q8="ALPHA_GAIN",
                 beta_q8="BETA_GAIN", max_dets="MAX_DETS")
    lib = TwsTracker(rtl_compat=rtl, **{names[k.lower()]: v for k, v in gen.items()})
    hist = []
    for dets in scans:
        want, act = o.scan(dets)
        got = lib.scan(np.array(dets, np.float64).reshape(-1, 3))
        assert lib.active_tracks == act
        assert len(got) == len(want)
        for g, w in zip(got, want):
            for k in ("id", "status", "quality", "range_q2", "doppler_q2", "vel_r", "vel_d", "last_mag", "age"):
                assert int(g[k]) == w[k], (k, g, w)
        hist.append((got, act))
    lib.close()
    return hist


@pytest.mark.parametrize("rtl", [False, True])
def test_tb_tws_tracker_scenario(rtl, tmp_path):
    """tb_tws_tracker.vhd generics (MAX_TRACKS 16, COAST_MAX 3) and its per-scan checks
    (:146-180): >= 2 tracks after scan 2 and 3, >= 3 after scan 6."""
    hist = run_both(T.tb_tws_scenario(), rtl, max_tracks=16, coast_max=3)
    act = [a for _, a in hist]
    assert act[1] >= 2 and act[2] >= 2 and act[5] >= 3
    if not rtl:
        # the intended tracker keeps targets 1 and 2 firm from scan 3 on, drops target 3
        # after COAST_MAX + 1 misses and holds the every-third-scan false alarm
        assert act[10] <= 3                                   # the scan-11 check (:173-178)
        firm = [{int(t["id"]) for t in trk if t["status"] == 2} for trk, _ in hist]
        assert {0, 1} <= firm[2] and all({0, 1} <= f for f in firm[2:])
        r1 = [int(t["range_q2"]) for trk, _ in hist[2:] for t in trk if t["id"] == 0]
        assert all(b < a for a, b in zip(r1, r1[1:]))         # approaching target 1
    f = tmp_path / "tracks.txt"
    formats.write_tracks(f, hist)
    tracks, counts = formats.read_tracks(f)
    assert counts == act
    assert sum(len(v) for v in tracks.values()) == sum(len(t) for t, _ in hist)


def random_scans(seed, n_scans=40, max_extra=8, burst=False):
    rng = np.random.default_rng(seed)
    tgt = [[rng.integers(20, 1000), rng.integers(5, 120), rng.integers(-6, 7), rng.integers(-2, 3)]
           for _ in range(6)]
    scans = []
    for s in range(n_scans):
        d = []
        for t in tgt:
            t[0] = int(np.clip(t[0] + t[2] + rng.integers(-1, 2), 0, 1023))
            t[1] = int(np.clip(t[1] + t[3] + rng.integers(-1, 2), 0, 127))
            if rng.random() < 0.85:
                d.append((t[0], t[1], int(rng.integers(1000, 200000))))
        for _ in range(int(rng.integers(0, max_extra))):
            d.append((int(rng.integers(0, 1024)), int(rng.integers(0, 128)), int(rng.integers(100, 5000))))
        if burst and s % 7 == 3:       # > 64 detections: the RTL's 6-bit counter wraps
            d += [(int(rng.integers(0, 1024)), int(rng.integers(0, 128)), 700) for _ in range(70)]
        rng.shuffle(d)
        scans.append(d)
    return scans


@pytest.mark.parametrize("rtl", [False, True])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_streams_match_oracle(rtl, seed):
    run_both(random_scans(seed), rtl)


@pytest.mark.parametrize("rtl", [False, True])
def test_overfull_scans_and_small_track_file(rtl):
    """> 64 detections per scan and a full track file (initiation finds no free slot)."""
    run_both(random_scans(9, burst=True), rtl, max_tracks=8, init_hits=1, coast_max=2)


def test_gate_and_gain_generics():
    run_both(random_scans(5, max_extra=3), False, gate_r=3, gate_d=2, alpha_q8=200, beta_q8=30)


def test_rejects_bad_generics():
    from fmcw import FmcwError
    for kw in (dict(MAX_TRACKS=0), dict(MAX_TRACKS=65), dict(MAX_DETS=65), dict(ALPHA_GAIN=256)):
        with pytest.raises(FmcwError):
            TwsTracker(**kw)
