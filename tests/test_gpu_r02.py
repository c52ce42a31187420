"""GPU parity, round 2: the configurations and paths round 1 left unexercised on hardware.

  * BASELINE config 5 at full geometry (1024 x 8192 fp16, 2-D OS-CFAR, k_cfar2d<1024>)
  * the rtl/old/tb_radar_core.vhd stimulus (exact VHDL RNG) vs data/radar_output.txt invariants
  * K2's AMBM magnitude end to end (magnitude_calc.vhd:57-81)
  * config 4's per-GPU share: 1024 config-2 frames in one fmcw_enqueue
  * detection-list overflow (2-D) and dropped-detection reporting; negative caller-map cells
  * RTL-compat CFAR (17-bit integer) and MTI (int16 saturating) vs the oracle's restatements
  * the C-ABI RCCL gather on a one-rank communicator; the CLI writing visualizer files

Tolerances as tests/test_gpu_parity.py: maps max|d|/max|ref| <= 1e-4 per frame plus 1e-4 per
bin above 1e-3 of the peak; detections bit-exact against the oracle CFAR on the GPU's map
(checked with oracle/fmcw_cpu.c where the NumPy oracle would need GBs: that C CFAR is itself
pinned bit-exact to the oracle by tests/test_cpu_backend.py).
"""
import subprocess
import sys

import numpy as np
import pytest

import cpu_backend as CB
import fmcw_oracle as O
from conftest import GOLDEN, PKG, rel_err
from fmcw import DET_DTYPE, DeviceBuffer, RadarCore, formats, synth
from fmcw.dist import RcclGather
from test_gpu_parity import check_map, oracle_dets, run_cfar_stage, run_range_ct, to_complex

pytestmark = pytest.mark.gpu


def _stage_dets(core, mag, cap=1 << 20):
    """fmcw_cfar on a host map; returns (records, found, dropped) without asserting."""
    nf = mag.shape[0]
    dm = DeviceBuffer(mag.nbytes)
    dm.upload(np.ascontiguousarray(mag, np.float32))
    dd = DeviceBuffer(cap * 16)
    dn = DeviceBuffer(16)
    core.cfar(dm, nf, dd, cap, dn)
    n, dropped = (int(x) for x in dn.download(np.uint32, (2,)))
    return dd.download(DET_DTYPE, (cap,))[: min(n, cap)], n, dropped


# ------------------------------------------------------------------------------------------
def test_config5_full_geometry():
    """BASELINE config 5: 1024 chirps x 8192 range bins, fp16 complex samples, 2-D OS-CFAR.
    The oracle is fed the fp16-dequantised input (SURVEY.md 7 "Hard parts")."""
    ns, nc = 8192, 1024
    cube = synth.frames(1, ns, nc, 1, "two_targets", dtype="f16")
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, in_dtype="f16", cfar="os2d", max_frames=1) as core:
        out = core.process(cube)
    ref = O.process(to_complex(cube[0], "f16"), None)["mag"]
    check_map(out.rd_map, ref[None])
    want = CB.cfar(out.rd_map, O.Cfar2D(), threads=16)
    np.testing.assert_array_equal(out.dets, want)
    hit = set(zip(out.dets["range"].tolist(), out.dets["doppler"].tolist()))
    assert (800, 5) in hit and (4000, nc - 10) in hit


def test_tb_radar_core_v3_stimulus():
    """rtl/old/tb_radar_core.vhd:86-141 (two CPIs, IEEE UNIFORM noise) through RadarCore as the
    raw ADC words: energy rows {99..101, 499..501} as data/radar_output.txt, Doppler peaks at
    natural bins 5 and 118; map and 1-D CFAR parity vs the oracle."""
    cpis = synth.tb_radar_core_v3_cpis()
    cube = cpis[:, None]                                   # [frame][rx][chirp][sample][2]
    with RadarCore(N_RANGE=1024, N_DOPPLER=128, in_dtype="i16", cfar="os1d", max_frames=2) as core:
        out = core.process(np.ascontiguousarray(cube))
    top = set(np.load(GOLDEN / "radar_output_profile.npz")["top_rows"].tolist())
    for f in range(2):
        m = out.rd_map[f]
        assert set(np.argsort(-m.sum(axis=1).astype(np.float64))[:6].tolist()) == top
        assert int(np.argmax(m[100])) == 5 and int(np.argmax(m[500])) == 118
    ref = np.stack([O.process(to_complex(cube[f], "i16"), None)["mag"] for f in range(2)])
    check_map(out.rd_map, ref)
    np.testing.assert_array_equal(out.dets, oracle_dets(out.rd_map, O.Cfar1D()))
    hit = {(int(r), int(d)) for r, d in zip(out.dets["range"], out.dets["doppler"])}
    assert (100, 5) in hit and (500, 118) in hit


@pytest.mark.parametrize("dtype", ["i16", "f32"])
def test_ambm_end_to_end(dtype):
    """K2 with magnitude_calc's alpha-max-beta-min (mx + floor(mn/4) + floor(mn/8),
    magnitude_calc.vhd:57-81) on the fp32 Doppler spectrum, vs the same formula on the oracle's
    fp64 spectrum; CFAR bit-exact on the GPU's AMBM map."""
    ns, nc = 512, 64
    cube = synth.frames(2, ns, nc, 1, "two_targets", dtype=dtype)
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, in_dtype=dtype, magnitude="ambm", cfar="os1d", max_frames=2) as core:
        out = core.process(cube)
    ref = []
    for f in range(2):
        rd = O.process(to_complex(cube[f], dtype), None)["rd"][0]
        ai, aq = np.abs(rd.real), np.abs(rd.imag)
        mx, mn = np.maximum(ai, aq), np.minimum(ai, aq)
        ref.append(mx + np.floor(mn / 4) + np.floor(mn / 8))
    check_map(out.rd_map, np.stack(ref))
    np.testing.assert_array_equal(out.dets, oracle_dets(out.rd_map, O.Cfar1D()))


def test_config4_share_1024_frames_one_enqueue():
    """Config 4's per-GPU share: 1024 config-2 frames in ONE fmcw_enqueue (8 chunks of 128).
    16 distinct frames tiled on the device; frames 0, 511, 1023 vs the oracle, every frame
    bit-identical to its source frame (maps and detections)."""
    ns, nc, F, U = 1024, 256, 1024, 16
    uniq = synth.frames(U, ns, nc, 1, "random_target", seed=901)
    fb = uniq[0].nbytes
    src = DeviceBuffer(uniq.nbytes)
    src.upload(uniq)
    cube = DeviceBuffer(F * fb)
    for f in range(F):
        cube.copy_from(src, fb, (f % U) * fb, f * fb)
    mb = ns * nc * 4
    dmap = DeviceBuffer(F * mb)
    cap = F * 4096
    ddet = DeviceBuffer(cap * 16)
    dn = DeviceBuffer(16)
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, cfar="os1d", max_frames=F) as core:
        core.enqueue(cube, F, dmap, ddet, cap, dn)
        n, dropped = (int(x) for x in dn.download(np.uint32, (2,)))
    assert dropped == 0 and n <= cap
    dets = ddet.download(DET_DTYPE, (n,))
    assert np.all(np.diff(dets["frame"].astype(np.int64)) >= 0)
    maps = {f: dmap.download(np.float32, (ns, nc), f * mb) for f in (0, 15, 511, 1023)}
    for f in (0, 511, 1023):
        ref = O.process(uniq[f % U], None)["mag"]
        check_map(maps[f][None], ref[None])
        np.testing.assert_array_equal(dets[dets["frame"] == f][["range", "doppler", "mag", "threshold"]],
                                      oracle_dets(maps[f][None], O.Cfar1D())[["range", "doppler", "mag", "threshold"]])
    np.testing.assert_array_equal(maps[511], maps[15])
    np.testing.assert_array_equal(maps[1023], maps[15])
    per_src = {}
    for f in range(F):
        d = dets[dets["frame"] == f][["range", "doppler", "mag", "threshold"]]
        if f % U in per_src:
            np.testing.assert_array_equal(d, per_src[f % U])
        else:
            per_src[f % U] = d


def test_cfar2d_dense_tiles_use_overflow_region():
    """the 2-D CFAR's phase B also spills tiles past their slot (1/32 of the tile's
    cells) into the shared overflow region; the list stays complete and ordered."""
    rng = np.random.default_rng(8)
    m = rng.rayleigh(1.0, (2, 128, 64)).astype(np.float32)
    m[:, ::4, ::4] = 100.0                     # 1/16 of the cells detect: 64 per 1024-cell tile
    with RadarCore(N_RANGE=128, N_DOPPLER=64, cfar="os2d", max_frames=2) as core:
        got = run_cfar_stage(core, m)
    want = oracle_dets(m, O.Cfar2D())
    assert len(want) > 900
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("det_capacity", [0, 65536])
def test_dropped_detections_are_reported(det_capacity):
    """A map on which 255 of every 256 cells detect.  With the default scratch (ABI 8: every
    cell) the whole list is stored and exact; with a bounded one (det_capacity = 65536 overflow
    records) the detections beyond it are counted in n_dets[1] (fmcw_process: FMCW_EDETCAP),
    never silently lost."""
    ns, nc = 1024, 256
    ramp = np.broadcast_to(np.arange(1, nc + 1, dtype=np.float32), (1, ns, nc)).copy()
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, cfar="os1d", cfar1d=(1, 0, 0, 1.0), max_frames=1,
                   det_capacity=det_capacity) as core:
        got, n, dropped = _stage_dets(core, ramp, cap=1 << 19)
        want = oracle_dets(ramp, O.Cfar1D(ref=1, guard=0, rank=0, alpha=1.0))
        assert n == len(want) == ns * (nc - 1)
        if det_capacity:
            # every detection is counted; those beyond the scratch (8192 slot + 65536 overflow
            # entries at max_frames 1) are reported as dropped
            assert dropped >= n - (8192 + det_capacity)
        else:
            assert dropped == 0
            np.testing.assert_array_equal(got, want)
        # the same map well inside the scratch is complete and exact
        small = ramp[:, :64].copy()
        got2, n2, dropped2 = _stage_dets(core, np.concatenate([small, np.zeros((1, ns - 64, nc), np.float32)], 1))
        assert dropped2 == 0
        np.testing.assert_array_equal(got2, oracle_dets(np.concatenate([small, np.zeros((1, ns - 64, nc), np.float32)], 1),
                                                        O.Cfar1D(ref=1, guard=0, rank=0, alpha=1.0)))


@pytest.mark.parametrize("kind", ["os1d", "os2d"])
def test_negative_and_negative_zero_cells(kind):
    """fmcw_cfar takes negative cells and -0.0 as +0 (the RTL's unsigned magnitude
    stream), identical to the oracle on the clamped map."""
    rng = np.random.default_rng(21)
    m = rng.normal(0.0, 3.0, (2, 128, 64)).astype(np.float32)
    m[:, :, 5] = -0.0
    m[0, 40, 10] = 200.0
    m[1, 70, 33] = 150.0
    clamped = np.where(m > 0, m, 0).astype(np.float32)
    cf = O.Cfar1D() if kind == "os1d" else O.Cfar2D()
    with RadarCore(N_RANGE=128, N_DOPPLER=64, cfar=kind, max_frames=2) as core:
        got = run_cfar_stage(core, m)
    np.testing.assert_array_equal(got, oracle_dets(clamped, cf))
    assert (40, 10) in set(zip(got["range"].tolist(), got["doppler"].tolist()))


def _rtl_dets(maps, cf):
    out = []
    for f in range(maps.shape[0]):
        if isinstance(cf, O.Cfar1D):
            det, thr = O.cfar_os1d_rtl(maps[f], cf)
        else:
            det, thr = O.cfar_os2d_rtl(maps[f], cf)
        out.append(O.detections_rtl(det, maps[f], thr, frame=f))
    return np.concatenate(out)


@pytest.mark.parametrize("kind", ["os1d", "os2d"])
def test_compat_cfar_stage(kind):
    """FMCW_COMPAT_CFAR through fmcw_cfar on maps whose cells span the 17-bit range (so the 1-D
    threshold wraps mod 2^17 and the 2-D bracket add wraps), fractions and out-of-range cells
    included; bit-exact vs cfar_os1d_rtl / cfar_os2d_rtl."""
    rng = np.random.default_rng(31)
    if kind == "os1d":
        m = rng.uniform(0, 140000, (2, 128, 128)).astype(np.float32)
        m[0, ::7, ::5] = rng.uniform(25000, 60000, m[0, ::7, ::5].shape)
    else:
        m = rng.uniform(5000, 15000, (2, 128, 128)).astype(np.float32)
        m[0, 50, 60], m[1, 60, 100], m[1, 90, 3] = 131000.0, 120000.0, 70000.5
        m[0, 10:12, :] = 150000.0                          # saturates at 2^17 - 1
        m[0, 100, 5:9] = 2.0 ** 17 - 1.5
    m[1, 20:40, 10:30] = rng.uniform(90000, 131000, (20, 20))   # mean ~1e5: the 17-bit bracket add wraps
    m[1, 30, 20] = 131071.0
    m[1, 50, 50] = -5.0
    cf = O.Cfar1D() if kind == "os1d" else O.Cfar2D()
    with RadarCore(N_RANGE=128, N_DOPPLER=128, cfar=kind, compat_rtl=("cfar",), max_frames=2) as core:
        got = run_cfar_stage(core, m)
    want = _rtl_dets(m, cf)
    assert len(want) > 0
    np.testing.assert_array_equal(got, want)


def test_compat_cfar_tb_map():
    """tb_os_cfar_2d.vhd's integer map with its generics in RTL-compat arithmetic: both
    targets found, bit-exact vs the integer restatement."""
    z = np.load(GOLDEN / "tb_cfar2d.npz")
    rr, gr, rd, gd = z["params"].tolist()
    p = O.Cfar2D(ref_range=rr, guard_range=gr, ref_doppler=rd, guard_doppler=gd)
    with RadarCore(N_RANGE=64, N_DOPPLER=32, CFAR_REF_R=rd, CFAR_GUARD_R=gd, CFAR_REF_D=rr,
                   CFAR_GUARD_D=gr, cfar="os2d", compat_rtl=("cfar",)) as core:
        got = run_cfar_stage(core, z["map"].astype(np.float32)[None])
    np.testing.assert_array_equal(got, _rtl_dets(z["map"].astype(np.float32)[None], p))
    pos = set(zip(got["range"].tolist(), got["doppler"].tolist()))
    assert (30, 16) in pos and (50, 8) in pos


def test_compat_cfar_fused_1d():
    """The 1-D compat CFAR fused into K2 (AMBM magnitude, int16 ADC words, range_shift so the
    map sits in the 17-bit range) == the integer restatement on the GPU's own map."""
    ns, nc = 1024, 128
    cube = synth.frames(2, ns, nc, 1, "random_target", dtype="i16")
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, in_dtype="i16", magnitude="ambm", cfar="os1d",
                   compat_rtl=("cfar",), range_shift=10, max_frames=2) as core:
        out = core.process(cube)
        exact = run_cfar_stage(core, out.rd_map)
    want = _rtl_dets(out.rd_map, O.Cfar1D())
    np.testing.assert_array_equal(out.dets, want)
    np.testing.assert_array_equal(exact, want)
    assert (out.rd_map < 131072).mean() > 0.99       # the map lives in the 17-bit word range


@pytest.mark.parametrize("mode", [2, 3])
def test_compat_mti(mode):
    """FMCW_COMPAT_MTI: the canceller on int16 words (doppler_notch.vhd:67-93) after the range
    FFT scaled by 2^-10 (the IP's scaling schedule).  Checked exactly against the oracle fed the
    GPU's own range spectrum (fmcw_range_ct; rounding to integers is then identical), and at
    frame level against the fp64 end-to-end oracle."""
    ns, nc = 1024, 128
    cube = synth.frames(2, ns, nc, 1, "random_target", dtype="i16")
    kw = dict(N_RANGE=ns, N_DOPPLER=nc, in_dtype="i16", cfar="os2d", mti_bypass=False, NOTCH_MODE=mode,
              compat_rtl=("mti",), range_shift=10, max_frames=2)
    with RadarCore(**kw) as core:
        out = core.process(cube)
        spec = run_range_ct(core, cube, 2)              # [f][rx][range][chirp], scaled, unwindowed in slow time
    for f in range(2):
        y = O.mti_spectrum_rtl(spec[f, 0].astype(np.complex128), mode)
        assert np.abs(y.real).max() <= 32767 and np.abs(y.imag).max() <= 32768
        ref = O.magnitude(O.doppler_fft(y[None]), rx_axis=0)
        check_map(out.rd_map[f][None], ref[None])
        e2e = O.process(to_complex(cube[f], "i16"), None, mti_mode=mode, range_shift=10, mti_rtl=True)["mag"]
        assert rel_err(out.rd_map[f], e2e) <= 1e-4
    np.testing.assert_array_equal(out.dets, oracle_dets(out.rd_map, O.Cfar2D()))


def test_rccl_gather_one_rank():
    """fmcw_gather_dets on a one-rank RCCL communicator: the pack, the root's self message and
    the device-side compaction (frame offset applied, count header, wire_cap overflow)."""
    rng = np.random.default_rng(5)
    n = 300
    recs = np.zeros(n, DET_DTYPE)
    recs["frame"] = np.sort(rng.integers(0, 8, n))
    recs["range"] = rng.integers(0, 1024, n)
    recs["doppler"] = rng.integers(0, 256, n)
    recs["mag"] = rng.uniform(0, 1e6, n)
    recs["threshold"] = rng.uniform(0, 1e6, n)
    dd = DeviceBuffer(n * 16)
    dd.upload(recs)
    dn = DeviceBuffer(16)
    dn.upload(np.array([n, 2], np.uint32))            # 2 records lost upstream
    wire = 512
    out = DeviceBuffer(wire * 16)
    on = DeviceBuffer(16)
    g = RcclGather(RcclGather.make_id(), 1, 0, 0, wire)
    try:
        g.gather(dd.ptr, n, dn.ptr, 1000, out.ptr, on.ptr, 0, 0)
        got_n = on.download(np.uint32, (2,))
        got = out.download(DET_DTYPE, (n,))
        want = recs.copy()
        want["frame"] += 1000
        assert list(got_n) == [n, 2]
        np.testing.assert_array_equal(got, want)
        # det_cap below the count (fmcw_enqueue stored only det_cap records): those travel,
        # the rest are counted lost
        g.gather(dd.ptr, 100, dn.ptr, 0, out.ptr, on.ptr, 0, 0)
        got_n = on.download(np.uint32, (2,))
        assert list(got_n) == [100, n - 100 + 2]
        np.testing.assert_array_equal(out.download(DET_DTYPE, (100,)), recs[:100])
    finally:
        g.close()
    # wire_cap below the count: the first wire_cap records travel, the rest are counted lost
    g = RcclGather(RcclGather.make_id(), 1, 0, 0, 100)
    try:
        g.gather(dd.ptr, n, dn.ptr, 0, out.ptr, on.ptr, 0, 0)
        assert list(on.download(np.uint32, (2,))) == [100, n - 100 + 2]
        np.testing.assert_array_equal(out.download(DET_DTYPE, (100,)), recs[:100])
    finally:
        g.close()


def _cli(*args):
    return subprocess.run([sys.executable, "-m", "fmcw.cli", *map(str, args)], cwd=str(PKG),
                          capture_output=True, text=True, timeout=300, check=True)


def test_cli_golden_chirp_writes_visualizer_files(tmp_path):
    """python -m fmcw.cli on data/golden_input_chirp.txt (config-1 framing): the detection file
    parses under the visualizer's rule (3 integer tokens) and equals RadarCore's own list; the
    map file is data/radar_output.txt's 5-column format; --doppler-centred shifts by N/2."""
    _cli(GOLDEN / "golden_input_chirp.txt", "--n-range", 256, "--n-doppler", 128, "--cfar", "os1d",
         "--out-dir", tmp_path, "--map-file", "radar_output.txt")
    iq = formats.read_adc_pairs(GOLDEN / "golden_input_chirp.txt")
    with RadarCore(N_RANGE=256, N_DOPPLER=128, cfar="os1d") as core:
        out = core.process(synth.golden_chirp_frame(iq, 128, 256)[None])
    got = formats.read_detections(tmp_path / "ADR_detections.txt")
    want = np.stack([out.dets["range"], out.dets["doppler"], np.rint(out.dets["mag"].astype(np.float64))], 1)
    np.testing.assert_array_equal(got, want.astype(np.int64))
    m = formats.read_rd_map(tmp_path / "radar_output.txt", 256, 128)
    np.testing.assert_array_equal(m, np.rint(out.rd_map[0].astype(np.float64)).astype(np.int64))
    assert np.unravel_index(np.argmax(m), m.shape) == (73, 0)
    cdir = tmp_path / "centred"
    _cli(GOLDEN / "golden_input_chirp.txt", "--n-range", 256, "--n-doppler", 128, "--cfar", "os1d",
         "--out-dir", cdir, "--map-file", "radar_output.txt", "--doppler-centred")
    mc = formats.read_rd_map(cdir / "radar_output.txt", 256, 128)
    assert np.unravel_index(np.argmax(mc), mc.shape) == (73, 64)      # zero Doppler at N/2
    gc = formats.read_detections(cdir / "ADR_detections.txt")
    np.testing.assert_array_equal(gc[:, 1], (got[:, 1] + 64) % 128)


def test_cli_axi_bin_stream(tmp_path):
    """A raw AXI word stream ({Q[31:16], I[15:0]}, tlast framing = whole chirps) of the
    tb_radar_core stimulus through the CLI == RadarCore on the int16 cube."""
    cpis = synth.tb_radar_core_v3_cpis()
    from fmcw.radar_core import pack_adc_words
    words = pack_adc_words(cpis[..., 0].reshape(-1), cpis[..., 1].reshape(-1)).astype("<u4")
    b = tmp_path / "stream.bin"
    words.tofile(b)
    _cli(b, "--n-range", 1024, "--n-doppler", 128, "--cfar", "os1d", "--out-dir", tmp_path)
    with RadarCore(N_RANGE=1024, N_DOPPLER=128, in_dtype="i16", cfar="os1d", max_frames=2) as core:
        out = core.process(np.ascontiguousarray(cpis[:, None]))
    got = formats.read_detections(tmp_path / "ADR_detections.txt")
    want = np.stack([out.dets["range"], out.dets["doppler"], np.rint(out.dets["mag"].astype(np.float64))], 1)
    np.testing.assert_array_equal(got, want.astype(np.int64))


def test_process_host_staging_is_reused():
    """fmcw_process with host buffers keeps its staging in the handle: repeated calls of
    different sizes give the same results as fresh handles."""
    ns, nc = 512, 64
    cube = synth.frames(4, ns, nc, 1, "random_target", seed=3)
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, cfar="os1d", max_frames=4) as core:
        a = core.process(cube[:1])
        b = core.process(cube)
        c = core.process(cube[:2])
    np.testing.assert_array_equal(a.rd_map[0], b.rd_map[0])
    np.testing.assert_array_equal(c.rd_map, b.rd_map[:2])
    np.testing.assert_array_equal(c.dets, b.dets[b.dets["frame"] < 2])


@pytest.mark.parametrize("chunk", [8, 5])
def test_repeated_launches_and_device_pointers(chunk):
    """Back-to-back launches on device buffers (the bench's pattern) with small K1 -> K2 chunks
    (several chunks per call, one short): every launch equals the first, batches of different
    sizes included, and equals the auto-chunked path."""
    ns, nc, F = 1024, 256, 64
    uniq = synth.frames(8, ns, nc, 1, "random_target", seed=44)
    cube = DeviceBuffer(F * uniq[0].nbytes)
    for f in range(F):
        cube.upload(uniq[f % 8], f * uniq[0].nbytes)
    dmap = DeviceBuffer(F * ns * nc * 4)
    cap = F * 4096
    ddet = DeviceBuffer(cap * 16)
    dn = DeviceBuffer(16)
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, cfar="os1d", max_frames=F, chunk_frames=chunk) as core:
        assert core.info("chunk") == chunk
        runs = []
        for nfr in (F, F, 17, F):
            core.enqueue(cube, nfr, dmap, ddet, cap, dn)
            n, dropped = (int(v) for v in dn.download(np.uint32, (2,)))
            assert dropped == 0
            runs.append((nfr, dmap.download(np.float32, (nfr, ns, nc)), ddet.download(DET_DTYPE, (n,))))
    _, m0, d0 = runs[0]
    for nfr, m, d in runs[1:]:
        np.testing.assert_array_equal(m, m0[:nfr])
        np.testing.assert_array_equal(d, d0[d0["frame"] < nfr])
    for f in range(8, F):
        np.testing.assert_array_equal(m0[f], m0[f % 8])
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, cfar="os1d", max_frames=F) as core:
        core.enqueue(cube, F, dmap, ddet, cap, dn)
        n, _ = (int(v) for v in dn.download(np.uint32, (2,)))
        np.testing.assert_array_equal(dmap.download(np.float32, (F, ns, nc)), m0)
        np.testing.assert_array_equal(ddet.download(DET_DTYPE, (n,)), d0)


@pytest.mark.parametrize("steps", ["1", "3", "7", "0"])
def test_cfar2d_strips_and_batched_launches(steps):
    """The 2-D CFAR walks strips of `steps` workgroup tiles through a ring of staged rows
    (cfar2d.hpp RowRing; 3 and 7 leave a short last strip per frame) and, on the caller's map,
    runs once per >= 16 frames (20 frames in chunks of 4: launches of 16 + 4).  Detections
    bit-exact vs the C oracle on the map the path wrote."""
    ns, nc, nf = 512, 128, 20
    cube = synth.frames(nf, ns, nc, 1, "two_targets")
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, cfar="os2d", max_frames=nf, chunk_frames=4) as core:
        core.set_param("cfar2d_steps", int(steps))
        out = core.process(cube)
        if steps != "0":
            assert core.info("cfar2d_steps") == int(steps)
    want = CB.cfar(out.rd_map, O.Cfar2D(), threads=16)
    np.testing.assert_array_equal(out.dets, want)
    assert out.n_dets > nf


@pytest.mark.parametrize("ns,nc,nrx,dtype,cfar,mti", [
    (8192, 1024, 1, "f16", "os2d", 0),   # BASELINE config 5 with the fp16 spectrum
    (1024, 256, 1, "f32", "os1d", 0),    # config 2 geometry
    (512, 64, 2, "i16", "os1d", 2),      # NCI over 2 rx, MTI 2-pulse on the fp16 spectrum
    (256, 128, 1, "i16", "os2d", 3),
])
def test_fp16_spectrum(ns, nc, nrx, dtype, cfar, mti):
    """FMCW_SPEC_F16 (fmcw.h): half2(X / N_range) between K1 and K2.  Map within the stated
    2e-3 of the fp64 oracle per frame; CFAR bit-exact vs the C oracle on the map produced."""
    nf = 1 if ns == 8192 else 2
    cube = synth.frames(nf, ns, nc, nrx, "two_targets", dtype=dtype)
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, N_RX=nrx, in_dtype=dtype, cfar=cfar, max_frames=nf,
                   mti_bypass=mti == 0, NOTCH_MODE=mti or 2, spectrum="f16") as core:
        out = core.process(cube)
    for f in range(nf):
        ref = O.process(to_complex(cube[f], dtype), None, mti_mode=mti)["mag"]
        assert rel_err(out.rd_map[f], ref) <= 2e-3
    p = O.Cfar2D() if cfar == "os2d" else O.Cfar1D()
    np.testing.assert_array_equal(out.dets, CB.cfar(out.rd_map, p, threads=16))
    assert out.n_dets >= nf


def test_fp16_spectrum_ambm_and_stage_api():
    """AMBM on the fp16 spectrum against the fp32-spectrum path's map (2e-3), and
    fmcw_range_ct still returning the fp32 spectrum (1e-4 vs the oracle) on an F16 handle."""
    ns, nc, nf = 512, 64, 3
    cube = synth.frames(nf, ns, nc, 1, "two_targets", dtype="i16")
    maps = {}
    for sp in ("f32", "f16"):
        with RadarCore(N_RANGE=ns, N_DOPPLER=nc, in_dtype="i16", magnitude="ambm", cfar="os1d",
                       max_frames=nf, spectrum=sp) as core:
            maps[sp] = core.process(cube).rd_map
            if sp == "f16":
                spec = run_range_ct(core, cube, nf)
    for f in range(nf):
        assert rel_err(maps["f16"][f], maps["f32"][f]) <= 2e-3
        ref = O.range_ct(to_complex(cube[f], "i16"))
        assert rel_err(spec[f], ref) <= 1e-4


@pytest.mark.parametrize("ref_r,guard_r,ref_d,guard_d,pct,scales,steps", [
    (4, 1, 4, 2, 75, (2, 4, 6), "2"),    # reference window: packed screen, strips of 2
    (4, 1, 4, 2, 90, (3, 4, 5), "0"),    # screen with need = 13, other scales
    (2, 1, 3, 1, 50, (1, 3, 5), "3"),    # other window: runtime-geometry phase A
    (3, 0, 5, 3, 75, (2, 2, 2), "1"),    # no range guard, equal scales
])
def test_cfar2d_geometries_and_ranks(ref_r, guard_r, ref_d, guard_d, pct, scales, steps):
    """2-D CFAR at several windows, ranks and scale sets (oracle naming: ref/guard along range
    and Doppler), Rayleigh clutter with targets and a quiet patch, 3 frames; bit-exact vs the
    C oracle.  The pivoting k-th select runs at ranks other than 96 here."""
    rng = np.random.default_rng(ref_r * 100 + pct)
    m = rng.rayleigh(10.0, (3, 256, 128)).astype(np.float32)
    m[:, 100:120, 20:40] = rng.rayleigh(150.0, (3, 20, 20))
    m[:, 200:230, 60:90] = 0.02
    m[0, 50, 7] = 900.0
    m[1, 180, 127] = 700.0
    m[2, 10:12, 64] = 800.0
    p = O.Cfar2D(ref_range=ref_r, guard_range=guard_r, ref_doppler=ref_d, guard_doppler=guard_d,
                 rank_pct=pct, scale_min=scales[0], scale_nom=scales[1], scale_max=scales[2])
    with RadarCore(N_RANGE=256, N_DOPPLER=128, CFAR_REF_R=ref_d, CFAR_GUARD_R=guard_d, CFAR_REF_D=ref_r,
                   CFAR_GUARD_D=guard_r, cfar_rank_pct=pct, cfar_scales=scales, cfar="os2d",
                   max_frames=3) as core:
        core.set_param("cfar2d_steps", int(steps))
        got, n, dropped = _stage_dets(core, m)
    assert dropped == 0
    want = CB.cfar(m, p, threads=16)
    np.testing.assert_array_equal(got, want)
    assert len(want) >= 3
