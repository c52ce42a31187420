"""Round-5 GPU tests (libfmcw.so on gfx950 through the C-ABI, checked against the CPU oracle).

  * The headline's own shape (round-4 verdict item 1): BASELINE config 2 exactly as bench.py
    runs it -- 1024 frames of 256 x 1024 fp32 in one fmcw_enqueue on device-resident buffers,
    the auto 104-frame chunks (ten K1 -> K2 launch pairs, the last of 88 frames), the fused 1-D
    OS-CFAR, the map written, one k_det_list over 256 look-back blocks.  Maps of frame 0, the
    first frame of chunk 6 and frame 1023 within 1e-4 of the fp64 oracle; every frame's map
    bit-identical to that of the frame it repeats (the bench tiles 16 distinct frames); all
    1024 frames' detections bit-exact vs the C oracle's 1-D OS-CFAR on the GPU's map.
    Semantics: rtl/old/os_cfar.vhd:98-137, rtl/old/radar_core_v3.vhd:373-381.
  * hipGraph capture of fmcw_enqueue / fmcw_cfar: one capture replayed on
    cubes with different detection counts, interleaved with direct calls on the same handle;
    every replay's list equals the direct call's (k_det_list keeps its call tag in device memory).
  * fmcw_comm_create with an injected buffer-allocation failure (round-4 verdict item 6).
"""
import ctypes as C

import numpy as np
import pytest

import cpu_backend as CB
import fmcw_oracle as O
from conftest import REPO
from fmcw import RadarCore, DeviceBuffer, DET_DTYPE, synth
from fmcw import _lib as L
from test_gpu_parity import check_map

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("spectrum", ["s48", "f32"])
def test_headline_shape_parity(gpu, spectrum):
    """(s48 is the bench's config-2 spectrum since round 5; f32 the fp32 path.)"""
    import sys
    if str(REPO) not in sys.path:
        sys.path.insert(0, str(REPO))
    import bench
    w = bench.WORKLOADS["c2"]
    F, ns, nc, nrx = w["frames"], w["ns"], w["nc"], w["nrx"]
    assert (F, ns, nc, nrx, w["dtype"], w["cfar"], w["spectrum"]) == (1024, 1024, 256, 1, "f32", "os1d", "s48")
    # bench.run_workload at rank 0: 16 distinct frames (seed 1234), tiled to F, resident in HBM
    n_u = 16
    u = np.ascontiguousarray(synth.frames(n_u, ns, nc, nrx, w["recipe"], seed=1234, dtype="f32"))
    fb = u.nbytes // n_u
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, N_RX=nrx, in_dtype="f32", cfar="os1d", max_frames=F,
                   spectrum=spectrum) as core:
        chunk = core.info("chunk")
        # f32: ten chunks of 104 frames, the last 88; s48 (6 B per point, same 208 MiB budget):
        # seven of 138, the last 58
        assert (chunk, F % chunk) == ((104, 88) if spectrum == "f32" else (138, 58))
        src = DeviceBuffer(u.nbytes)
        src.upload(u)
        cube = DeviceBuffer(F * fb)
        for k in range(F // n_u):
            cube.copy_from(src, u.nbytes, dst_offset=k * u.nbytes)
        del src
        rd = DeviceBuffer(F * ns * nc * 4)
        cap = F * 4096
        dd = DeviceBuffer(cap * 16)
        dn = DeviceBuffer(16)
        core.enqueue(cube, F, rd_map=rd, dets=dd, det_cap=cap, n_dets=dn)
        st = dn.download(np.uint32, (4,))
        n = int(st[0])
        assert st[1] == 0 and st[2] == 0 and st[3] == 0
        dets = dd.download(DET_DTYPE, (n,))
        del cube, dd
        rd_map = rd.download(np.float32, (F, ns, nc))
    # maps: frames 0, 6 x chunk (first of chunk 6) and 1023 vs the fp64 oracle of the frame they repeat
    for f in (0, 6 * chunk, F - 1):
        ref = O.process(u[f % n_u].astype(np.complex128), None)["mag"]
        check_map(rd_map[f:f + 1], ref[None])
    # every frame bit-identical to its source frame's map (no chunk mixes frames up)
    for f in range(n_u, F):
        assert np.array_equal(rd_map[f], rd_map[f % n_u]), f"frame {f} differs from frame {f % n_u}"
    # all 1024 frames' detections bit-exact vs the C oracle's CFAR on the GPU's map
    want = CB.cfar(rd_map, O.Cfar1D(), threads=16, cap=1 << 24)
    assert n == len(want) >= 2 * F
    np.testing.assert_array_equal(dets, want)
    assert set(dets["frame"].tolist()) == set(range(F))


# ---- hipGraph capture -------------------------------------------------------------------------
class _Hip:
    """The few HIP runtime calls a graph capture needs, bound with ctypes (no torch)."""
    CAPTURE_RELAXED = 2   # hipStreamCaptureModeRelaxed

    def __init__(self):
        self.lib = C.CDLL("libamdhip64.so")
        for name in ("hipStreamCreate", "hipStreamDestroy", "hipStreamBeginCapture", "hipStreamEndCapture",
                     "hipGraphInstantiate", "hipGraphLaunch", "hipGraphExecDestroy", "hipGraphDestroy",
                     "hipStreamSynchronize"):
            getattr(self.lib, name).restype = C.c_int
        self.lib.hipStreamBeginCapture.argtypes = [C.c_void_p, C.c_int]
        self.lib.hipStreamEndCapture.argtypes = [C.c_void_p, C.POINTER(C.c_void_p)]
        self.lib.hipGraphInstantiate.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, C.c_void_p, C.c_void_p,
                                                 C.c_size_t]
        self.lib.hipGraphLaunch.argtypes = [C.c_void_p, C.c_void_p]
        self.lib.hipStreamSynchronize.argtypes = [C.c_void_p]
        self.lib.hipStreamDestroy.argtypes = [C.c_void_p]
        self.lib.hipGraphExecDestroy.argtypes = [C.c_void_p]
        self.lib.hipGraphDestroy.argtypes = [C.c_void_p]

    def ok(self, rc):
        assert rc == 0, f"HIP error {rc}"

    def stream(self):
        s = C.c_void_p()
        self.ok(self.lib.hipStreamCreate(C.byref(s)))
        return s

    def capture(self, s, fn):
        self.ok(self.lib.hipStreamBeginCapture(s, self.CAPTURE_RELAXED))
        try:
            fn()
        finally:
            g = C.c_void_p()
            rc = self.lib.hipStreamEndCapture(s, C.byref(g))
        self.ok(rc)
        exe = C.c_void_p()
        self.ok(self.lib.hipGraphInstantiate(C.byref(exe), g, None, None, 0))
        return g, exe

    def replay(self, exe, s):
        self.ok(self.lib.hipGraphLaunch(exe, s))
        self.ok(self.lib.hipStreamSynchronize(s))


def _cubes(ns, nc, nf):
    """Cubes with clearly different detection counts (two targets vs one strong random target per
    frame vs pure noise)."""
    a = synth.frames(nf, ns, nc, 1, "two_targets", seed=71)
    b = synth.frames(nf, ns, nc, 1, "random_target", seed=72)
    c = np.ascontiguousarray(synth.frames(nf, ns, nc, 1, "two_targets", seed=73))
    c[: nf // 2] *= 0.0    # frames without any energy: no detection there
    return [np.ascontiguousarray(x) for x in (a, b, c)]


@pytest.mark.parametrize("cfar", ["os1d", "os2d"])
def test_graph_capture_replay(gpu, cfar):
    """fmcw_enqueue captured once (16 frames of 256 x 1024: 4096 detection tiles, 4 look-back
    blocks) and replayed on three cubes with different detection counts, a direct call on the
    same handle between replays, and the first cube again: every replay's status words and list
    equal the direct call's on the same cube, and the direct calls equal the C oracle's CFAR on
    their maps."""
    ns, nc, nf = 1024, 256, 16
    cubes = _cubes(ns, nc, nf)
    cf = O.Cfar1D() if cfar == "os1d" else O.Cfar2D()
    hip = _Hip()
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, cfar=cfar, max_frames=nf, chunk_frames=6) as core:
        want = []
        for x in cubes:
            out = core.process(x)
            np.testing.assert_array_equal(out.dets, CB.cfar(out.rd_map, cf, threads=16))
            want.append(out)
        assert len({w.n_dets for w in want}) == 3, [w.n_dets for w in want]
        cube = DeviceBuffer(cubes[0].nbytes)
        rd = DeviceBuffer(nf * ns * nc * 4)
        cap = nf * 4096
        dd = DeviceBuffer(cap * 16)
        dn = DeviceBuffer(16)
        s = hip.stream()
        g, exe = hip.capture(s, lambda: core.enqueue(cube, nf, rd_map=rd, dets=dd, det_cap=cap, n_dets=dn,
                                                     stream=s.value))
        try:
            for k in (0, 1, 2, 0, 1):
                cube.upload(cubes[k])
                hip.replay(exe, s)
                st = dn.download(np.uint32, (4,))
                assert int(st[0]) == want[k].n_dets and st[1] == 0, (k, st, want[k].n_dets)
                np.testing.assert_array_equal(dd.download(DET_DTYPE, (int(st[0]),)), want[k].dets)
                np.testing.assert_array_equal(rd.download(np.float32, (nf, ns, nc)), want[k].rd_map)
                # a direct call between replays (another cube), checked too
                j = (k + 1) % 3
                out = core.process(cubes[j])
                np.testing.assert_array_equal(out.dets, want[j].dets)
        finally:
            hip.lib.hipGraphExecDestroy(exe)
            hip.lib.hipGraphDestroy(g)
            hip.lib.hipStreamDestroy(s)


def test_graph_capture_cfar_stage(gpu):
    """fmcw_cfar (2-D, a caller map) captured once and replayed on maps with very different
    detection counts (1280 detection tiles: two look-back blocks): each replay equals the oracle.
    (The dense map stays within the handle's detection scratch: its tiles of > 32 detections go
    to the shared overflow region, 64 Ki records here.)"""
    ns, nc, nf = 1024, 256, 5
    rng = np.random.default_rng(81)
    maps = []
    for dense in (False, True, False):
        m = rng.rayleigh(1.0, (nf, ns, nc)).astype(np.float32)
        if dense:
            m[:, ::6, ::6] = 50.0
        else:
            m[:, 100, 40] = 80.0
        maps.append(m)
    want = [CB.cfar(m, O.Cfar2D(), threads=16) for m in maps]
    assert len(want[1]) > 20 * (len(want[0]) + 1)
    hip = _Hip()
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, cfar="os2d", max_frames=nf) as core:
        dm = DeviceBuffer(maps[0].nbytes)
        cap = 1 << 20
        dd = DeviceBuffer(cap * 16)
        dn = DeviceBuffer(16)
        s = hip.stream()
        g, exe = hip.capture(s, lambda: core.cfar(dm, nf, dd, cap, dn, stream=s.value))
        try:
            for k in (0, 1, 2, 1, 0):
                dm.upload(maps[k])
                hip.replay(exe, s)
                st = dn.download(np.uint32, (4,))
                assert int(st[0]) == len(want[k]) and st[1] == 0
                np.testing.assert_array_equal(dd.download(DET_DTYPE, (int(st[0]),)), want[k])
        finally:
            hip.lib.hipGraphExecDestroy(exe)
            hip.lib.hipGraphDestroy(g)
            hip.lib.hipStreamDestroy(s)


def test_comm_create_alloc_failure_one_rank(gpu):
    """An injected buffer-allocation failure in fmcw_comm_create returns FMCW_ENOMEM (after the
    communicator is built: the same path a multi-rank job takes into its collective check) and
    leaves nothing behind; the next create succeeds."""
    from fmcw.dist import RcclGather
    lib = L.load()
    uid = RcclGather.make_id()
    assert lib.fmcw_comm_fail_next_alloc_for_test(1) == 0
    with pytest.raises(L.FmcwError) as e:
        RcclGather(uid, 1, 0, 0, 64)
    assert e.value.code == L.FMCW_ENOMEM and "per rank" in str(e.value)
    rg = RcclGather(RcclGather.make_id(), 1, 0, 0, 64)
    rg.close()


# ---- FMCW_SPEC_S48: the 6-byte corner-turned spectrum (round-4 verdict item 5) ------------------
@pytest.mark.parametrize("ns,nc,nf,dtype,cfar,recipe", [
    (1024, 256, 6, "f32", "os1d", "two_targets"),      # config 2's geometry
    (1024, 256, 6, "f32", "os1d", "random_target"),
    (1024, 256, 4, "i16", "os2d", "random_target"),
    (1024, 64, 4, "f16", "os1d", "two_targets"),       # P = 4: one lane quad per row
    (512, 128, 4, "f32", "os2d", "two_targets"),       # T = 8
    (128, 1024, 3, "f32", "os2d", "random_target"),    # T = 16, NC = 1024 (no prefetch)
    (1024, 512, 3, "f32", "os1d", "random_target"),
    # the pair form (K1 tiles of T = 2 chirps, n_range >= 2048): k_range, k_range_sq, k_range_px
    (2048, 256, 3, "f32", "os1d", "random_target"),
    (4096, 128, 2, "i16", "os2d", "two_targets"),
    (4096, 64, 2, "f32", "os1d", "random_target"),     # P = 4
    (8192, 64, 2, "f16", "os1d", "two_targets"),
    (8192, 128, 2, "f32", "os2d", "random_target"),
])
def test_s48_parity(gpu, ns, nc, nf, dtype, cfar, recipe):
    """Maps within the north star's 1e-4 (per frame and per bin above 1e-3 of the frame peak) of
    the fp64 oracle, the same bound as the fp32 spectrum; detections bit-exact vs the C oracle's
    CFAR on the GPU's map."""
    from test_gpu_parity import to_complex
    cube = synth.frames(nf, ns, nc, 1, recipe, seed=2025 + ns + nc, dtype=dtype)
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, in_dtype=dtype, cfar=cfar, max_frames=nf, spectrum="s48") as core:
        out = core.process(cube)
    for f in range(nf):
        ref = O.process(to_complex(cube[f], dtype), None)["mag"]
        check_map(out.rd_map[f:f + 1], ref[None])
    cf = O.Cfar1D() if cfar == "os1d" else O.Cfar2D()
    np.testing.assert_array_equal(out.dets, CB.cfar(out.rd_map, cf, threads=16))
    assert out.n_dets >= nf


def test_s48_bench_shape_two_chunks(gpu):
    """Config 2 with the S48 spectrum at 208 frames in one call (two auto chunks of 104 frames at
    6 B per point: the chunk keeps its 208 MiB budget, so more frames fit), device-resident:
    maps of the first / last frame vs the oracle, every frame's map bit-identical to its source
    frame's, detections bit-exact vs the C oracle on the map."""
    ns, nc, F, n_u = 1024, 256, 208, 16
    u = np.ascontiguousarray(synth.frames(n_u, ns, nc, 1, "two_targets", seed=1234, dtype="f32"))
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, cfar="os1d", max_frames=F, spectrum="s48") as core:
        chunk = core.info("chunk")
        assert chunk == min(F, (208 << 20) // (ns * nc * 6)) and chunk > 104
        src = DeviceBuffer(u.nbytes)
        src.upload(u)
        cube = DeviceBuffer(F * u.nbytes // n_u)
        for k in range(F // n_u):
            cube.copy_from(src, u.nbytes, dst_offset=k * u.nbytes)
        rd = DeviceBuffer(F * ns * nc * 4)
        cap = F * 4096
        dd = DeviceBuffer(cap * 16)
        dn = DeviceBuffer(16)
        core.enqueue(cube, F, rd_map=rd, dets=dd, det_cap=cap, n_dets=dn)
        st = dn.download(np.uint32, (4,))
        n = int(st[0])
        assert st[1] == 0
        dets = dd.download(DET_DTYPE, (n,))
        rd_map = rd.download(np.float32, (F, ns, nc))
    for f in (0, F - 1):
        ref = O.process(u[f % n_u].astype(np.complex128), None)["mag"]
        check_map(rd_map[f:f + 1], ref[None])
    for f in range(n_u, F):
        assert np.array_equal(rd_map[f], rd_map[f % n_u])
    np.testing.assert_array_equal(dets, CB.cfar(rd_map, O.Cfar1D(), threads=16, cap=1 << 22))


@pytest.mark.parametrize("wl", ["c3", "c5"])
def test_s48_bench_shape_parity(wl):
    """Configs 3 and 5 at the bench's own shape (16 frames, one call) on the S48 spectrum in its
    pair form: 48 MiB per frame, so the auto chunk takes 4 frames (16 = 4 x 4, no one-frame tail
    launch).  Maps of the first and last frame within 1e-4 of the fp64 oracle, every detection
    bit-exact vs the C oracle's 2-D OS-CFAR on the GPU's map (as test_gpu_r04's fp32 case)."""
    import sys
    if str(REPO) not in sys.path:
        sys.path.insert(0, str(REPO))
    import bench
    from test_gpu_parity import to_complex
    w = bench.WORKLOADS[wl]
    F, ns, nc, nrx, dtype = w["frames"], w["ns"], w["nc"], w["nrx"], w["dtype"]
    cube = synth.frames(F, ns, nc, nrx, w["recipe"], seed=1234, dtype=dtype)
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, N_RX=nrx, in_dtype=dtype, cfar=w["cfar"], max_frames=F,
                   spectrum="s48") as core:
        assert core.info("chunk") == 4
        out = core.process(cube)
    for f in (0, F - 1):
        ref = O.process(to_complex(cube[f], dtype), None)["mag"]
        check_map(out.rd_map[f:f + 1], ref[None])
    np.testing.assert_array_equal(out.dets, CB.cfar(out.rd_map, O.Cfar2D(), threads=16))
    assert set(out.dets["frame"].tolist()) == set(range(F))
