"""Round-3 GPU tests (libfmcw.so on gfx950 vs the CPU oracle, through the C-ABI):

  * the range-stage kernel family that ships for each N (k_range, k_range_sq at 4096, k_range_px
    at 8192; fmcw.h FMCW_INFO_RANGE_KERNEL) is the one selected, and is on parity with the oracle
    at N = 2048..8192;
  * the status words of the RTL-compat paths (fmcw.h n_dets_dev[2], [3]; the reference's sticky
    status_overflow, rtl/src/radar_core.vhd:447-456) count exactly what the integer oracle
    predicts, and stay 0 on the fp32 path;
  * the detection gather's device side (fmcw_gather_pack_for_test / _compact_for_test) for 2, 3
    and 8 synthetic ranks against a NumPy model of fmcw.h's gather contract.
"""
import numpy as np
import pytest

import fmcw_oracle as O
from conftest import rel_err
from fmcw import RadarCore, DeviceBuffer, DET_DTYPE, synth
from fmcw import _lib as L
from test_gpu_parity import check_map, oracle_dets, run_range_ct, to_complex

pytestmark = pytest.mark.gpu

KINDS = {"single": 0, "seq": 2, "px": 3}   # FMCW_INFO_RANGE_KERNEL (1 = k_range2, retired)


@pytest.mark.parametrize("ns,nc,nrx,dtype,mti,kind", [
    (8192, 32, 1, "f16", 0, "px"),      # config 5's range length
    (8192, 64, 1, "i16", 2, "px"),      # MTI on: the Doppler window is applied by K2, not folded into K1
    (8192, 32, 1, "i16", 0, "px"),
    (4096, 64, 2, "f32", 0, "seq"),     # config 3's range length: radix-16 first pass from 8-B loads
    (4096, 32, 1, "i16", 3, "seq"),
    (2048, 64, 1, "f32", 0, "single"),  # below both: k_range
])
def test_shipped_range_kernel_families(ns, nc, nrx, dtype, mti, kind):
    """The release library selects exactly one K1 family per N (no environment knob since ABI 6)
    and its map is on parity with the oracle (1e-4), detections bit-exact vs the oracle CFAR on
    the GPU's map.  (k_range at N = 4096 / 8192 ships for the Q15 and fp16-spectrum paths and is
    tested there: test_range_ct_q15_rtl, test_fp16_spectrum.)"""
    nf = 2
    cube = synth.frames(nf, ns, nc, nrx, "two_targets", dtype=dtype, seed=17)
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, N_RX=nrx, in_dtype=dtype, cfar="os1d", max_frames=nf,
                   mti_bypass=mti == 0, NOTCH_MODE=mti or 2) as core:
        assert core.info("range_kernel") == KINDS[kind]
        out = core.process(cube)
    ref = np.stack([O.process(to_complex(cube[f], dtype), None, mti_mode=mti)["mag"] for f in range(nf)])
    check_map(out.rd_map, ref)
    np.testing.assert_array_equal(out.dets, oracle_dets(out.rd_map, O.Cfar1D()))


@pytest.mark.parametrize("dtype", ["f16", "f32", "i16"])
def test_range_ct_px_many_groups(dtype):
    """k_range_px (N = 8192) over many chirp groups per workgroup and an odd group count per
    launch, every input word type: the canonical corner-turned spectrum vs the oracle, both chirps
    of every group (the permlane last pass and the half-wave tile stores)."""
    ns, nc, nf = 8192, 128, 11     # 704 chirp pairs: more than one per resident workgroup
    cube = synth.frames(nf, ns, nc, 1, "random_target", dtype=dtype, seed=29)
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, in_dtype=dtype, cfar="none", max_frames=nf) as core:
        assert core.info("range_kernel") == KINDS["px"]
        din = DeviceBuffer(cube.nbytes)
        din.upload(cube)
        spec = DeviceBuffer(nf * ns * nc * 8)
        core.range_ct(din, spec, nf)
        got = spec.download(np.complex64, (nf, 1, ns, nc))
    for f in range(nf):
        ref = O.range_ct(to_complex(cube[f], dtype))
        assert rel_err(got[f], ref) <= 1e-4, f


def test_range_ct_seq_many_groups():
    """k_range_sq over many chirp groups per workgroup (the grid-stride loop with the one-chirp
    lookahead crossing group boundaries), an odd number of groups per launch: the canonical
    corner-turned spectrum vs the oracle, both chirps of every group."""
    ns, nc, nf = 4096, 128, 5
    cube = synth.frames(nf, ns, nc, 1, "random_target", dtype="f32", seed=23)
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, cfar="none", max_frames=nf) as core:
        assert core.info("range_kernel") == KINDS["seq"]
        din = DeviceBuffer(cube.nbytes)
        din.upload(cube)
        spec = DeviceBuffer(nf * ns * nc * 8)
        core.range_ct(din, spec, nf)
        got = spec.download(np.complex64, (nf, 1, ns, nc))
    for f in range(nf):
        ref = O.range_ct(to_complex(cube[f], "f32"))
        assert rel_err(got[f], ref) <= 1e-4


# ---- status words (saturation counts) ------------------------------------------------------
def _enqueue_status(core, cube):
    nf = cube.shape[0]
    c = core.cfg
    din = DeviceBuffer(cube.nbytes)
    din.upload(cube)
    dmap = DeviceBuffer(nf * c.n_range * c.n_doppler * 4)
    cap = nf * 4096
    dd = DeviceBuffer(cap * 16)
    dn = DeviceBuffer(4 * L.STATUS_WORDS)
    dn.upload(np.full(L.STATUS_WORDS, 0xDEADBEEF, np.uint32))   # every call rewrites all words
    core.enqueue(din, nf, dmap, dd, cap, dn)
    st = dn.download(np.uint32, (L.STATUS_WORDS,))
    return st, dmap.download(np.float32, (nf, c.n_range, c.n_doppler))


def test_status_words_zero_on_fp32_path():
    cube = synth.frames(2, 1024, 128, 1, "two_targets", dtype="i16", seed=3)
    with RadarCore(N_RANGE=1024, N_DOPPLER=128, in_dtype="i16", cfar="os2d", max_frames=2) as core:
        st, _ = _enqueue_status(core, cube)
        out = core.process(cube)
    assert st[1] == 0 and st[2] == 0 and st[3] == 0 and st[0] == out.n_dets
    assert out.window_saturations == 0 and out.word_saturations == 0 and not out.status_overflow


def test_range_window_saturation_count():
    """Full-scale int16 ADC words through the RTL-compat Q15 range window (2x gain): every sample
    whose I or Q leaves int16 is one win1_saturation event (window_multiplier.vhd:152-158).
    range_shift 13 keeps the spectrum words small, so words and the Doppler window never clip:
    status word 2 is the range window's count exactly, word 3 is 0."""
    ns, nc, nf = 256, 64, 2
    rng = np.random.default_rng(8)
    cube = rng.integers(-32768, 32768, size=(nf, 1, nc, ns, 2)).astype(np.int16)
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, in_dtype="i16", window="q15_rtl", cfar="os1d",
                   cfar1d=(8, 2, 12, 4.0), max_frames=nf, range_shift=13) as core:
        st, rd = _enqueue_status(core, cube)
        out = core.process(cube)
        spec = run_range_ct(core, cube, nf)
    want = [O.saturation_counts(cube[f], 13) for f in range(nf)]
    assert sum(w for w, _ in want) > 1000 and all(n == 0 for _, n in want)
    assert st[2] == sum(w for w, _ in want) and st[3] == 0
    assert out.window_saturations == st[2] and out.word_saturations == 0 and out.status_overflow
    _check_q15_map(rd, spec, cube, 13)


def _check_q15_map(rd, spec, cube, shift, mti=0):
    """Map of an integer-window run vs the oracle: the Doppler stage from the GPU's own range
    spectrum (its 16-bit words round exactly as on the GPU), and frame-level vs fp64 end to end."""
    nf = cube.shape[0]
    ref = np.stack([O.magnitude(O.doppler_stage(spec[f].astype(np.complex128), mti_mode=mti, q15_rtl=True),
                                rx_axis=0) for f in range(nf)])
    check_map(rd, ref)
    e2e = np.stack([O.process(cube[f], None, mti_mode=mti, q15_rtl=True, range_shift=shift)["mag"]
                    for f in range(nf)])
    assert rel_err(rd, e2e) <= 1e-4


def test_word_and_canceller_saturation_count():
    """FMCW_COMPAT_MTI on chirps that are constants of alternating sign (window none): range bin
    0 of every chirp is +-A*N beyond int16 (a clipped spectrum word each), the other bins are 0,
    and the 2-pulse canceller's difference of consecutive clipped words leaves int16 at every
    chirp c >= 1: status word 3 = nf * (2 nc - 1), as the integer oracle counts."""
    ns, nc, nf, a = 256, 32, 2, 1000
    cube = np.zeros((nf, 1, nc, ns, 2), np.int16)
    cube[..., 0] = (a * np.where(np.arange(nc) % 2 == 0, 1, -1))[None, None, :, None]
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, in_dtype="i16", window="none", cfar="os2d", max_frames=nf,
                   mti_bypass=False, NOTCH_MODE=2, compat_rtl=("mti",), range_shift=0) as core:
        st, rd = _enqueue_status(core, cube)
    want = [O.saturation_counts(cube[f], 0, mti_mode=2, q15_rtl=False, mti_rtl=True) for f in range(nf)]
    assert [w for w, _ in want] == [0] * nf and sum(n for _, n in want) == nf * (2 * nc - 1)
    assert st[2] == 0 and st[3] == nf * (2 * nc - 1)
    ref = np.stack([O.process(to_complex(cube[f], "i16"), None, window=False, mti_mode=2, mti_rtl=True)["mag"]
                    for f in range(nf)])
    check_map(rd, ref)


def test_doppler_window_saturation_count():
    """FMCW_WIN_Q15_RTL on both axes: constant chirps whose range-bin-0 words sit near int16
    full scale after range_shift, so the integer Doppler window (2x gain, u_doppler_window,
    radar_core.vhd:340-349) clips where the ROM coefficient exceeds ~1/2: status word 2 counts
    those (the range window itself cannot clip at this amplitude), word 3 the clipped words --
    both exactly as the integer oracle predicts; the map is on parity with the oracle."""
    ns, nc, nf = 256, 64, 2
    cube = np.zeros((nf, 1, nc, ns, 2), np.int16)
    cube[..., 0] = 12000
    cube[..., 1] = -7000
    cube[1, 0, ::3, :, 0] = -16000                        # some chirps of frame 1 of opposite sign
    shift = 7
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, in_dtype="i16", window="q15_rtl", cfar="os2d", max_frames=nf,
                   range_shift=shift) as core:
        st, rd = _enqueue_status(core, cube)
        spec = run_range_ct(core, cube, nf)
    want = [O.saturation_counts(cube[f], shift) for f in range(nf)]
    assert want[0][0] > 0 and want[0][1] == 0 and want[1][1] > 0
    assert st[2] == sum(w for w, _ in want) and st[3] == sum(n for _, n in want)
    _check_q15_map(rd, spec, cube, shift)


# ---- detection gather, device side ---------------------------------------------------------
def _records(rng, n, frames):
    r = np.zeros(n, DET_DTYPE)
    r["frame"] = np.sort(rng.integers(0, frames, n))
    r["range"] = rng.integers(0, 1024, n)
    r["doppler"] = rng.integers(0, 256, n)
    r["mag"] = rng.uniform(0, 1e6, n)
    r["threshold"] = rng.uniform(0, 1e6, n)
    return r


@pytest.mark.parametrize("n_ranks", [2, 3, 8])
def test_gather_pack_and_compact_multi_rank(n_ranks):
    """Each synthetic rank has its own (found, lost, det_cap): 0 detections, a few, more than
    wire_cap, more than its buffer (det_cap < found, the records past it never written), and
    scratch losses.  fmcw_gather_pack_for_test builds each rank's message, the messages are laid
    end to end as the root's receive buffer, fmcw_gather_compact_for_test packs them: the output
    is every rank's first min(found, det_cap, wire_cap) records in rank order with its frame
    offset, out_n = (records written, records not sent + scratch losses) -- fmcw.h's contract."""
    rng = np.random.default_rng(100 + n_ranks)
    wire = 96
    frames_per_rank = 16
    specs = [(0, 0, 64), (5, 0, 64), (200, 3, 400), (150, 0, 40), (40, 7, 64), (96, 0, 96), (97, 1, 128),
             (1, 0, 1)][:n_ranks]
    msg_bytes = (1 + wire) * 16
    recv = DeviceBuffer(n_ranks * msg_bytes)
    want_recs, want_lost = [], 0
    keep = []
    for r, (found, lost, det_cap) in enumerate(specs):
        recs = _records(rng, max(found, 1), frames_per_rank)[:found]
        stored = recs[:min(found, det_cap)]
        dd = DeviceBuffer(max(det_cap, 1) * 16)
        if len(stored):
            dd.upload(stored)
        dn = DeviceBuffer(16)
        dn.upload(np.array([found, lost, 0, 0], np.uint32))
        L.check(L.load().fmcw_gather_pack_for_test(dd.ptr, det_cap, dn.ptr, wire, r * frames_per_rank,
                                                   recv.ptr + r * msg_bytes, None))
        keep += [dd, dn]
        n = min(found, det_cap, wire)
        w = recs[:n].copy()
        w["frame"] += r * frames_per_rank
        want_recs.append(w)
        want_lost += found - n + lost
    out = DeviceBuffer(n_ranks * wire * 16)
    on = DeviceBuffer(16)
    L.check(L.load().fmcw_gather_compact_for_test(recv.ptr, n_ranks, wire, out.ptr, on.ptr, None))
    want = np.concatenate(want_recs)
    got_n = on.download(np.uint32, (2,))
    assert list(got_n) == [len(want), want_lost]
    np.testing.assert_array_equal(out.download(DET_DTYPE, (len(want),)), want)
    # message headers as the wire carries them: (sent, not sent + lost, 0, 0)
    for r, (found, lost, det_cap) in enumerate(specs):
        hdr = recv.download(np.uint32, (4,), offset=r * msg_bytes)
        n = min(found, det_cap, wire)
        assert list(hdr) == [n, found - n + lost, 0, 0]
