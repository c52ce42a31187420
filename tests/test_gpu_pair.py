"""GPU parity of the round-2 session-2 kernel variants: the dual-chirp range kernel (k_range2,
default for N >= 4096) against the one-chirp kernel, and the paired K1 + K2 launches
(csrc/pair.hpp, opt-in at BASELINE config 2's geometry): launch i runs the range stage of chunk i beside the Doppler stage of chunk i - 1 on
double-buffered spectra.  The arithmetic is k_range's and k_doppler's, so maps and detection
lists must be bit-identical to the serial K1 -> K2 path (FMCW_PAIR=0), and on parity with the
oracle (maps within 1e-4 per frame, detections bit-exact against the oracle CFAR on the map)."""
import numpy as np
import pytest

import cpu_backend as CB
import fmcw_oracle as O
from fmcw import DET_DTYPE, DeviceBuffer, RadarCore, synth
from test_gpu_parity import check_map, to_complex

pytestmark = pytest.mark.gpu


def _run(monkeypatch, pair, cube, dtype, cfar, chunk=None, **kw):
    monkeypatch.setenv("FMCW_PAIR", "1" if pair else "0")
    if chunk:
        monkeypatch.setenv("FMCW_PAIR_CHUNK", str(chunk))
    else:
        monkeypatch.delenv("FMCW_PAIR_CHUNK", raising=False)
    with RadarCore(N_RANGE=1024, N_DOPPLER=256, in_dtype=dtype, cfar=cfar, max_frames=cube.shape[0], **kw) as core:
        pc = core.info("pair_chunk")
        out = core.process(cube)
    return pc, out


@pytest.mark.parametrize("dtype,cfar,nf,chunk", [
    ("f32", "os1d", 109, None),   # auto chunk (48 frames): 3 launches of both halves, a ragged last chunk
    ("i16", "os1d", 23, 5),       # the AXI word format, 6 launches of 5 frames
    ("f16", "none", 11, 4),       # no CFAR, map only
])
def test_pair_matches_serial_and_oracle(monkeypatch, dtype, cfar, nf, chunk):
    cube = synth.frames(nf, 1024, 256, 1, "two_targets", dtype=dtype, seed=7)
    pc, paired = _run(monkeypatch, True, cube, dtype, cfar, chunk)
    assert pc == (chunk or pc) and 0 < pc < nf, "the paired path must be active"
    pc0, serial = _run(monkeypatch, False, cube, dtype, cfar)
    assert pc0 == 0
    np.testing.assert_array_equal(paired.rd_map, serial.rd_map)
    np.testing.assert_array_equal(paired.dets, serial.dets)
    for f in (0, pc - 1, pc, nf - 1):
        ref = O.process(to_complex(cube[f], dtype), None)["mag"]
        check_map(paired.rd_map[f:f + 1], ref[None])
    if cfar == "os1d":
        np.testing.assert_array_equal(paired.dets, CB.cfar(paired.rd_map, O.Cfar1D(), threads=16))
        assert paired.n_dets > nf  # both targets in every frame


def test_pair_repeated_enqueues_device_buffers(monkeypatch):
    """The bench's pattern: back-to-back fmcw_enqueue on device buffers, batch sizes that end on
    a full, a ragged and a single-frame last chunk; every run equals the first."""
    monkeypatch.setenv("FMCW_PAIR", "1")
    monkeypatch.setenv("FMCW_PAIR_CHUNK", "12")
    ns, nc, F = 1024, 256, 61
    uniq = synth.frames(8, ns, nc, 1, "random_target", seed=45)
    cube = DeviceBuffer(F * uniq[0].nbytes)
    for f in range(F):
        cube.upload(uniq[f % 8], f * uniq[0].nbytes)
    dmap = DeviceBuffer(F * ns * nc * 4)
    cap = F * 4096
    ddet = DeviceBuffer(cap * 16)
    dn = DeviceBuffer(16)
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, cfar="os1d", max_frames=F) as core:
        assert core.info("pair_chunk") == 12
        runs = []
        for nfr in (F, 48, 25, 13, F):
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


@pytest.mark.parametrize("ns,nc,dtype,mti", [
    (4096, 64, "f32", 0),
    (4096, 32, "i16", 3),   # MTI on: the Doppler window is not folded into the range stage
    (8192, 32, "f16", 0),
    (8192, 64, "i16", 2),
])
def test_dual_range_kernel_matches_single(monkeypatch, ns, nc, dtype, mti):
    """K1's dual-chirp kernel (k_range2, T = 2 geometries: both chirps per thread, tiles stored
    from registers) is bit-identical to the one-chirp-per-thread kernel (FMCW_K1_SINGLE=1): the
    same passes in the same order.  Checked on the full map and the CFAR detections."""
    nf = 2
    cube = synth.frames(nf, ns, nc, 1, "two_targets", dtype=dtype, seed=11)
    outs = []
    for single in ("0", "1"):
        if single == "1":
            monkeypatch.setenv("FMCW_K1_SINGLE", "1")
        else:
            monkeypatch.delenv("FMCW_K1_SINGLE", raising=False)
        with RadarCore(N_RANGE=ns, N_DOPPLER=nc, in_dtype=dtype, cfar="os1d", max_frames=nf,
                       mti_bypass=mti == 0, NOTCH_MODE=mti or 2) as core:
            outs.append(core.process(cube))
    np.testing.assert_array_equal(outs[0].rd_map, outs[1].rd_map)
    np.testing.assert_array_equal(outs[0].dets, outs[1].dets)
    for f in range(nf):
        ref = O.process(to_complex(cube[f], dtype), None, mti_mode=mti)["mag"]
        check_map(outs[0].rd_map[f:f + 1], ref[None])
