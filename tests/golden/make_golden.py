#!/usr/bin/env python3
"""Regenerate the committed golden fixtures in tests/golden/.

Run in the development container (where /root/reference is mounted):
    python tests/golden/make_golden.py [--reference /root/reference]

Inputs it reads from the reference are DATA only (no reference code is imported or run):
  data/golden_input_chirp.txt       2000 "I Q" lines          -> golden_input_chirp.txt (copy)
  data/radar_output.txt             1024x128 map, 5 columns    -> radar_output_profile.npz
                                                                   (per-row / per-residue sums)
The known-answer vectors below are the literal test vectors of the reference's testbenches:
  rtl/src/tb_magnitude_calc.vhd:49-73   17 (I, Q) pairs, model mx + mn/4 + mn/8 (:32-40)
  rtl/src/tb_os_cfar_2d.vhd:14-19,52-75 64x32 synthetic map + window generics
  rtl/src/tb_corner_turner.vhd:12-13,36-49  16x8 encode chirp*256+sample
Expected outputs are computed by the oracle (oracle/fmcw_oracle.py) and stored beside them;
the tests recompute them to pin the oracle, and the GPU tests compare against them.
"""
from __future__ import annotations

import argparse
import json
import shutil
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO / "oracle"))
import fmcw_oracle as O  # noqa: E402

# rtl/src/tb_magnitude_calc.vhd:49-73
MAG_KAT_IQ = [(1000, 0), (0, 1000), (-1000, 0), (0, -1000), (1000, 1000), (-1000, 1000),
              (-1000, -1000), (1000, -1000), (5000, 3000), (-8000, 6000), (100, 100),
              (32000, 32000), (0, 0), (1, 0), (1, 1), (30000, 100), (100, 30000)]


def tb_amb_ref(i, q):
    """The testbench's own integer model (tb_magnitude_calc.vhd:32-40): VHDL '/' truncates."""
    ai, aq = abs(i), abs(q)
    mx, mn = (ai, aq) if ai >= aq else (aq, ai)
    return mx + mn // 4 + mn // 8


def tb_cfar2d_map(n_range=64, n_doppler=32, noise=100, amp=5000, t1=(30, 16), t2=(50, 8)):
    """rtl/src/tb_os_cfar_2d.vhd:52-75 make_map()."""
    m = np.zeros((n_range, n_doppler), np.int64)
    for r in range(n_range):
        for d in range(n_doppler):
            m[r, d] = noise + ((r * 7 + d * 13) % 30)
    for (tr, td) in (t1, t2):
        for dr in (-1, 0, 1):
            for dd in (-1, 0, 1):
                if 0 <= tr + dr < n_range and 0 <= td + dd < n_doppler:
                    m[tr + dr, td + dd] = amp if (dr == 0 and dd == 0) else amp // 3
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    ref = Path(args.reference)

    # 1. magnitude KAT
    kat = [{"i": i, "q": q, "expect": tb_amb_ref(i, q)} for (i, q) in MAG_KAT_IQ]
    (HERE / "mag_kat.json").write_text(json.dumps(kat, indent=1) + "\n")

    # 2. corner-turner KAT (16 range x 8 Doppler): value = chirp*256 + sample
    n_r, n_d = 16, 8
    enc = np.array([[c * 256 + s for s in range(n_r)] for c in range(n_d)], np.int64)
    np.savez(HERE / "ct_kat.npz", chirp_major=enc, range_major=enc.T.copy())

    # 3. window: Hamming ROM (Q15) for the testbench size and the core sizes; fp32 tables
    win = {str(n): {"q15_rom": O.hamming_q15(n).tolist(),
                    "f32": O.window_f32(n).tolist()} for n in (64, 128, 256, 1024)}
    (HERE / "window.json").write_text(json.dumps(win) + "\n")

    # 4. golden chirp (BASELINE config 1): copy the data file, store oracle outputs
    src = ref / "data" / "golden_input_chirp.txt"
    shutil.copyfile(src, HERE / "golden_input_chirp.txt")
    iq = np.loadtxt(src, dtype=np.int64).reshape(-1, 2)
    z = iq[:, 0] + 1j * iq[:, 1]
    peaks = {str(n): int(np.argmax(np.abs(np.fft.fft(z[:n])))) for n in (128, 256, 1024)}
    cube = (z[:256][None, None, :] * np.ones((1, 128, 1))).astype(np.complex64)  # 128 x 256
    res1 = O.process(cube, O.Cfar1D())
    res2 = O.process(cube, O.Cfar2D())
    np.savez_compressed(HERE / "golden_chirp_c1.npz", cube=cube, mag=res1["mag"],
                        dets_os1d=res1["dets"], dets_os2d=res2["dets"],
                        spec_peak=np.array([peaks["128"], peaks["256"], peaks["1024"]]))

    # 5. data/radar_output.txt coarse profile (the only things it pins)
    a = np.loadtxt(ref / "data" / "radar_output.txt", dtype=np.int64)
    m = np.zeros((1024, 128), np.int64)
    m[a[:, 0], a[:, 1]] = a[:, 4]
    row_energy = m.astype(np.float64).sum(axis=1)
    resid = np.stack([m[:, k::4].sum(axis=1) for k in range(4)], axis=1)
    np.savez_compressed(HERE / "radar_output_profile.npz", row_energy=row_energy,
                        doppler_residue_energy=resid, top_rows=np.argsort(-row_energy)[:6])

    # 6. tb_os_cfar_2d map + oracle detections with the testbench generics
    #    (REF_R=3, REF_D=2, GUARD_R=1, GUARD_D=1 as the RTL applies them: along Doppler
    #    ref 3 / guard 1, along range rows ref 2 / guard 1)
    m2 = tb_cfar2d_map()
    p = O.Cfar2D(ref_range=2, guard_range=1, ref_doppler=3, guard_doppler=1)
    det, thr = O.cfar_os2d(m2.astype(np.float32), p)
    dets = O.detections(det, m2.astype(np.float32), thr)
    np.savez(HERE / "tb_cfar2d.npz", map=m2, dets=dets,
             params=np.array([p.ref_range, p.guard_range, p.ref_doppler, p.guard_doppler]))
    print(f"wrote fixtures to {HERE}: golden peaks {peaks}, tb_cfar2d dets {len(dets)}, "
          f"C1 dets os1d {len(res1['dets'])} os2d {len(res2['dets'])}")


if __name__ == "__main__":
    main()
