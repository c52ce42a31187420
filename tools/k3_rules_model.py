#!/usr/bin/env python3
"""NumPy model of k_cfar2d_lv's screen (cfar2d.hpp, round 5): the fraction of config-5 bench-map
cells that survive the s_min rule and the scale rules A / B, per pair of level quantiles (QA, QB;
QB clamped to 1.5 QA as the kernel does), with the kernel's bounds for levels C (16 cells around a
group of 4 CUTs) and D (the lane's 11 x 32 window).  The map is the bench's synthetic config-5 frame
(seed 1234) through the C restatement (oracle/fmcw_cpu.c); 4 x 48 CUT rows.
usage: python tools/k3_rules_model.py [--pairs 0.56:0.68,0.50:0.74] [--law bench|rayleigh|exponential|lognormal|uniform]
(--law: synthetic clutter instead of the bench frame, as tools/cfar2d_bench.py --maps; the share of
survivors that truly detect is printed beside them)"""
import argparse
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "fpga-fmcw-radar-processor_amd"))
sys.path.insert(0, str(REPO / "oracle"))
HR, GR, HD, GD, NEED, NROWS = 5, 1, 6, 2, 32, 48


def k16(v):
    return (np.asarray(v, np.float32).view(np.uint32) >> 16).astype(np.int64)


def lo(k):
    return (np.asarray(k, np.uint32) << 16).view(np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", default="0.56:0.68,0.52:0.68,0.56:0.74,0.50:0.74,0.48:0.76")
    ap.add_argument("--law", default="bench")
    ap.add_argument("--kd", type=int, default=2, help="level D = QB + kd octaves (the kernel: 2)")
    ap.add_argument("--rb", default="63:32", help="rule B bounds C_B:C_C")
    ap.add_argument("--ra", default="80:40:8", help="rule A bounds C_A:C_B:C_C")
    a = ap.parse_args()
    pairs = [tuple(float(x) for x in p.split(":")) for p in a.pairs.split(",")]
    import cpu_backend as CB
    import fmcw_oracle as O
    from fmcw import synth
    if a.law == "bench":
        cube = synth.frames(1, 8192, 1024, 1, "two_targets", seed=1234, dtype="f16")
        if not np.iscomplexobj(cube):
            x = cube.astype(np.float32)
            cube = x[..., 0] + 1j * x[..., 1]
        m = CB.process(cube.astype(np.complex64), None, threads=8)[0][0]
    else:
        rng = np.random.default_rng(7)
        sh = (8192, 1024)
        m = {"rayleigh": lambda: rng.rayleigh(1.0, sh), "exponential": lambda: rng.exponential(5.0, sh),
             "lognormal": lambda: rng.lognormal(1.0, 1.2, sh), "uniform": lambda: rng.uniform(9.0, 11.0, sh)}[a.law]()
        m = m.astype(np.float32)
    dets = {}
    for r0 in [20, 2055, 4096, 6124]:
        d, _ = O.cfar_os2d(m[r0 - HR:r0 + NROWS + HR], O.Cfar2D())
        dets[r0] = d[HR:-HR]
    s_min, s2 = np.float32(2.0), np.float32(4.0)
    tot = {p: [] for p in pairs}
    for r0 in [20, 2055, 4096, 6124]:
        K = k16(m[r0 - HR:r0 + NROWS + HR])
        cut = K[HR:-HR]

        def rows_of(Q):
            b = (K >= Q).astype(np.int64)
            return b, sum(b[HR + dr: HR + dr + NROWS] for dr in range(-HR, HR + 1))

        def box(Q):  # refs at or above Q in the 11 x 13 box minus the 3 x 5 guard block
            b, _ = rows_of(Q)
            acc = np.zeros(cut.shape, np.int64)
            for dr in range(-HR, HR + 1):
                for dd in range(-HD, HD + 1):
                    if abs(dr) <= GR and abs(dd) <= GD:
                        continue
                    acc += np.roll(b[HR + dr: HR + dr + NROWS], -dd, axis=1)
            return acc

        def window(Q, step, a0, a1):  # cells a0 .. a1 - 1 around each group of `step` CUTs, 11 rows
            _, rows = rows_of(Q)
            out = np.zeros(cut.shape, np.int64)
            for d0 in range(0, 1024, step):
                out[:, d0:d0 + step] = rows[:, np.arange(d0 + a0, d0 + a1) % 1024].sum(1)[:, None]
            return out

        k7 = (m[r0:r0 + 4].view(np.uint32) >> 19).astype(np.int64).ravel()
        for p in pairs:
            QA = int(np.quantile(k7, p[0])) * 8
            QB = max(QA, min(int(np.quantile(k7, p[1])) * 8, int(k16(np.float32(1.5) * lo(QA)))))
            QC, QD = QB + 128, QB + 128 * a.kd
            CA, CB_ = box(QA), box(QB)
            CC, nzD = window(QC, 4, -6, 10), window(QD, 16, -8, 24) > 0
            UA, UB = int(k16(s_min * lo(QA))), int(k16(s_min * lo(QB)))
            U2A, U2B = int(k16(s2 * lo(QA))), int(k16(s2 * lo(QB)))
            rule_a = lo(QB) <= 1.5 * lo(QA)
            smin = ((CA >= NEED) & (cut < UA)) | ((CB_ >= NEED) & (cut < UB))
            b1, b2 = (int(x) for x in a.rb.split(":"))
            a1, a2, a3 = (int(x) for x in a.ra.split(":"))
            rB = (CB_ >= NEED) & (CB_ <= b1) & (CC <= b2) & ~nzD & (cut < U2B)
            rA = rule_a & (CA >= NEED) & (CA <= a1) & (CB_ <= a2) & (CC <= a3) & ~nzD & (cut < U2A)
            surv = ~(smin | rA | rB)
            assert not (dets[r0] & ~surv).any(), "the screen dropped a detection"
            tot[p].append((surv.mean(), dets[r0].mean()))
    print(a.law, {f"{p[0]:.2f}/{p[1]:.2f}": "survivors %.4f %% (detect %.4f %%)" % (100 * np.mean([x[0] for x in v]),
                                                                         100 * np.mean([x[1] for x in v]))
                  for p, v in tot.items()})


if __name__ == "__main__":
    main()
