#!/usr/bin/env python3
"""Phase timeline of the fused range + Doppler kernel (fused.hpp) on config 2.

Runs FMCW_FUSED_TRACE=1 launches of 512 frames (64 per XCD) on device-resident input and
prints, per XCD, the mean time per frame and the mean of each phase (µs, 100 MHz counter):
  A: frame start -> past the wait for B to free S -> ready signalled (first range workgroup)
  B: wait start -> ready seen -> freed signalled -> tile done (first Doppler workgroup)
usage: python tools/fused_trace.py [--frames 512] [--launches 3]"""
import argparse
import ctypes as C
import os
import sys
from pathlib import Path

os.environ["FMCW_FUSED_TRACE"] = "1"
os.environ.setdefault("FMCW_FUSED", "1")
REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "fpga-fmcw-radar-processor_amd"))

import numpy as np  # noqa: E402

from fmcw import DeviceBuffer, RadarCore, synth  # noqa: E402
from fmcw import _lib as L  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=512)
    ap.add_argument("--launches", type=int, default=3)
    ap.add_argument("--ns", type=int, default=1024)
    ap.add_argument("--nc", type=int, default=256)
    a = ap.parse_args()
    ns, nc, F = a.ns, a.nc, a.frames
    uniq = synth.frames(8, ns, nc, 1, "two_targets")
    cube = DeviceBuffer(F * uniq[0].nbytes)
    for f in range(F):
        cube.upload(uniq[f % 8], f * uniq[0].nbytes)
    dmap = DeviceBuffer(F * ns * nc * 4)
    cap = F * 4096
    ddet = DeviceBuffer(cap * 16)
    dn = DeviceBuffer(16)
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, cfar="os1d", max_frames=F) as core:
        print("fused", core.info("fused"), "group", core.info("fused_group"))
        core.set_profiling(True)
        for _ in range(a.launches):
            core.enqueue(cube, F, dmap, ddet, cap, dn)
        kt = core.kernel_times()
        print("kernel times", {k: (round(v[0] / max(1, v[1]), 4), v[1]) for k, v in kt.items() if v[1]})
        buf = (C.c_uint64 * 4096)()
        L.check(L.load().fmcw_get_fused_trace(core._h, buf, 4096))
    t = np.frombuffer(buf, np.uint64).reshape(8, 64, 8).astype(np.int64)
    t0 = t[t > 0].min()
    us = (t - t0) / 100.0  # 100 MHz -> µs
    nk = min(64, (F + 7) // 8)
    for x in range(8):
        u = us[x, :nk]
        per = np.diff(u[:, 2])
        print(f"XCD {x}: frame period {per[2:].mean():6.2f} us | A wait {np.mean(u[1:,1]-u[1:,0]):5.2f} "
              f"A store->ready {np.mean(u[:,2]-u[:,1]):5.2f} lastA {np.mean(u[:,7]-u[:,1]):5.2f} | "
              f"B data {np.mean(u[:,4]-u[:,3]):5.2f} B pass1 {np.mean(u[:,5]-u[:,4]):5.2f} "
              f"B rest {np.mean(u[:,6]-u[:,5]):5.2f} B iter {np.mean(np.diff(u[:,6])):5.2f} | first ready {u[0,2]:.2f}")
    print("XCD 0 frames 0..7 (us):")
    for k in range(8):
        print(" ", " ".join(f"{v:8.2f}" for v in us[0, k]))


if __name__ == "__main__":
    main()
