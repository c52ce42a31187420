#!/usr/bin/env python3
"""Ablation timing of the hot path on one GPU: per-kernel HIP-event times for config-2
frames under switches that need no rebuild (CFAR kind, map store, chunk size, MTI).

usage: python tools/ablate.py [--frames 1024] [--steps 5]
Prints one JSON line per variant.
"""
import argparse
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "fpga-fmcw-radar-processor_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--ns", type=int, default=1024)
    ap.add_argument("--nc", type=int, default=256)
    ap.add_argument("--variants", default="base,nocfar,nomap,bare,os2d,chunk16,chunk64,chunk128,mti2")
    ap.add_argument("--spectrum", default="f32", help="f32 | f16 | s48 (the bench runs config 2 on s48)")
    a = ap.parse_args()
    import numpy as np
    import torch
    from fmcw import RadarCore, synth

    F, ns, nc = a.frames, a.ns, a.nc
    dev = torch.device("cuda", 0)
    u = synth.frames(16, ns, nc, 1, "two_targets").view(np.float32)
    cube = torch.from_numpy(np.ascontiguousarray(u)).to(dev).repeat((F // 16, 1, 1, 1))
    rd_map = torch.empty((F, ns, nc), dtype=torch.float32, device=dev)
    dets = torch.empty((F * 4096, 4), dtype=torch.int32, device=dev)
    nd = torch.zeros(4, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    variants = {
        "base": dict(cfar="os1d", map=True, chunk=0, mti=False),
        "nocfar": dict(cfar="none", map=True, chunk=0, mti=False),
        "nomap": dict(cfar="os1d", map=False, chunk=0, mti=False),
        "bare": dict(cfar="none", map=False, chunk=0, mti=False),
        "os2d": dict(cfar="os2d", map=True, chunk=0, mti=False),
        "chunk16": dict(cfar="os1d", map=True, chunk=16, mti=False),
        "chunk32": dict(cfar="os1d", map=True, chunk=32, mti=False),
        "chunk64": dict(cfar="os1d", map=True, chunk=64, mti=False),
        "chunk128": dict(cfar="os1d", map=True, chunk=128, mti=False),
        "chunk256": dict(cfar="os1d", map=True, chunk=256, mti=False),
        "chunk1024": dict(cfar="os1d", map=True, chunk=1024, mti=False),
        "mti2": dict(cfar="os1d", map=True, chunk=0, mti=True),
        # CFAR phase split: impossible scale / alpha -> no survivors, counting pass only
        "os1d_a": dict(cfar="os1d", map=True, chunk=0, mti=False, cfar1d=(8, 2, 12, 1000.0)),
        "os2d_a": dict(cfar="os2d", map=True, chunk=0, mti=False, ovr=7),
        "os2d_nom": dict(cfar="os2d", map=True, chunk=0, mti=False, ovr=4),
    }
    for name in a.variants.split(","):
        v = variants[name]
        extra = {"cfar1d": v["cfar1d"]} if "cfar1d" in v else {}
        core = RadarCore(N_RANGE=ns, N_DOPPLER=nc, cfar=v["cfar"], max_frames=F, chunk_frames=v["chunk"],
                         mti_bypass=not v["mti"], cfar_scale_ovr=v.get("ovr", 0), spectrum=a.spectrum, **extra)

        def step():
            core.enqueue(cube.data_ptr(), F, rd_map.data_ptr() if v["map"] else 0, dets.data_ptr(),
                         F * 4096, nd.data_ptr(), stream)
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / a.steps
        core.reset_kernel_times()
        core.set_profiling(True)
        for _ in range(a.steps):
            step()
        kt = core.kernel_times()
        core.close()
        out = {"variant": name, "spectrum": a.spectrum, "frames_per_s": round(F / el), "ms_per_step": round(el * 1e3, 3),
               "dets_per_frame": round(int(nd[0].item()) / F, 1)}
        for k, (ms, n) in kt.items():
            if n:
                out[k + "_us_per_frame"] = round(ms * 1e3 / (F * a.steps), 4)
                out[k + "_launches"] = n // a.steps
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
