#!/usr/bin/env python3
"""Time the 2-D OS-CFAR stage (k_cfar2d) alone on the bench's config-3 / config-5 maps.

Builds each workload's linear map once through the whole path (bench.py's synthetic frames),
then runs fmcw_cfar on it repeatedly with the library's per-kernel HIP-event timing and prints
one JSON line per (workload, scale override): mean k_cfar2d time per launch, launches, the
detection count and a hash of the ordered detection list (A/B variants must agree bit for bit).
usage: python tools/cfar2d_bench.py [--workloads c3,c5] [--iters 20] [--ovr 0,7] [--steps 0,16,32]
                                   [--maps bench,rayleigh,exponential,lognormal,uniform,sparse]
(--maps: the bench's own map, or synthetic clutter of the workload's shape drawn on the device --
 the clutter laws of tests/test_gpu_r05_k3.py::test_lv_clutter_shapes, scaled to the bench's size,
 with the same planted targets per frame)
(--steps: strip lengths through fmcw_set_param, 0 = the library's cost model)
(FMCW_LIB=lib/var_<name>.so selects a variant library built by tools/build_variants.sh)"""
import argparse
import hashlib
import json
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "fpga-fmcw-radar-processor_amd"))

GEOM = {"c3": dict(ns=4096, nc=512, nrx=4, dtype="f32"), "c5": dict(ns=8192, nc=1024, nrx=1, dtype="f16")}


def clutter(law, F, ns, nc, dev):
    """Synthetic clutter maps on the device (test_lv_clutter_shapes' laws), targets planted in
    every frame: exponential (power-like), lognormal (wide), uniform (narrow), sparse (2 % of cells
    non-zero), rayleigh (|X| of complex noise)."""
    import torch
    g = torch.Generator(device=dev)
    g.manual_seed({"rayleigh": 79, "exponential": 81, "lognormal": 83, "uniform": 85, "sparse": 87}[law])
    m = torch.empty((F, ns, nc), dtype=torch.float32, device=dev)
    if law == "exponential":
        m.exponential_(1 / 5.0, generator=g)
    elif law == "lognormal":
        m.log_normal_(1.0, 1.2, generator=g)
    elif law == "uniform":
        m.uniform_(9.0, 11.0, generator=g)
    elif law == "rayleigh":
        m.exponential_(1.0, generator=g)
        m.mul_(2.0).sqrt_()
    elif law == "sparse":
        m.exponential_(1.0, generator=g)
        m.mul_(2.0).sqrt_().mul_(10.0)
        keep = torch.empty_like(m).uniform_(0.0, 1.0, generator=g) < 0.02
        m.mul_(keep)
        del keep
    else:
        raise ValueError(law)
    m[:, 60, 100] = 4000.0
    m[:, 200, nc - 4] = 3000.0
    m[:, 120:124, 400 % nc:460 % nc or nc] *= 30.0
    return m


def time_k3(core_args, steps, rd_map, F, dets, cap, nd, stream, iters, tag):
    """fmcw_cfar on one map: mean K3 (k_cfar2d + decide + emit) time per launch, one JSON line."""
    import torch
    from fmcw import RadarCore
    with RadarCore(**core_args) as core:
        cnt = {}
        core.set_param("cfar2d_steps", steps)
        if os.environ.get("FMCW_K3_COUNTS"):  # a FMCW_LAB + FMCW_K3_COUNT variant library
            import ctypes as C

            def rd(k):
                v = C.c_int64(0)
                core._lib.fmcw_get_info(core._h, k, C.byref(v))
                return v.value
            s0, c0 = rd(100), rd(101)
        core.cfar(rd_map, F, dets, cap, nd, stream=stream)  # warm-up
        torch.cuda.synchronize()
        if os.environ.get("FMCW_K3_COUNTS"):
            cnt = {"screen_survivors": rd(100) - s0, "candidates": rd(101) - c0, "cells": rd_map.numel()}
        core.set_profiling(True)
        core.reset_kernel_times()
        for _ in range(iters):
            core.cfar(rd_map, F, dets, cap, nd, stream=stream)
        torch.cuda.synchronize()
        kt = core.kernel_times()
        n = int(nd[0].item())
        h = hashlib.sha1(dets[:min(n, cap)].cpu().numpy().tobytes()).hexdigest()[:16]
        ms, calls = kt["k_cfar"]
        print(json.dumps({**tag, "steps": core.info("cfar2d_steps"), "frames": F,
                          "k_cfar2d_us_per_launch": round(1e3 * ms / max(1, calls), 2), "launches": calls,
                          "frames_per_launch": F * iters / max(1, calls),
                          "us_per_frame": round(1e3 * ms / (F * iters), 2),
                          "n_dets": n, "lost": int(nd[1].item()), "dets_sha1": h, **cnt}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="c3,c5")
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--ovr", default="0,7")
    ap.add_argument("--steps", default="0")
    ap.add_argument("--maps", default="bench")
    a = ap.parse_args()
    import numpy as np
    import torch
    from fmcw import RadarCore, synth

    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    for w in a.workloads.split(","):
        g = GEOM[w]
        F, ns, nc, nrx = a.frames, g["ns"], g["nc"], g["nrx"]
        u = synth.frames(min(16, F), ns, nc, nrx, "two_targets", seed=1234, dtype=g["dtype"])
        if g["dtype"] == "f32":
            u = u.view(np.float32)
        ut = torch.from_numpy(np.ascontiguousarray(u)).to(dev)
        cube = ut.repeat((F // ut.shape[0],) + (1,) * (ut.dim() - 1)).contiguous()
        del ut
        rd_map = torch.empty((F, ns, nc), dtype=torch.float32, device=dev)
        cap = F * 65536
        dets = torch.empty((cap, 4), dtype=torch.int32, device=dev)
        nd = torch.zeros(4, dtype=torch.int32, device=dev)
        with RadarCore(N_RANGE=ns, N_DOPPLER=nc, N_RX=nrx, in_dtype=g["dtype"], cfar="os2d",
                       max_frames=F) as core:
            core.enqueue(cube, F, rd_map, dets, cap, nd, stream=stream)
            torch.cuda.synchronize()
        del cube
        bench_map = rd_map
        for mp in a.maps.split(","):
            rd_map = bench_map if mp == "bench" else clutter(mp, F, ns, nc, dev)
            for ovr, st in [(int(o), int(x)) for o in a.ovr.split(",") for x in a.steps.split(",")]:
                time_k3(core_args=dict(N_RANGE=ns, N_DOPPLER=nc, N_RX=nrx, in_dtype=g["dtype"], cfar="os2d",
                                       max_frames=F, cfar_scale_ovr=ovr),
                        steps=st, rd_map=rd_map, F=F, dets=dets, cap=cap, nd=nd, stream=stream, iters=a.iters,
                        tag={"workload": w, "map": mp, "ovr": ovr})
            rd_map = None
        del bench_map, dets


if __name__ == "__main__":
    main()
