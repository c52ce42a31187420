#!/usr/bin/env python3
"""bench.py -- radar frames/s of the MI355X FMCW hot path (BASELINE.json metric).

One step = one pass of the hot path (window -> range FFT -> corner turn -> Doppler FFT ->
|X| map -> OS-CFAR -> ordered detection list) over one batch of synthetic frames already
resident in HBM.  Headline workload at N=1: BASELINE config 2 -- 256 chirps x 1024 samples,
fp32 complex, 1 Rx, 1-D OS-CFAR 16 ref / 4 guard -- in batches of 1024 frames per GPU per step
(= config 4's per-GPU share of 8192 frames at 8 GPUs; weak scaling).  With N > 1 each rank
processes its own 1024 frames (frame sharding, no data-path collective) and the detection
lists are gathered over RCCL inside the step (config 4).

The same JSON line carries sub-records "config3" and "config5" (BASELINE configs 3 and 5, 16
frames per GPU per step, 2-D OS-CFAR), timed the same way in the same process, each with the
roofline of ITS dominant kernel (the kernel with the most time per step).

Launch: `python bench.py [--gpus N --steps K --warmup W]`, or for N > 1
`python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1
 --master-port P bench.py --gpus N ...`.  Rank 0 prints ONE JSON line.

Warm-up: the W untimed steps, then more untimed steps until --prewarm-s (0.3 s) of sustained work
has run, the same count on every rank; "warmup_steps_run" reports the total.  The MI355X reaches
its steady clocks only after ~0.1 s of load, so timing K=10 steps after 3 warm-up steps (4 ms)
read 7-10 % low (profiles/r04/warmup/).  --prewarm-s 0 restores the W-only warm-up.

roofline: the dominant kernel's algorithmic bytes per launch / its average launch duration,
from HIP events the library records on the launch stream (fmcw_set_profiling: the dispatches'
own begin / end timestamps, hipExtLaunchKernelGGL) over a profiled repeat of the timed steps.  traffic: HBM bytes per launch from rocprofv3 PMC passes
(profiles/pmc_r05.json, per frame x the launch's mean frames; tools/pmc_summary.py), or null.
The 2-D CFAR (k_cfar2d) is bound by VALU work, not bytes: its roofline is SQ_INSTS_VALU per
launch (same profile file) / launch time against the chip's VALU issue rate (2 wave-instructions
per CU per clock at 2.4 GHz), its map bytes beside.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "fpga-fmcw-radar-processor_amd"))

HBM_PEAK_GBPS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
CLOCK_GHZ = 2.4             # MI355X peak engine clock
PMC_FILE = "pmc_r06.json"   # per-frame HBM bytes and SQ counts per workload (tools/pmc_summary.py)

WORKLOADS = {
    "c2": dict(ns=1024, nc=256, nrx=1, dtype="f32", cfar="os1d", frames=1024, recipe="two_targets", spectrum="s48",
               desc="BASELINE config 2: 256 chirps x 1024 samples fp32, 1 Rx, OS-CFAR 1-D 16 ref / 4 guard"),
    "c3": dict(ns=4096, nc=512, nrx=4, dtype="f32", cfar="os2d", frames=16, recipe="two_targets", spectrum="f32",
               desc="BASELINE config 3: 512 chirps x 4096 samples fp32, 4 Rx NCI, 2-D OS-CFAR"),
    "c5": dict(ns=8192, nc=1024, nrx=1, dtype="f16", cfar="os2d", frames=16, recipe="two_targets", spectrum="f32",
               desc="BASELINE config 5: 1024 chirps x 8192 range bins, fp16 complex samples, 2-D OS-CFAR"),
}
SUB = {"c3": "config3", "c5": "config5"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--prewarm-s", type=float, default=0.3,
                    help="untimed warm-up continues past --warmup steps until this much sustained work has run")
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--frames", type=int, default=0, help="frames per GPU per step (0 = workload default)")
    ap.add_argument("--chunk", type=int, default=0, help="frames per kernel chunk (0 = library auto)")
    ap.add_argument("--no-sub", action="store_true", help="skip the config-3 / config-5 sub-records")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--gather", default="rccl", choices=["rccl", "torch"],
                    help="N > 1: libfmcw's RCCL gather-to-root (no host sync) or torch all_gather")
    ap.add_argument("--no-h2d", action="store_true", help="skip the H2D-inclusive measurement")
    ap.add_argument("--spectrum", default=None, choices=["f32", "f16", "s48"],
                    help="element type of the corner-turned spectrum (fmcw.h fmcw_spectrum_dtype); default: "
                         "the workload's (WORKLOADS: s48 at config 2, where A/B measured it faster, f32 at "
                         "configs 3 / 5, where it was not)")
    return ap.parse_args()


def load_pmc():
    f = REPO / "profiles" / PMC_FILE
    if f.exists():
        try:
            return json.loads(f.read_text())
        except Exception:  # noqa: BLE001 -- a damaged file means "no counters"
            return {}
    return {}


def kernel_rooflines(wl, name, F, steps, kt, spectrum, n_cu, pmc):
    """Per-kernel rooflines from the HIP-event times of `steps` profiled steps of F frames."""
    ns, nc, nrx = wl["ns"], wl["nc"], wl["nrx"]
    b_in = 8 if wl["dtype"] == "f32" else 4
    b_sp = {"f16": 4, "s48": 6}.get(spectrum, 8)
    px = ns * nc * nrx
    frames = F * steps
    # algorithmic bytes per frame: K1 cube in + spectrum out; K2 spectrum in + map
    # out; K3 map in (+ detections, negligible)
    alg = {"k_range": px * (b_in + b_sp), "k_doppler": px * b_sp + ns * nc * 4, "k_cfar": ns * nc * 4}
    what = {"k_range": "k_range (window + range FFT + corner turn)",
            "k_doppler": "k_doppler (Doppler FFT + |X|" + (" NCI" if nrx > 1 else "") + " + map"
                         + (" + 1-D CFAR)" if wl["cfar"] == "os1d" else ")"),
            "k_cfar": "k_cfar2d (2-D OS-CFAR, 128 refs, adaptive scale)",
            "k_compact": "k_det_list (ordered detection list, one-pass look-back scan)"}
    pw = (pmc.get("workloads") or {}).get(name, {})
    pk = pw.get("kernels", {})
    out = {}
    for k, (ms, n) in kt.items():
        if not n:
            continue
        per_step_ms = ms / steps
        r = {"kernel": what.get(k, k), "launches_per_step": n // steps, "avg_launch_ms": round(ms / n, 5),
             "ms_per_step": round(per_step_ms, 4)}
        fpl = frames / n                                   # mean frames per launch
        if k in alg:
            bpl = alg[k] * fpl
            gbps = bpl / (ms / n * 1e-3) / 1e9
            traffic = pk.get(k, {}).get("hbm_bytes_per_frame")
            r.update({"bound": "hbm", "achieved": round(gbps, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                      "frac": round(gbps / HBM_PEAK_GBPS, 4), "bytes_per_launch": int(bpl),
                      "frames_per_launch": round(fpl, 3),
                      "traffic": int(traffic * fpl) if traffic else None})
        if k == "k_cfar" and wl["cfar"] == "os2d":
            # VALU issue: a SIMD retires a 32-bit wave64 VALU instruction every 2 cycles with >= 2
            # waves on it (MI355X_MICROARCH.md, "Per-instruction cycle constants": v_fma_f32 2 cyc,
            # SIMD-32), so 4 SIMDs give 2 wave-instructions per CU per clock
            hbm = dict(r)
            sq = pk.get("k_cfar", {}).get("SQ_INSTS_VALU_per_frame")
            peak = n_cu * CLOCK_GHZ * 2                        # G wave-instructions / s
            ach = sq * fpl / (ms / n * 1e-3) / 1e9 if sq else None
            r.update({"bound": "valu", "achieved": round(ach, 1) if ach else None, "peak": round(peak, 1),
                      "unit": "G VALU wave-instructions/s", "frac": round(ach / peak, 4) if ach else None,
                      "SQ_INSTS_VALU_per_launch": int(sq * fpl) if sq else None,
                      "map_GBps": hbm["achieved"], "map_frac_of_hbm": hbm["frac"],
                      "traffic": hbm["traffic"]})
        out[k] = r
    return out


SPECTRUM_FORMAT = {  # fmcw.h fmcw_spectrum_dtype; every arithmetic step is fp32 either way
    "f32": "complex fp32, 8 B per point",
    "f16": "half2 of X / N_range, 4 B per point (map within 2e-3)",
    "s48": "6 B per point: 23-bit significands sharing an 8-bit exponent per chirp quad of a range bin "
           "(22-bit per pair above n_range 1024); map within the north star's 1e-4 of the fp64 oracle (tested)",
}


def shard_plan(world, rank, F):
    """Frame sharding of one step (SURVEY.md 8e, weak scaling): every rank runs F frames of its
    own, global frames [rank * F, (rank + 1) * F); its synthetic input is seeded by its first global
    frame (seed 1234 + frame), and its detection records carry global frame ids
    (frame_offset) on the wire, whose fixed message holds 128 records per frame."""
    first = rank * F
    return {"first_global": first, "seed": 1234 + first, "frames": F, "frame_offset": first,
            "wire_cap": F * 128, "global_frames": world * F}


def spectrum_of(wl, args, primary):
    """The corner-turned spectrum format a workload runs: --spectrum for the primary workload if
    given, else the workload's own (WORKLOADS)."""
    return args.spectrum if primary and args.spectrum else wl["spectrum"]


def run_workload(name, args, world, rank, dev, primary, pmc, n_cu):
    import numpy as np
    import torch
    import torch.distributed as dist
    from fmcw import RadarCore, synth
    from fmcw.dist import RcclGather, gather_detections

    wl = dict(WORKLOADS[name])
    if primary and args.frames:
        wl["frames"] = args.frames
    F, ns, nc, nrx = wl["frames"], wl["ns"], wl["nc"], wl["nrx"]
    steps, warmup = args.steps, args.warmup  # the sub-records are timed like the headline
    local = dev.index
    core = RadarCore(N_RANGE=ns, N_DOPPLER=nc, N_RX=nrx, in_dtype=wl["dtype"], cfar=wl["cfar"],
                     max_frames=F, chunk_frames=args.chunk if primary else 0, device=local,
                     spectrum=spectrum_of(wl, args, primary))
    # synthetic input: 16 distinct frames (seed 1234 + global frame), tiled to F, resident in HBM
    n_u = min(16, F)
    plan = shard_plan(world, rank, F)
    first_global = plan["first_global"]
    u = synth.frames(n_u, ns, nc, nrx, wl["recipe"], seed=plan["seed"], dtype=wl["dtype"])
    if wl["dtype"] == "f32":
        u = u.view(np.float32)
    ut = torch.from_numpy(np.ascontiguousarray(u)).to(dev)
    reps = (F + n_u - 1) // n_u
    cube = ut.repeat((reps,) + (1,) * (ut.dim() - 1))[:F].contiguous()
    del ut
    rd_map = torch.empty((F, ns, nc), dtype=torch.float32, device=dev)
    det_cap = F * 4096
    # two detection buffers: step i+1 may be enqueued while step i's list is still gathered;
    # status words (fmcw.h FMCW_STATUS_WORDS): found, lost, window / word saturations
    bufs = [(torch.empty((det_cap, 4), dtype=torch.int32, device=dev), torch.zeros(4, dtype=torch.int32, device=dev))
            for _ in range(2)]
    dets, n_dets = bufs[0]
    cstream = torch.cuda.current_stream(dev)
    stream = cstream.cuda_stream
    gather = primary and world > 1 and not args.no_gather
    gather_kind = None
    rg = None
    rccl_info = None
    wire_cap = plan["wire_cap"]        # records per rank on the wire: 128 per frame (~64 found)
    use_rccl = args.gather == "rccl" and os.environ.get("FMCW_BENCH_BACKEND", "nccl") == "nccl"
    if gather and use_rccl:
        # libfmcw's fmcw_gather_dets: fixed-size ncclSend/ncclRecv to rank 0, device-side
        # compaction; stream-ordered after the step, no host synchronisation per step
        try:
            obj = [RcclGather.make_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            rg = RcclGather(obj[0], world, rank, local, wire_cap)
            gather_kind = "libfmcw fmcw_gather_dets (RCCL send/recv to rank 0, fixed wire_cap, no host sync)"
            # what RCCL itself reports (fmcw_comm_info: ncclCommCount / UserRank / CuDevice), from
            # every rank: the line then proves the gather spans `world` distinct GPUs
            mine = rg.info()
            infos = [None] * world
            dist.all_gather_object(infos, mine)
            rccl_info = {"rccl_ranks": mine["rccl_ranks"], "rccl_user_ranks": [i["rccl_rank"] for i in infos],
                         "rccl_devices": [i["rccl_device"] for i in infos], "wire_cap": mine["wire_cap"]}
        except Exception as e:  # noqa: BLE001 -- reported, then the torch path is used
            print(f"rank {rank}: RCCL gather unavailable ({e}); using torch all_gather", file=sys.stderr)
            rg = None
    if gather and rg is None:
        gather_kind = (("rccl" if dist.get_backend() == "nccl" else dist.get_backend())
                       + " all_gather via torch.distributed, one step behind the compute")
    root_out = torch.empty((world * wire_cap, 4), dtype=torch.int32, device=dev) if rg is not None else None
    root_n = torch.zeros(4, dtype=torch.int32, device=dev) if rg is not None else None
    gstream = torch.cuda.Stream(dev) if gather else None
    # RCCL path: the gather of step i runs on gstream behind step i (event), and step i + 2 (same
    # detection buffer) waits for it on the device: no host synchronisation anywhere
    g_done = [None, None]
    last = {"i": 0, "pending": None}

    def do_gather(d, nd, ev):
        with torch.cuda.stream(gstream):
            gstream.wait_event(ev)
            allr, counts = gather_detections(d, nd[:2], first_global)
            last["total"] = int(allr.shape[0])

    def step():
        b = last["i"] % 2
        d, nd = bufs[b]
        last["i"] += 1
        if rg is not None and g_done[b] is not None:
            cstream.wait_event(g_done[b])
        core.enqueue(cube.data_ptr(), F, rd_map.data_ptr(), d.data_ptr(), det_cap, nd.data_ptr(), stream)
        if rg is not None:
            ev = torch.cuda.Event()
            ev.record(cstream)
            gstream.wait_event(ev)
            rg.gather(d.data_ptr(), det_cap, nd.data_ptr(), first_global,
                      root_out.data_ptr() if rank == 0 else None, root_n.data_ptr() if rank == 0 else None,
                      0, gstream.cuda_stream)
            g_done[b] = torch.cuda.Event()
            g_done[b].record(gstream)
        elif gather:
            ev = torch.cuda.Event()
            ev.record(cstream)
            prev, last["pending"] = last["pending"], (d, nd, ev)
            if prev is not None:
                do_gather(*prev)

    def flush():
        if last["pending"] is not None:
            prev, last["pending"] = last["pending"], None
            do_gather(*prev)

    def timed(k):
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(k):
            step()
        flush()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
        return float(el.item())

    # untimed warm-up: the W steps asked for, then more steps until args.prewarm_s of sustained
    # work has run (the same number on every rank: the gather is collective).  The MI355X reaches
    # its steady clocks only after ~0.1 s of load: with 3 warm-up steps (4 ms) the timed steps ran
    # 7-10 % slower than with 100 (profiles/r04/warmup/).
    t_w = time.perf_counter()
    for _ in range(warmup):
        step()
    flush()
    torch.cuda.synchronize(dev)
    n_warm = warmup
    if args.prewarm_s > 0:  # same branch on every rank (args are shared)
        t1 = time.perf_counter()  # one more step, timed on its own: the first ones carry one-time costs
        step()
        flush()
        torch.cuda.synchronize(dev)
        per = max(time.perf_counter() - t1, 1e-6)
        n_warm += 1
        spent = time.perf_counter() - t_w
        extra = torch.tensor([max(0, int((args.prewarm_s - spent) / per) + 1)], dtype=torch.int64, device=dev)
        if world > 1:
            dist.all_reduce(extra, op=dist.ReduceOp.MAX)
        for _ in range(int(extra.item())):
            step()
        flush()
        n_warm += int(extra.item())
    elapsed = timed(steps)
    st = n_dets.tolist()
    n_det_step = int(st[0])

    # profiled repeat: per-kernel durations from HIP events on the launch stream
    core.reset_kernel_times()
    core.set_profiling(True)
    elapsed_prof = timed(steps)
    kt = core.kernel_times()
    core.set_profiling(False)
    spectrum = spectrum_of(wl, args, primary)
    kern = kernel_rooflines(wl, name, F, steps, kt, spectrum, n_cu, pmc)
    dom = max((k for k in kern if k in ("k_range", "k_doppler", "k_cfar")), key=lambda k: kern[k]["ms_per_step"])
    value = world * F * steps / elapsed
    b_in = 8 if wl["dtype"] == "f32" else 4
    e2e_bytes = F * (ns * nc * nrx * b_in + ns * nc * 4) + 16 * n_det_step
    rec = {
        "metric": "radar frames/sec (range-Doppler+CFAR)",
        "value": round(value, 1), "unit": "frames/s", "n_gpus": world, "steps": steps, "warmup": warmup,
        "warmup_steps_run": n_warm, "prewarm_s": args.prewarm_s,
        "ms_per_step": round(elapsed / steps * 1e3, 4),
        "dtype": wl["dtype"],
        "config": {"workload": wl["desc"], "frames_per_gpu_step": F, "n_chirps": nc,
                   "n_samples": ns, "n_rx": nrx, "cfar": wl["cfar"], "rd_map": "linear fp32, written",
                   "spectrum": spectrum,
                   "spectrum_format": SPECTRUM_FORMAT[spectrum],
                   "detection_gather": gather_kind if gather else "none",
                   "parallelism": f"frame-sharded x{world}"},
        "range_kernel": core.info("range_kernel"),
        "chunk_frames": core.info("chunk"),
        "detections_per_step": n_det_step,
        "status_words": [int(x) for x in st],
        "e2e_GBps_algorithmic": round(e2e_bytes * steps * world / elapsed / 1e9, 1),
        "e2e_frac_of_peak": round(e2e_bytes * steps / elapsed / 1e9 / HBM_PEAK_GBPS, 4),
        "roofline": {k: v for k, v in kern[dom].items() if k not in ("launches_per_step",)},
        "kernels": kern,
        "profiled_step_ms": round(elapsed_prof / steps * 1e3, 4),
    }
    from fmcw._lib import RANGE_KERNELS
    rec["range_kernel"] = RANGE_KERNELS[rec["range_kernel"]]

    if primary and not args.no_h2d and world == 1:
        # H2D-inclusive rate: the cube streamed from pinned host memory inside each step (copy of
        # batch i+1 on a copy stream overlapping the compute of batch i), PCIe-bound by design
        Fh = min(F, 256)
        host = torch.empty((Fh,) + tuple(cube.shape[1:]), dtype=cube.dtype, pin_memory=True)
        host.copy_(cube[:Fh].cpu())
        dbuf = [torch.empty_like(cube[:Fh]) for _ in range(2)]
        cps = torch.cuda.Stream(dev)
        used = [None, None]
        d_h, nd_h = bufs[0]
        n_h = 8

        def h2d_run():
            for i in range(n_h):
                b = i % 2
                with torch.cuda.stream(cps):
                    if used[b] is not None:
                        cps.wait_event(used[b])
                    dbuf[b].copy_(host, non_blocking=True)
                    ready = torch.cuda.Event()
                    ready.record(cps)
                cstream.wait_event(ready)
                core.enqueue(dbuf[b].data_ptr(), Fh, rd_map.data_ptr(), d_h.data_ptr(), det_cap, nd_h.data_ptr(),
                             stream)
                used[b] = torch.cuda.Event()
                used[b].record(cstream)

        h2d_run()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        h2d_run()
        torch.cuda.synchronize(dev)
        th = time.perf_counter() - t0
        rec["h2d_inclusive"] = {"frames_per_s_per_gpu": round(n_h * Fh / th, 1),
                                "GBps_h2d": round(n_h * host.numel() * host.element_size() / th / 1e9, 1),
                                "sample": f"{n_h} batches of {Fh} frames from pinned host memory, copy/compute overlapped"}
        del host, dbuf
    if rccl_info is not None:
        rec["config"]["rccl"] = rccl_info
        rec["rccl_ranks"] = rccl_info["rccl_ranks"]
    if rg is not None and rank == 0:
        torch.cuda.synchronize(dev)
        rec["config"]["gathered_records_last_step"] = int(root_n[0].item())
        rec["config"]["gather_lost_last_step"] = int(root_n[1].item())
        rec["gathered_records_last_step"] = int(root_n[0].item())
    core.close()
    if rg is not None:
        rg.close()
    del cube, rd_map, bufs
    torch.cuda.empty_cache()
    return rec


def cpu_baseline(args, wl):
    import numpy as np
    from fmcw import synth
    sys.path.insert(0, str(REPO / "oracle"))
    import cpu_baseline as cb
    import fmcw_oracle as O
    # C backend (oracle/fmcw_cpu.c) on the same workload: single core and the job's CPU share
    ns, nc, nrx = wl["ns"], wl["nc"], wl["nrx"]
    nt = cb.threads_allowed()
    batch = max(8, nt)
    uu = synth.frames(min(16, batch), ns, nc, nrx, wl["recipe"], seed=1234, dtype="f32")
    ucube = np.concatenate([uu] * ((batch + len(uu) - 1) // len(uu)))[:batch]
    cf = O.Cfar1D() if wl["cfar"] == "os1d" else O.Cfar2D()
    mc = cb.measure_c(ucube, cf, runs=20, budget_s=args.cpu_seconds / 2)
    ac = mc["all_core"]
    cpu = {"value": round(ac["frames_per_s"], 2), "unit": "frames/s", "cores": ac["threads"],
           "kind": "port",
           "single_core_frames_per_s": round(mc["single_core"]["frames_per_s"], 2),
           "nproc": mc["nproc"], "cpus_allowed": mc["affinity"], "omp_num_threads": mc["omp_num_threads"],
           "cpu_model": mc["cpu_model"],
           "sample": (f"C restatement of the oracle (oracle/fmcw_cpu.c, OpenMP, fp32), {batch} frames of "
                      f"{ns}x{nc}x{nrx} per run, median of {ac['runs']} runs at {ac['threads']} threads and "
                      f"{mc['single_core']['runs']} runs at 1 thread")}
    # the whole node's CPUs: the job runs on a 16-CPU share of the node (gpurun box rule), so the
    # all-affinity figure is the measured per-thread rate at 16 threads times the CPUs the
    # affinity mask lists -- an extrapolation, labelled as such, not a measurement
    aff = mc["affinity"] if isinstance(mc["affinity"], int) else None
    if aff and ac["threads"] > 0:
        cpu["all_affinity_cpus_estimate"] = {
            "cpus": aff, "frames_per_s": round(ac["frames_per_s"] / ac["threads"] * aff, 1),
            "how": f"{ac['threads']}-thread rate x {aff}/{ac['threads']} (linear; not run: the job's CPU share "
                   f"is {ac['threads']} CPUs)"}
    if args.workload == "c2":
        # config-3 leg (2-D OS-CFAR, 4 rx NCI): one frame per run
        u3 = synth.frames(1, 4096, 512, 4, "two_targets", seed=1234, dtype="f32")
        m3 = cb.measure_c(u3, O.Cfar2D(), runs=20, budget_s=args.cpu_seconds / 2)
        cpu["config3_2d_cfar"] = {
            "all_core_frames_per_s": round(m3["all_core"]["frames_per_s"], 3),
            "single_core_frames_per_s": round(m3["single_core"]["frames_per_s"], 3),
            "threads": m3["all_core"]["threads"],
            "sample": f"1 frame of 4096x512x4 (NCI, 2-D OS-CFAR) per run, median of "
                      f"{m3['all_core']['runs']} / {m3['single_core']['runs']} runs"}
    return cpu


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; the modulo only matters for a rehearsal of N ranks on fewer GPUs
    # (with FMCW_BENCH_BACKEND=gloo, since RCCL needs distinct devices)
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        backend = os.environ.get("FMCW_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    pmc = load_pmc()

    rec = run_workload(args.workload, args, world, rank, dev, True, pmc, n_cu)
    subs = {}
    if not args.no_sub and args.workload == "c2":
        for w in ("c3", "c5"):
            subs[SUB[w]] = run_workload(w, args, world, rank, dev, False, pmc, n_cu)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, WORKLOADS[args.workload])

    out = {
        "metric": rec["metric"], "value": rec["value"], "unit": "frames/s", "n_gpus": world,
        "steps": rec["steps"], "warmup": rec["warmup"], "warmup_steps_run": rec["warmup_steps_run"],
        "prewarm_s": rec["prewarm_s"], "ms_per_step": rec["ms_per_step"],
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": rec["dtype"],
        "data": "synthetic (tb_radar_core-style point targets + uniform noise, int16-quantised)",
        "config": rec["config"],
        "roofline": rec["roofline"],
        "cpu_baseline": cpu,
    }
    for k in ("range_kernel", "chunk_frames", "detections_per_step", "status_words", "e2e_GBps_algorithmic",
              "e2e_frac_of_peak", "kernels", "profiled_step_ms", "h2d_inclusive", "rccl_ranks",
              "gathered_records_last_step"):
        if k in rec:
            out[k] = rec[k]
    out["h2d_inclusive_fps"] = rec.get("h2d_inclusive", {}).get("frames_per_s_per_gpu")
    out.update(subs)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
