#!/usr/bin/env python3
"""Per-frame HBM traffic and SQ instruction counts of the bench's kernels, from rocprofv3 PMC
passes of ONE bench.py command (MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE and WRITE_SIZE
each in its own run; the SQ counters in a third).

Normalisation: every counter is summed over all launches of a kernel in the run and divided by
the frames that kernel processed in the run (--frames w=N, known from the command: warm-up +
timed + profiled steps x frames per step), so the numbers do not depend on how the frames were
split into launches.  bench.py multiplies them by a launch's mean frames.

Kernels are assigned to workloads by their template arguments (N / NC differ between configs
2, 3 and 5): c2 = k_range*<1024>, k_doppler<256>; c3 = k_range*<4096>, k_doppler<512>,
k_cfar2d<512>; c5 = k_range*<8192>, k_doppler<1024>, k_cfar2d<1024>.

gfx950 correction: FETCH_SIZE reports half the bytes of a wide coalesced streaming read, so it
is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.  Units of both: KiB.

usage: python tools/pmc_summary.py --fetch F.csv --write W.csv [--sq SQ.csv]
       --frames c2=5120 --frames c3=80 --frames c5=80 [--spectrum c2=s48] --out profiles/pmc_r05.json
"""
import argparse
import collections
import csv
import json
import re

PATTERNS = {
    "c2": {"k_range": r"k_range\w*<1024,", "k_doppler": r"k_doppler<256,"},
    # K3 = the three launches of a 2-D CFAR batch (k_cfar2d, k_cfar2d_decide, k_cfar2d_emit; round 4)
    "c3": {"k_range": r"k_range\w*<4096,", "k_doppler": r"k_doppler<512,", "k_cfar": r"k_cfar2d(_decide|_emit)?<512[,>]"},
    "c5": {"k_range": r"k_range(\w*<8192,|_px<)", "k_doppler": r"k_doppler<1024,",
           "k_cfar": r"k_cfar2d(_lv|_decide|_emit)?<1024[,>]"},
}
ALG = {  # algorithmic bytes per frame, fp32 spectrum
    "c2": {"k_range": 1024 * 256 * 16, "k_doppler": 1024 * 256 * 12},
    "c3": {"k_range": 4096 * 512 * 4 * 16, "k_doppler": 4096 * 512 * (4 * 8 + 4), "k_cfar": 4096 * 512 * 4},
    "c5": {"k_range": 8192 * 1024 * 12, "k_doppler": 8192 * 1024 * 12, "k_cfar": 8192 * 1024 * 4},
}


def read(path):
    """{kernel name: {counter: [values per dispatch]}}"""
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("fmcw::", "").replace(" ", "")
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def classify(name):
    for w, pats in PATTERNS.items():
        for k, p in pats.items():
            if re.search(p, name):
                return w, k
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--sq", default=None)
    ap.add_argument("--frames", action="append", default=[], help="workload=frames processed in the run")
    ap.add_argument("--command", default="python3 bench.py --steps 2 --warmup 1 --prewarm-s 0 --no-cpu-baseline --no-h2d")
    ap.add_argument("--out", default="profiles/pmc_r05.json")
    ap.add_argument("--spectrum", action="append", default=[],
                    help="workload=f32|s48: the spectrum format the run used (algorithmic bytes; default f32)")
    a = ap.parse_args()
    frames = {k: int(v) for k, v in (x.split("=") for x in a.frames)}
    spec = dict(x.split("=") for x in a.spectrum)
    for w, fmt in spec.items():  # K1 writes and K2 reads b_sp bytes per point instead of 8
        b_sp = {"f32": 8, "f16": 4, "s48": 6}[fmt]
        px = {"c2": 1024 * 256, "c3": 4096 * 512 * 4, "c5": 8192 * 1024}[w]
        ALG[w]["k_range"] += px * (b_sp - 8)
        ALG[w]["k_doppler"] += px * (b_sp - 8)
    tables = [read(a.fetch), read(a.write)] + ([read(a.sq)] if a.sq else [])
    out = {"method": "rocprofv3 --pmc FETCH_SIZE, --pmc WRITE_SIZE and --pmc SQ_* in separate runs of `"
                     + a.command + "`; per kernel: sum over its launches / frames it processed; "
                     "FETCH_SIZE x2 (gfx950 wide-read correction), KiB -> bytes",
           "frames": frames, "spectrum": {w: spec.get(w, "f32") for w in frames}, "workloads": {}}
    # several kernel names may map to one (workload, kernel) entry (K3's three launches): the counters
    # are summed over all of them
    tot = collections.defaultdict(float)
    for t in tables:
        for name, ctrs in t.items():
            w, k = classify(name)
            if not w or w not in frames:
                continue
            ent = out["workloads"].setdefault(w, {"kernels": {}})["kernels"].setdefault(k, {"names": []})
            if name not in ent["names"]:
                ent["names"].append(name)
            for c, vals in ctrs.items():
                tot[(w, k, c)] += sum(vals)
                if c in ("FETCH_SIZE", "WRITE_SIZE") and re.search(r"k_cfar2d<|k_range|k_doppler", name):
                    ent["launches"] = len(vals)
    for (w, k, c), v in tot.items():
        ent = out["workloads"][w]["kernels"][k]
        if c == "FETCH_SIZE":
            ent["fetch_bytes_per_frame"] = v * 2 * 1024 / frames[w]
        elif c == "WRITE_SIZE":
            ent["write_bytes_per_frame"] = v * 1024 / frames[w]
        else:
            ent[c + "_per_frame"] = v / frames[w]
    for w, d in out["workloads"].items():
        for k, e in d["kernels"].items():
            if "fetch_bytes_per_frame" in e and "write_bytes_per_frame" in e:
                e["hbm_bytes_per_frame"] = e["fetch_bytes_per_frame"] + e["write_bytes_per_frame"]
                e["algorithmic_bytes_per_frame"] = ALG[w].get(k)
                if e["algorithmic_bytes_per_frame"]:
                    e["traffic_over_algorithmic"] = round(e["hbm_bytes_per_frame"] / e["algorithmic_bytes_per_frame"], 4)
            for key in list(e):
                if isinstance(e[key], float) and key != "traffic_over_algorithmic":
                    e[key] = round(e[key], 1)
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
