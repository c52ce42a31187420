#!/usr/bin/env python3
"""Per-launch HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE, each in
its own run -- MI355X_MICROARCH.md "HBM [CDNA4]": the two do not fit one TCC pass).

Units are KiB.  gfx950 correction: FETCH_SIZE reports half the bytes of a wide coalesced
streaming read, so it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.

usage: python tools/pmc_summary.py FETCH_CSV WRITE_CSV --workload c2 --frames-per-launch 32
       [--out profiles/pmc_r01.json]
"""
import argparse
import collections
import csv
import json


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        if "fmcw::" not in name:
            continue
        short = name.split("fmcw::", 1)[1].split("(", 1)[0]
        acc[short].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--frames-per-launch", type=int, required=True)
    ap.add_argument("--out", default="profiles/pmc_r01.json")
    a = ap.parse_args()
    fetch = per_kernel(a.fetch_csv, "FETCH_SIZE")
    write = per_kernel(a.write_csv, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, 0.0) * 2 * 1024
        w = write.get(k, 0.0) * 1024
        kernels[k] = {"fetch_bytes": round(f), "write_bytes": round(w), "hbm_bytes": round(f + w)}
    rng = next((v for k, v in kernels.items() if k.startswith("k_range")), None)
    out = {
        "workload": a.workload,
        "frames_per_launch": a.frames_per_launch,
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of bench.py; "
                  "KiB -> bytes; FETCH x2 (gfx950 wide-read correction); mean over launches",
        "k_range_bytes_per_launch": rng["hbm_bytes"] if rng else None,
        "kernels": kernels,
    }
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
