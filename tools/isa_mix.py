#!/usr/bin/env python3
"""Static instruction mix of one kernel in a hipcc --cuda-device-only -S listing.

usage: python tools/isa_mix.py <file.s> <substring of mangled kernel name> [--top N]
Prints the counts of VALU / SALU / LDS / VMEM instructions and the most common VALU opcodes
(static counts: loops are counted once)."""
import collections
import re
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 30
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(key) + r"\S*:", l))
    body = []
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        if l.startswith("\t") and not l.strip().startswith((".", ";")):
            body.append(l.split()[0])
    kinds = collections.Counter()
    for op in body:
        kinds["valu" if op.startswith("v_") else "salu" if op.startswith("s_") else
              "lds" if op.startswith("ds_") else
              "vmem" if op.startswith(("global_", "buffer_", "flat_", "scratch_")) else "other"] += 1
    print(lines[start][:90], len(body), dict(kinds))
    for op, n in collections.Counter(o for o in body if o.startswith(("v_", "ds_", "global_"))).most_common(top):
        print(f"  {op:28s} {n}")


if __name__ == "__main__":
    main()
