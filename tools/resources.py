#!/usr/bin/env python3
"""Per-kernel VGPR / scratch / occupancy / LDS report for libfmcw (hipcc remarks).

usage: python tools/resources.py [filter-substring]
"""
import re
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent.parent / "fpga-fmcw-radar-processor_amd"
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-fvisibility=hidden",
       *sys.argv[2:], "--cuda-device-only", "-c", "-o", "/tmp/fmcw_res.o", str(PKG / "csrc" / "fmcw_api.hip"),
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    if cur is None:
        continue
    for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                     ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
        m = re.search(pat, line)
        if m:
            cur[key] = int(m.group(1))


def short(n):
    """Demangle the fmcw kernel names to name<args> (c++filt, template args only)."""
    try:
        d = subprocess.run(["c++filt", n], capture_output=True, text=True).stdout.strip()
    except OSError:
        return n
    d = d.replace("fmcw::", "").replace("void ", "")
    return d.split("(", 1)[0].replace(" ", "")


flt = sys.argv[1] if len(sys.argv) > 1 else ""
for r in rows:
    s = short(r["name"])
    if flt in s:
        print(f"{s:34s} vgpr={r.get('vgpr', '?'):>3} agpr={r.get('agpr', 0):>3} scratch={r.get('scratch', '?'):>4} "
              f"occ={r.get('occ', '?')} lds={r.get('lds', '?')}")
