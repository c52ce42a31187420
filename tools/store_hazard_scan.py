#!/usr/bin/env python3
"""Scan gfx950 assembly (hipcc --cuda-device-only -S, or llvm-objdump -d of a code object) for a VALU write of a wide VMEM store's data
VGPRs within 2 wait states of the store (the hazard hipcc pads with `s_nop 1` itself, but missed
after a dwordx3 store followed by a late-expanded `v_max_f32 vX, |vY|, |vY|` in ROCm 7.2 -- which
corrupted S48 spectrum tiles intermittently).  Prints every unpadded case;
exit status 1 if any.   usage: tools/store_hazard_scan.py file.s ...
(tests/test_abi.py runs it over the disassembly of libfmcw.so's gfx950 code objects.)"""
import re
import sys


def regs_in(op):
    out = set()
    for m in re.finditer(r'v\[(\d+):(\d+)\]', op):
        out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
    for m in re.finditer(r'(?<![\w\[:])v(\d+)\b', op):
        out.add(int(m.group(1)))
    return out


bad = 0
for path in sys.argv[1:]:
    lines = [l.split('//')[0] for l in open(path).read().split('\n')]  # objdump: drop the encoding comments
    fn = None
    for k, l in enumerate(lines):
        m = re.match(r'^(?:[0-9a-f]+ <)?(_Z\w+)>?:', l)
        if m:
            fn = m.group(1)
        t = l.strip()
        if not re.match(r'(buffer|global|flat)_store_dword(x3|x4)\b', t):
            continue
        ops = t.split(None, 1)[1].split(',')
        data = regs_in(ops[0] if t.startswith('buffer') else ops[1])
        ws, n = 0, k + 1
        while ws < 2 and n < len(lines):
            nt = lines[n].strip()
            n += 1
            if not nt or nt.startswith((';', '.')):
                continue
            if nt.startswith('s_nop'):
                ws += int(nt.split()[1], 0) + 1
                continue
            if nt.startswith('v_'):
                dst = regs_in(nt.split(None, 1)[1].split(',')[0])
                if dst & data:
                    print(f"{path}: {fn}: '{t[:60]}' then '{nt[:60]}' ({ws} wait states)")
                    bad += 1
                    break
            ws += 1
print(f"{bad} unpadded wide-store data hazards")
sys.exit(1 if bad else 0)
