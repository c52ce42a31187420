#!/usr/bin/env python3
"""Where the S48 pair form goes wrong at 8192 x 1024 (GPU box): per-frame map error for several
chunk sizes, and for a bad frame the range rows whose Doppler spectrum is off."""
import sys
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, "oracle")
sys.path.insert(0, "fpga-fmcw-radar-processor_amd")
import fmcw_oracle as O
from fmcw import RadarCore, synth
from test_gpu_parity import to_complex
from conftest import rel_err

ns, nc, nf = 8192, 1024, 4
for dt in ("f16",):
    cube = synth.frames(nf, ns, nc, 1, "two_targets", seed=1234, dtype=dt)
    refs = [O.process(to_complex(cube[f], dt), None)["mag"] for f in range(nf)]
    for ch in (0, 2, 1):
        for sp in ("s48",):
            with RadarCore(N_RANGE=ns, N_DOPPLER=nc, in_dtype=dt, cfar="none", max_frames=nf, spectrum=sp,
                           chunk_frames=ch) as core:
                out = core.process(cube)
                chunk = core.info("chunk")
            errs = [rel_err(out.rd_map[f], refs[f]) for f in range(nf)]
            print(dt, sp, "chunk", chunk, "err", ["%.3g" % e for e in errs], flush=True)
            for f in range(nf):
                if errs[f] > 1e-3:
                    d = np.abs(out.rd_map[f] - refs[f]) / np.abs(refs[f]).max()
                    rows = np.nonzero(d.max(axis=1) > 1e-4)[0]
                    cols = np.nonzero(d.max(axis=0) > 1e-4)[0]
                    print("  frame", f, "bad rows", len(rows), rows[:12], rows[-4:], "bad cols", len(cols), cols[:8],
                          flush=True)
                    zero = np.nonzero(np.abs(out.rd_map[f]).max(axis=1) == 0)[0]
                    print("  all-zero rows", len(zero), zero[:8], flush=True)
