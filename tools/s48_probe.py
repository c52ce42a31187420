#!/usr/bin/env python3
"""Map error of the S48 spectrum against the fp64 oracle over a few geometries (GPU box; a
localisation aid for the pair form: K1 family x K2 size x frames per launch)."""
import sys
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, "oracle")
sys.path.insert(0, "fpga-fmcw-radar-processor_amd")
import fmcw_oracle as O
from fmcw import RadarCore, synth
from test_gpu_parity import to_complex
from conftest import rel_err

CASES = [  # ns, nc, frames, dtype, chunk
    (8192, 1024, 1, "f16", 0), (8192, 1024, 4, "f16", 0), (8192, 128, 8, "f16", 0),
    (4096, 1024, 2, "f32", 0), (2048, 1024, 2, "f32", 0), (1024, 1024, 2, "f32", 0),
    (8192, 512, 2, "f16", 0), (8192, 256, 2, "f16", 0),
]
for ns, nc, nf, dt, ch in CASES:
    cube = synth.frames(nf, ns, nc, 1, "two_targets", seed=1234, dtype=dt)
    for sp in ("f32", "s48"):
        with RadarCore(N_RANGE=ns, N_DOPPLER=nc, in_dtype=dt, cfar="none", max_frames=nf, spectrum=sp,
                       chunk_frames=ch) as core:
            out = core.process(cube)
            chunk = core.info("chunk")
        errs = []
        for f in sorted({0, nf - 1}):
            ref = O.process(to_complex(cube[f], dt), None)["mag"]
            errs.append(rel_err(out.rd_map[f], ref))
        print(ns, nc, nf, dt, sp, "chunk", chunk, "err", ["%.3g" % e for e in errs], flush=True)
