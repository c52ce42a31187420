#!/usr/bin/env python3
"""Per-frame map error of the S48 pair form by K1 family / K2 size / chunk (GPU box)."""
import sys
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, "oracle")
sys.path.insert(0, "fpga-fmcw-radar-processor_amd")
import fmcw_oracle as O
from fmcw import RadarCore, synth
from test_gpu_parity import to_complex
from conftest import rel_err

CASES = [(8192, 1024, 8, 4, "f16"), (8192, 1024, 6, 3, "f16"), (8192, 512, 8, 4, "f16"),
         (4096, 1024, 4, 4, "f32"), (2048, 1024, 4, 4, "f32"), (8192, 1024, 4, 4, "f32")]
for ns, nc, nf, ch, dt in CASES:
    cube = synth.frames(nf, ns, nc, 1, "two_targets", seed=1234, dtype=dt)
    with RadarCore(N_RANGE=ns, N_DOPPLER=nc, in_dtype=dt, cfar="none", max_frames=nf, spectrum="s48",
                   chunk_frames=ch) as core:
        out = core.process(cube)
    errs = [rel_err(out.rd_map[f], O.process(to_complex(cube[f], dt), None)["mag"]) for f in range(nf)]
    print(ns, nc, nf, "chunk", ch, dt, "err", ["%.2g" % e for e in errs], flush=True)
