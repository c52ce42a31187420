"""fmcw CLI -- run the MI355X hot path on a file and write the reference's output formats.

    python -m fmcw.cli INPUT [--n-range 1024 --n-doppler 128 --cfar os2d|os1d|none]
                             [--out-dir DIR] [--quick] [--map-file radar_output.txt]

INPUT formats (by extension):
  .txt   "I Q" integer lines (data/golden_input_chirp.txt); a frame is N_DOPPLER chirps of
         N_RANGE samples; a file shorter than one frame is framed as N_DOPPLER identical
         chirps of its first N_RANGE samples (BASELINE config 1)
  .npy   complex64 [frames][rx][chirp][sample] or [chirp][sample], or int16 [..., 2]
  .bin   raw 32-bit AXI words {Q[31:16], I[15:0]} (radar_core.vhd:25-29), frame-major

Outputs in --out-dir (names the visualizer searches, model/visualize_radar_targets.py:37-107):
  ADR_detections.txt (or ADR_quick_det.txt with --quick): "r d mag" per detection
  radar_output.txt (with --map-file): "r d 0 0 mag" map of the first frame
  --doppler-centred shifts Doppler bins by N/2 (fftshift) in both files
  ADR_tracks.txt (with --tracks): the track-while-scan log, one scan per frame
                 ("TRK id R= D= Q=" / "SCAN_END ACTIVE=n", tb_radar_core.vhd:163-180)
"""
from __future__ import annotations

import argparse
from pathlib import Path

import numpy as np

from . import formats, synth
from .radar_core import RadarCore, adc_words_to_cube
from .tracker import TwsTracker


def load_cube(path: Path, ns: int, nc: int):
    if path.suffix == ".txt":
        iq = formats.read_adc_pairs(path)
        per = ns * nc
        if len(iq) < per:
            return synth.golden_chirp_frame(iq, nc, ns)[None], "f32"
        nf = len(iq) // per
        z = (iq[: nf * per, 0] + 1j * iq[: nf * per, 1]).astype(np.complex64)
        return z.reshape(nf, 1, nc, ns), "f32"
    if path.suffix == ".npy":
        a = np.load(path, allow_pickle=False)
        if a.dtype == np.int16:
            return a.reshape(-1, 1, nc, ns, 2) if a.ndim <= 4 else a, "i16"
        a = a.astype(np.complex64)
        return a.reshape(-1, 1, nc, ns) if a.ndim <= 3 else a, "f32"
    if path.suffix == ".bin":
        w = np.fromfile(path, dtype="<u4")
        nf = len(w) // (ns * nc)
        return adc_words_to_cube(w[: nf * ns * nc].reshape(nf, nc * ns), nc, ns).reshape(nf, 1, nc, ns, 2), "i16"
    raise SystemExit(f"unsupported input {path}")


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("input", type=Path)
    ap.add_argument("--n-range", type=int, default=1024)
    ap.add_argument("--n-doppler", type=int, default=128)
    ap.add_argument("--cfar", default="os2d", choices=["os2d", "os1d", "none"])
    ap.add_argument("--out-dir", type=Path, default=Path("."))
    ap.add_argument("--quick", action="store_true", help="write ADR_quick_det.txt (128x32 geometry)")
    ap.add_argument("--map-file", default=None)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--tracks", action="store_true", help="run the TWS tracker, write ADR_tracks.txt")
    ap.add_argument("--tracker-rtl", action="store_true", help="tracker in RTL-compat mode")
    ap.add_argument("--window", default="hamming", choices=["hamming", "none", "q15_rtl"])
    ap.add_argument("--doppler-centred", action="store_true",
                    help="write Doppler bins fftshifted (zero Doppler at N/2, as the visualizer assumes)")
    a = ap.parse_args(argv)
    cube, dt = load_cube(a.input, a.n_range, a.n_doppler)
    nf = cube.shape[0]
    with RadarCore(N_RANGE=a.n_range, N_DOPPLER=a.n_doppler, N_RX=cube.shape[1], in_dtype=dt,
                   cfar=a.cfar, max_frames=nf, device=a.device, window=a.window) as core:
        out = core.process(np.ascontiguousarray(cube))
    a.out_dir.mkdir(parents=True, exist_ok=True)
    det_name = "ADR_quick_det.txt" if a.quick else "ADR_detections.txt"
    n = formats.write_detections(a.out_dir / det_name, out.dets, doppler_centred=a.doppler_centred,
                                 n_doppler=a.n_doppler)
    if a.map_file:
        formats.write_rd_map(a.out_dir / a.map_file, out.rd_map[0], doppler_centred=a.doppler_centred)
    print(f"{nf} frame(s) {a.n_doppler}x{a.n_range}: {n} detections -> {a.out_dir / det_name}")
    if a.tracks:
        with TwsTracker(rtl_compat=a.tracker_rtl) as trk:
            hist = []
            for f in range(nf):
                tracks = trk.scan(out.dets[out.dets["frame"] == f])
                hist.append((tracks, trk.active_tracks))
        formats.write_tracks(a.out_dir / "ADR_tracks.txt", hist)


if __name__ == "__main__":
    main()
