"""Text formats of the reference's simulation outputs, so model/ visualizers read our results.

  detections  "r d mag" -- exactly 3 integer tokens per line (model/visualize_radar_targets.py:
              117-120), searched under the names ADR_quick_det.txt / ADR_detections.txt
              (:37-107); "quick" in the name selects the 128x32 geometry (:392-394).
              Writer of record: the monitor process of rtl/old/tb_radar_core.vhd:173-208.
  rd map      "r d 0 0 mag" -- 5 columns, range-major, as data/radar_output.txt.
              The visualizer's parser rejects 5-token lines; this is the data/ format.
  ADC input   "I Q" integer pairs, one sample per line, as data/golden_input_chirp.txt.

Doppler order.  The library emits natural FFT order (bin 0 = zero Doppler).
The visualizer centres zero Doppler at N_DOPPLER/2 (bin_to_velocity_mps,
visualize_radar_targets.py:174-182) and the ADR stimuli pre-offset by +N/2
(rtl/old/ADR_tb_quick.vhd:149-157); the writers' ``doppler_centred=True`` applies that
fftshift, d' = (d + N/2) mod N, so that the visualizer converts zero Doppler to 0 m/s.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np


def centre_doppler(d, n_doppler: int):
    """Natural-order Doppler bins -> centred order (fftshift): (d + N/2) mod N."""
    return (np.asarray(d, np.int64) + n_doppler // 2) % n_doppler


def write_detections(path, dets, frame: int | None = None, doppler_centred: bool = False,
                     n_doppler: int | None = None) -> int:
    """Write detections as 'r d mag' integer lines (optionally only one frame's)."""
    d = dets if frame is None else dets[dets["frame"] == frame]
    mag = np.rint(np.asarray(d["mag"], np.float64)).astype(np.int64)
    dop = np.asarray(d["doppler"], np.int64)
    if doppler_centred:
        if not n_doppler:
            raise ValueError("doppler_centred needs n_doppler")
        dop = centre_doppler(dop, n_doppler)
    with open(path, "w") as f:
        for r, dd, m in zip(d["range"].tolist(), dop.tolist(), mag.tolist()):
            f.write(f"{r} {dd} {m}\n")
    return len(d)


def read_detections(path) -> np.ndarray:
    """Parse like load_detections() (visualize_radar_targets.py:109-122): 3-token lines only."""
    rows = []
    for line in Path(path).read_text().splitlines():
        p = line.split()
        if len(p) == 3:
            rows.append([int(p[0]), int(p[1]), int(p[2])])
    return np.array(rows, dtype=np.int64).reshape(-1, 3)


def write_rd_map(path, rd_map: np.ndarray, doppler_centred: bool = False) -> None:
    """One frame [range][doppler] -> 'r d 0 0 mag' lines, range-major, integer magnitudes."""
    m = np.rint(np.asarray(rd_map, np.float64)).astype(np.int64)
    if doppler_centred:
        m = np.fft.fftshift(m, axes=-1)         # column d' holds natural bin (d' - N/2) mod N
    nr, nd = m.shape
    r = np.repeat(np.arange(nr), nd)
    d = np.tile(np.arange(nd), nr)
    z = np.zeros_like(r)
    np.savetxt(path, np.stack([r, d, z, z, m.ravel()], axis=1), fmt="%d")


def read_rd_map(path, n_range: int = 1024, n_doppler: int = 128) -> np.ndarray:
    """data/radar_output.txt -> [range][doppler] int map (columns r d 0 0 mag)."""
    a = np.loadtxt(path, dtype=np.int64)
    out = np.zeros((n_range, n_doppler), np.int64)
    out[a[:, 0], a[:, 1]] = a[:, 4]
    return out


def read_adc_pairs(path) -> np.ndarray:
    """'I Q' integer lines (data/golden_input_chirp.txt) -> int array [n, 2]."""
    return np.loadtxt(path, dtype=np.int64).reshape(-1, 2)


def write_adc_pairs(path, iq: np.ndarray) -> None:
    np.savetxt(path, np.asarray(iq, np.int64).reshape(-1, 2), fmt="%d")


def write_tracks(path, scans) -> None:
    """Track log as rtl/src/tb_radar_core.vhd:163-180 writes it: per scan, one
    'TRK id R=range D=doppler Q=quality' line per reported track (R, D = the Q2 trk_range /
    trk_doppler words as signed integers), then 'SCAN_END ACTIVE=n'.  scans: iterable of
    (tracks, active) with tracks in fmcw.tracker.TRACK_DTYPE."""
    with open(path, "w") as f:
        for tracks, active in scans:
            for t in tracks:
                f.write(f"TRK {int(t['id'])} R={int(t['range_q2'])} D={int(t['doppler_q2'])} "
                        f"Q={int(t['quality'])}\n")
            f.write(f"SCAN_END ACTIVE={int(active)}\n")


def read_tracks(path):
    """Parse like load_tracks() (model/visualize_radar_targets.py:124-166): returns
    ({id: [(scan, R, D, Q), ...]}, [active per scan])."""
    tracks, counts, scan = {}, [], 0
    for line in Path(path).read_text().splitlines():
        p = line.split()
        if not p:
            continue
        if p[0] == "TRK":
            q = next((int(x.split("=")[1]) for x in p[4:] if x.startswith("Q=")), 0)
            tracks.setdefault(int(p[1]), []).append(
                (scan, int(p[2].split("=")[1]), int(p[3].split("=")[1]), q))
        elif p[0] == "SCAN_END":
            counts.append(int(p[1].split("=")[1]))
            scan += 1
    return tracks, counts
