"""File adapters: the text formats the reference's visualizer parses.

The visualizer itself may not be imported (recorded denial); its parse rules
are restated in fmcw.formats (read_detections = load_detections, visualize_radar_targets.py:
109-122: exactly 3 integer tokens; read_tracks = load_tracks, :124-168) and checked here on
files the writers produce.  The CLI end-to-end runs are GPU tests (test_gpu_r02.py)."""
import numpy as np

from fmcw import formats
from fmcw.radar_core import DET_DTYPE, adc_words_to_cube, pack_adc_words


def _dets():
    d = np.zeros(5, DET_DTYPE)
    d["frame"] = [0, 0, 1, 1, 1]
    d["range"] = [3, 100, 7, 500, 1023]
    d["doppler"] = [0, 5, 127, 118, 64]
    d["mag"] = [10.4, 99999.6, 1.5, 2.5, 0.0]
    d["threshold"] = 1.0
    return d


def test_detection_lines_parse_like_the_visualizer(tmp_path):
    p = tmp_path / "ADR_detections.txt"
    n = formats.write_detections(p, _dets())
    assert n == 5
    lines = p.read_text().splitlines()
    assert all(len(line.split()) == 3 for line in lines)          # :118 accepts 3 tokens only
    got = formats.read_detections(p)
    # magnitudes are written as integers (round half to even, the rint of np)
    np.testing.assert_array_equal(got, [[3, 0, 10], [100, 5, 100000], [7, 127, 2], [500, 118, 2],
                                        [1023, 64, 0]])
    one = tmp_path / "f1.txt"
    assert formats.write_detections(one, _dets(), frame=1) == 3


def test_doppler_centred_writer(tmp_path):
    """visualize_radar_targets.py:174-182 centres zero Doppler at N/2: the centred writer puts
    natural bin d at (d + N/2) mod N, so bin 0 -> 64 (0 m/s) and 118 (= -10) -> 54."""
    p = tmp_path / "ADR_detections.txt"
    formats.write_detections(p, _dets(), doppler_centred=True, n_doppler=128)
    got = formats.read_detections(p)
    np.testing.assert_array_equal(got[:, 1], [64, 69, 63, 54, 0])
    assert np.all(got[:, 1] - 64 == ((_dets()["doppler"].astype(int) + 64) % 128) - 64)


def test_rd_map_roundtrip_and_centring(tmp_path):
    rng = np.random.default_rng(2)
    m = rng.uniform(0, 5000, (16, 8)).astype(np.float32)
    p = tmp_path / "radar_output.txt"
    formats.write_rd_map(p, m)
    rows = np.loadtxt(p, dtype=np.int64)
    assert rows.shape == (128, 5) and np.all(rows[:, 2:4] == 0)       # "r d 0 0 mag"
    assert np.array_equal(rows[:8, 0], np.zeros(8)) and np.array_equal(rows[:8, 1], np.arange(8))
    np.testing.assert_array_equal(formats.read_rd_map(p, 16, 8), np.rint(m).astype(np.int64))
    formats.write_rd_map(p, m, doppler_centred=True)
    np.testing.assert_array_equal(formats.read_rd_map(p, 16, 8), np.fft.fftshift(np.rint(m).astype(np.int64), -1))


def test_tracks_format(tmp_path):
    from fmcw.tracker import TRACK_DTYPE
    t = np.zeros(2, TRACK_DTYPE)
    t["id"] = [1, 4]
    t["range_q2"] = [400, -8]
    t["doppler_q2"] = [20, 3]
    t["quality"] = [3, 15]
    p = tmp_path / "ADR_tracks.txt"
    formats.write_tracks(p, [(t, 2), (t[:0], 0)])
    tracks, counts = formats.read_tracks(p)
    assert counts == [2, 0]
    assert tracks[1] == [(0, 400, 20, 3)] and tracks[4] == [(0, -8, 3, 15)]


def test_adc_text_and_axi_words(tmp_path):
    rng = np.random.default_rng(0)
    iq = rng.integers(-32768, 32768, (300, 2))
    p = tmp_path / "adc.txt"
    formats.write_adc_pairs(p, iq)
    np.testing.assert_array_equal(formats.read_adc_pairs(p), iq)
    # the AXI word {Q[31:16], I[15:0]} (tb_radar_core.vhd:115-118) round trip through a .bin
    words = pack_adc_words(iq[:256, 0], iq[:256, 1])
    b = tmp_path / "adc.bin"
    words.astype("<u4").tofile(b)
    cube = adc_words_to_cube(np.fromfile(b, "<u4"), 16, 16)
    np.testing.assert_array_equal(cube.reshape(-1, 2), iq[:256])
    assert (int(words[0]) & 0xFFFF) == (int(iq[0, 0]) & 0xFFFF)
