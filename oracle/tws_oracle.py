"""CPU oracle of the track-while-scan tracker -- TEST INFRASTRUCTURE ONLY.

Restates rtl/src/tws_tracker.vhd (states COLLECT -> PREDICT -> ASSOCIATE/UPDATE per track ->
INITIATE -> MAINTAIN -> OUTPUT, :129-298) one scan per call, as the checker of the library's
host-side tracker (fmcw_tws_*, csrc/tws_tracker.cpp).  Only tests/ may import it.

Two modes:

rtl=True   literal RTL semantics, including what the VHDL does rather than what it says:
  - field widths wrap: range_pos signed 12, dopp_pos signed 9, range_vel signed 10, dopp_vel
    signed 8 (:49-53); hit/miss/quality 4-bit, age 8-bit; det range 10 / Doppler 7 /
    magnitude 17 bits (:25-27); the 6-bit det counter wraps at 64 (:132, :137);
  - numeric_std RESIZE of a signed value keeps the sign bit and the low n-1 bits (:190-197);
  - ASSOCIATE reads `best_distance` as a SIGNAL (:160-177): every comparison in the loop sees
    the value left by the previous active track's association (all ones at power-up, never
    reset), and the LAST qualifying detection wins, not the nearest;
  - the measured position is signed in UPDATE/INITIATE (:185-186, :241-244) but unsigned in
    ASSOCIATE's distance (:165-168).
rtl=False  the intended semantics (the build's default): unbounded integers, the first max_dets
  detections of a scan, nearest-neighbour association (smallest |dr| + |dd| inside the gate,
  lowest index on ties).  Everything else -- the Q2 fixed point, Q8 gains with floor shifts,
  the INIT_HITS / COAST_MAX / quality rules read on the pre-update values -- is the RTL's.
"""
from __future__ import annotations

from dataclasses import dataclass, field

FREE, TENTATIVE, FIRM, COAST = 0, 1, 2, 3
STATUS_NAMES = {FREE: "FREE", TENTATIVE: "TENT", FIRM: "FIRM", COAST: "COAST"}


def wrap(x: int, n: int) -> int:
    """n-bit two's complement wrap (signed + / - / shift_left, numeric_std)."""
    m = 1 << n
    x &= m - 1
    return x - m if x >= m >> 1 else x


def resize_s(x: int, n: int) -> int:
    """numeric_std RESIZE(signed, n) when shrinking: sign bit + the low n-1 bits."""
    low = x & ((1 << (n - 1)) - 1)
    return low - (1 << (n - 1)) if x < 0 else low


@dataclass
class TwsParams:
    """tws_tracker generics (:11-19); radar_core instantiates the defaults (:424-432)."""
    max_tracks: int = 32
    max_dets: int = 64
    init_hits: int = 2
    coast_max: int = 5
    gate_r: int = 10
    gate_d: int = 5
    alpha_q8: int = 128
    beta_q8: int = 64
    rtl: bool = False


@dataclass
class Track:
    active: bool = False
    status: int = FREE
    range_pos: int = 0
    dopp_pos: int = 0
    range_vel: int = 0
    dopp_vel: int = 0
    hit: int = 0
    miss: int = 0
    quality: int = 0
    age: int = 0
    last_mag: int = 0


@dataclass
class TwsOracle:
    p: TwsParams = field(default_factory=TwsParams)

    def __post_init__(self):
        self.tracks = [Track() for _ in range(self.p.max_tracks)]
        self.best_distance = 0xFFFF   # power-up value, not reset by aresetn (:92-93)
        self.best_idx = 63

    # width helpers: identity in the intended mode
    def _w(self, x, n):
        return wrap(x, n) if self.p.rtl else x

    def _rs(self, x, n):
        return resize_s(x, n) if self.p.rtl else x

    def _u(self, x, n):
        return x & ((1 << n) - 1) if self.p.rtl else x

    def scan(self, dets):
        """dets: iterable of (range_bin, doppler_bin, magnitude).  Returns (tracks reported
        by OUTPUT as dicts, active count after MAINTAIN)."""
        p = self.p
        # ST_COLLECT (:130-141)
        buf = []
        if p.rtl:
            slots = [None] * 64
            cnt = 0
            for r, d, m in dets:
                if cnt < p.max_dets:          # the 6-bit counter: < 64 always holds at 64
                    slots[cnt] = [self._u(int(r), 10), self._u(int(d), 7), self._u(int(m), 17), False]
                    cnt = (cnt + 1) & 63
            buf = slots
            det_count = cnt
        else:
            for r, d, m in list(dets)[:p.max_dets]:
                buf.append([int(r), int(d), int(m), False])
            det_count = len(buf)
        # ST_PREDICT (:143-156)
        for t in self.tracks:
            if t.active:
                t.range_pos = self._w(t.range_pos + t.range_vel, 12)
                t.dopp_pos = self._w(t.dopp_pos + t.dopp_vel, 9)
                t.age = self._u(t.age + 1, 8)
        # ST_ASSOCIATE / ST_UPDATE per track (:158-232)
        for t in self.tracks:
            if t.active:
                if p.rtl:
                    b_old = self.best_distance
                    best_d, best_i = 0xFFFF, 63
                    for i, e in enumerate(buf):
                        if e is None or e[3]:
                            continue
                        dr = abs(t.range_pos - ((e[0] << 2) & 0xFFF))
                        dd = abs(t.dopp_pos - ((e[1] << 2) & 0x1FF))
                        if dr < p.gate_r * 4 and dd < p.gate_d * 4:
                            dist = (dr + dd) & 0xFFFF
                            if dist < b_old:
                                best_d, best_i = dist, i
                    self.best_distance, self.best_idx = best_d, best_i
                    hit = best_i < p.max_dets and best_d < 0xFFFF
                else:
                    best_d, best_i = None, -1
                    for i, e in enumerate(buf):
                        if e[3]:
                            continue
                        dr = abs(t.range_pos - 4 * e[0])
                        dd = abs(t.dopp_pos - 4 * e[1])
                        if dr < p.gate_r * 4 and dd < p.gate_d * 4 and (best_d is None or dr + dd < best_d):
                            best_d, best_i = dr + dd, i
                    hit = best_d is not None
                if hit:
                    e = buf[best_i]
                    e[3] = True
                    meas_r = self._w(4 * e[0], 12)
                    meas_d = self._w(4 * e[1], 9)
                    ir = self._w(meas_r - t.range_pos, 12)
                    idd = self._w(meas_d - t.dopp_pos, 9)
                    old_hit, old_status = t.hit, t.status
                    t.range_pos = self._w(t.range_pos + self._rs((ir * p.alpha_q8) >> 8, 12), 12)
                    t.dopp_pos = self._w(t.dopp_pos + self._rs((idd * p.alpha_q8) >> 8, 9), 9)
                    t.range_vel = self._w(t.range_vel + self._rs((ir * p.beta_q8) >> 8, 10), 10)
                    t.dopp_vel = self._w(t.dopp_vel + self._rs((idd * p.beta_q8) >> 8, 8), 8)
                    t.hit = self._u(old_hit + 1, 4)
                    t.miss = 0
                    t.last_mag = e[2]
                    if old_status == TENTATIVE and old_hit >= p.init_hits:
                        t.status = FIRM
                    elif old_status == COAST:
                        t.status = FIRM
                    if t.quality < 15:
                        t.quality += 1
                else:
                    old_miss = t.miss
                    t.miss = self._u(old_miss + 1, 4)
                    if t.status == FIRM:
                        t.status = COAST
                    if old_miss >= p.coast_max:
                        t.active = False
                        t.status = FREE
                    if t.quality > 0:
                        t.quality -= 1
        # ST_INITIATE (:234-263): detection indices 0 .. det_count-1
        # (RTL: the state is entered at index 0 even when the 6-bit counter reads 0, :259)
        for i in (range(det_count) if det_count or not p.rtl else [0]):
            e = buf[i]
            if e is None or e[3]:
                continue
            free = next((k for k, t in enumerate(self.tracks) if not t.active), -1)
            if free >= 0:
                self.tracks[free] = Track(active=True, status=TENTATIVE,
                                          range_pos=self._w(4 * e[0], 12), dopp_pos=self._w(4 * e[1], 9),
                                          hit=1, quality=1, last_mag=e[2])
        # ST_MAINTAIN / ST_OUTPUT (:265-295)
        active = sum(t.active for t in self.tracks)
        out = []
        for k, t in enumerate(self.tracks):
            if t.active and t.status in (FIRM, COAST):
                out.append(dict(id=k, status=t.status, quality=t.quality, range_q2=t.range_pos,
                                doppler_q2=t.dopp_pos, vel_r=t.range_vel, vel_d=t.dopp_vel,
                                last_mag=t.last_mag, age=t.age))
        return out, active


def tb_tws_scenario():
    """Detections of rtl/src/tb_tws_tracker.vhd:113-142, one list per scan (12 scans):
    target 1 R = 200 - 5 (scan-1) D 40; target 2 R 600 D 80; target 3 R = 400 + 3 (scan-4)
    D 60 in scans 4-7; a false alarm (900, 10) every third scan."""
    scans = []
    for scan in range(1, 13):
        d = []
        t1 = 200 - (scan - 1) * 5
        if t1 > 0:
            d.append((t1, 40, 5000))
        d.append((600, 80, 8000))
        if 4 <= scan <= 7:
            d.append((400 + (scan - 4) * 3, 60, 3000))
        if scan % 3 == 0:
            d.append((900, 10, 2000))
        scans.append(d)
    return scans
