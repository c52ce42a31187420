"""Host-side models of the HIP kernels' algorithms, checked against the oracle on CPU.

These pin the *reformulations* the kernels rely on, independent of any GPU:
  * the Stockham pass plan and padded LDS addressing of fft_device.hpp,
  * the counting form of OS-CFAR (no sort) used by k_doppler / k_cfar1d / k_cfar2d,
  * the order-preserving float keys + radix select used for the ranked threshold,
  * the tiled corner-turn layout inter[rb][cb][RB][T].
"""
import numpy as np
import pytest

import fmcw_oracle as O


def pad16(i):
    return i + (i >> 4)


def plan(n, first):
    out, L = [], first
    while L < n:
        rem = n // L
        r = 16 if rem >= 16 else rem
        out.append((r, L))
        L *= r
    return out


def stockham_model(x, k1_style):
    """fft_device.hpp: pass 0 radix-8 from registers (K1) or all passes from LDS (K2)."""
    n = len(x)
    p = n // 16
    buf = np.zeros(pad16(n) + 8, complex)
    if k1_style:
        for t in range(p):
            for e in range(2):
                j = 2 * t + e
                v = np.fft.fft(np.array([x[j + (n // 8) * m] for m in range(8)]))
                for m in range(8):
                    buf[pad16(j * 8 + m)] = v[m]
        passes = plan(n, 8)
    else:
        for i in range(n):
            buf[pad16(i)] = x[i]
        passes = plan(n, 1)
    for (r, L) in passes:
        vals = {}
        for t in range(p):
            for g in range(16 // r):
                j = t + p * g
                vals[j] = np.array([buf[pad16(j + m * (n // r))] for m in range(r)])
        for j, v in vals.items():
            k = j % L
            tw = np.exp(-2j * np.pi * np.arange(r) * k / (L * r))
            V = np.fft.fft(v * tw)
            base = (j // L) * L * r + k
            for m in range(r):
                buf[pad16(base + m * L)] = V[m]
    return np.array([buf[pad16(i)] for i in range(n)])


@pytest.mark.parametrize("n", [32, 64, 128, 256, 512, 1024, 2048, 4096, 8192])
def test_stockham_plan(n):
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    ref = np.fft.fft(x)
    if n >= 64:
        assert np.abs(stockham_model(x, True) - ref).max() < 1e-9 * np.abs(ref).max()
    assert np.abs(stockham_model(x, False) - ref).max() < 1e-9 * np.abs(ref).max()


def test_padded_offsets_affine():
    """Every LDS access of every plan satisfies pad16(x + m*S) == pad16(x) + padoff(m*S)."""
    def padoff(o):
        return o + o // 16
    for n in [32, 64, 128, 256, 512, 1024, 2048, 4096, 8192]:
        p = n // 16
        for first in ((8, 1) if n >= 64 else (1,)):
            for (r, L) in plan(n, first):
                s = n // r
                for t in range(p):
                    for g in range(16 // r):
                        j = t + p * g
                        base = (j // L) * L * r + j % L
                        for m in range(r):
                            assert pad16(j + m * s) == pad16(j) + padoff(m * s)
                            assert pad16(base + m * L) == pad16(base) + padoff(m * L)


def cfar1d_counting(mag, p):
    m = np.asarray(mag, np.float32)
    offs = [-(p.guard + 1 + i) for i in range(p.ref)] + [p.guard + 1 + i for i in range(p.ref)]
    cnt = np.zeros(m.shape, np.int64)
    for o in offs:
        cnt += (np.float32(p.alpha) * np.roll(m, -o, axis=-1)) >= m
    return cnt < (2 * p.ref - p.rank)


@pytest.mark.parametrize("seed", range(4))
def test_cfar1d_counting_equals_sort(seed):
    rng = np.random.default_rng(seed)
    mag = rng.rayleigh(1.0, (64, 256)).astype(np.float32)
    mag[10, 40] = 50.0
    mag[20, ::7] = 9.0                          # ties and near-threshold structure
    mag[30] = np.float32(2.5)                   # a constant row: all ties
    p = O.Cfar1D()
    det_sort, _ = O.cfar_os1d(mag, p)
    np.testing.assert_array_equal(cfar1d_counting(mag, p), det_sort)
    assert det_sort[10, 40]


def cfar2d_counting(mag, p):
    """k_cfar2d's decision procedure, vectorised: phase A (s_min), then mean / bracket /
    final counts; returns (det, ranked-threshold for detections)."""
    m = np.asarray(mag, np.float32)
    nr, nd = m.shape
    hr = p.ref_range + p.guard_range
    rows = np.arange(hr, nr - hr)
    offs = O.cfar2d_offsets(p)
    refs = np.stack([np.roll(m[rows + dr], -dd, axis=-1) for dr, dd in offs])
    cut = m[rows]
    n, k = len(offs), p.rank
    need = n - k
    s_min = np.float32(p.scale_override or min(p.scale_min, p.scale_nom, p.scale_max))
    surv = ((s_min * refs) >= cut).sum(0) < need
    mean = (O.tree_sum_f32(refs) / np.float32(n)).astype(np.float32)
    if p.scale_override:
        sc = np.full(cut.shape, np.float32(p.scale_override))
    else:
        half = (mean * np.float32(0.5)).astype(np.float32)
        hi = (mean + half).astype(np.float32)
        n_hi = (refs > hi).sum(0)
        n_lo = (refs < half).sum(0)
        sc = np.where(n_hi >= need, np.float32(p.scale_max),
                      np.where(n_lo >= k + 1, np.float32(p.scale_min), np.float32(p.scale_nom)))
    det_rows = surv & (((sc.astype(np.float32) * refs) >= cut).sum(0) < need)
    det = np.zeros((nr, nd), bool)
    det[rows] = det_rows
    return det


@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("override", [0, 3])
def test_cfar2d_counting_equals_sort(seed, override):
    rng = np.random.default_rng(100 + seed)
    mag = rng.rayleigh(1.0, (48, 128)).astype(np.float32)
    mag[20, 30] = 40.0
    mag[21, 30:34] = 12.0
    mag[5:9, 60:70] = rng.rayleigh(8.0, (4, 10))   # clutter patch -> scale_max bracket
    mag[30:40, 100:110] = 0.01                       # quiet patch -> scale_min bracket
    p = O.Cfar2D(scale_override=override)
    det_sort, _ = O.cfar_os2d(mag, p)
    np.testing.assert_array_equal(cfar2d_counting(mag, p), det_sort)
    assert det_sort[20, 30]


def f2key(f):
    u = np.asarray(f, np.float32).view(np.uint32).astype(np.uint64)
    return np.where(u & 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000).astype(np.uint32)


def test_radix_select_keys():
    rng = np.random.default_rng(7)
    for _ in range(50):
        v = (rng.standard_normal(128) * rng.choice([1e-3, 1, 1e6])).astype(np.float32)
        v[:5] = [0.0, -0.0, 1.0, 1.0, -1.0]
        keys = f2key(v)
        k = int(rng.integers(0, 128))
        prefix, kk = 0, k                      # k_cfar2d's 32-step radix select
        for bit in range(31, -1, -1):
            hmask = 0 if bit == 31 else (~((2 << bit) - 1)) & 0xFFFFFFFF
            z = ((keys & hmask) == prefix) & (((keys >> bit) & 1) == 0)
            c0 = int(z.sum())
            if kk >= c0:
                kk -= c0
                prefix |= 1 << bit
        u = np.uint32(prefix)
        back = np.array([(u & 0x7FFFFFFF) if (u & 0x80000000) else (~u) & 0xFFFFFFFF],
                        np.uint32).view(np.float32)[0]
        assert back == np.sort(v)[k] or (back == 0 and np.sort(v)[k] == 0)


@pytest.mark.parametrize("ns,nc,T", [(1024, 256, 8), (256, 128, 16), (4096, 512, 2), (64, 64, 32)])
def test_tiled_corner_turn_layout(ns, nc, T):
    """inter[rb][cb][RB][T] with RB = 128/T holds exactly the transposed spectrum."""
    rb_ = 128 // T
    spec = np.arange(nc * ns).reshape(nc, ns)          # [chirp][range]
    inter = np.empty(ns * nc, np.int64)
    ncb = nc // T
    for c in range(nc):
        for r in range(ns):
            off = ((r // rb_ * ncb + c // T) * rb_ + r % rb_) * T + c % T
            inter[off] = spec[c, r]
    assert len(np.unique(inter)) == ns * nc
    # un-blocking recovers the corner turner's [range][chirp]
    out = np.empty((ns, nc), np.int64)
    for r in range(ns):
        for c in range(nc):
            out[r, c] = inter[((r // rb_ * ncb + c // T) * rb_ + r % rb_) * T + c % T]
    np.testing.assert_array_equal(out, spec.T)


def cfar1d_screened(mag, p):
    """k_doppler's 1-D decision with its screen: a cell whose groups of 4 consecutive refs give
    4 * #{groups with fl(alpha * min4) >= cut} >= need cannot detect and is never counted; the
    rest use the exact count.  Returns (detections, screen survivors)."""
    m = np.asarray(mag, np.float32)
    a = np.float32(p.alpha)
    g = np.minimum(np.minimum(m, np.roll(m, -1, -1)), np.minimum(np.roll(m, -2, -1), np.roll(m, -3, -1)))
    starts = [-(p.guard + p.ref) + 4 * q for q in range(p.ref // 4)] + \
             [p.guard + 1 + 4 * q for q in range(p.ref // 4)]
    ng = sum(((a * np.roll(g, -s, -1)) >= m).astype(np.int64) for s in starts)
    surv = 4 * ng < (2 * p.ref - p.rank)
    return surv & cfar1d_counting(m, p), surv


@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("rank", [12, 10, 14])
def test_cfar1d_screen_is_exact(seed, rank):
    """The groups-of-4 screen never clears a detecting cell (decisions equal the sort)."""
    rng = np.random.default_rng(50 + seed)
    mag = rng.rayleigh(1.0, (64, 256)).astype(np.float32)
    mag[10, 40] = 50.0
    mag[20, ::7] = 9.0
    mag[30] = np.float32(2.5)
    p = O.Cfar1D(rank=rank)
    det_sort, _ = O.cfar_os1d(mag, p)
    det, surv = cfar1d_screened(mag, p)
    np.testing.assert_array_equal(det, det_sort)
    assert det_sort[10, 40]
    if rank == 12:
        assert surv.mean() < 0.05      # the screen clears almost every noise cell
