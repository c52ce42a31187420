// cfar2d.hpp -- K3: 2-D OS-CFAR (rtl/src/os_cfar_2d.vhd:140-217) over the linear magnitude
// map, for gfx950.  Included from inside namespace fmcw by kernels.hpp (uses DetSink,
// det_reserve_wave, wave_excl_scan, lt_bit, opaque, the magnitude-row format midx / moff /
// mrow_floats / load_cells and DopplerGeom declared there).
//
// Tiles.  The detection unit is K2's wave tile: WR = 1024/NC range rows x NC Doppler cells
// (16 cells per lane), so the 1-D and 2-D CFAR share one sink layout and one (frame, range,
// doppler) order.  A workgroup (4 waves) takes 4 consecutive wave tiles of one frame and
// stages their rows plus +-hr halo rows in LDS once, in the magnitude-row format (16-cell
// circular Doppler halos, 4 pad floats per 16 cells).  After that the waves run on their own.
// Doppler is circular; a CUT row is tested only if its whole range extent lies inside the map
// (build spec).
//
// Phase A (every cell, one lane per 16 consecutive cells): for each of the 2 hr + 1 window
// rows the lane reads that row's 16 + 2 hd span once (16-B LDS reads), scales it by s_min,
// and counts for each of its 16 CUTs the refs with fl(s_min * ref) < cut (guard rows skip
// |dd| <= gd).  #{fl(s_min * ref) >= cut} >= n_ref - k proves cut <= fl(s * ranked) for
// every admissible scale s >= s_min, so such a cell cannot detect; the others are candidates.
// Phase B (candidates, one whole wave per cell, in cell order): lanes hold refs l and l + 64
// (fixed order: dr outer, dd inner); the mean is the fixed fp32 halving tree (one add, then
// xor-shuffles 32..1 == oracle tree_sum_f32); the scale bracket comes from ballot counts
// (ranked > M <=> #{ref > M} >= n_ref - k; ranked < M' <=> #{ref < M'} >= k + 1); detect <=>
// #{fl(s * ref) >= cut} < n_ref - k.  Pass 1 decides and counts, the wave reserves its sink
// range, pass 2 walks its detections again and finds the exact ranked value by a 32-step radix
// select over order-preserving keys (threshold = fl(s * ranked), dbg_threshold).  No per-cell
// list is kept, so LDS holds only the rows.
#pragma once

struct Cfar2DArgs {
  int hr, gr, hd, gd;  // half extents (ref + guard) and guards, range / Doppler
  int n_ref, rank;
  float s_min, sc_min, sc_nom, sc_max;
  int override_;
  int compat;          // FMCW_COMPAT_CFAR: 17-bit integer cells, integer mean and brackets
};

template <int NC> struct Cfar2DGeom {
  static constexpr int NT = 256;
  static constexpr int WPB = 4;                   // wave tiles per workgroup tile
  static constexpr int WR = DopplerGeom<NC>::WR;  // CUT rows per wave tile
  static constexpr int TR = WPB * WR;             // CUT rows per workgroup tile
  static constexpr int RS = mrow_floats<NC>();    // LDS row stride (floats)
  static constexpr int TPR = NC / 16;             // lanes per row
};

// The staged rows of one step: a ring of nr = TR + 2 hr rows of rs floats.  Tile row x (0 = the
// first halo row of the current step) lives in slot (x + base) mod nr, so a strip of steps
// keeps the 2 hr rows it shares with the next step and loads only TR new ones.
struct RowRing {
  float* tile;
  int base, nr, rs;
  __device__ __forceinline__ int slot(int x) const {
    const int y = x + base;
    return y >= nr ? y - nr : y;
  }
  __device__ __forceinline__ float* row(int x) const { return tile + slot(x) * rs; }
};

__device__ __forceinline__ uint32_t f2key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

#ifndef FMCW_CFAR2D_SCREEN  // phase A: packed 16-bit pair screen (2), fp32 pair screen (1), exact (0);
#define FMCW_CFAR2D_SCREEN 2  // the screens are followed by the exact count of their survivors
#endif
#ifndef FMCW_CFAR2D_PREFETCH  // load a strip's next rows during the current step (1)
#define FMCW_CFAR2D_PREFETCH 1
#endif
constexpr int kCfar2dList = 2 * 256 + 16;  // u32 after the rows: round list, verdicts / positions, counts

template <int NC>
constexpr size_t cfar2d_smem_bytes(int hr) {
  using G = Cfar2DGeom<NC>;
  return (size_t)(G::TR + 2 * hr) * G::RS * 4 + kCfar2dList * 4;
}

// Phase A screen (compile-time HD / GD): disjoint PAIRS of Doppler-adjacent references.  A pair
// with fl(s_min * min) >= cut holds 2 references with fl(s_min * ref) >= cut (fl(s x) is
// monotone), so 2 * #{such pairs} is a lower bound on the exact count and a cell whose bound
// reaches n_ref - k cannot detect.  A reference row of 2 HD + 1 cells gives HD pairs (its last
// cell is left out), a guard row two segments of HD - GD cells, (HD - GD) / 2 pairs each.
// On noise + targets about 5 % of the cells pass (0.6 % pass the exact count) at half the
// compares; the survivors are then counted exactly, one per lane.
template <int NC, int HD, int GD>
__device__ __forceinline__ uint32_t cfar2d_screen(const RowRing& rr, int rl, int d0, const Cfar2DArgs& a,
                                                  int need) {
  static_assert(HD <= MH, "the window stays inside the row halos");
  constexpr int W = 16 + 2 * HD;
  constexpr int O0 = floor4(-HD);
  constexpr int NV = (W + (-HD - O0) + 3) / 4;
  constexpr int SEG = HD - GD, NPS = SEG / 2;   // guard-row segment length, pairs per segment
  const float* lb = rr.row(rl + a.hr) + midx(d0);
  uint32_t cb[16], nlt[16];  // cut bits; #{pairs with fl(s_min * min) < cut}
  {
    float c[16];
    load_cells<4>(lb, 0, c);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      cb[i] = __float_as_uint(c[i]);
      nlt[i] = 0;
    }
  }
  for (int dr = -a.hr; dr <= a.hr; ++dr) {
    float v[4 * NV];
    load_cells<NV>(rr.row(rl + a.hr + dr) + midx(d0), O0, v);
    uint32_t pm[W - 1];  // pm[k] = fl(s_min * min(cell k, cell k + 1)), cell 0 = d0 - HD
#pragma unroll
    for (int k = 0; k < W - 1; ++k)
      pm[k] = __float_as_uint(a.s_min * fminf(v[-HD - O0 + k], v[-HD - O0 + k + 1]));
    if (dr >= -a.gr && dr <= a.gr) {  // guard row (uniform branch)
#pragma unroll
      for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int j = 0; j < NPS; ++j)
          nlt[i] += lt_bit(pm[i + 2 * j], cb[i]) + lt_bit(pm[i + HD + GD + 1 + 2 * j], cb[i]);
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int j = 0; j < HD; ++j) nlt[i] += lt_bit(pm[i + 2 * j], cb[i]);
    }
  }
  const int n_guard = 2 * a.gr + 1;
  const int np = (2 * a.hr + 1 - n_guard) * HD + n_guard * 2 * NPS;  // pairs per cell
  uint32_t bits = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) bits |= (2 * (np - (int)nlt[i]) < need ? 1u : 0u) << i;
  return bits;
}

// Phase A screen on packed 16-bit keys, two CUTs per VALU op, over disjoint PAIRS of
// Doppler-adjacent references.  A pair whose MAX satisfies fl(s_min * max) >= cut holds at
// least one reference that does, so #{such pairs} is a lower bound on the exact count
// E(s_min) = #{fl(s_min * ref) >= cut}; a cell whose bound reaches n_ref - k cannot detect at
// any admissible scale.  (The max bound beats 2 * #{pairs whose min qualifies} exactly where it
// matters: for a reference exceeding the cut's level with probability p it rejects from
// p ~ 0.32 instead of p ~ 0.52; on single-channel Rayleigh maps 1.9 % of the cells survive it
// instead of 4.8 %.)  A reference row of 2 HD + 1 cells gives HD pairs (its last cell is left
// out), a guard row two segments of HD - GD cells, (HD - GD) / 2 pairs each.
// The key of a cell is the high half of its bit pattern (cells are non-negative: sign 0, 8
// exponent and 7 mantissa bits), monotone in the value, so max() commutes with it.  Each CUT
// gets the key of q = fl(cut / s_min) + 8 ulps (cut * fl(1 / s_min): <= 2 ulps of error), and
// a pair counts only if its max key is STRICTLY above that key: then max > q > cut / s_min in
// reals, so s_min * max > cut and fl(s_min * max) >= cut (the key's 2^-7 resolution only makes
// the screen a little weaker).  Per window row: 27 byte-perms build hi16 pairs, 26
// v_pk_max_u16 the packed pair maxima, and each (two CUTs, one pair) step is v_pk_sub_u16 +
// v_pk_lshrrev_b16 + v_pk_add_u16 (bit 15 of pairmax - (key + 1) is set iff pairmax <= key).
// The survivors are then counted exactly, one per lane.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

template <int NC, int HD, int GD>
__device__ __forceinline__ uint32_t cfar2d_screen16(const RowRing& rr, int rl, int d0, const Cfar2DArgs& a,
                                                    int need) {
  static_assert(HD <= MH, "the window stays inside the row halos");
  constexpr int W = 16 + 2 * HD;
  constexpr int O0 = floor4(-HD);
  constexpr int NV = (W + (-HD - O0) + 3) / 4;
  constexpr int SEG = HD - GD, NPS = SEG / 2;
  const float* lb = rr.row(rl + a.hr) + midx(d0);
  const float inv_s = 1.0f / a.s_min;
  u16x2 ck[8], nlt[8];  // (key + 1) of CUTs 2p, 2p + 1; #{pairs not counted}
  {
    float c[16];
    load_cells<4>(lb, 0, c);
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const uint32_t k0 = min((__float_as_uint(c[2 * p] * inv_s) + 8u) >> 16, 0x7fffu) + 1u;
      const uint32_t k1 = min((__float_as_uint(c[2 * p + 1] * inv_s) + 8u) >> 16, 0x7fffu) + 1u;
      ck[p] = __builtin_bit_cast(u16x2, k0 | (k1 << 16));
      nlt[p] = (u16x2)(0);
    }
  }
  for (int dr = -a.hr; dr <= a.hr; ++dr) {
    float v[4 * NV];
    load_cells<NV>(rr.row(rl + a.hr + dr) + midx(d0), O0, v);
    u16x2 P[W - 2];  // P[k] = (pairmax key k, pairmax key k + 1), cell 0 = d0 - HD
    {
      uint32_t V[W - 1];  // V[k] = (key of cell k, key of cell k + 1)
#pragma unroll
      for (int k = 0; k < W - 1; ++k)
        V[k] = __builtin_amdgcn_perm(__float_as_uint(v[-HD - O0 + k + 1]), __float_as_uint(v[-HD - O0 + k]),
                                     0x07060302u);
#pragma unroll
      for (int k = 0; k < W - 2; ++k)
        P[k] = __builtin_elementwise_max(__builtin_bit_cast(u16x2, V[k]), __builtin_bit_cast(u16x2, V[k + 1]));
    }
    if (dr >= -a.gr && dr <= a.gr) {  // guard row (uniform branch)
#pragma unroll
      for (int p = 0; p < 8; ++p)
#pragma unroll
        for (int j = 0; j < NPS; ++j) {
          nlt[p] += (u16x2)(P[2 * p + 2 * j] - ck[p]) >> (unsigned short)15;
          nlt[p] += (u16x2)(P[2 * p + HD + GD + 1 + 2 * j] - ck[p]) >> (unsigned short)15;
        }
    } else {
#pragma unroll
      for (int p = 0; p < 8; ++p)
#pragma unroll
        for (int j = 0; j < HD; ++j) nlt[p] += (u16x2)(P[2 * p + 2 * j] - ck[p]) >> (unsigned short)15;
    }
  }
  const int n_guard = 2 * a.gr + 1;
  const int np = (2 * a.hr + 1 - n_guard) * HD + n_guard * 2 * NPS;  // pairs per cell
  uint32_t bits = 0;
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    bits |= (np - (int)nlt[p].x < need ? 1u : 0u) << (2 * p);
    bits |= (np - (int)nlt[p].y < need ? 1u : 0u) << (2 * p + 1);
  }
  return bits;
}

// Candidate test of one screen survivor (CUT row rl of the group tile, Doppler d), one lane per
// cell; it keeps every cell that can detect.  With E(s) = #{fl(s * ref) >= cut}, the cell can
// only detect if E(s) < need for the scale s it gets.  E(s_min) >= need rules every scale out.
// The scale is sc_min only when #{ref < mean / 2} >= rank + 1 (os_cfar_2d.vhd:195-199);
// otherwise it is >= s2 = min(sc_nom, sc_max) and E(s2) >= need rules the cell out too.
// E(s_min) and E(s2) are bounded from below with the screen's 16-bit keys, both in one packed
// op per reference (a reference counts if its key is strictly above key(cut / s) + 8 ulps), and
// #{ref < mean / 2} from above with an any-order fp32 sum x (1 + 2^-15) (the sum of <= 128
// non-negative terms in another order differs by < 2^-16 relative; compat's integer sums are
// exact).  On single-channel (Rayleigh) maps this leaves ~0.3 % of the cells E(s_min) alone
// would pass.  Addresses: midx(d + dd) with a runtime d.
template <int NC, int HD, int GD>
__device__ __forceinline__ bool cfar2d_exact_a(const RowRing& rr, int rl, int d, const Cfar2DArgs& a, int need,
                                               int sub, int L) {
  const float* crow = rr.row(rl + a.hr);
  const int x = d + MH;
  auto at = [&](const float* row, int dd) { return row[(x + dd) + (((x + dd) >> 4) << 2)]; };
  const float cut = at(crow, 0);
  const float s2 = a.override_ ? a.s_min : fminf(a.sc_nom, a.sc_max);
  const uint32_t k1 = min((__float_as_uint(cut * (1.0f / a.s_min)) + 8u) >> 16, 0x7fffu) + 1u;
  const uint32_t k2 = min((__float_as_uint(cut * (1.0f / s2)) + 8u) >> 16, 0x7fffu) + 1u;
  const u16x2 kk = __builtin_bit_cast(u16x2, k1 | (k2 << 16));
  u16x2 nlt = (u16x2)(0);  // #{refs not counted} for (s_min, s2)
  float sum = 0.f;
  auto visit = [&](auto&& fn) {  // this lane's rows: dr = -hr + sub, every L-th
    for (int dr = -a.hr + sub; dr <= a.hr; dr += L) {
      const float* row = rr.row(rl + a.hr + dr);
      if (dr >= -a.gr && dr <= a.gr) {
#pragma unroll
        for (int dd = -HD; dd <= HD; ++dd)
          if (dd < -GD || dd > GD) fn(at(row, dd));
      } else {
#pragma unroll
        for (int dd = -HD; dd <= HD; ++dd) fn(at(row, dd));
      }
    }
  };
  visit([&](float v) {
    const uint32_t kv = __builtin_amdgcn_perm(__float_as_uint(v), __float_as_uint(v), 0x07060302u);
    nlt += (u16x2)(__builtin_bit_cast(u16x2, kv) - kk) >> (unsigned short)15;
    sum += v;
  });
  for (int x = 1; x < L; x <<= 1) {  // the cell's L lanes are adjacent and aligned
    nlt += __builtin_bit_cast(u16x2, __shfl_xor(__builtin_bit_cast(int, nlt), x, 64));
    sum += __shfl_xor(sum, x, 64);
  }
  if (a.n_ref - (int)nlt.x >= need) return false;                // E(s_min) >= need
  if (a.n_ref - (int)nlt.y < need || a.override_) return true;   // E(s2) may be < need
  const float half_up = sum * (1.0f + 1.0f / 32768.0f) / (float)a.n_ref * 0.5f;
  // >= need refs lie above cut / s2; if cut / s2 >= mean / 2 they all lie above the half, so
  // n_lo <= n_ref - need = rank < rank + 1 without counting (most noise survivors: their cut
  // is high).  (1 - 2^-20) covers the product's rounding.
  if (cut * (1.0f / s2) * (1.0f - 1.0f / 1048576.0f) >= half_up) return false;
  int n_lo = 0;
  visit([&](float v) { n_lo += v < half_up ? 1 : 0; });
  for (int x = 1; x < L; x <<= 1) n_lo += __shfl_xor(n_lo, x, 64);
  return n_lo >= a.rank + 1;                                     // sc_min still possible
}

// Phase A for a compile-time Doppler extent HD / guard GD; returns this lane's candidate bits.
// `rl` is the CUT row within the workgroup tile (tile row rl + hr).
template <int NC, int HD, int GD>
__device__ __forceinline__ uint32_t cfar2d_phase_a(const RowRing& rr, int rl, int d0, const Cfar2DArgs& a,
                                                   int need) {
  static_assert(HD <= MH, "the window stays inside the row halos");
  constexpr int W = 16 + 2 * HD;
  constexpr int O0 = floor4(-HD);
  constexpr int NV = (W + (-HD - O0) + 3) / 4;
  const float* lb = rr.row(rl + a.hr) + midx(d0);
  uint32_t cb[16], lt[16];   // cut bits; #{fl(s_min * ref) < cut} (lt_bit: no SGPR masks)
  {
    float c[16];
    load_cells<4>(lb, 0, c);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      cb[i] = __float_as_uint(c[i]);
      lt[i] = 0;
    }
  }
  for (int dr = -a.hr; dr <= a.hr; ++dr) {
    float v[4 * NV];
    load_cells<NV>(rr.row(rl + a.hr + dr) + midx(d0), O0, v);
    uint32_t sb[W];
#pragma unroll
    for (int k = 0; k < W; ++k) sb[k] = __float_as_uint(a.s_min * v[-HD - O0 + k]);
    if (dr >= -a.gr && dr <= a.gr) {  // guard row: skip |dd| <= GD (uniform branch)
#pragma unroll
      for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int dd = -HD; dd <= HD; ++dd)
          if (dd < -GD || dd > GD) lt[i] += lt_bit(sb[i + HD + dd], cb[i]);
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int dd = -HD; dd <= HD; ++dd) lt[i] += lt_bit(sb[i + HD + dd], cb[i]);
    }
  }
  // candidate <=> #{fl(s_min * ref) >= cut} < need  <=>  lt > n_ref - need
  uint32_t bits = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) bits |= ((int)lt[i] > a.n_ref - need ? 1u : 0u) << i;
  return bits;
}

// Phase A, runtime geometry (any window the LDS budget allows; Doppler wraps explicitly).
template <int NC>
__device__ __forceinline__ uint32_t cfar2d_phase_a_generic(const RowRing& rr, int rl, int d0,
                                                           const Cfar2DArgs& a, int need) {
  const float* crow = rr.row(rl + a.hr);
  uint32_t bits = 0;
  for (int i = 0; i < 16; ++i) {
    const int d = d0 + i;
    const uint32_t c = __float_as_uint(crow[midx(d)]);
    uint32_t lt = 0;
    for (int dr = -a.hr; dr <= a.hr; ++dr) {
      const float* row = rr.row(rl + a.hr + dr);
      const bool grow = dr >= -a.gr && dr <= a.gr;
      for (int dd = -a.hd; dd <= a.hd; ++dd) {
        if (grow && dd >= -a.gd && dd <= a.gd) continue;
        lt += lt_bit(__float_as_uint(a.s_min * row[midx((d + dd) & (NC - 1))]), c);
      }
    }
    bits |= ((int)lt > a.n_ref - need ? 1u : 0u) << i;
  }
  return bits;
}

// Reference j of the fixed order (dr ascending outer, dd ascending inner, guard block
// skipped; oracle cfar2d_offsets) -> (dr, dd).  Run once per lane per kernel.
__device__ __forceinline__ void cfar2d_ref_offset(const Cfar2DArgs& a, int j, int& dr, int& dd) {
  dr = 0;
  dd = 0;
  int n = 0;
  for (int r = -a.hr; r <= a.hr; ++r) {
    const bool grow = r >= -a.gr && r <= a.gr;
    const int side = a.hd - a.gd;
    const int cnt = grow ? 2 * side : 2 * a.hd + 1;
    if (j < n + cnt) {
      const int k = j - n;
      dr = r;
      dd = grow ? (k < side ? -a.hd + k : a.gd + 1 + (k - side)) : -a.hd + k;
      return;
    }
    n += cnt;
  }
}

// ---- Workgroup-cooperative rounds over a set of cells.  Each lane owns up to 16 cells (bits of
// `m`); the workgroup's cells, in (wave, lane, bit) order == tile order, are listed 256 per round
// in `list` as (wave << 10 | lane << 4 | bit) and handed to fn(n) between two barriers.  With
// `pos` the entry's running position pos0 + (its index among the lane's bits) goes alongside.
// Every wave of the workgroup must call this (barriers); `cnt` holds 4 words of its own.
constexpr int kCoopRound = 256;
template <class Fn>
__device__ __forceinline__ void coop_rounds(uint32_t m, uint32_t* cnt, uint32_t* list, uint32_t* pos,
                                            uint32_t pos0, Fn&& fn) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int n_w;
  const int ex = wave_excl_scan(__popc(m), n_w);
  if (lane == 0) cnt[wv] = (uint32_t)n_w;
  __syncthreads();
  int off = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = (int)cnt[i];
    off += i < wv ? c : 0;
    tot += c;
  }
  for (int b0 = 0; b0 < tot; b0 += kCoopRound) {  // uniform over the workgroup
    int o = off + ex, t = 0;
    for (uint32_t mm = m; mm; mm &= mm - 1, ++o, ++t)
      if (o >= b0 && o < b0 + kCoopRound) {
        list[o - b0] = ((uint32_t)wv << 10) | ((uint32_t)lane << 4) | (uint32_t)__builtin_ctz(mm);
        if (pos) pos[o - b0] = pos0 + (uint32_t)t;
      }
    __syncthreads();
    fn(min(kCoopRound, tot - b0));
    __syncthreads();  // the next round rewrites the list
  }
}

// k-th smallest (0-based) of the wave's keys ka (lanes in ma) and kb (lanes in mb), by
// pivoting: the pivot is the median of three active keys, ballots count the keys below and
// equal to it, and the active set shrinks to the side holding rank k.  Every step removes at
// least the pivot's equals, so it ends; on these windows it takes ~6-10 steps where a bitwise
// radix select takes 32.  Wave-uniform control flow; needs k < #active.
__device__ __forceinline__ uint32_t wave_select_kth(uint32_t ka, uint32_t kb, uint64_t ma, uint64_t mb, int k) {
  for (int it = 0; it < 256; ++it) {  // bound: >= 1 key leaves per step, 128 keys
    const uint64_t m1 = ma ? ma : mb;
    const uint32_t v1 = ma ? ka : kb;
    const uint32_t p1 = (uint32_t)__builtin_amdgcn_readlane((int)v1, __builtin_ctzll(m1));
    const uint32_t p2 = (uint32_t)__builtin_amdgcn_readlane((int)v1, 63 - __builtin_clzll(m1));
    const uint64_t m3 = mb ? mb : ma;
    const uint32_t v3 = mb ? kb : ka;
    const uint64_t m3r = m3 & (m3 - 1);  // second active lane when there is one
    const uint32_t p3 = (uint32_t)__builtin_amdgcn_readlane((int)v3, __builtin_ctzll(m3r ? m3r : m3));
    const uint32_t p = max(min(p1, p2), min(max(p1, p2), p3));
    const uint64_t la = __ballot(ka < p) & ma, ea = __ballot(ka == p) & ma;
    const uint64_t lb = __ballot(kb < p) & mb, eb = __ballot(kb == p) & mb;
    const int lt = __popcll(la) + __popcll(lb), eq = __popcll(ea) + __popcll(eb);
    if (k < lt) {
      ma = la;
      mb = lb;
    } else if (k < lt + eq) {
      return p;
    } else {
      k -= lt + eq;
      ma &= ~(la | ea);
      mb &= ~(lb | eb);
    }
  }
  return 0u;  // unreachable for k < #active
}

template <int NC, int HD, int GD>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3)))
k_cfar2d(const float* __restrict__ map, int ns, int n_strips, int steps, int frame0, int tile0, Cfar2DArgs a,
         DetSink sink) {
  using Gm = Cfar2DGeom<NC>;
  constexpr int WR = Gm::WR, NT = Gm::NT, RS = Gm::RS, TPR = Gm::TPR, WPB = Gm::WPB, TR = Gm::TR;
  static_assert(TR * NC == 4 * 4 * NT, "a step's new rows are 4 float4 per thread");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* const tile = smem;

  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // this lane's two reference cells (index lane and lane + 64 of the fixed order)
  int dra, dda, drb, ddb;
  cfar2d_ref_offset(a, lane, dra, dda);
  cfar2d_ref_offset(a, lane + 64, drb, ddb);
  const bool oka = lane < a.n_ref, okb = lane + 64 < a.n_ref;
  const int need = a.n_ref - a.rank;
  const int wt_per_frame = ns / WR;                      // wave tiles per frame
  const int wg_per_frame = (wt_per_frame + WPB - 1) / WPB;
  const int spf = (wg_per_frame + steps - 1) / steps;    // strips per frame
  const int nf = n_strips / spf;
  const int nr = TR + 2 * a.hr;                          // ring rows
  uint32_t* const list = reinterpret_cast<uint32_t*>(tile + nr * RS);
  uint32_t* const aux = list + kCoopRound;
  uint32_t* const cnt = aux + kCoopRound;
  const int tid = opaque(threadIdx.x);

  // one float4 of cells (row x, Doppler d..d+3) into the ring, with its circular-halo copy
  auto put4 = [&](const RowRing& rr, int x, int d, float4 v) {
    v = a.compat ? q17x4(v) : nonneg4(v);
    float* row = rr.row(x);
    *reinterpret_cast<float4*>(row + midx(d)) = v;
    if (d < MH) *reinterpret_cast<float4*>(row + midx(NC + d)) = v;
    if (d >= NC - MH) *reinterpret_cast<float4*>(row + midx(d - NC)) = v;
  };

  for (int g = blockIdx.x; g < n_strips; g += gridDim.x) {
    // a strip: `steps` consecutive workgroup tiles of one frame (frame-minor order, as K2:
    // hot rows spread over all workgroups); each step tests TR rows and loads only TR new ones
    const int f = g % nf;
    const int t_beg = (g / nf) * steps, t_end = min(t_beg + steps, wg_per_frame);
    const float* fm = map + (size_t)f * ns * NC;
    RowRing rr{tile, 0, nr, RS};
    float4 pre[4];
    for (int t = t_beg; t < t_end; ++t) {
      const int wt0 = t * WPB;                             // first wave tile of this step
      const int n_wt = min(WPB, wt_per_frame - wt0);
      const int r0 = wt0 * WR;                             // first CUT row of this step
      __syncthreads();  // the previous step's waves are done with the rows and the lists
      if (t == t_beg) {
        // rows r0-hr .. r0+TR+hr-1 (zero outside the map), 4 float4 loads in flight per lane
        const int n4 = nr * (NC / 4);
        for (int b = tid; b < n4; b += 4 * NT) {
          float4 v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int e4 = b + u * NT;
            const int x = e4 / (NC / 4), d = (e4 - x * (NC / 4)) * 4;
            const int r = r0 - a.hr + x;
            v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (e4 < n4 && r >= 0 && r < ns) v[u] = *reinterpret_cast<const float4*>(fm + (size_t)r * NC + d);
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int e4 = b + u * NT;
            const int x = e4 / (NC / 4), d = (e4 - x * (NC / 4)) * 4;
            if (e4 < n4) put4(rr, x, d, v[u]);
          }
        }
      } else {
        // the ring turns by TR rows; the TR new rows (prefetched during the previous step) go
        // into the slots of the TR rows that left
        rr.base += TR;
        if (rr.base >= nr) rr.base -= nr;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int e4 = tid + u * NT;
          const int i = e4 / (NC / 4), d = (e4 - i * (NC / 4)) * 4;
          if (!FMCW_CFAR2D_PREFETCH) {
            const int rn = r0 + a.hr + i;  // new row of this step (zero past the map)
            pre[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (rn < ns) pre[u] = *reinterpret_cast<const float4*>(fm + (size_t)rn * NC + d);
          }
          put4(rr, nr - TR + i, d, pre[u]);
        }
      }
      if (FMCW_CFAR2D_PREFETCH && t + 1 < t_end) {  // prefetch the next step's new rows r0 + TR + hr ..
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int e4 = tid + u * NT;
          const int i = e4 / (NC / 4), d = (e4 - i * (NC / 4)) * 4;
          const int r = r0 + TR + a.hr + i;
          pre[u] = make_float4(0.f, 0.f, 0.f, 0.f);
          if (r < ns) pre[u] = *reinterpret_cast<const float4*>(fm + (size_t)r * NC + d);
        }
      }
      __syncthreads();
      const bool has_tile = wv < n_wt;  // uniform per wave; waves without a tile still join the barriers

      // ---- Phase A: candidates among this lane's 16 cells
      const int rlw = wv * WR + lane / TPR;    // CUT row within the group tile
      const int d0 = (lane % TPR) * 16;
      const int r = r0 + rlw;
      uint32_t cand = 0;
      // cell of a round-list entry (wave << 10 | lane << 4 | bit) -> group-tile row, Doppler bin
      auto cell_of = [&](uint32_t e, int& trow, int& d) {
        const int we = (int)(e >> 10), le = (int)((e >> 4) & 63u);
        trow = we * WR + le / TPR;
        d = (le % TPR) * 16 + (int)(e & 15u);
      };
      const bool tested = has_tile && r >= a.hr && r < ns - a.hr;
      if (tested) {
        if constexpr (HD > 0) {
          if constexpr (FMCW_CFAR2D_SCREEN == 2) cand = cfar2d_screen16<NC, HD, GD>(rr, rlw, d0, a, need);
          else if constexpr (FMCW_CFAR2D_SCREEN) cand = cfar2d_screen<NC, HD, GD>(rr, rlw, d0, a, need);
          else cand = cfar2d_phase_a<NC, HD, GD>(rr, rlw, d0, a, need);
        } else {
          cand = cfar2d_phase_a_generic<NC>(rr, rlw, d0, a, need);
        }
      }
#ifdef FMCW_CFAR2D_ABLATE
      if (FMCW_CFAR2D_ABLATE != 4)
#endif
      if constexpr (HD > 0 && FMCW_CFAR2D_SCREEN) {
        // survivors of the screen -> candidate test, 256 per round over the whole workgroup (a
        // hot tile's survivors spread over all four waves).  A round of <= 32 / 64 / 128 cells
        // gives each cell 8 / 4 / 2 adjacent lanes that split its rows: a step usually has a
        // few dozen survivors, and one lane walking all 128 references of a cell alone set the
        // critical path of the step (config 5: 89 -> 71 us per frame).
        aux[threadIdx.x] = 0u;
        const uint32_t scr = cand;
        coop_rounds(scr, cnt, list, nullptr, 0u, [&](int n) {
          const int L = n <= 32 ? 8 : n <= 64 ? 4 : n <= 128 ? 2 : 1;
          const int j = (int)threadIdx.x / L, sub = (int)threadIdx.x % L;
          if (j < n) {  // whole aligned groups of L lanes
            int trow, d;
            const uint32_t e = list[j];
            cell_of(e, trow, d);
            if (cfar2d_exact_a<NC, HD, GD>(rr, trow, d, a, need, sub, L) && sub == 0)
              atomicOr(&aux[e >> 4], 1u << (e & 15u));
          }
        });
        cand = aux[threadIdx.x];
        __syncthreads();  // every lane has its bits before aux is cleared again
      }

      // ---- Phase B: one whole wave per candidate cell.  Lanes hold refs l and l + 64 of the fixed
      // order; the mean is the fixed fp32 halving tree; the scale bracket comes from ballot counts.
      auto refs_of = [&](int trow, int d, float& va, float& vb) {
        va = oka ? rr.row(trow + a.hr + dra)[midx((d + dda) & (NC - 1))] : 0.f;
        vb = okb ? rr.row(trow + a.hr + drb)[midx((d + ddb) & (NC - 1))] : 0.f;
      };
      auto scale_of = [&](float va, float vb) -> float {
        float sum = va + vb;
#pragma unroll
        for (int x = 32; x >= 1; x >>= 1) sum += __shfl_xor(sum, x, 64);
        if (a.override_) return (float)a.override_;
        float half, hi;
        if (a.compat) {
          // integer cells < 2^17, <= 128 of them: every partial sum < 2^24 is exact in fp32.
          // mean = floor(sum / N_REF) (os_cfar_2d.vhd:189); the bracket add is 17 bits wide (:193)
          const uint32_t mean = (uint32_t)sum / (uint32_t)a.n_ref;
          half = (float)(mean >> 1);
          hi = (float)((mean + (mean >> 1)) & kQ17Mask);
        } else {
          const float mean = sum / (float)a.n_ref;
          half = mean * 0.5f;
          hi = mean + half;
        }
        const int n_hi = __popcll(__ballot(oka && va > hi)) + __popcll(__ballot(okb && vb > hi));
        const int n_lo = __popcll(__ballot(oka && va < half)) + __popcll(__ballot(okb && vb < half));
        return (n_hi >= need) ? a.sc_max : (n_lo >= a.rank + 1) ? a.sc_min : a.sc_nom;
      };
#ifdef FMCW_CFAR2D_ABLATE  // timing experiments only: 1 = no phase B, 2 = no ranked-value select
      if (FMCW_CFAR2D_ABLATE == 1) cand = 0;
#endif

      // Pass 1: decide every candidate; the four waves take the round's entries in turn
      aux[threadIdx.x] = 0u;
      coop_rounds(cand, cnt + 4, list, nullptr, 0u, [&](int n) {
        for (int j = wv; j < n; j += WPB) {
          int trow, d;
          const uint32_t e = list[j];
          cell_of(e, trow, d);
          const float cut = rr.row(trow + a.hr)[midx(d)];
          float va, vb;
          refs_of(trow, d, va, vb);
          const float sc = scale_of(va, vb);
          const int n_ge = __popcll(__ballot(oka && sc * va >= cut)) + __popcll(__ballot(okb && sc * vb >= cut));
#ifdef FMCW_CFAR2D_ABLATE  // 3 / 4: every candidate / screen survivor is reported (counting)
          if (FMCW_CFAR2D_ABLATE >= 3 && lane == 0) atomicOr(&aux[e >> 4], 1u << (e & 15u));
#endif
          if (n_ge < need && lane == 0) atomicOr(&aux[e >> 4], 1u << (e & 15u));
        }
      });
      const uint32_t detw = aux[threadIdx.x];
      int total;
      const int dx = wave_excl_scan(__popc(detw), total);
      const int wtile = tile0 + f * wt_per_frame + wt0 + wv;
      const uint32_t base = has_tile ? det_reserve_wave(sink, wtile, total) : 0u;
      __syncthreads();  // aux now carries sink positions

      // Pass 2: exact ranked value (k-th smallest) of each detection by a pivoting select on the
      // bit patterns (cells are non-negative: unsigned order == value order), then the record
      coop_rounds(detw, cnt + 8, list, aux, base + (uint32_t)dx, [&](int n) {
        for (int j = wv; j < n; j += WPB) {
          int trow, d;
          cell_of(list[j], trow, d);
          const uint32_t slot = aux[j];
          float va, vb;
          refs_of(trow, d, va, vb);
          const float sc = scale_of(va, vb);
          uint32_t ranked = 0;
#ifdef FMCW_CFAR2D_ABLATE
          if (FMCW_CFAR2D_ABLATE != 2)
#endif
          ranked = wave_select_kth(oka ? __float_as_uint(va) : 0u, okb ? __float_as_uint(vb) : 0u,
                                   __ballot(oka), __ballot(okb), a.rank);
          if (lane == 0 && slot < sink.cap) {
            fmcw_det dd;
            dd.frame = (uint32_t)(frame0 + f);
            dd.range = (uint16_t)(r0 + trow);
            dd.doppler = (uint16_t)d;
            dd.mag = rr.row(trow + a.hr)[midx(d)];
            dd.threshold = sc * __uint_as_float(ranked);
            sink.scratch[slot] = dd;
          }
        }
      });
    }  // steps
  }    // strips
}
