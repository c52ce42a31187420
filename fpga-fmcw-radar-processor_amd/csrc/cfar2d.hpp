// cfar2d.hpp -- K3: 2-D OS-CFAR (rtl/src/os_cfar_2d.vhd:140-217) over the linear magnitude
// map, for gfx950.  Included from inside namespace fmcw by kernels.hpp (uses DetSink,
// det_reserve_wave, wave_excl_scan, lt_bit, opaque, nonneg / q17, MH and DopplerGeom declared
// there).
//
// Tiles.  The detection unit is K2's wave tile: WR = 1024/NC range rows x NC Doppler cells
// (16 cells per lane), so the 1-D and 2-D CFAR share one sink layout and one (frame, range,
// doppler) order.  A workgroup (4 waves) takes 4 consecutive wave tiles of one frame (a step)
// and walks a strip of such steps through a ring of staged rows (the TR rows of the step plus
// +-hr halo rows).  Doppler is circular; a CUT row is tested only if its whole range extent
// lies inside the map (build spec).
//
// Three stages, each conservative (it never drops a cell that can detect), the last exact:
//  1. Screen (every cell, one lane per 16 consecutive cells), on 7-bit PAIR-MAX keys staged in
//     LDS: 4 CUTs per 32-bit VALU op (cfar2d_screen7).
//  2. Candidate test of the screen's survivors (~1.3 % of noise cells), L lanes per cell, on the
//     exact fp32 cells of the map in global memory (L2 / MALL-resident: the rows were staged
//     moments before): exact E(s) counts and a bound on the mean (cfar2d_exact_a).
//  3. Phase B (the candidates, one whole wave per cell, in cell order): lanes hold refs l and
//     l + 64 (fixed order: dr outer, dd inner); the mean is the fixed fp32 halving tree (one
//     add, then xor-shuffles 32..1 == oracle tree_sum_f32); the scale bracket comes from ballot
//     counts (ranked > M <=> #{ref > M} >= n_ref - k; ranked < M' <=> #{ref < M'} >= k + 1);
//     detect <=> #{fl(s * ref) >= cut} < n_ref - k.  Pass 1 decides and counts, the wave
//     reserves its sink range, pass 2 walks its detections again and finds the exact ranked
//     value by a pivoting select (threshold = fl(s * ranked), dbg_threshold).
#pragma once

struct Cfar2DArgs {
  int hr, gr, hd, gd;  // half extents (ref + guard) and guards, range / Doppler
  int n_ref, rank;
  float s_min, sc_min, sc_nom, sc_max;
  int override_;
  int compat;          // FMCW_COMPAT_CFAR: 17-bit integer cells, integer mean and brackets
};

// The candidate list of one 2-D CFAR launch (capacity: every cell of the launch, so it cannot
// overflow): cell[i] = (frame in the launch x ns + range) x NC + doppler, runs of one wave tile in
// cell order; thr[i] = the threshold of a detection, -1 for a rejected candidate (k_cfar2d_decide);
// tiles[] = the wave tiles with candidates; ctr[0] = candidates, ctr[1] = such tiles (zeroed before
// the launch).
struct Cfar2Cands {
  uint32_t* cell;
  float* thr;
  uint32_t* tiles;
  uint32_t* ctr;
  // k_cfar2d_lv's strip-private spill regions (room for every cell / wave tile of the launch: a
  // strip's part starts at its first cell / wave tile), copied into cell / tiles at the strip's end
  uint32_t* pcell;
  uint32_t* ptile;   // 2 words per wave tile
};

// 7-bit keys.  key(v) = clamp((bits(v) >> SH) - base, 0, 127) for a non-negative fp32 cell v:
// 2^(23 - SH) levels per octave (16 at SH = 19) over a 128-level window that starts `base`
// levels up; base is set per strip from the mean level of its first step's cells minus LOW
// (kK3KeyLow, 64: the window spans 4 octaves below the mean level to 4 above, where
// Rayleigh noise and the cut / s_min levels it is tested against lie).  The key is monotone
// non-decreasing in v, with clamping at both ends, and NaN maps to 0 (a NaN reference never
// counts), so key(ref) > key(q) implies ref > q.  Cells above the window all get 127: they
// count as references, and as CUTs they are never screened out (no key is above 127).
constexpr int kK3KeyShift = 19, kK3KeyLow = 64;
__device__ __forceinline__ uint32_t key7(float v, int base) {
  const uint32_t b = __float_as_uint(v);
  const int k = b > 0x7f800000u ? -1 : (int)(b >> kK3KeyShift) - base;
  return (uint32_t)min(max(k, 0), 127);
}
// key(q) + 1 for q = fl(c * inv_s) + 8 ulps (c * fl(1 / s): <= 2 ulps of error), c = the CUT:
// a pair max whose key is >= this has max > q > c / s in reals, so fl(s * max) >= c.
// (No NaN test: a NaN cut gets 128, which no key reaches, so this round-3 screen never screens it
// out; the level screens do -- NaN cells are outside the specification, fmcw.h fmcw_cfar.)
__device__ __forceinline__ uint32_t cut_key7(float c, float inv_s, int base) {
  const int k = (int)((__float_as_uint(c * inv_s) + 8u) >> kK3KeyShift) - base;
  return (uint32_t)min(max(k, 0), 127) + 1u;
}

// 16-bit keys (the candidate test's): the high half of the bit pattern of a non-negative cell
// (sign 0, 8 exponent and 7 mantissa bits), NaN -> 0; lo(k) = float(k << 16) <= cell <=
// hi(k) = float(k << 16 | 0xffff).
__device__ __forceinline__ uint32_t key16(float v) {
  const uint32_t b = __float_as_uint(v);
  return b > 0x7f800000u ? 0u : b >> 16;
}
__device__ __forceinline__ float key_lo(uint32_t k) { return __uint_as_float(k << 16); }
__device__ __forceinline__ float key_hi(uint32_t k) {  // the inf key bounds as +inf
  return __uint_as_float(min((k << 16) | 0xffffu, 0x7f800000u));
}
// (key16 + 1) of q = fl(c * inv_s) + 8 ulps: a reference whose key16 is strictly above key(q)
// has ref > q > c / s in reals, so fl(s * ref) >= c.  Clamped so that a packed 16-bit
// difference never wraps.
__device__ __forceinline__ uint32_t cut_key16(float c, float inv_s) {
  return min((__float_as_uint(c * inv_s) + 8u) >> 16, 0x7fffu) + 1u;
}
// LDS key16 row: cell d (-MH <= d < NC + MH, circular halos) at k16idx(d), unpadded (the
// candidate test's reads are scattered anyway; the LDS budget keeps 3 workgroups per CU).
__host__ __device__ constexpr int k16idx(int d) { return d + MH; }
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// LDS byte row: the pair-max key of cell d (-MH <= d < NC + MH, circular halos) at byte
// b7idx(d), with bit 7 set: pm(d) = max(key(d), key(d + 1)) | 0x80.  A lane's 32-byte window
// (cells d0 - 8 .. d0 + 23) is two aligned 16-B reads.
__host__ __device__ constexpr int b7idx(int d) { return d + MH + 8; }

template <int NC> struct Cfar2DGeom {
  static constexpr int NT = 256;
  static constexpr int WPB = 4;                   // wave tiles per workgroup tile
  static constexpr int WR = DopplerGeom<NC>::WR;  // CUT rows per wave tile
  static constexpr int TR = WPB * WR;             // CUT rows per workgroup tile
  static constexpr int RB = NC + 2 * MH + 16;     // LDS pair-max row stride (bytes)
  static constexpr int KRS = NC + 2 * MH;        // LDS key16 row stride (keys)
  static constexpr int TPR = NC / 16;             // lanes per row
  static_assert(RB % 16 == 0 && KRS % 8 == 0 && MH >= 8, "rows stay 16-B aligned; the window is inside the halos");
};

// The staged rows of one step: a ring of nr = TR + 2 hr slots, each a pair-max byte row (rs
// bytes) and a key16 row (ks keys).  Tile row x (0 = the first halo row of the current step)
// lives in slot (x + base) mod nr, so a strip of steps keeps the 2 hr rows it shares with the
// next step and loads only TR new ones.
struct RowRing {
  uint8_t* tile;
  uint16_t* keys;
  int base, nr, rs, ks;
  __device__ __forceinline__ int slot(int x) const {
    const int y = x + base;
    return y >= nr ? y - nr : y;
  }
  __device__ __forceinline__ uint8_t* row(int x) const { return tile + slot(x) * rs; }
  __device__ __forceinline__ uint16_t* krow(int x) const { return keys + slot(x) * ks; }
};

constexpr int kCfar2dList = 2 * 256 + 16;  // u32 after the rows: round list, verdicts / positions, counts

template <int NC>
constexpr size_t cfar2d_smem_bytes(int hr) {
  using G = Cfar2DGeom<NC>;
  return (size_t)(G::TR + 2 * hr) * (G::RB + 2 * G::KRS) + kCfar2dList * 4;
}

// ---- Level screen (round 4; the reference window: HD 6, GD 2, HR <= 7, GR <= 1) ----------------
// Exact reference counts at two fixed LEVELS per strip instead of a pair bound per CUT threshold.
// For a level key Q, count_Q(c) = #{ref r of CUT c : key16(r) >= Q} is a box count: (2 HR + 1) x
// 13 window minus the 3 x 5 guard block, separable into column sums over the staged rows and
// sliding row sums of those.  Every ref counted lies >= lo(Q), so fl(s_min r) >= P = fl(s_min lo(Q))
// (rounding is monotone); a CUT with key16(cut) < U = key16(P) has cut < lo(U) <= P.  So
// key16(cut) < U and count_Q >= need give E(s_min) >= need: the cell cannot detect at any scale
// >= s_min.  Two levels A <= B per strip, at the kK3LvQA / _QB quantiles (50 % / 66 %) of
// the key7 levels of the strip's first 4096 cells: a CUT is screened out if either level rules it
// out.  Quantiles, not offsets from the mean, so the levels follow the clutter's spread (config 3's
// 4-rx NCI cells are far narrower than config 5's Rayleigh ones).  Survivors on the bench maps
// (tests' fixed seed, NumPy model of this screen, round 4's 56 % / 68 %): config 5 1.6 %, config 2 1.7 %, config 3
// 0.014 % -- the round-3 pair screen 1.9 %, 2.0 %, 0.010 % -- at about a quarter of its VALU work.
// Ring rows hold per cell one byte: bit 0 = key >= QA, bit 4 = key >= QB, so both levels' column
// sums (<= 2 HR + 1 <= 15) add in the nibbles of one 32-bit add; the 13-cell row sums (<= 143) of
// each level are taken from byte prefix sums, the guard block's 5-cell sums (<= 15) in nibbles.
// the two levels: quantiles (per mille) of the strip's first-step cells; rows of the level
// screen's LDS reads in flight ahead of the accumulation (round 5: 2 or 3 measured alike, 2 keeps
// k_cfar2d_lv spill-free at 4 waves per SIMD)
// (k_cfar2d: 50 % / 66 % since late round 5 -- NumPy model of the screen on config 3's map 0.014 % ->
// 0.006 % survivors; config-3 K3 73.5-74.1 -> 68.2-69.2 us, lab, two passes; 52 / 66 70.9-71.4,
// 50 / 64 69.6)
constexpr int kK3LvQA = 500, kK3LvQB = 660, kK3ScreenAhead = 2;
// k_cfar2d_lv's two levels (its scale rules change the optimum): the 50 % / 74 % quantiles, B clamped
// to 1.5 A so that rule A stays available.  NumPy model of the rules on the config-5 bench map
// (tools/k3_rules_model.py, 4 x 48 rows): survivors 0.0356 % at 56 / 68, 0.0041 % at 50 / 74; 48 / 76, where B passes 1.5 A
// unclamped, 2.2 %.
constexpr int kK3RulesQA = 500, kK3RulesQB = 740;
// k_cfar2d: odd strips of a frame walk upwards (round 5; see the strip loop)
constexpr bool kK3AltDir = true;
// level nibbles of 4 cells from their key16 pairs (cells d, d + 1 | d + 2, d + 3): (k | 0x8000) - Q has
// bit 15 set iff k >= Q (k < 0x8000, 1 <= Q <= 0x8000: no borrow across the halves); the byte
// permute collects bits 15 / 31 of both words as bit 7 of 4 bytes
__device__ __forceinline__ uint32_t lv_nibbles(uint2 kw, uint32_t qa2, uint32_t qb2) {
  const uint32_t x0 = kw.x | 0x80008000u, x1 = kw.y | 0x80008000u;
  const uint32_t pa = __builtin_amdgcn_perm(x1 - qa2, x0 - qa2, 0x07050301u);
  const uint32_t pb = __builtin_amdgcn_perm(x1 - qb2, x0 - qb2, 0x07050301u);
  return ((pa >> 7) & 0x01010101u) | ((pb >> 3) & 0x10101010u);
}
// the same from sanitised keys (k <= 0x7f80) with ca2 / cb2 = (0x8000 - Q) in both halves: k + 0x8000 - Q
// has bit 15 set iff k >= Q and stays below 0x10000 (no carry into the upper half)
__device__ __forceinline__ uint32_t lv_nibbles_add(uint2 kw, uint32_t ca2, uint32_t cb2) {
  const uint32_t pa = __builtin_amdgcn_perm(kw.y + ca2, kw.x + ca2, 0x07050301u);
  const uint32_t pb = __builtin_amdgcn_perm(kw.y + cb2, kw.x + cb2, 0x07050301u);
  return ((pa >> 7) & 0x01010101u) | ((pb >> 3) & 0x10101010u);
}
// byte-wise inclusive prefix sums of a word (bytes <= 63: no carry)
__device__ __forceinline__ uint32_t byte_prefix(uint32_t x) {
  x += x << 8;
  return x + (x << 16);
}
// 13-cell sums of one level's column counts: b[i] = cell d0 - 6 + i in X[0..6]; out m (0..3) byte t
// = sum b[4m + t .. 4m + t + 12] = (T_m - PE_m[t]) + T_{m+1} + T_{m+2} + PF_{m+3}[t] with T = word sums,
// PF / PE the inclusive / exclusive byte prefixes (PE = PF - X); every byte stays in 0..143
__device__ __forceinline__ void lv_sum13(const uint32_t (&X)[7], uint32_t (&H)[4]) {
  uint32_t PF[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) PF[k] = byte_prefix(X[k]);
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const uint32_t t3 = PF[m] + PF[m + 1] + PF[m + 2];           // byte 3 = T_m + T_{m+1} + T_{m+2} (<= 132)
    const uint32_t tb = __builtin_amdgcn_perm(t3, t3, 0x03030303u);  // broadcast
    H[m] = tb - PF[m] + X[m] + PF[m + 3];
  }
}
// Survivor bits (bit j = cell d0 + j may detect) of this lane's 16 CUTs, CUT row rl of the group
// tile.  wa2 / wb2 = per level (U | 0x80008000) - 0x00010001 in both halves: W - key16 has bit 15
// set iff key16 < U.
template <int NC, int HR, int GR>
__device__ __forceinline__ uint32_t cfar2d_screen_lv(const RowRing& rr, int rl, int d0, int need, uint32_t wa2,
                                                     uint32_t wb2) {
  static_assert(2 * HR + 1 <= 15 && 5 * (2 * GR + 1) <= 15, "nibble column sums and guard-row sums");
  // column sums of the nibble rows: V over the 2 HR + 1 window rows (cells d0 - 8 .. d0 + 23), G over
  // the 2 GR + 1 guard rows (cells d0 - 4 .. d0 + 19 = V words 1..6)
  uint32_t V[8], G[6];
#pragma unroll
  for (int k = 0; k < 8; ++k) V[k] = 0u;
#pragma unroll
  for (int k = 0; k < 6; ++k) G[k] = 0u;
  // The 2 HR + 1 rows' 32-byte windows, with at most kK3ScreenAhead rows' loads in flight: left to
  // itself the scheduler issued all 22 LDS reads first (88 VGPRs of loads, the kernel's register
  // peak); the scheduling barriers keep a rolling window of loads ahead of the accumulation.
  constexpr int NW = 2 * HR + 1, AH = kK3ScreenAhead < NW ? kK3ScreenAhead : NW;
  int sl = rr.slot(rl);  // ring slot of window row dr = -HR, advanced with wrap
  uint4 q0[AH], q1[AH];
  auto load_row = [&](int j) {
    const uint8_t* rp = rr.tile + sl * rr.rs + b7idx(d0 - 8);
    q0[j % AH] = *reinterpret_cast<const uint4*>(rp);
    q1[j % AH] = *reinterpret_cast<const uint4*>(rp + 16);
    sl = sl + 1 == rr.nr ? 0 : sl + 1;
  };
#pragma unroll
  for (int j = 0; j < AH; ++j) load_row(j);
#pragma unroll
  for (int j = 0; j < NW; ++j) {
    const int dr = j - HR;
    if constexpr (kK3ScreenAhead < 2 * HR + 1) __builtin_amdgcn_sched_barrier(0);
    const uint4 a0 = q0[j % AH], a1 = q1[j % AH];
    const uint32_t D[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    if (j + AH < NW) load_row(j + AH);
#pragma unroll
    for (int k = 0; k < 8; ++k) V[k] += D[k];
    if (dr >= -GR && dr <= GR) {
#pragma unroll
      for (int k = 0; k < 6; ++k) G[k] += D[k + 1];
    }
    if constexpr (kK3ScreenAhead < 2 * HR + 1) {
      // the row's sums now (no reassociation into one add tree after every load)
#pragma unroll
      for (int k = 0; k < 8; ++k) asm volatile("" : "+v"(V[k]));
#pragma unroll
      for (int k = 0; k < 6; ++k) asm volatile("" : "+v"(G[k]));
    }
  }
  if constexpr (kK3ScreenAhead < 2 * HR + 1) __builtin_amdgcn_sched_barrier(0);
  // 13-cell window per level: realign so that word k byte t = cell d0 - 6 + 4k + t, then unpack
  uint32_t HA[4], HB[4];
  {
    uint32_t XA[7], XB[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const uint32_t w = __builtin_amdgcn_alignbyte(V[k + 1], V[k], 2);
      XA[k] = w & 0x0F0F0F0Fu;
      XB[k] = (w >> 4) & 0x0F0F0F0Fu;
    }
    lv_sum13(XA, HA);
    lv_sum13(XB, HB);
  }
  // guard block (3 x 5 around the CUT) per level, both levels in the nibbles (sums <= 15):
  // g[i] = cell d0 - 2 + i; out m byte t = g[4m + t .. 4m + t + 4]
  uint32_t H5[4];
  {
    uint32_t Gp[5], S2[5], S4[4];
#pragma unroll
    for (int k = 0; k < 5; ++k) Gp[k] = __builtin_amdgcn_alignbyte(G[k + 1], G[k], 2);
#pragma unroll
    for (int k = 0; k < 5; ++k) S2[k] = Gp[k] + __builtin_amdgcn_alignbyte(k < 4 ? Gp[k + 1] : 0u, Gp[k], 1);
#pragma unroll
    for (int k = 0; k < 4; ++k) S4[k] = S2[k] + __builtin_amdgcn_alignbyte(S2[k + 1], S2[k], 2);
#pragma unroll
    for (int m = 0; m < 4; ++m) H5[m] = S4[m] + Gp[m + 1];
  }
  // the CUTs' key16 (the staged row): W - key16 bit 15 = key16(cut) < U, gathered as byte bit 7
  const uint16_t* kr = rr.krow(rl + HR) + k16idx(d0);
  const uint4 ka = *reinterpret_cast<const uint4*>(kr), kc = *reinterpret_cast<const uint4*>(kr + 8);
  const uint32_t kw[8] = {ka.x, ka.y, ka.z, ka.w, kc.x, kc.y, kc.z, kc.w};
  const uint32_t add_need = (uint32_t)(128 - need) * 0x01010101u;  // count >= need <=> bit 7 of count + 128 - need
  uint32_t bits = 0;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const uint32_t ca = __builtin_amdgcn_perm(wa2 - kw[2 * m + 1], wa2 - kw[2 * m], 0x07050301u);
    const uint32_t cb = __builtin_amdgcn_perm(wb2 - kw[2 * m + 1], wb2 - kw[2 * m], 0x07050301u);
    const uint32_t na = HA[m] - (H5[m] & 0x0F0F0F0Fu) + add_need;
    const uint32_t nb = HB[m] - ((H5[m] >> 4) & 0x0F0F0F0Fu) + add_need;
    const uint32_t surv = ~((na & ca) | (nb & cb)) & 0x80808080u;
    bits |= ((surv * 0x00204081u) >> 28) << (4 * m);  // bit 7 of byte t -> bit 28 + t
  }
  return bits;
}

// Screen, runtime geometry (any window the LDS budget allows; Doppler wraps explicitly): the
// same pair bound, one byte read per (CUT, pair).
template <int NC>
__device__ __forceinline__ uint32_t cfar2d_screen7_generic(const RowRing& rr, int rl, int d0, const Cfar2DArgs& a,
                                                           int need, const uint32_t (&Y)[4]) {
  const int nps = (a.hd - a.gd) / 2;
  uint32_t bits = 0;
  for (int i = 0; i < 16; ++i) {
    const int d = d0 + i;
    const uint32_t y = (Y[i >> 2] >> (8 * (i & 3))) & 0xffu;
    int n = 0;
    auto pm = [&](const uint8_t* row, int c) { return (uint32_t)row[b7idx(c & (NC - 1))] >= y + 128u ? 1 : 0; };
    for (int dr = -a.hr; dr <= a.hr; ++dr) {
      const uint8_t* row = rr.row(rl + a.hr + dr);
      if (dr >= -a.gr && dr <= a.gr) {
        for (int j = 0; j < nps; ++j) n += pm(row, d - a.hd + 2 * j) + pm(row, d + a.gd + 1 + 2 * j);
      } else {
        for (int j = 0; j < a.hd; ++j) n += pm(row, d - a.hd + 2 * j);
      }
    }
    bits |= (n < need ? 1u : 0u) << i;
  }
  return bits;
}

// Candidate test of one screen survivor (CUT row rl of the group tile, Doppler d; `cut` = the
// cut or an upper bound of it, here hi(key16): every bound below holds with it, since the
// references counted lie above cut / s and the half-mean test compares the same value), by L
// adjacent lanes that split the window rows; it keeps every cell that can
// detect.  With E(s) = #{fl(s * ref) >= cut}, the cell can only detect if E(s) < need for the
// scale s it gets.  E(s_min) >= need rules every scale out.  The scale is sc_min only when
// #{ref < mean / 2} >= rank + 1 (os_cfar_2d.vhd:195-199); otherwise it is >= s2 =
// min(sc_nom, sc_max) and E(s2) >= need rules the cell out too.  On the key16 rows: E(s_min)
// and E(s2) are bounded from below (a reference counts if its key is >= cut_key16; E(s2) and
// the rest decided only for the survivors E(s_min) does not rule out), the mean from above by an
// any-order fp32 sum of lo(key) x (1 + 2^-7 + 2^-14) + 2^-119
// (<= 128 non-negative terms: any order is within 2^-16 relative; compat's floor(sum / n) >> 1
// is below the real half), and #{ref < mean / 2} from above by #{lo(key) < half_up}.
// Compile-time HD: the window is inside the row halos; HD == 0 (runtime geometry): Doppler
// wraps explicitly.
template <int NC, int HD, int GD>
__device__ __forceinline__ bool cfar2d_exact_a(const RowRing& rr, int rl, float cut, int d, const Cfar2DArgs& a,
                                               int need, int sub, int L) {
  const float s2 = a.override_ ? a.s_min : fminf(a.sc_nom, a.sc_max);
  const uint32_t k1 = cut_key16(cut, 1.0f / a.s_min);
  const uint32_t k2 = cut_key16(cut, 1.0f / s2);
  auto visit = [&](auto&& fn) {  // this lane's rows: dr = -hr + sub, every L-th
    for (int dr = -a.hr + sub; dr <= a.hr; dr += L) {
      const uint16_t* row = rr.krow(rl + a.hr + dr);
      const bool grow = dr >= -a.gr && dr <= a.gr;
      if constexpr (HD > 0) {
        if (grow) {
#pragma unroll
          for (int dd = -HD; dd <= HD; ++dd)
            if (dd < -GD || dd > GD) fn((uint32_t)row[k16idx(d + dd)]);
        } else {
#pragma unroll
          for (int dd = -HD; dd <= HD; ++dd) fn((uint32_t)row[k16idx(d + dd)]);
        }
      } else {
        for (int dd = -a.hd; dd <= a.hd; ++dd)
          if (!grow || dd < -a.gd || dd > a.gd) fn((uint32_t)row[k16idx((d + dd) & (NC - 1))]);
      }
    }
  };
  // one walk: #{refs not counted} at s_min and at s2, and the mean bound.  (Two walks -- the
  // second only for cells E(s_min) does not rule out -- read every key twice in practice: a
  // round's wave runs the second walk whenever any of its cells needs it, which is nearly always.)
  int n1 = 0, n2 = 0;
  float sum = 0.f;
  visit([&](uint32_t kv) {
    n1 += kv < k1 ? 1 : 0;
    n2 += kv < k2 ? 1 : 0;
    sum += key_lo(kv);  // hi(k) <= lo(k) (1 + 2^-7) for normal keys; the bound below widens by that
  });
  for (int x = 1; x < L; x <<= 1) {  // the cell's L lanes are adjacent and aligned
    n1 += __shfl_xor(n1, x, 64);
    n2 += __shfl_xor(n2, x, 64);
    sum += __shfl_xor(sum, x, 64);
  }
  if (a.n_ref - n1 >= need) return false;                         // E(s_min) >= need
  if (a.n_ref - n2 < need || a.override_) return true;            // E(s2) may be < need
  // upper bound of mean / 2: sum of lo(key) x (1 + 2^-7 + 2^-14) (key precision, then the any-order
  // fp32 sum of <= 128 non-negative terms, within 2^-16) + 2^-119 (the subnormal keys, where
  // hi / lo is unbounded: 128 x 2^-126)
  const float half_up = (sum * (1.0f + 1.0f / 128.0f + 1.0f / 16384.0f) + 0x1p-119f) / (float)a.n_ref * 0.5f;
  // >= need refs lie above cut / s2; if that is >= mean / 2 they all lie above the half, so
  // n_lo <= n_ref - need = rank < rank + 1 without counting (most noise survivors: their cut
  // is high).  (1 - 2^-20) covers the product's rounding.
  if (cut * (1.0f / s2) * (1.0f - 1.0f / 1048576.0f) >= half_up) return false;
  int n_lo = 0;
  visit([&](uint32_t kv) { n_lo += key_lo(kv) < half_up ? 1 : 0; });
  for (int x = 1; x < L; x <<= 1) n_lo += __shfl_xor(n_lo, x, 64);
  return n_lo >= a.rank + 1;                                     // sc_min still possible
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


// HD > 0: the reference window (HD 6, GD 2, compile-time HR / GR) with the level screen; HD == 0:
// any window, runtime geometry, the pair screen on 7-bit keys (cfar2d_screen7_generic).
template <int NC, int HD, int GD, int HR = 0, int GR = 0>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
k_cfar2d(const float* __restrict__ map, int ns, int n_strips, int steps, int frame0, int tile0, Cfar2DArgs a,
         DetSink sink, Cfar2Cands cands) {
  (void)frame0;
  constexpr bool LV = HD > 0;
  static_assert(!LV || (HD == 6 && GD == 2 && HR >= 1), "the level screen is built for the reference window");
  using Gm = Cfar2DGeom<NC>;
  constexpr int WR = Gm::WR, NT = Gm::NT, RB = Gm::RB, TPR = Gm::TPR, WPB = Gm::WPB, TR = Gm::TR;
  static_assert(TR * NC == 4 * 4 * NT, "a step's new rows are 4 float4 per thread");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem8[];
  uint8_t* const tile = smem8;

  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int need = a.n_ref - a.rank;
  const int wt_per_frame = ns / WR;                      // wave tiles per frame
  const int wg_per_frame = (wt_per_frame + WPB - 1) / WPB;
  const int spf = (wg_per_frame + steps - 1) / steps;    // strips per frame
  const int nf = n_strips / spf;
  const int nr = TR + 2 * a.hr;                          // ring rows
  uint16_t* const keys = reinterpret_cast<uint16_t*>(tile + nr * RB);
  uint32_t* const list = reinterpret_cast<uint32_t*>(keys + nr * Gm::KRS);
  uint32_t* const aux = list + kCoopRound;
  uint32_t* const cnt = aux + kCoopRound;
  const int tid = opaque(threadIdx.x);

  // The ring rows of one float4 of cells (row x, Doppler d..d+3), each with its circular-halo copy:
  // put_k16 the key16 row (returns the 4 keys), put_scr 4 bytes of the screen row -- LV: level
  // nibbles; else the pair-max 7-bit keys (which need the cell d + 4 after it, circularly).
  // Per strip: LV level words (qa2, qb2), else the 7-bit key base kb.
  uint32_t qa2 = 0u, qb2 = 0u;
  int kb = 0;
  auto put_k16 = [&](const RowRing& rr, int x, int d, float4 v) -> uint2 {
    v = a.compat ? q17x4(v) : nonneg4(v);
    const uint2 kw = make_uint2(key16(v.x) | (key16(v.y) << 16), key16(v.z) | (key16(v.w) << 16));
    uint16_t* krow = rr.krow(x);
    *reinterpret_cast<uint2*>(krow + k16idx(d)) = kw;
    if (d < MH) *reinterpret_cast<uint2*>(krow + k16idx(NC + d)) = kw;
    if (d >= NC - MH) *reinterpret_cast<uint2*>(krow + k16idx(d - NC)) = kw;
    return kw;
  };
  auto put_scr = [&](const RowRing& rr, int x, int d, uint32_t w) {
    uint8_t* row = rr.row(x);
    *reinterpret_cast<uint32_t*>(row + b7idx(d)) = w;
    if (d < MH) *reinterpret_cast<uint32_t*>(row + b7idx(NC + d)) = w;
    if (d >= NC - MH) *reinterpret_cast<uint32_t*>(row + b7idx(d - NC)) = w;
  };
  // 7-bit pair-max keys of cells d..d+3 from the key16 of cells d..d+4 (key7 = key16 >> 3 - kb)
  auto pm_word = [&](uint2 kw, uint32_t k4) {
    auto k7 = [&](uint32_t k16) { return (uint32_t)min(max((int)(k16 >> 3) - kb, 0), 127); };
    const uint32_t k0 = k7(kw.x & 0xffffu), k1 = k7(kw.x >> 16), k2 = k7(kw.y & 0xffffu), k3 = k7(kw.y >> 16),
                   k5 = k7(k4);
    return max(k0, k1) | (max(k1, k2) << 8) | (max(k2, k3) << 16) | (max(k3, k5) << 24) | 0x80808080u;
  };

  for (int g = blockIdx.x; g < n_strips; g += gridDim.x) {
    // a strip: `steps` consecutive workgroup tiles of one frame (frame-minor order, as K2:
    // hot rows spread over all workgroups); each step tests TR rows and loads only TR new ones
    const int f = g % nf;
    const int t_beg = (g / nf) * steps, t_end = min(t_beg + steps, wg_per_frame);
    const float* fm = map + (size_t)f * ns * NC;
    RowRing rr{tile, keys, 0, nr, RB, Gm::KRS};
    float4 pre[4];
    float pre4[4];
    uint32_t wa2 = 0u, wb2 = 0u;  // LV: the CUT bounds of the two levels (cfar2d_screen_lv)
    // Odd strips of a frame walk upwards (kK3AltDir): the two strips on either side of a strip
    // boundary then stage the halo rows they share at the same time -- at both strips' start or
    // both strips' end -- and workgroups g and g + nf (neighbouring strips of one frame) sit on one
    // XCD when nf % 8 == 0, so the second load of those rows hits its L2 (config 3: map traffic
    // 1.125x -> 1.01x of the algorithmic bytes).
    const bool up = kK3AltDir && ((g / nf) & 1);
    for (int k = 0; k < t_end - t_beg; ++k) {
      const int t = up ? t_end - 1 - k : t_beg + k;
      const bool first = k == 0, last = k + 1 == t_end - t_beg;
      const int wt0 = t * WPB;                             // first wave tile of this step
      const int n_wt = min(WPB, wt_per_frame - wt0);
      const int r0 = wt0 * WR;                             // first CUT row of this step
      // this lane's 16 CUT cells: row r0 + rlw, Doppler d0..d0+15
      const int rlw = wv * WR + lane / TPR;    // CUT row within the group tile
      const int d0 = (lane % TPR) * 16;
      const int r = r0 + rlw;
      __syncthreads();  // the previous step's waves are done with the rows and the lists
      if (first) {
        // rows r0-hr .. r0+TR+hr-1 (zero outside the map), 4 float4 loads in flight per lane: the
        // key16 rows first, then the strip's levels (or key base) from the staged keys of the first
        // step's CUT rows, then the screen rows from the keys
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
            if (e4 < n4) put_k16(rr, x, d, v[u]);
          }
        }
        if (threadIdx.x == 0) cnt[12] = 0u;
        if (LV && threadIdx.x < 128) list[threadIdx.x] = 0u;
        __syncthreads();
        // the first step's CUT rows (TR x NC = 4096 cells; ring rows hr .. hr + TR - 1): their mean
        // level key16 >> 3 (= bits >> 19: 16 levels per octave), then (LV) the kK3LvQA / _QB
        // quantiles of a 128-level histogram around that mean
        uint32_t k7[16];
        {
          uint32_t sum = 0;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int e4 = tid + u * NT;
            const int i = e4 / (NC / 4), d = (e4 - i * (NC / 4)) * 4;
            const uint2 kw = *reinterpret_cast<const uint2*>(rr.krow(a.hr + i) + k16idx(d));
            k7[4 * u] = (kw.x & 0xffffu) >> 3;
            k7[4 * u + 1] = kw.x >> 19;
            k7[4 * u + 2] = (kw.y & 0xffffu) >> 3;
            k7[4 * u + 3] = kw.y >> 19;
            sum += k7[4 * u] + k7[4 * u + 1] + k7[4 * u + 2] + k7[4 * u + 3];
          }
#pragma unroll
          for (int x = 32; x >= 1; x >>= 1) sum += (uint32_t)__shfl_xor((int)sum, x, 64);
          if (lane == 0) atomicAdd(&cnt[12], sum);
        }
        __syncthreads();
        const int mean7 = (int)(cnt[12] / (uint32_t)(TR * NC));
        if constexpr (LV) {
          const int h0 = mean7 - 64;  // histogram bin 0
#pragma unroll
          for (int i = 0; i < 16; ++i) atomicAdd(&list[min(max((int)k7[i] - h0, 0), 127)], 1u);
          __syncthreads();
          if (wv == 0) {
            // bins 2 lane, 2 lane + 1: inclusive counts; the quantile bin = the first reaching p N
            const uint32_t c0 = list[2 * lane], c1 = list[2 * lane + 1];
            int tot;
            const uint32_t ex = (uint32_t)wave_excl_scan((int)(c0 + c1), tot);
            const uint32_t cum0 = ex + c0, cum1 = ex + c0 + c1;
            const uint32_t na = (uint32_t)(kK3LvQA * (TR * NC) / 1000), nb = (uint32_t)(kK3LvQB * (TR * NC) / 1000);
            const uint64_t ba0 = __ballot(cum0 >= na), ba1 = __ballot(cum1 >= na);
            const uint64_t bb0 = __ballot(cum0 >= nb), bb1 = __ballot(cum1 >= nb);
            // first bin: lane l's bin 2l if its cum0 qualifies, else 2l + 1
            auto first_bin = [](uint64_t m0, uint64_t m1) {
              const int l = __builtin_ctzll(m1);  // cum1 is reached by every qualifying lane
              return (m0 >> l) & 1u ? 2 * l : 2 * l + 1;
            };
            if (lane == 0) {
              cnt[14] = (uint32_t)first_bin(ba0, ba1);
              cnt[15] = (uint32_t)first_bin(bb0, bb1);
            }
          }
          __syncthreads();
          // level keys QA <= QB (key16 units: key7 << 3) and the CUT bounds U = key16(fl(s_min lo(Q))),
          // as the words lv_nibbles / cfar2d_screen_lv compare against
          const uint32_t QA = (uint32_t)min(max((h0 + (int)cnt[14]) * 8, 1), 0x7f80);
          const uint32_t QB = (uint32_t)min(max((h0 + (int)cnt[15]) * 8, 1), 0x7f80);
          qa2 = QA | (QA << 16);
          qb2 = QB | (QB << 16);
          const uint32_t UA = key16(a.s_min * key_lo(QA)), UB = key16(a.s_min * key_lo(QB));
          wa2 = ((UA | 0x8000u) - 1u) * 0x00010001u;
          wb2 = ((UB | 0x8000u) - 1u) * 0x00010001u;
        } else {
          kb = mean7 - kK3KeyLow;
        }
        // the screen rows of the whole ring from its key16 rows (halos included)
        for (int e4 = tid; e4 < n4; e4 += NT) {
          const int x = e4 / (NC / 4), d = (e4 - x * (NC / 4)) * 4;
          const uint16_t* kr = rr.krow(x) + k16idx(d);
          const uint2 kw = *reinterpret_cast<const uint2*>(kr);
          if constexpr (LV) put_scr(rr, x, d, lv_nibbles(kw, qa2, qb2));
          else put_scr(rr, x, d, pm_word(kw, (uint32_t)kr[4]));
        }
      } else {
        // the ring turns by TR rows (downwards: tile row x moves to x - TR; upwards: to x + TR);
        // the TR new rows (prefetched during the previous step) go into the slots of the TR rows
        // that left, at the bottom (rows nr - TR ..) or the top (rows 0 .. TR - 1) of the tile
        rr.base += up ? nr - TR : TR;
        if (rr.base >= nr) rr.base -= nr;
        const int x0 = up ? 0 : nr - TR;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int e4 = tid + u * NT;
          const int i = e4 / (NC / 4), d = (e4 - i * (NC / 4)) * 4;
          const uint2 kw = put_k16(rr, x0 + i, d, pre[u]);
          if constexpr (LV) {
            put_scr(rr, x0 + i, d, lv_nibbles(kw, qa2, qb2));
          } else {
            const float v4 = a.compat ? q17(pre4[u]) : nonneg(pre4[u]);
            put_scr(rr, x0 + i, d, pm_word(kw, key16(v4)));
          }
        }
      }
      if (!last) {  // prefetch the next step's new rows: r0 + TR + hr .. or r0 - TR - hr .. (zero off the map)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int e4 = tid + u * NT;
          const int i = e4 / (NC / 4), d = (e4 - i * (NC / 4)) * 4;
          const int r = (up ? r0 - TR - a.hr : r0 + TR + a.hr) + i;
          pre[u] = make_float4(0.f, 0.f, 0.f, 0.f);
          pre4[u] = 0.f;
          if (r >= 0 && r < ns) {
            pre[u] = *reinterpret_cast<const float4*>(fm + (size_t)r * NC + d);
            if constexpr (!LV) pre4[u] = fm[(size_t)r * NC + ((d + 4) & (NC - 1))];
          }
        }
      }
      __syncthreads();
      const bool has_tile = wv < n_wt;  // uniform per wave; waves without a tile still join the barriers

      // ---- Phase A: candidates among this lane's 16 cells
      uint32_t cand = 0;
      // cell of a round-list entry (wave << 10 | lane << 4 | bit) -> group-tile row, Doppler bin
      auto cell_of = [&](uint32_t e, int& trow, int& d) {
        const int we = (int)(e >> 10), le = (int)((e >> 4) & 63u);
        trow = we * WR + le / TPR;
        d = (le % TPR) * 16 + (int)(e & 15u);
      };
      const bool tested = has_tile && r >= a.hr && r < ns - a.hr;
      if (tested) {
        if constexpr (LV) {
          cand = cfar2d_screen_lv<NC, HR, GR>(rr, rlw, d0, need, wa2, wb2);
        } else {
          // cut_key7 of this lane's 16 CUTs, 4 per dword, from their staged key16 (an upper bound of
          // the cut, as the candidate test uses: a higher threshold only keeps more cells)
          uint32_t Y[4];
          const float inv_s = 1.0f / a.s_min;
          const uint16_t* kr = rr.krow(rlw + a.hr) + k16idx(d0);
          const uint4 ka = *reinterpret_cast<const uint4*>(kr), kc = *reinterpret_cast<const uint4*>(kr + 8);
          const uint32_t kw[8] = {ka.x, ka.y, ka.z, ka.w, kc.x, kc.y, kc.z, kc.w};
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            const uint32_t w0 = kw[2 * p], w1 = kw[2 * p + 1];
            Y[p] = cut_key7(key_hi(w0 & 0xffffu), inv_s, kb) | (cut_key7(key_hi(w0 >> 16), inv_s, kb) << 8) |
                   (cut_key7(key_hi(w1 & 0xffffu), inv_s, kb) << 16) | (cut_key7(key_hi(w1 >> 16), inv_s, kb) << 24);
          }
          cand = cfar2d_screen7_generic<NC>(rr, rlw, d0, a, need, Y);
        }
      }
      uint32_t n_cand = 1u;  // candidates in the workgroup's step (nonzero: phase B runs)
      {
        // (Measured and dropped: each wave testing its own survivors without workgroup barriers,
        // 643 vs 623 us per 16 frames at config 5 -- the rounds balance the waves' survivors.)
        // survivors of the screen -> candidate test, 256 per round over the whole workgroup (a
        // hot tile's survivors spread over all four waves).  A round of <= 32 / 64 / 128 cells
        // gives each cell 8 / 4 / 2 adjacent lanes that split its rows: a step usually has a
        // few dozen survivors, and one lane walking all 128 references of a cell alone set the
        // critical path of the step.
        const uint32_t scr = cand;
        aux[threadIdx.x] = 0u;
        if (threadIdx.x == 0) cnt[13] = 0u;  // candidates of the step (read after the rounds' barriers)
        coop_rounds(scr, cnt, list, nullptr, 0u, [&](int n) {
          const int L = n <= 32 ? 8 : n <= 64 ? 4 : n <= 128 ? 2 : 1;
          const int j = (int)threadIdx.x / L, sub = (int)threadIdx.x % L;
          if (j < n) {  // whole aligned groups of L lanes
            int trow, d;
            const uint32_t e = list[j];
            cell_of(e, trow, d);
            const uint32_t kc = rr.krow(trow + a.hr)[k16idx(d)];
            // a +0 CUT never detects (every reference is >= it: E(s) = n_ref), but with key16 0 it passes
            // every key bound; the exact cell decides (only key-0 cells load it: blank / sparse maps)
            bool live = true;
            if (kc == 0u) {
              const float v = fm[(size_t)(r0 + trow) * NC + d];
              live = (a.compat ? q17(v) : nonneg(v)) > 0.f;
            }
            if (live && cfar2d_exact_a<NC, HD, GD>(rr, trow, key_hi(kc), d, a, need, sub, L) && sub == 0)
            {
              atomicOr(&aux[e >> 4], 1u << (e & 15u));
              atomicAdd(&cnt[13], 1u);
            }
          }
        });
        cand = aux[threadIdx.x];
        n_cand = cnt[13];
        __syncthreads();  // every lane has its bits (and the count) before aux / cnt[13] change
      }
      const int wtile = tile0 + f * wt_per_frame + wt0 + wv;
      // ---- Emission: the wave tile's candidates, in (range, doppler) order, go to the launch's
      // candidate list as one contiguous run (k_cfar2d_decide decides them, k_cfar2d_emit writes
      // the tile's records); (wg_base, wg_count) = (run start, run length) until then.  An empty
      // tile is final here.
      // One reservation (two atomics) per workgroup step with candidates, not per wave tile (round 6:
      // on heavy-tailed clutter, where most wave tiles have candidates, the per-tile atomics on the
      // launch's two counters serialised; n_cand != 0 is uniform over the workgroup).
      if (n_cand != 0u) {
        const uint32_t mine = has_tile ? cand : 0u;  // bits of this lane's candidates (aux after the test)
        int k_w;
        const int ex = wave_excl_scan(__popc(mine), k_w);
        if (lane == 0) cnt[8 + wv] = has_tile ? (uint32_t)k_w : 0u;
        __syncthreads();
        uint32_t T = 0, woff = 0, ti = 0, nt = 0;
#pragma unroll
        for (int i = 0; i < WPB; ++i) {
          const uint32_t c = cnt[8 + i];
          woff += i < wv ? c : 0u;
          ti += (i < wv && c) ? 1u : 0u;
          T += c;
          nt += c ? 1u : 0u;
        }
        if (threadIdx.x == 0) {
          cnt[6] = atomicAdd(&cands.ctr[0], T);
          cnt[7] = atomicAdd(&cands.ctr[1], nt);
        }
        __syncthreads();
        const uint32_t p0 = cnt[6] + woff, q0 = cnt[7] + ti;
        if (has_tile) {
          if (k_w == 0) {
            if (lane == 0) {
              sink.wg_base[wtile] = (uint32_t)wtile * sink.slot_cap;
              sink.wg_count[wtile] = 0u;
            }
          } else {
            if (lane == 0) {
              cands.tiles[q0] = (uint32_t)wtile;
              sink.wg_base[wtile] = p0;
              sink.wg_count[wtile] = (uint32_t)k_w;
            }
            const uint32_t cbase = ((uint32_t)f * (uint32_t)ns + (uint32_t)r) * (uint32_t)NC + (uint32_t)d0;
            uint32_t o = p0 + (uint32_t)ex;
            for (uint32_t m = mine; m; m &= m - 1, ++o) cands.cell[o] = cbase + (uint32_t)__builtin_ctz(m);
          }
        }
        __syncthreads();  // cnt[6 .. 11] are read before the next step rewrites them
      } else if (has_tile && lane == 0) {
        sink.wg_base[wtile] = (uint32_t)wtile * sink.slot_cap;
        sink.wg_count[wtile] = 0u;
      }
    }  // steps
  }    // strips
}

// ---- K3a for the reference window (HD 6, GD 2, compile-time HR / GR; round 5): the level screen
// with the scale rules, and no candidate test inside the launch -- its survivors go straight to
// K3b's exact decision.
//
// Round 4's screen ruled a cell out only at the smallest scale s_min (= sc_min 2): with Rayleigh
// clutter 1.6 % of the cells (config 5) have cut >= 2 x the 68 % level, and a candidate test on LDS
// keys (~40 % of the launch) sorted them out again.  A cell gets sc_min only when #{ref < mean / 2}
// >= rank + 1 (os_cfar_2d.vhd:195-199).  If C_Q refs lie at or above a level q = lo(Q) and the mean
// is at most 2 q, those C_Q >= need refs are not below mean / 2, so at most rank refs are: the
// scale is >= s2 = min(sc_nom, sc_max), and E(s2) >= C_Q >= need rules the cell out when cut <
// fl(s2 q), i.e. key16(cut) < U2 = key16(fl(s2 q)).  The mean is bounded from counts at two more
// levels per strip, C = QB + 1 octave (2 b) and D = QB + 2 octaves (4 b), b = lo(QB), a = lo(QA):
// with no cell of the 11 x 13 box at or above D, every ref is < a, < b, < 2 b or < 4 b by its level, so
//   rule B: sum < b (n + C_B + 2 C_C)            <= 255 b   when C_B <= 63, C_C <= 32
//   rule A: sum < a (n + (b/a - 1) C_A + (b/a) C_B + 2 (b/a) C_C)
//                                                <= 252 a   when b <= 1.5 a, C_A <= 80, C_B <= 40, C_C <= 8
// (n = 128; C_A / C_B count refs, C_C / C_D the whole box), and the fp32 tree mean then stays below
// 2 q (the tree sum of 128 non-negative terms is within 2^-21 of the sum).  RTL-compat cells: the
// integer mean floor(sum / n) >> 1 is below the same bound.  NumPy model on the bench's maps (round
// 5 at 56 % / 68 % levels): survivors 1.60 % -> 0.033 % (config 5), 0.014 % -> 0.009 % (config 3);
// at the rules kernel's own levels (below) 0.004 % at config 5 (tools/k3_rules_model.py).
//
// LDS per ring row: two nibble PREFIX rows and a cut-code row (a nibble per cell: key16 < UA, UB, U2A,
// U2B).  A prefix row holds per cell one byte of two 4-bit counters: nibble 0 = #{rows y of the strip
// so far, in its walk order, with key16 >= QA} mod 16, nibble 1 the same for QB (second row: QC / QD),
// with circular halos.  A window's column count (<= 2 HR + 1 = 11 < 16) is then the nibble-wise
// difference of two rows mod 16 (round 5; before: the sum of the 11 rows' level bits, 44 LDS reads
// and 194 adds per lane and step, now 12 reads and 22 nibble differences), at 2.5 B per cell; the
// ring holds one row more (TR + 2 HR + 1) for the difference.  Every rule is exact in its own right; a
// cell that passes none of them goes to K3b (key16(cut) is an upper bound: the rules only ever keep
// more cells).
template <int NC, int HR, int GR> struct LvGeom {
  static constexpr int NT = 256, WPB = 4, WR = DopplerGeom<NC>::WR, TR = WPB * WR, TPR = NC / 16;
  static constexpr int RB = NC + 16;            // prefix row (bytes): cell d (-8 <= d < NC + 8) at byte d + 8
  static constexpr int CS = NC / 2;             // cut-code row (a nibble per cell, no halos)
  static constexpr int ROWB = 2 * RB + CS;      // one ring slot: A / B prefixes, C / D prefixes, cut codes
  static constexpr int NR = TR + 2 * HR + 1;    // ring rows
  static constexpr int N_REF = (2 * HR + 1) * 13 - (2 * GR + 1) * 5;
  static constexpr int HIST = 128 + 16;         // u32: level histogram + counters
  static constexpr int CAPB = 192, CAPT = 64;   // strip buffer: survivor cells, (tile, run) pairs
  static constexpr size_t SMEM = (size_t)NR * ROWB + (HIST + CAPB + 2 * CAPT) * 4;
  static_assert(RB % 16 == 0 && ROWB % 16 == 0 && TR * NC == 16 * NT, "a step's rows are 16 cells per thread");
};
__host__ __device__ constexpr int pidx(int d) { return d + 8; }

template <int NC, int HR, int GR>
constexpr size_t cfar2d_lv_smem_bytes() { return LvGeom<NC, HR, GR>::SMEM; }

// nibble-wise (p + w) mod 16 for w with nibbles 0 / 1
__device__ __forceinline__ uint32_t nib_add(uint32_t p, uint32_t w) { return ((p & 0x77777777u) + w) ^ (p & 0x88888888u); }
// nibble-wise (a - b) mod 16: (a | 8) - (b & 7) never borrows; bit 3 flips where a and b agree in it
__device__ __forceinline__ uint32_t nib_sub(uint32_t a, uint32_t b) {
  return ((a | 0x88888888u) - (b & 0x77777777u)) ^ (~(a ^ b) & 0x88888888u);
}

// The four cut-code flags of 4 cells (kw: their key16 pairs) as a 16-bit word of nibbles (cell j in
// bits 4j .. 4j + 3; bit k = key16 < U_k, W_k = (U_k | 0x8000) - 1 in both halves, as
// cfar2d_screen_lv's CUT side)
__device__ __forceinline__ uint32_t lv_cut_code(uint2 kw, const uint32_t (&W)[4]) {
  uint32_t n = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t f = __builtin_amdgcn_perm(W[k] - kw.y, W[k] - kw.x, 0x07050301u);  // bit 7 of byte j
    n |= (f >> (7 - k)) & (0x01010101u << k);
  }
  const uint32_t t = n | (n >> 4);        // byte 0 = cells 0, 1; byte 2 = cells 2, 3
  return (t & 0xffu) | ((t >> 8) & 0xff00u);
}
// The same when U_1 = QC and U_3 = QD (the default scales, s_min = 2 and s2 = 4: fl(2 lo(QB)) and
// fl(4 lo(QB)) are lo(QB + 128) and lo(QB + 256)): flags 1 and 3 are then the complements of the
// cells' own C / D level bits, which staging has already formed (wcd: byte j bit 0 = key16 >= QC,
// bit 4 = key16 >= QD), so only flags 0 and 2 take compares.
__device__ __forceinline__ uint32_t lv_cut_code_cd(uint2 kw, const uint32_t (&W)[4], uint32_t wcd) {
  uint32_t n = (((wcd << 1) & 0x02020202u) | ((wcd >> 1) & 0x08080808u)) ^ 0x0a0a0a0au;
#pragma unroll
  for (int k = 0; k < 4; k += 2) {
    const uint32_t f = __builtin_amdgcn_perm(W[k] - kw.y, W[k] - kw.x, 0x07050301u);
    n |= (f >> (7 - k)) & (0x01010101u << k);
  }
  const uint32_t t = n | (n >> 4);
  return (t & 0xffu) | ((t >> 8) & 0xff00u);
}

// Survivor bits (bit j: cell d0 + j may detect) of a lane's 16 CUTs from the prefix rows: hiA / loA
// (A / B levels) and hiC / loC (C / D) the 32-byte windows (cells d0 - 8 .. d0 + 23) of the two rows
// whose difference is the window's column counts, hiG / loG those of the guard rows, cw the CUTs' 16
// code nibbles.
template <int HR, int GR>
__device__ __forceinline__ uint32_t cfar2d_screen_prefix(const uint8_t* hiA, const uint8_t* loA, const uint8_t* hiC,
                                                         const uint8_t* loC, const uint8_t* hiG, const uint8_t* loG,
                                                         uint2 cw, int need, bool ruleA) {
  static_assert((2 * HR + 1) * 13 - (2 * GR + 1) * 5 == 128 && 2 * HR + 1 <= 15 && 5 * (2 * GR + 1) <= 15,
                "thresholds below are for n_ref 128");
  uint32_t V[8], G[6], W[8];
  {
    const uint4 a0 = *reinterpret_cast<const uint4*>(hiA), a1 = *reinterpret_cast<const uint4*>(hiA + 16);
    const uint4 b0 = *reinterpret_cast<const uint4*>(loA), b1 = *reinterpret_cast<const uint4*>(loA + 16);
    const uint4 c0 = *reinterpret_cast<const uint4*>(hiC), c1 = *reinterpret_cast<const uint4*>(hiC + 16);
    const uint4 e0 = *reinterpret_cast<const uint4*>(loC), e1 = *reinterpret_cast<const uint4*>(loC + 16);
    const uint4 g0 = *reinterpret_cast<const uint4*>(hiG), g1 = *reinterpret_cast<const uint4*>(hiG + 16);
    const uint4 h0 = *reinterpret_cast<const uint4*>(loG), h1 = *reinterpret_cast<const uint4*>(loG + 16);
    const uint32_t A[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    const uint32_t B[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    const uint32_t C[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    const uint32_t E[8] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
    const uint32_t Gh[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
    const uint32_t Gl[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      V[k] = nib_sub(A[k], B[k]);
      W[k] = nib_sub(C[k], E[k]);
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) G[k] = nib_sub(Gh[k + 1], Gl[k + 1]);
  }
  // 13-cell window sums of levels A and B (bytes: cell d0 + 4m + t in word m byte t).  Levels C and D
  // only enter the rules through upper bounds, so they are counted over supersets of the boxes (the
  // rules hold as well with them): C over the 16 cells around each group of 4 CUTs, D as "any cell of
  // the lane's whole 11 x 32 window at D".  On the bench maps (NumPy model of the rules) the survivors
  // do not change: D cells lie far out in the clutter's tail, C cells are rare enough.
  uint32_t HA[4], HB[4], okC32[4], okC8[4];
  {
    uint32_t XA[7], XB[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const uint32_t w = __builtin_amdgcn_alignbyte(V[k + 1], V[k], 2);
      XA[k] = w & 0x0F0F0F0Fu;
      XB[k] = (w >> 4) & 0x0F0F0F0Fu;
    }
    lv_sum13(XA, HA);
    lv_sum13(XB, HB);
    // C: word k byte t = cell d0 - 6 + 4k + t; group m's 13-cell boxes lie in words m .. m + 3
    uint32_t XC[7], P2[6];
#pragma unroll
    for (int k = 0; k < 7; ++k) XC[k] = __builtin_amdgcn_alignbyte(W[k + 1], W[k], 2) & 0x0F0F0F0Fu;
#pragma unroll
    for (int k = 0; k < 6; ++k) P2[k] = XC[k] + XC[k + 1];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const uint32_t g = __builtin_amdgcn_sad_u8(P2[m] + P2[m + 2], 0u, 0u);  // <= 176
      okC32[m] = g <= 32u ? 0x80808080u : 0u;
      okC8[m] = g <= 8u ? 0x80808080u : 0u;
    }
  }
  const uint32_t orD = (W[0] | W[1] | W[2] | W[3] | W[4] | W[5] | W[6] | W[7]) & 0xF0F0F0F0u;
  const uint32_t okD = orD ? 0u : 0x80808080u;  // bit 7: no D cell in the window (lane-uniform)
  // guard block (3 x 5 around the CUT) of levels A / B in the nibbles
  uint32_t H5[4];
  {
    uint32_t Gp[5], S2[5], S4[4];
#pragma unroll
    for (int k = 0; k < 5; ++k) Gp[k] = __builtin_amdgcn_alignbyte(G[k + 1], G[k], 2);
#pragma unroll
    for (int k = 0; k < 5; ++k) S2[k] = Gp[k] + __builtin_amdgcn_alignbyte(k < 4 ? Gp[k + 1] : 0u, Gp[k], 1);
#pragma unroll
    for (int k = 0; k < 4; ++k) S4[k] = S2[k] + __builtin_amdgcn_alignbyte(S2[k + 1], S2[k], 2);
#pragma unroll
    for (int m = 0; m < 4; ++m) H5[m] = S4[m] + Gp[m + 1];
  }
  constexpr uint32_t H = 0x80808080u;
  auto K = [](int v) { return (uint32_t)v * 0x01010101u; };
  const uint32_t k_need = K(128 - need);
  const uint32_t okA = ruleA ? okD : 0u;
  // the CUTs' code nibbles as bytes: word m byte t = cell 4m + t's code
  const uint32_t cx4 = cw.x >> 4, cy4 = cw.y >> 4;
  uint32_t sv[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const uint32_t src = m < 2 ? cw.x : cw.y, s4 = m < 2 ? cx4 : cy4;
    // bytes (b, b >> 4, b', b' >> 4) of code bytes b = 2 (m & 1), b' = b + 1, then the low nibbles
    const uint32_t nb = __builtin_amdgcn_perm(src, s4, (m & 1) ? 0x03070206u : 0x01050004u) & 0x0F0F0F0Fu;
    const uint32_t CA = HA[m] - (H5[m] & 0x0F0F0F0Fu), CB = HB[m] - ((H5[m] >> 4) & 0x0F0F0F0Fu);
    const uint32_t na = CA + k_need, nb2 = CB + k_need;                     // bit 7: C_A / C_B >= need
    const uint32_t smin = (na & (nb << 7)) | (nb2 & (nb << 6));             // E(s_min) >= need at A or B
    const uint32_t rB = nb2 & ~(CB + K(64)) & okC32[m] & okD & (nb << 4);   // C_B <= 63, C_C <= 32
    const uint32_t rA = na & ~(CA + K(47)) & ~(CB + K(87)) & okC8[m] & okA & (nb << 5);  // 80, 40, 8
    sv[m] = ~(smin | rA | rB) & H;
  }
  // the survivor bits in cell order, only where there are any (a few lanes in a thousand)
  uint32_t bits = 0;
  if (sv[0] | sv[1] | sv[2] | sv[3]) {
#pragma unroll
    for (int m = 0; m < 4; ++m) bits |= ((sv[m] * 0x00204081u) >> 28) << (4 * m);  // bit 7 of byte t -> bit 28 + t
  }
  return bits;
}

// k_cfar2d_lv at NC = 1024 (CMP: the RTL-compat 17-bit integer cells, a.compat, as a template
// switch: the staging's per-row branch cost copies): thread t stages cells 4t .. 4t + 3 of every ring row (NC / 4 = NT), so
// it carries its column's two running prefixes from row to row in registers.  Ring tile row x is
// map row r0 - HR - xo + x (xo = 1 walking downwards, 0 upwards: the extra row lies on the side the
// prefix starts from); the strip's first step stages all NR rows in walk order, every later step
// the TR new ones (prefetched a step ahead: buffer loads whose range check returns the zero rows
// off the map).  For CUT row rl the window's column counts are P[rl + 2 HR + 1] - P[rl] (downwards;
// upwards the prefix runs the other way and the difference flips), the guard rows'
// P[rl + HR + GR + 1] - P[rl + HR - GR], the CUT row is tile row rl + HR + xo.
template <int NC, int HR, int GR, bool CMP>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
k_cfar2d_lv(const float* __restrict__ map, int ns, int n_strips, int steps, int frame0, int tile0, Cfar2DArgs a,
            DetSink sink, Cfar2Cands cands) {
  (void)frame0;
  using Gm = LvGeom<NC, HR, GR>;
  static_assert(NC == 1024 && Gm::WR == 1 && NC / 4 == Gm::NT, "a thread stages one 4-cell column of every row");
  constexpr int WR = Gm::WR, NT = Gm::NT, RB = Gm::RB, ROWB = Gm::ROWB, TPR = Gm::TPR, WPB = Gm::WPB, TR = Gm::TR;
  constexpr int NR = Gm::NR;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem8[];
  uint8_t* const ring = smem8;
  uint32_t* const hist = reinterpret_cast<uint32_t*>(ring + NR * ROWB);
  uint32_t* const cnt = hist + 128;    // [0..3] wave counts, [4] / [5] buffer fill, [6] / [7] list bases,
                                       // [8] / [9] private-region fill
  uint32_t* const buf = cnt + 16;      // the strip's survivor cells (Gm::CAPB)
  uint32_t* const bt = buf + Gm::CAPB; // their wave tiles: (tile, offset << 16 | count) (Gm::CAPT)
  constexpr int CAPB = Gm::CAPB, CAPT = Gm::CAPT;
  // The candidate list takes a strip's survivors in ONE reservation at the strip's end (two atomics):
  // an atomic per wave tile on the launch's two counters -- every workgroup on the same two words --
  // cost ~0.5 ms per launch with ~10^5 survivors (config 5, measured), and round 5's flush of a full
  // LDS buffer (two atomics per flush) and its dense steps (two per wave tile) serialised on those
  // words at 3.0 ms per 16-frame launch on heavy-tailed clutter (round 6, tools/cfar2d_bench.py
  // --maps).  Survivors collect in the LDS buffer (a few per step on radar maps); a full buffer, and a
  // step with more survivors than it holds, go to the strip's PRIVATE region of cands.pcell / .ptile
  // (room for every cell and wave tile of the strip: no atomic), which the strip's end copies behind
  // the buffer's remainder.  pcell / ptile hold (cell) and (rel tile | count << 16, run offset).
  auto spill = [&](uint32_t pc0, uint32_t pt0) {  // uniform: the LDS buffer -> the private region
    const uint32_t n = cnt[4], m = cnt[5], pn = cnt[8], pm = cnt[9];
    if (n == 0u) return;
    for (uint32_t i = threadIdx.x; i < n; i += NT) cands.pcell[pc0 + pn + i] = buf[i];
    for (uint32_t j = threadIdx.x; j < m; j += NT) {
      const uint32_t oc = bt[2 * j + 1];
      cands.ptile[2 * (pt0 + pm + j)] = (bt[2 * j] - (uint32_t)tile0 - pt0) | ((oc & 0xffffu) << 16);
      cands.ptile[2 * (pt0 + pm + j) + 1] = pn + (oc >> 16);
    }
    __syncthreads();  // every thread has read cnt and the buffer
    if (threadIdx.x == 0) {
      cnt[8] = pn + n;
      cnt[9] = pm + m;
      cnt[4] = cnt[5] = 0u;
    }
    __syncthreads();
  };
  auto finish = [&](uint32_t pc0, uint32_t pt0) {  // uniform; the strip's end
    const uint32_t n = cnt[4], m = cnt[5], pn = cnt[8], pm = cnt[9];
    if (n + pn == 0u) return;
    __syncthreads();  // every thread has read cnt[4], [5], [8], [9]
    if (threadIdx.x == 0) {
      cnt[6] = atomicAdd(&cands.ctr[0], n + pn);
      cnt[7] = atomicAdd(&cands.ctr[1], m + pm);
      cnt[4] = cnt[5] = cnt[8] = cnt[9] = 0u;
    }
    __syncthreads();
    const uint32_t p0 = cnt[6], q0 = cnt[7];
    // the private region first (written by this workgroup's waves before the barriers above)
    for (uint32_t i = threadIdx.x; i < pn; i += NT) cands.cell[p0 + i] = cands.pcell[pc0 + i];
    for (uint32_t i = threadIdx.x; i < n; i += NT) cands.cell[p0 + pn + i] = buf[i];
    for (uint32_t j = threadIdx.x; j < pm; j += NT) {
      const uint32_t w0 = cands.ptile[2 * (pt0 + j)], off = cands.ptile[2 * (pt0 + j) + 1];
      const uint32_t wt = (uint32_t)tile0 + pt0 + (w0 & 0xffffu);
      cands.tiles[q0 + j] = wt;
      sink.wg_base[wt] = p0 + off;
      sink.wg_count[wt] = w0 >> 16;
    }
    for (uint32_t j = threadIdx.x; j < m; j += NT) {
      const uint32_t wt = bt[2 * j], oc = bt[2 * j + 1];
      cands.tiles[q0 + pm + j] = wt;
      sink.wg_base[wt] = p0 + pn + (oc >> 16);
      sink.wg_count[wt] = oc & 0xffffu;
    }
    __syncthreads();  // the buffer is free again
  };
  if (threadIdx.x == 0) cnt[4] = cnt[5] = cnt[8] = cnt[9] = 0u;

  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int need = a.n_ref - a.rank;
  const int wt_per_frame = ns / WR;
  const int wg_per_frame = (wt_per_frame + WPB - 1) / WPB;
  const int spf = (wg_per_frame + steps - 1) / steps;
  const int nf = n_strips / spf;
  const int dt = 4 * (int)threadIdx.x;            // this thread's staged cells dt .. dt + 3
  const bool halo_lo = dt < 8, halo_hi = dt >= NC - 8;
  const int d0 = (lane % TPR) * 16;               // the lane's 16 CUTs (row wv of the step)

  // per strip: level words and cut-code thresholds (uniform)
  uint32_t qa2 = 0, qb2 = 0, qc2 = 0, qd2 = 0;
  uint32_t Wc[4] = {0, 0, 0, 0};
  bool ruleA = false;
  bool cd_codes = false;  // U_B == QC and U2_B == QD: lv_cut_code_cd
  // zero-aware strip (most of its first step's cells are +0 or tiny: a sparse or blank map): the
  // screen's survivors lose their +0 CUTs -- E(s) counts every reference of a +0 CUT (refs >= +0), so
  // it cannot detect.  Without it every +0 cell of such a strip survived the level rules (its refs
  // are mostly below every level) and K3b decided all of them: 26.8 ms per 16-frame launch on a map
  // with 98 % zeros (round 6, tools/cfar2d_bench.py --maps sparse).  The filter re-reads the
  // survivors' cells from the map (L2, just staged) behind a uniform branch, so the staging and the
  // screen carry no zero-aware work (as a cut code 0x1 set in staging and ruled out by the screen:
  // 228 against 226 us per config-5 launch on the bench map, profiles/r06/k3_zaware/).
  bool zaware = false;
  uint32_t pab = 0, pcd = 0;  // this column's running prefixes (A / B, C / D)
  // one ring slot's cells dt .. dt + 3: level bits into the prefixes, prefixes and cut codes to LDS
  auto stage = [&](int slot, float4 v) {
    if constexpr (CMP) v = q17x4(v);
    // key16 without the NaN / negative cells (-> 0): a sign or NaN bit pattern is above inf's.  The
    // cut codes use the same keys, so a NaN CUT is screened out: NaN cells are outside the
    // specification (fmcw.h, fmcw_cfar), where the sorting and the counting OS-CFAR disagree
    const uint32_t b0 = __float_as_uint(v.x), b1 = __float_as_uint(v.y), b2 = __float_as_uint(v.z),
                   b3 = __float_as_uint(v.w);
    const uint32_t s0 = b0 <= 0x7f800000u ? b0 : 0u, s1 = b1 <= 0x7f800000u ? b1 : 0u;
    const uint32_t s2 = b2 <= 0x7f800000u ? b2 : 0u, s3 = b3 <= 0x7f800000u ? b3 : 0u;
    const uint2 kw = make_uint2(__builtin_amdgcn_perm(s1, s0, 0x07060302u), __builtin_amdgcn_perm(s3, s2, 0x07060302u));
    const uint32_t wcd = lv_nibbles_add(kw, qc2, qd2);
    pab = nib_add(pab, lv_nibbles_add(kw, qa2, qb2));
    pcd = nib_add(pcd, wcd);
    uint8_t* const rp = ring + slot * ROWB;
    *reinterpret_cast<uint32_t*>(rp + pidx(dt)) = pab;
    *reinterpret_cast<uint32_t*>(rp + RB + pidx(dt)) = pcd;
    if (halo_lo) {
      *reinterpret_cast<uint32_t*>(rp + pidx(dt + NC)) = pab;
      *reinterpret_cast<uint32_t*>(rp + RB + pidx(dt + NC)) = pcd;
    }
    if (halo_hi) {
      *reinterpret_cast<uint32_t*>(rp + pidx(dt - NC)) = pab;
      *reinterpret_cast<uint32_t*>(rp + RB + pidx(dt - NC)) = pcd;
    }
    const uint32_t code = cd_codes ? lv_cut_code_cd(kw, Wc, wcd) : lv_cut_code(kw, Wc);  // (uniform)
    *reinterpret_cast<uint16_t*>(rp + 2 * RB + dt / 2) = (uint16_t)code;
  };

  for (int g = blockIdx.x; g < n_strips; g += gridDim.x) {
    const int f = g % nf;
    const int t_beg = (g / nf) * steps, t_end = min(t_beg + steps, wg_per_frame);
    const float* fm = map + (size_t)f * ns * NC;
    // the frame's map: rows off it (negative offsets wrap) read as zero by the range check
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(fm), (short)0, ns * NC * 4, 0x00020000);
    auto load_row = [&](int row) {  // cells dt .. dt + 3 of map row `row` (uniform)
      return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(row * (NC * 4) + 4 * dt), 0, 0));
    };
    int base = 0;  // ring slot of tile row 0
    float4 pre[TR];
    const bool up = kK3AltDir && ((g / nf) & 1);  // odd strips walk upwards, as k_cfar2d's
    // the strip's private region: its first cell and first wave tile in the launch
    const uint32_t pc0 = ((uint32_t)f * (uint32_t)ns + (uint32_t)(t_beg * TR)) * (uint32_t)NC;
    const uint32_t pt0 = (uint32_t)(f * wt_per_frame + t_beg * WPB);
    const int xo = up ? 0 : 1;
    for (int k = 0; k < t_end - t_beg; ++k) {
      const int t = up ? t_end - 1 - k : t_beg + k;
      const bool first = k == 0, last = k + 1 == t_end - t_beg;
      const int wt0 = t * WPB;
      const int n_wt = min(WPB, wt_per_frame - wt0);
      const int r0 = wt0 * WR;
      const int r = r0 + wv;
      // the previous step's waves are done with the rows: at a strip's start by the barrier after the
      // last strip, later by the emission's barrier (every wave passes it after its screen)
      if (first) __syncthreads();
      if (first) {
        // levels: the mean key7 level of the first step's CUT rows (this thread's 16 cells), then the
        // kK3RulesQA / _QB quantiles of a 128-bin histogram around it
        float4 v[TR];
#pragma unroll
        for (int u = 0; u < TR; ++u) v[u] = load_row(r0 + u);
        if (threadIdx.x == 0) cnt[12] = 0u;
        if (threadIdx.x < 128) hist[threadIdx.x] = 0u;
        uint32_t k7[16];
        uint32_t sum = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float4 w = CMP ? q17x4(v[u]) : nonneg4(v[u]);
          k7[4 * u] = key16(w.x) >> 3;
          k7[4 * u + 1] = key16(w.y) >> 3;
          k7[4 * u + 2] = key16(w.z) >> 3;
          k7[4 * u + 3] = key16(w.w) >> 3;
          sum += k7[4 * u] + k7[4 * u + 1] + k7[4 * u + 2] + k7[4 * u + 3];
        }
#pragma unroll
        for (int x = 32; x >= 1; x >>= 1) sum += (uint32_t)__shfl_xor((int)sum, x, 64);
        __syncthreads();  // counters zeroed
        if (lane == 0) atomicAdd(&cnt[12], sum);
        __syncthreads();
        const int mean7 = (int)(cnt[12] / (uint32_t)(TR * NC));
        const int h0 = mean7 - 64;
#pragma unroll
        for (int i = 0; i < 16; ++i) atomicAdd(&hist[min(max((int)k7[i] - h0, 0), 127)], 1u);
        __syncthreads();
        if (wv == 0) {
          const uint32_t c0 = hist[2 * lane], c1 = hist[2 * lane + 1];
          int tot;
          const uint32_t ex = (uint32_t)wave_excl_scan((int)(c0 + c1), tot);
          const uint32_t cum0 = ex + c0, cum1 = ex + c0 + c1;
          const uint32_t na = (uint32_t)(kK3RulesQA * (TR * NC) / 1000), nb = (uint32_t)(kK3RulesQB * (TR * NC) / 1000);
          const uint64_t ba0 = __ballot(cum0 >= na), ba1 = __ballot(cum1 >= na);
          const uint64_t bb0 = __ballot(cum0 >= nb), bb1 = __ballot(cum1 >= nb);
          auto first_bin = [](uint64_t m0, uint64_t m1) {
            const int l = __builtin_ctzll(m1);
            return (m0 >> l) & 1u ? 2 * l : 2 * l + 1;
          };
          if (lane == 0) {
            cnt[14] = (uint32_t)first_bin(ba0, ba1);
            cnt[15] = (uint32_t)first_bin(bb0, bb1);
          }
        }
        __syncthreads();
        const int h0u = __builtin_amdgcn_readfirstlane(h0);
        const uint32_t QA = (uint32_t)min(max((h0u + (int)__builtin_amdgcn_readfirstlane(cnt[14])) * 8, 1), 0x7f80);
        // B at most 1.5 A (key16 truncates: lo(key16(x)) <= x), at least A
        const uint32_t QB = max(QA, min((uint32_t)min(max((h0u + (int)__builtin_amdgcn_readfirstlane(cnt[15])) * 8, 1), 0x7f80),
                                        key16(1.5f * key_lo(QA))));
        // C / D one and two octaves above QB (exact: key16 + 128 doubles lo); the scale rules need them
        // inside the finite range and no scale override
        const bool s2ok = !a.override_ && QB + 256u < 0x7f80u;
        const uint32_t QC = min(QB + 128u, 0x7f80u), QD = min(QB + 256u, 0x7f80u);
        qa2 = (0x8000u - QA) * 0x00010001u;  // lv_nibbles_add's level constants
        qb2 = (0x8000u - QB) * 0x00010001u;
        qc2 = (0x8000u - QC) * 0x00010001u;
        qd2 = (0x8000u - QD) * 0x00010001u;
        const float s2 = fminf(a.sc_nom, a.sc_max);
        const uint32_t UA = key16(a.s_min * key_lo(QA)), UB = key16(a.s_min * key_lo(QB));
        const uint32_t U2A = s2ok ? key16(s2 * key_lo(QA)) : 0u, U2B = s2ok ? key16(s2 * key_lo(QB)) : 0u;
        ruleA = s2ok && key_lo(QB) <= 1.5f * key_lo(QA);
        // equal thresholds make "key16 < U" and "not key16 >= Q" the same predicate, whatever the scales
        cd_codes = UB == QC && U2B == QD;
        zaware = QA < 16u;  // the 50 % quantile level below 2^-124: at least half the cells are ~zero
        const uint32_t U[4] = {UA, UB, U2A, U2B};
#pragma unroll
        for (int k2 = 0; k2 < 4; ++k2) Wc[k2] = ((U[k2] | 0x8000u) - 1u) * 0x00010001u;
        // the whole ring in walk order (tile rows 0 .. NR - 1 downwards, NR - 1 .. 0 upwards), 4 rows'
        // loads in flight; the prefixes start at the strip's first row
        base = 0;
        pab = pcd = 0u;
#pragma unroll
        for (int j0 = 0; j0 < NR; j0 += 4) {
          float4 w[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int x = up ? NR - 1 - (j0 + u) : j0 + u;
            if (j0 + u < NR) w[u] = load_row(r0 - HR - xo + x);
          }
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (j0 + u < NR) stage(up ? NR - 1 - (j0 + u) : j0 + u, w[u]);
        }
      } else {
        // the ring turns by TR rows; the TR new rows (prefetched in walk order) go into the slots of the
        // rows that left: tile rows NR - TR .. NR - 1 (downwards) or TR - 1 .. 0 (upwards)
        base += up ? NR - TR : TR;
        if (base >= NR) base -= NR;
#pragma unroll
        for (int j = 0; j < TR; ++j) {
          int x = (up ? TR - 1 - j : NR - TR + j) + base;
          x = x >= NR ? x - NR : x;
          stage(x, pre[j]);
        }
      }
      if (!last) {  // prefetch the next step's new rows in walk order: r0 + TR + HR + j or r0 - HR - 1 - j
#pragma unroll
        for (int j = 0; j < TR; ++j) pre[j] = load_row(up ? r0 - HR - 1 - j : r0 + TR + HR + j);
      }
      __syncthreads();
      const bool has_tile = wv < n_wt;
      uint32_t surv = 0;
      if (has_tile && r >= HR && r < ns - HR) {
        auto slot = [&](int x) {
          const int y = x + base;
          return y >= NR ? y - NR : y;
        };
        const uint8_t* const p_lo = ring + slot(wv) * ROWB + d0;                // pidx(d0 - 8) = d0
        const uint8_t* const p_hi = ring + slot(wv + 2 * HR + 1) * ROWB + d0;
        const uint8_t* const g_lo = ring + slot(wv + HR - GR) * ROWB + d0;
        const uint8_t* const g_hi = ring + slot(wv + HR + GR + 1) * ROWB + d0;
        const uint2 cw = *reinterpret_cast<const uint2*>(ring + slot(wv + HR + xo) * ROWB + 2 * RB + d0 / 2);
        const uint8_t* const hA = up ? p_lo : p_hi;
        const uint8_t* const lA = up ? p_hi : p_lo;
        const uint8_t* const hG = up ? g_lo : g_hi;
        const uint8_t* const lG = up ? g_hi : g_lo;
        surv = cfar2d_screen_prefix<HR, GR>(hA, lA, hA + RB, lA + RB, hG, lG, cw, need, ruleA);
        if (zaware && surv) {  // uniform flag: drop the +0 CUTs, re-read from the map (L2: just staged)
          uint32_t z = 0;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            float4 q = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)((r * NC + d0 + 4 * u) * 4), 0, 0));
            if constexpr (CMP) q = q17x4(q);
            const float e[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const uint32_t b = __float_as_uint(e[j]);  // s == 0 after staging's sanitising
              z |= (b == 0u || b > 0x7f800000u ? 1u : 0u) << (4 * u + j);
            }
          }
          surv &= ~z;
        }
      }
      // emission: each wave tile's survivors, in (range, doppler) order, as one run of the strip
      // buffer (flushed to the candidate list when full and at the strip's end); an empty tile is
      // final here.  (wg_base, wg_count) = (run start, run length) until k_cfar2d_emit.
      const int wtile = tile0 + f * wt_per_frame + wt0 + wv;
      int k_w = 0;
      const int ex = wave_excl_scan(has_tile ? __popc(surv) : 0, k_w);
      if (lane == 0) cnt[wv] = (uint32_t)k_w;
      if (has_tile && k_w == 0 && lane == 0) {
        sink.wg_base[wtile] = (uint32_t)wtile * sink.slot_cap;
        sink.wg_count[wtile] = 0u;
      }
      __syncthreads();
      uint32_t T = 0, woff = 0, ti = 0, nt = 0;
#pragma unroll
      for (int i = 0; i < WPB; ++i) {
        const uint32_t c = cnt[i];
        woff += i < wv ? c : 0u;
        ti += (i < wv && c) ? 1u : 0u;
        T += c;
        nt += c ? 1u : 0u;
      }
      if (T != 0u) {  // uniform
        if (cnt[4] + T > (uint32_t)CAPB || cnt[5] + nt > (uint32_t)CAPT) spill(pc0, pt0);
        const uint32_t bn = cnt[4], tn = cnt[5];
        const uint32_t cbase = ((uint32_t)f * (uint32_t)ns + (uint32_t)r) * (uint32_t)NC + (uint32_t)d0;
        if (T > (uint32_t)CAPB) {  // a dense step: straight into the private region (the buffer is empty)
          if (k_w) {
            const uint32_t pn = cnt[8] + woff, pm = cnt[9] + ti;
            if (lane == 0) {
              cands.ptile[2 * (pt0 + pm)] = ((uint32_t)wtile - (uint32_t)tile0 - pt0) | ((uint32_t)k_w << 16);
              cands.ptile[2 * (pt0 + pm) + 1] = pn;
            }
            uint32_t o = pc0 + pn + (uint32_t)ex;
            for (uint32_t m = surv; m; m &= m - 1, ++o) cands.pcell[o] = cbase + (uint32_t)__builtin_ctz(m);
          }
        } else if (k_w) {
          uint32_t o = bn + woff + (uint32_t)ex;
          for (uint32_t m = surv; m; m &= m - 1, ++o) buf[o] = cbase + (uint32_t)__builtin_ctz(m);
          if (lane == 0) {
            bt[2 * (tn + ti)] = (uint32_t)wtile;
            bt[2 * (tn + ti) + 1] = ((bn + woff) << 16) | (uint32_t)k_w;
          }
        }
        __syncthreads();  // every thread has read cnt[0 .. 9]
        if (threadIdx.x == 0) {
          if (T <= (uint32_t)CAPB) {
            cnt[4] = bn + T;
            cnt[5] = tn + nt;
          } else {
            cnt[8] += T;
            cnt[9] += nt;
          }
        }
      }
    }  // steps
    __syncthreads();
    finish(pc0, pt0);  // the strip's runs into the candidate list
  }    // strips
}

// ---- K3b: the exact decision of every candidate of a launch, one whole wave per candidate, all
// waves of the GPU sharing the list (round 4: inside k_cfar2d the 4 waves of the workgroup that
// met a target's rows decided its dozens of candidates one after the other, and that step set the
// critical path of the launch).  On the exact fp32 cells of the map: lanes hold refs l and l + 64 of
// the fixed order (dr ascending outer, dd ascending inner, guard block skipped; oracle
// cfar2d_offsets); the mean is the fixed fp32 halving tree (one add, then xor-shuffles 32..1 ==
// oracle tree_sum_f32); the scale bracket comes from ballot counts (ranked > M <=> #{ref > M} >=
// n_ref - k; os_cfar_2d.vhd:189-213); detect <=> #{fl(s ref) >= cut} < n_ref - k; a detection's
// ranked value (k-th smallest) by the pivoting select, threshold = fl(s ranked) (dbg_threshold).
// The fixed fp32 halving tree of a wave's values (xor partners 32, 16, .., 1: oracle tree_sum_f32),
// every lane ending with the sum.  Steps 8 .. 1 are DPP row rotations: after the steps above it, the
// lane a rotation by x reaches holds the xor partner's value bit for bit (fp32 addition commutes).
__device__ __forceinline__ float wave_tree_sum(float s, int a32, int a16) {
  s += __int_as_float(__builtin_amdgcn_ds_bpermute(a32, __float_as_int(s)));
  s += __int_as_float(__builtin_amdgcn_ds_bpermute(a16, __float_as_int(s)));
  s += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s), 0x128, 0xf, 0xf, false));  // row_ror:8
  s += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s), 0x124, 0xf, 0xf, false));  // row_ror:4
  s += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s), 0x122, 0xf, 0xf, false));  // row_ror:2
  s += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s), 0x121, 0xf, 0xf, false));  // row_ror:1
  return s;
}
__device__ __forceinline__ int ballot_count(bool p) { return __popcll(__builtin_amdgcn_ballot_w64(p)); }

template <int NC, bool CMP>
__device__ __forceinline__ void cfar2d_decide_run(const float* __restrict__ map, const Cfar2DArgs& a,
                                                  const Cfar2Cands& cands) {
  const int lane = threadIdx.x & 63;
  int dra, dda, drb, ddb;
  cfar2d_ref_offset(a, lane, dra, dda);
  cfar2d_ref_offset(a, lane + 64, drb, ddb);
  const bool oka = lane < a.n_ref, okb = lane + 64 < a.n_ref;
  const int need = a.n_ref - a.rank;
  const int a32 = (lane ^ 32) * 4, a16 = (lane ^ 16) * 4;
  // fl(sum / n): with n a power of two the product with 1 / n is the same correctly rounded value
  const bool n_pow2 = (a.n_ref & (a.n_ref - 1)) == 0;
  const float inv_n = 1.0f / (float)a.n_ref;
  const uint32_t n = cands.ctr[0];
  const uint32_t w0 = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
  auto cell = [](float v) { return CMP ? q17(v) : nonneg(v); };
  // Software-pipelined (round 5): the next candidate's cut and refs are in flight while this one is
  // decided, the one after next's cell index a step earlier still (the refs' addresses depend on it);
  // the windows mostly come from HBM / MALL again, K3a having streamed the launch's frames through.
  // (Branch-free: lanes past n_ref read their row's first cell and the last candidate stands in past
  // the list's end, so the waits can count the loads in flight.)
  struct Pend {
    float cut, va, vb;
  };
  auto fetch = [&](uint32_t c) {  // c = (f ns + r) NC + d; rows r + dr stay inside the frame
    const uint32_t fr = c / (uint32_t)NC, d = c & (uint32_t)(NC - 1);
    Pend p;
    p.cut = map[c];  // c in a VGPR (opaque below): a vector load, counted with the refs'
    p.va = map[oka ? (fr + dra) * (uint32_t)NC + ((d + dda) & (uint32_t)(NC - 1)) : fr * (uint32_t)NC];
    p.vb = map[okb ? (fr + drb) * (uint32_t)NC + ((d + ddb) & (uint32_t)(NC - 1)) : fr * (uint32_t)NC];
    return p;
  };
  // the loop counter is scalar; the cell indices are read by vector loads (opaque lane offsets), so
  // that the shuffles' LDS waits do not also wait for them
  uint32_t i = __builtin_amdgcn_readfirstlane(w0);
  if (i >= n) return;
  const uint32_t* const cl = cands.cell;
  uint32_t c_next = cl[opaque(0) + min(i + nw, n - 1)];
  Pend cur = fetch(cl[opaque(0) + i]);
  for (; i < n; i += nw) {
    const uint32_t c_after = cl[opaque(0) + min(i + 2 * nw, n - 1)];
    const Pend nxt = fetch(c_next);
    const float cut = cell(cur.cut);
    const float va = oka ? cell(cur.va) : 0.f;
    const float vb = okb ? cell(cur.vb) : 0.f;
    cur = nxt;
    c_next = c_after;
    const float sum = wave_tree_sum(va + vb, a32, a16);
    float sc = (float)a.override_;
    if (!a.override_) {
      float half, hi;
      if constexpr (CMP) {
        // integer cells < 2^17, <= 128 of them: every partial sum < 2^24 is exact in fp32.
        // mean = floor(sum / N_REF) (os_cfar_2d.vhd:189); the bracket add is 17 bits wide (:193)
        const uint32_t mean = (uint32_t)sum / (uint32_t)a.n_ref;
        half = (float)(mean >> 1);
        hi = (float)((mean + (mean >> 1)) & kQ17Mask);
      } else {
        const float mean = n_pow2 ? sum * inv_n : sum / (float)a.n_ref;
        half = mean * 0.5f;
        hi = mean + half;
      }
      const int n_hi = ballot_count(oka && va > hi) + ballot_count(okb && vb > hi);
      const int n_lo = ballot_count(oka && va < half) + ballot_count(okb && vb < half);
      sc = (n_hi >= need) ? a.sc_max : (n_lo >= a.rank + 1) ? a.sc_min : a.sc_nom;
    }
    const int n_ge = ballot_count(oka && sc * va >= cut) + ballot_count(okb && sc * vb >= cut);
    float thr = -1.f;
    if (n_ge < need) {  // uniform
      const uint32_t ranked = wave_select_kth(oka ? __float_as_uint(va) : 0u, okb ? __float_as_uint(vb) : 0u,
                                              __ballot(oka), __ballot(okb), a.rank);
      thr = sc * __uint_as_float(ranked);
    }
    if (lane == 0) cands.thr[i] = thr;
  }
}
template <int NC>
__global__ void __launch_bounds__(256)
k_cfar2d_decide(const float* __restrict__ map, int ns, Cfar2DArgs a, Cfar2Cands cands) {
  (void)ns;
  if (a.compat) cfar2d_decide_run<NC, true>(map, a, cands);
  else cfar2d_decide_run<NC, false>(map, a, cands);
}

// ---- K3c: per wave tile with candidates, its detections in order into the sink (det_reserve_wave:
// the tile's slot, or the overflow region).  One lane per tile first (round 5): most tiles' few
// candidates were all rejected, and such a tile is final with (slot, 0) -- a wave per tile spent
// three dependent loads on each.  Tiles with detections, or with more than kEmitLaneRun candidates,
// then go through the whole wave one after the other, 64 candidates per round.
constexpr uint32_t kEmitLaneRun = 8;
template <int NC>
__global__ void __launch_bounds__(256)
k_cfar2d_emit(const float* __restrict__ map, int ns, int frame0, Cfar2DArgs a, Cfar2Cands cands, DetSink sink) {
  const int lane = threadIdx.x & 63;
  const uint32_t nt = cands.ctr[1];
  const uint32_t w0 = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
  // lane l of wave w takes list entries w + nw (l + 64 i): consecutive entries (a target's tiles,
  // which carry the detections) go to different waves
  for (uint32_t t0 = 0; t0 < nt; t0 += nw * 64u) {
    const uint32_t ti = t0 + (uint32_t)lane * nw + w0;
    int tile = 0;
    uint32_t p0 = 0, k = 0;
    bool wave = false;
    if (ti < nt) {
      tile = (int)cands.tiles[ti];
      p0 = sink.wg_base[tile];  // the candidate run (k_cfar2d)
      k = sink.wg_count[tile];
      bool det = k > kEmitLaneRun;
      float t[kEmitLaneRun];
#pragma unroll
      for (uint32_t j = 0; j < kEmitLaneRun; ++j) t[j] = cands.thr[p0 + min(j, k - 1u)];  // k >= 1
#pragma unroll
      for (uint32_t j = 0; j < kEmitLaneRun; ++j) det |= t[j] >= 0.f;
      if (det) {
        wave = true;
      } else {
        sink.wg_base[tile] = (uint32_t)tile * sink.slot_cap;
        sink.wg_count[tile] = 0u;
      }
    }
    for (uint64_t m = __ballot(wave); m; m &= m - 1) {  // uniform
      const int l = __builtin_ctzll(m);
      const int tl = __shfl(tile, l, 64);
      const uint32_t pl = (uint32_t)__shfl((int)p0, l, 64), kl = (uint32_t)__shfl((int)k, l, 64);
      int total = 0;
      for (uint32_t j0 = 0; j0 < kl; j0 += 64) {
        const bool det = j0 + lane < kl && cands.thr[pl + j0 + lane] >= 0.f;
        total += (int)__popcll(__ballot(det));
      }
      const uint32_t base = det_reserve_wave(sink, tl, total);
      uint32_t o = base;
      for (uint32_t j0 = 0; j0 < kl && total; j0 += 64) {
        const uint32_t j = j0 + lane;
        const float thr = j < kl ? cands.thr[pl + j] : -1.f;
        const uint64_t bal = __ballot(thr >= 0.f);
        if (thr >= 0.f) {
          const uint32_t slot = o + (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
          if (slot < sink.cap) {
            const uint32_t c = cands.cell[pl + j];
            const uint32_t fr = c / (uint32_t)NC;
            const float v = map[c];
            fmcw_det dd;
            dd.frame = (uint32_t)frame0 + fr / (uint32_t)ns;
            dd.range = (uint16_t)(fr % (uint32_t)ns);
            dd.doppler = (uint16_t)(c & (uint32_t)(NC - 1));
            dd.mag = a.compat ? q17(v) : nonneg(v);
            dd.threshold = thr;
            sink.scratch[slot] = dd;
          }
        }
        o += (uint32_t)__popcll(bal);
      }
    }
  }
}
