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

__device__ __forceinline__ uint32_t f2key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

#ifndef FMCW_CFAR2D_SCREEN  // phase A as pair screen + exact count of the survivors (1) or exact (0)
#define FMCW_CFAR2D_SCREEN 1
#endif
constexpr int kCfar2dList = 128;  // u32 per wave after the rows: 64 survivor cells + 64 verdicts

template <int NC>
constexpr size_t cfar2d_smem_bytes(int hr) {
  using G = Cfar2DGeom<NC>;
  return (size_t)(G::TR + 2 * hr) * G::RS * 4 + (FMCW_CFAR2D_SCREEN ? G::WPB * kCfar2dList * 4 : 0);
}

// Phase A screen (compile-time HD / GD): disjoint PAIRS of Doppler-adjacent references.  A pair
// with fl(s_min * min) >= cut holds 2 references with fl(s_min * ref) >= cut (fl(s x) is
// monotone), so 2 * #{such pairs} is a lower bound on the exact count and a cell whose bound
// reaches n_ref - k cannot detect.  A reference row of 2 HD + 1 cells gives HD pairs (its last
// cell is left out), a guard row two segments of HD - GD cells, (HD - GD) / 2 pairs each.
// On noise + targets about 5 % of the cells pass (0.6 % pass the exact count) at half the
// compares; the survivors are then counted exactly, one per lane.
template <int NC, int HD, int GD>
__device__ __forceinline__ uint32_t cfar2d_screen(const float* tile, int rl, int d0, const Cfar2DArgs& a,
                                                  int need) {
  constexpr int RS = Cfar2DGeom<NC>::RS;
  static_assert(HD <= MH, "the window stays inside the row halos");
  constexpr int W = 16 + 2 * HD;
  constexpr int O0 = floor4(-HD);
  constexpr int NV = (W + (-HD - O0) + 3) / 4;
  constexpr int SEG = HD - GD, NPS = SEG / 2;   // guard-row segment length, pairs per segment
  const float* lb = tile + (rl + a.hr) * RS + midx(d0);
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
    load_cells<NV>(lb + dr * RS, O0, v);
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

// Exact phase-A test of one cell (CUT row rl of the group tile, Doppler d): candidate <=>
// #{fl(s_min * ref) >= cut} < need.  Addresses: midx(d + dd) with a runtime d.
template <int NC, int HD, int GD>
__device__ __forceinline__ bool cfar2d_exact_a(const float* tile, int rl, int d, const Cfar2DArgs& a, int need) {
  constexpr int RS = Cfar2DGeom<NC>::RS;
  const float* crow = tile + (rl + a.hr) * RS;
  const int x = d + MH;
  auto at = [&](const float* row, int dd) { return row[(x + dd) + (((x + dd) >> 4) << 2)]; };
  const uint32_t cbits = __float_as_uint(at(crow, 0));
  uint32_t lt = 0;
  for (int dr = -a.hr; dr <= a.hr; ++dr) {
    const float* row = crow + dr * RS;
    if (dr >= -a.gr && dr <= a.gr) {
#pragma unroll
      for (int dd = -HD; dd <= HD; ++dd)
        if (dd < -GD || dd > GD) lt += lt_bit(__float_as_uint(a.s_min * at(row, dd)), cbits);
    } else {
#pragma unroll
      for (int dd = -HD; dd <= HD; ++dd) lt += lt_bit(__float_as_uint(a.s_min * at(row, dd)), cbits);
    }
  }
  return (int)lt > a.n_ref - need;
}

// Phase A for a compile-time Doppler extent HD / guard GD; returns this lane's candidate bits.
// `rl` is the CUT row within the workgroup tile (tile row rl + hr).
template <int NC, int HD, int GD>
__device__ __forceinline__ uint32_t cfar2d_phase_a(const float* tile, int rl, int d0, const Cfar2DArgs& a,
                                                   int need) {
  constexpr int RS = Cfar2DGeom<NC>::RS;
  static_assert(HD <= MH, "the window stays inside the row halos");
  constexpr int W = 16 + 2 * HD;
  constexpr int O0 = floor4(-HD);
  constexpr int NV = (W + (-HD - O0) + 3) / 4;
  const float* lb = tile + (rl + a.hr) * RS + midx(d0);
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
    load_cells<NV>(lb + dr * RS, O0, v);
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
__device__ __forceinline__ uint32_t cfar2d_phase_a_generic(const float* tile, int rl, int d0,
                                                           const Cfar2DArgs& a, int need) {
  constexpr int RS = Cfar2DGeom<NC>::RS;
  const float* crow = tile + (rl + a.hr) * RS;
  uint32_t bits = 0;
  for (int i = 0; i < 16; ++i) {
    const int d = d0 + i;
    const uint32_t c = __float_as_uint(crow[midx(d)]);
    uint32_t lt = 0;
    for (int dr = -a.hr; dr <= a.hr; ++dr) {
      const float* row = crow + dr * RS;
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

template <int NC, int HD, int GD>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3)))
k_cfar2d(const float* __restrict__ map, int ns, int n_wg_tiles, int frame0, int tile0, Cfar2DArgs a,
         DetSink sink) {
  using Gm = Cfar2DGeom<NC>;
  constexpr int WR = Gm::WR, NT = Gm::NT, RS = Gm::RS, TPR = Gm::TPR, WPB = Gm::WPB;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* const tile = smem;

  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // this lane's two reference cells (index lane and lane + 64 of the fixed order)
  int dra, dda, drb, ddb;
  cfar2d_ref_offset(a, lane, dra, dda);
  cfar2d_ref_offset(a, lane + 64, drb, ddb);
  const bool oka = lane < a.n_ref, okb = lane + 64 < a.n_ref;
  const int offa = dra * RS, offb = drb * RS;
  const int need = a.n_ref - a.rank;
  const int wt_per_frame = ns / WR;                      // wave tiles per frame
  const int wg_per_frame = (wt_per_frame + WPB - 1) / WPB;
  const int nf = n_wg_tiles / wg_per_frame;

  for (int g = blockIdx.x; g < n_wg_tiles; g += gridDim.x) {
    // frame-minor order (as K2): hot rows (targets) spread over all workgroups
    const int f = g % nf;
    const int wt0 = (g / nf) * WPB;                      // first wave tile of this group
    const int n_wt = min(WPB, wt_per_frame - wt0);
    const int r0 = wt0 * WR;                             // first CUT row of this group
    const int rows_in = n_wt * WR + 2 * a.hr;
    const int tid = opaque(threadIdx.x);
    __syncthreads();  // the previous group's waves are done with the rows
    {
      // rows r0-hr .. r0+n_wt*WR+hr-1 (zero outside the map), 4 float4 loads in flight per lane
      const float* fm = map + (size_t)f * ns * NC;
      const int n4 = rows_in * (NC / 4);
      for (int b = tid; b < n4; b += 4 * NT) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int e4 = b + u * NT;
          const int rl = e4 / (NC / 4), d = (e4 - rl * (NC / 4)) * 4;
          const int r = r0 - a.hr + rl;
          v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
          if (e4 < n4 && r >= 0 && r < ns) v[u] = *reinterpret_cast<const float4*>(fm + (size_t)r * NC + d);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int e4 = b + u * NT;
          if (e4 < n4) {
            const int rl = e4 / (NC / 4), d = (e4 - rl * (NC / 4)) * 4;
            *reinterpret_cast<float4*>(tile + rl * RS + midx(d)) = a.compat ? q17x4(v[u]) : nonneg4(v[u]);
          }
        }
      }
    }
    __syncthreads();
    for (int e = tid; e < rows_in * 2 * MH; e += NT) {   // circular Doppler halos
      const int rl = e / (2 * MH), j = e - rl * (2 * MH);
      const int dst = j < MH ? NC + j : j - 2 * MH;
      const int src = j < MH ? j : NC + j - 2 * MH;
      tile[rl * RS + midx(dst)] = tile[rl * RS + midx(src)];
    }
    __syncthreads();
    if (wv >= n_wt) continue;  // uniform per wave: no wave tile left in this frame

    // ---- Phase A: candidates among this lane's 16 cells
    const int rlw = wv * WR + lane / TPR;    // CUT row within the group tile
    const int d0 = (lane % TPR) * 16;
    const int r = r0 + rlw;
    uint32_t cand = 0;
    if (r >= a.hr && r < ns - a.hr) {
      if constexpr (HD > 0) {
        if constexpr (FMCW_CFAR2D_SCREEN) cand = cfar2d_screen<NC, HD, GD>(tile, rlw, d0, a, need);
        else cand = cfar2d_phase_a<NC, HD, GD>(tile, rlw, d0, a, need);
      } else {
        cand = cfar2d_phase_a_generic<NC>(tile, rlw, d0, a, need);
      }
    }
    if constexpr (HD > 0 && FMCW_CFAR2D_SCREEN) {
      // survivors of the screen -> exact test, 64 per round, one per lane, in cell order
      uint32_t* const lst = reinterpret_cast<uint32_t*>(tile + (Gm::TR + 2 * a.hr) * RS) + wv * kCfar2dList;
      uint32_t* const ver = lst + 64;
      const uint32_t scr = cand;
      cand = 0;
      int n_s;
      const int sx = wave_excl_scan(__popc(scr), n_s);
      for (int base_s = 0; base_s < n_s; base_s += 64) {  // uniform
        {
          int o = sx;
          for (uint32_t m = scr; m; m &= m - 1, ++o)
            if (o >= base_s && o < base_s + 64) lst[o - base_s] = ((uint32_t)lane << 4) | (uint32_t)__builtin_ctz(m);
        }
        pass_sync<false>();
        if (base_s + lane < n_s) {
          const uint32_t e = lst[lane];
          const int src = (int)(e >> 4), i = (int)(e & 15u);
          ver[lane] = cfar2d_exact_a<NC, HD, GD>(tile, wv * WR + src / TPR, (src % TPR) * 16 + i, a, need) ? 1u : 0u;
        }
        pass_sync<false>();
        {
          int o = sx;
          for (uint32_t m = scr; m; m &= m - 1, ++o)
            if (o >= base_s && o < base_s + 64 && ver[o - base_s]) cand |= 1u << __builtin_ctz(m);
        }
        pass_sync<false>();  // the next round rewrites lst / ver
      }
    }

    // ---- Phase B helpers: the wave's view of candidate cell (row l0 / TPR of the wave, d)
    auto refs_of = [&](int l0, int d, float& va, float& vb) {
      const float* crow = tile + (wv * WR + l0 / TPR + a.hr) * RS;
      va = oka ? crow[offa + midx((d + dda) & (NC - 1))] : 0.f;
      vb = okb ? crow[offb + midx((d + ddb) & (NC - 1))] : 0.f;
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

    // ---- Phase B pass 1: decide every candidate (cell order); detections -> owner's bits
    uint32_t detw = 0;
    {
      uint64_t nz = __ballot(cand != 0);
      while (nz) {
        const int l0 = __builtin_ctzll(nz);
        nz &= nz - 1;
        uint32_t bits = (uint32_t)__shfl((int)cand, l0, 64);
        while (bits) {
          const int i = __builtin_ctz(bits);
          bits &= bits - 1;
          const int d = (l0 % TPR) * 16 + i;
          const float cut = tile[(wv * WR + l0 / TPR + a.hr) * RS + midx(d)];
          float va, vb;
          refs_of(l0, d, va, vb);
          const float sc = scale_of(va, vb);
          const int n_ge = __popcll(__ballot(oka && sc * va >= cut)) + __popcll(__ballot(okb && sc * vb >= cut));
          if (n_ge < need && lane == l0) detw |= 1u << i;
        }
      }
    }
    int total;
    (void)wave_excl_scan(__popc(detw), total);
    const int wtile = tile0 + f * wt_per_frame + wt0 + wv;
    const uint32_t base = det_reserve_wave(sink, wtile, total);

    // ---- Phase B pass 2: exact ranked value (k-th smallest) of each detection, in order
    uint32_t o = 0;
    uint64_t nz = __ballot(detw != 0);
    while (nz) {
      const int l0 = __builtin_ctzll(nz);
      nz &= nz - 1;
      uint32_t bits = (uint32_t)__shfl((int)detw, l0, 64);
      while (bits) {
        const int i = __builtin_ctz(bits);
        bits &= bits - 1;
        const int d = (l0 % TPR) * 16 + i;
        const int rl = wv * WR + l0 / TPR;
        float va, vb;
        refs_of(l0, d, va, vb);
        const float sc = scale_of(va, vb);
        const uint32_t ka = f2key(va), kb = f2key(vb);
        uint32_t prefix = 0;
        int k = a.rank;
        for (int bit = 31; bit >= 0; --bit) {
          const uint32_t hmask = bit == 31 ? 0u : ~((2u << bit) - 1u);
          const bool za = oka && ((ka & hmask) == prefix) && !((ka >> bit) & 1u);
          const bool zb = okb && ((kb & hmask) == prefix) && !((kb >> bit) & 1u);
          const int c0 = __popcll(__ballot(za)) + __popcll(__ballot(zb));
          if (k >= c0) {
            k -= c0;
            prefix |= 1u << bit;
          }
        }
        const uint32_t slot = base + o;
        if (lane == 0 && slot < sink.cap) {
          fmcw_det dd;
          dd.frame = (uint32_t)(frame0 + f);
          dd.range = (uint16_t)(r0 + rl);
          dd.doppler = (uint16_t)d;
          dd.mag = tile[(rl + a.hr) * RS + midx(d)];
          dd.threshold = sc * key2f(prefix);
          sink.scratch[slot] = dd;
        }
        ++o;
      }
    }
  }
}
