// cfar2d.hpp -- K3: 2-D OS-CFAR (rtl/src/os_cfar_2d.vhd:140-217) over the linear magnitude
// map, for gfx950.  Included by kernels.hpp (needs DetSink, det_reserve, block_excl_scan1).
//
// One workgroup = TR = 4096/NC CUT rows x all NC Doppler cells of one frame; rows
// r0-hr .. r0+TR-1+hr sit in LDS, each row padded one float per 16 (index pad16(d)), so
// lanes that start 16 cells apart hit distinct banks.  Doppler is circular; a CUT row is
// tested only if its whole range extent lies inside the map (build spec).
//
// Phase A (every cell): thread t owns 16 consecutive cells of one row.  For each of the
// 2 hr + 1 window rows it loads that row's 16 + 2 hd span once, scales it by s_min, and
// counts for each of its 16 CUTs the refs with fl(s_min * ref) >= cut (guard rows skip
// |dd| <= gd).  #{..} >= n_ref - k proves cut <= fl(s * ranked) for every admissible scale
// s >= s_min, so the cell cannot detect; the rest (survivors) go to a bitmap.
// Phase B (survivors, in (row, doppler) order): one whole wave per cell.  Lanes hold refs
// l and l + 64 (fixed order: dr outer, dd inner); the mean is the fixed fp32 halving tree
// (one add + xor-shuffles 32..1 == oracle tree_sum_f32); the scale bracket from ballot counts
// (ranked > M <=> #{ref > M} >= n_ref - k; ranked < M' <=> #{ref < M'} >= k + 1); detect
// <=> #{fl(s * ref) >= cut} < n_ref - k; for detections the exact ranked value by a 32-step
// radix select over order-preserving keys (threshold = fl(s * ranked), dbg_threshold).
//
// Included from inside namespace fmcw by kernels.hpp (uses DetSink, det_reserve,
// block_excl_scan1, opaque, pad16 declared there).
#pragma once

struct Cfar2DArgs {
  int hr, gr, hd, gd;  // half extents (ref + guard) and guards, range / Doppler
  int n_ref, rank;
  float s_min, sc_min, sc_nom, sc_max;
  int override_;
};

template <int NC> struct Cfar2DGeom {
  static constexpr int NT = 256;
  static constexpr int TR = 4096 / NC;   // CUT rows per workgroup (4096 cells, 16 per thread)
  static constexpr int CW = 4096 / 4;    // cells per wave
  static constexpr int RS = padded(NC);  // LDS row stride (floats)
  static constexpr int TPR = NC / 16;    // threads per row
};

__device__ __forceinline__ uint32_t f2key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

template <int NC>
constexpr size_t cfar2d_smem_bytes(int hr) {
  using G = Cfar2DGeom<NC>;
  return (size_t)(G::TR + 2 * hr) * G::RS * 4      // tile
         + (size_t)G::TR * NC / 16 * 2               // survivor bitmap (u16 per 16 cells)
         + 4 * (size_t)G::CW * 8                     // per-wave detection lists
         + 128 * 4 + 16 * 4;                         // offsets, scan scratch
}

// Phase A for a compile-time Doppler extent HD / guard GD; returns this thread's survivor bits.
template <int NC, int HD, int GD>
__device__ __forceinline__ uint32_t cfar2d_phase_a(const float* tile, int rl, int d0, const Cfar2DArgs& a,
                                                   int need) {
  constexpr int RS = Cfar2DGeom<NC>::RS;
  constexpr int W = 16 + 2 * HD;
  const float* crow = tile + (rl + a.hr) * RS;
  uint32_t cb[16], lt[16];   // cut bits; #{fl(s_min * ref) < cut} (lt_bit: no SGPR masks)
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    cb[i] = __float_as_uint(crow[pad16(d0 + i)]);
    lt[i] = 0;
  }
  for (int dr = -a.hr; dr <= a.hr; ++dr) {
    const float* row = crow + dr * RS;
    uint32_t sb[W];
#pragma unroll
    for (int k = 0; k < W; ++k) sb[k] = __float_as_uint(a.s_min * row[pad16((d0 - HD + k) & (NC - 1))]);
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
  // survivor <=> #{fl(s_min * ref) >= cut} < need  <=>  lt > n_ref - need
  uint32_t bits = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) bits |= ((int)lt[i] > a.n_ref - need ? 1u : 0u) << i;
  return bits;
}

// Phase A, runtime geometry (any window the LDS budget allows).
template <int NC>
__device__ __forceinline__ uint32_t cfar2d_phase_a_generic(const float* tile, int rl, int d0,
                                                           const Cfar2DArgs& a, int need) {
  constexpr int RS = Cfar2DGeom<NC>::RS;
  const float* crow = tile + (rl + a.hr) * RS;
  uint32_t bits = 0;
  for (int i = 0; i < 16; ++i) {
    const int d = d0 + i;
    const uint32_t c = __float_as_uint(crow[pad16(d)]);
    uint32_t lt = 0;
    for (int dr = -a.hr; dr <= a.hr; ++dr) {
      const float* row = crow + dr * RS;
      const bool grow = dr >= -a.gr && dr <= a.gr;
      for (int dd = -a.hd; dd <= a.hd; ++dd) {
        if (grow && dd >= -a.gd && dd <= a.gd) continue;
        lt += lt_bit(__float_as_uint(a.s_min * row[pad16((d + dd) & (NC - 1))]), c);
      }
    }
    bits |= ((int)lt > a.n_ref - need ? 1u : 0u) << i;
  }
  return bits;
}

template <int NC, int HD, int GD>
__global__ void __launch_bounds__(256)
k_cfar2d(const float* __restrict__ map, int ns, int n_tiles, int frame0, int tile0, Cfar2DArgs a,
         DetSink sink) {
  using Gm = Cfar2DGeom<NC>;
  constexpr int TR = Gm::TR, CW = Gm::CW, NT = Gm::NT, RS = Gm::RS, TPR = Gm::TPR;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int rows_in = TR + 2 * a.hr;
  float* tile = smem;
  uint16_t* surv = reinterpret_cast<uint16_t*>(tile + rows_in * RS);
  uint2* lists = reinterpret_cast<uint2*>(surv + TR * NC / 16);     // 8-B aligned: TR*NC/16*2 % 8 == 0
  short2* offs = reinterpret_cast<short2*>(lists + 4 * CW);
  int* s_scan = reinterpret_cast<int*>(offs + 128);

  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // reference-cell offsets in the fixed order (dr outer, dd inner, guard skipped)
  if (threadIdx.x == 0) {
    int n = 0;
    for (int dr = -a.hr; dr <= a.hr; ++dr)
      for (int dd = -a.hd; dd <= a.hd; ++dd) {
        if (dr >= -a.gr && dr <= a.gr && dd >= -a.gd && dd <= a.gd) continue;
        offs[n++] = make_short2((short)dr, (short)dd);
      }
  }
  const int need = a.n_ref - a.rank;
  const int tiles_per_frame = (ns + TR - 1) / TR;

  for (int tl = blockIdx.x; tl < n_tiles; tl += gridDim.x) {
    const int tid = opaque(threadIdx.x);
    const int f = tl / tiles_per_frame;
    const int r0 = (tl - f * tiles_per_frame) * TR;
    __syncthreads();
    // load rows r0-hr .. r0+TR+hr-1 (zero outside the map), padded
    const float* fm = map + (size_t)f * ns * NC;
    for (int e = 4 * tid; e < rows_in * NC; e += 4 * NT) {
      const int rl = e / NC, d = e - rl * NC;
      const int r = r0 - a.hr + rl;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r >= 0 && r < ns) v = *reinterpret_cast<const float4*>(fm + (size_t)r * NC + d);
      float* dst = tile + rl * RS + pad16(d);  // d % 4 == 0: the 4 floats share a 16-block
      dst[0] = v.x;
      dst[1] = v.y;
      dst[2] = v.z;
      dst[3] = v.w;
    }
    __syncthreads();

    // Phase A
    {
      const int rl = tid / TPR, d0 = (tid % TPR) * 16;
      const int r = r0 + rl;
      uint32_t bits = 0;
      if (r >= a.hr && r < ns - a.hr) {
        if constexpr (HD > 0)
          bits = cfar2d_phase_a<NC, HD, GD>(tile, rl, d0, a, need);
        else
          bits = cfar2d_phase_a_generic<NC>(tile, rl, d0, a, need);
      }
      surv[tid] = (uint16_t)bits;  // word tid covers cells tid*16 .. tid*16+15
    }
    __syncthreads();

    // Phase B: wave wv walks its 64 words (= its 1024 cells) in cell order
    int ndet = 0;
    uint2* mylist = lists + wv * CW;
    const uint32_t word = surv[wv * 64 + lane];
    uint64_t nz = __ballot(word != 0);
    while (nz) {
      const int l0 = __builtin_ctzll(nz);
      nz &= nz - 1;
      uint32_t bits = (uint32_t)__shfl((int)word, l0, 64);
      while (bits) {
        const int i = __builtin_ctz(bits);
        bits &= bits - 1;
        const int cell = (wv * 64 + l0) * 16 + i;
        const int rl = cell / NC, d = cell - rl * NC;
        const float* crow = tile + (rl + a.hr) * RS;
        const float cut = crow[pad16(d)];
        float va = 0.f, vb = 0.f;
        const bool oka = lane < a.n_ref, okb = lane + 64 < a.n_ref;
        if (oka) { const short2 o = offs[lane]; va = crow[o.x * RS + pad16((d + o.y) & (NC - 1))]; }
        if (okb) { const short2 o = offs[lane + 64]; vb = crow[o.x * RS + pad16((d + o.y) & (NC - 1))]; }
        float sum = va + vb;
#pragma unroll
        for (int x = 32; x >= 1; x >>= 1) sum += __shfl_xor(sum, x, 64);
        const float mean = sum / (float)a.n_ref;
        float sc;
        if (a.override_) {
          sc = (float)a.override_;
        } else {
          const float half = mean * 0.5f;
          const float hi = mean + half;
          const int n_hi = __popcll(__ballot(oka && va > hi)) + __popcll(__ballot(okb && vb > hi));
          const int n_lo = __popcll(__ballot(oka && va < half)) + __popcll(__ballot(okb && vb < half));
          sc = (n_hi >= need) ? a.sc_max : (n_lo >= a.rank + 1) ? a.sc_min : a.sc_nom;
        }
        const int n_ge = __popcll(__ballot(oka && sc * va >= cut)) + __popcll(__ballot(okb && sc * vb >= cut));
        if (n_ge < need) {
          // exact k-th smallest (k = rank) by radix select on order keys
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
          if (lane == 0) mylist[ndet] = make_uint2((uint32_t)cell, __float_as_uint(sc * key2f(prefix)));
          ++ndet;
        }
      }
    }
    // ordered emission: waves in row order, each list in cell order
    int total;
    const int excl = block_excl_scan1<NT>(lane == 0 ? ndet : 0, s_scan, total);
    const int wexcl = __shfl(excl, 0, 64);
    const uint32_t base = det_reserve(sink, tile0 + tl, total, s_scan + NT / 64 + 1);
    for (int i = lane; i < ndet; i += 64) {
      const uint2 rec = mylist[i];
      const uint32_t slot = base + (uint32_t)(wexcl + i);
      if (slot < sink.cap) {
        const int cell = (int)rec.x;
        const int rl = cell / NC, d = cell - rl * NC;
        fmcw_det dd;
        dd.frame = (uint32_t)(frame0 + f);
        dd.range = (uint16_t)(r0 + rl);
        dd.doppler = (uint16_t)d;
        dd.mag = tile[(rl + a.hr) * RS + pad16(d)];
        dd.threshold = __uint_as_float(rec.y);
        sink.scratch[slot] = dd;
      }
    }
  }
}
