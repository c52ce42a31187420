// pair.hpp -- K12p k_pair: K1 of chunk c and K2 of chunk c - 1 in ONE launch.
// Included from inside namespace fmcw by kernels.hpp (k_range's and k_doppler's building blocks).
//
// Why.  K1 (window + range FFT + corner turn) streams HBM; K2 (Doppler FFT + |X| + map + 1-D
// OS-CFAR) is VALU-bound (round 2 SQ counters: ~75 % of the issue slots) and reads its spectrum
// from the Infinity Cache when the chunk fits there (auto_chunk).  Back to back, each kernel
// leaves the other's resource idle and every launch pays its own ramp and tail.  Here one
// launch holds both, with no dependency between them: K1 writes chunk c's spectrum into buffer
// c % 2 while K2 reads chunk c - 1's from buffer (c - 1) % 2 (written by the previous launch; the
// kernel boundary is the only synchronisation, as between K1 and K2 today).  Every workgroup
// alternates a K1 item (T chirps of one frame) and a K2 item (4 wave tiles of one frame), so
// the waves on a CU mix HBM streaming with FFT / CFAR arithmetic.
//
// The reference's analogue is the ping-pong corner turner (rtl/src/corner_turner.vhd:98-166):
// the range stage fills one bank while the Doppler stage drains the other.
//
// Both halves are k_range / k_doppler's code paths (MTI off, one rx, FAST K2: |X|, no dB map,
// 1-D CFAR at the reference geometry or none); the results are bit-identical to K1 + K2.
#pragma once

struct PairArgs {
  // K1 half: chunk c (n_groups = 0 in the last launch)
  const void* cube;        // chunk c's frames [frame][chirp][sample]
  float2* inter_w;         // spectrum buffer written (k_range's tiled corner-turn layout)
  const float* win_r;      // range window [N]
  const float* chirp_w;    // Doppler window [NC], folded into the range stage
  int n_groups;            // chirp groups of T chirps
  // K2 half: chunk c - 1 (n_tiles = 0 in the first launch)
  const float2* inter_r;   // spectrum buffer read
  int n_tiles;             // Doppler wave tiles (WR range rows x NC cells each)
  int frame0, tile0;       // chunk c - 1's first frame / wave tile in the batch
  float* lin_map;          // chunk c - 1's linear map [frame][range][doppler], or null
  Cfar1DArgs cf;
  DetSink sink;
};

template <int N, int NC> struct PairGeom {
  using RG = RangeGeom<N>;
  using DG = DopplerGeom<NC>;
  static constexpr int LDS_A = RG::T * RG::REG * 2;   // floats
  static constexpr int LDS_B = DG::WPB * DG::WFL;
  static constexpr int LDS = LDS_A > LDS_B ? LDS_A : LDS_B;
  static constexpr bool OK = RG::NT == 256 && DG::NT == 256 && !RG::WG_SYNC;
};

#ifndef FMCW_PAIR_K2PF   // K2 unit's points loaded during the K1 item before it (1) or at its start (0)
#define FMCW_PAIR_K2PF 0
#endif
#ifndef FMCW_PAIR_WAVES  // waves per SIMD asked of the register allocator
#define FMCW_PAIR_WAVES 3
#endif
template <int N, int NC, typename LD>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FMCW_PAIR_WAVES)))
k_pair(PairArgs a) {
  using G = PairGeom<N, NC>;
  static_assert(G::OK, "pair geometry: 256-thread range and Doppler workgroups");
  using RG = RangeGeom<N>;
  using DG = DopplerGeom<NC>;
  __shared__ __attribute__((aligned(16))) float ldsf[G::LDS];

  // ---------------- K1 state (k_range) ----------------
  constexpr int P1 = RG::P, T = RG::T, RB = RG::RB, REG = RG::REG;
  constexpr int ncb = NC / T;
  float2* const lds1 = reinterpret_cast<float2*>(ldsf);
  const int tid = threadIdx.x;
  const int q = tid / P1;
  const int t10 = tid % P1;
  const int e0 = 2 * tid;
  const int chunk0 = e0 / (RB * T);
  const int win0 = e0 - chunk0 * (RB * T);
  const int r0c = chunk0 * RB + win0 / T;
  const int c0 = win0 % T;
  constexpr int CI = T * N / 1024;
  const int rd0_off = c0 * REG + pad16(r0c);
  auto cw_index = [](int i) { return P1 >= 64 ? __builtin_amdgcn_readfirstlane(i) : i; };

  // ---------------- K2 state (k_doppler, FAST, MTI off, one rx) ----------------
  constexpr int P2 = DG::P, WR = DG::WR, WPB = DG::WPB, REGD = DG::REGD, REGM = DG::REGM;
  constexpr int LR = DG::LR, LG = DG::LG;
  constexpr int lgT = __builtin_ctz(T), lgRB = __builtin_ctz(RB), lgncb = __builtin_ctz(NC) - lgT;
  constexpr int TPF = N / WR;                       // wave tiles per frame
  static_assert(TPF % WPB == 0, "whole workgroup units per frame");
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane0 = tid & 63;
  const int rr = lane0 / P2;
  const int t20 = lane0 % P2;
  float* const mags = ldsf + wv * DG::WFL;
  float2* const wreg = reinterpret_cast<float2*>(mags);
  uint32_t* const list = reinterpret_cast<uint32_t*>(mags + DG::LIST);
  constexpr bool TWH = NC / 16 <= 16 && P2 % 16 == 0;
  GroupTwiddles<NC / 16, NC> twh;
  if constexpr (TWH) twh.init(t20 & 15);
  const int n_units = a.n_tiles / WPB;
  const int nf2 = a.n_tiles / TPF;                  // frames of the K2 half

  // K2 unit u (WPB consecutive wave tiles of one frame, frame-minor over units: k_doppler's
  // FMCW_K2_ORDER 1) -> this wave's tile: frame f, first range row r0
  auto unit_tile = [&](int u, int& f, int& lt) {
    f = u % nf2;
    lt = (u / nf2) * WPB + wv;
  };
  // the 16 points c = t + P m of this lane's range row of wave tile (f, lt)
  float2 nxt[16];
  auto load_tile = [&](int u) {
    int f, lt;
    unit_tile(u, f, lt);
    const int r = lt * WR + rr;
    const uint32_t rbase = (uint32_t)(r >> lgRB) << lgncb;
    const uint32_t rin = (uint32_t)(r & ((1 << lgRB) - 1));
    const float2* src = a.inter_r + (size_t)f * N * NC;
    const int tq = opaque(t20);
    if constexpr ((P2 & (T - 1)) == 0) {
      const float2* p = src + ((((rbase + ((uint32_t)tq >> lgT)) << lgRB) + rin) << lgT) +
                        ((uint32_t)tq & (uint32_t)(T - 1));
      constexpr uint32_t S = (uint32_t)(P2 >> lgT) << (lgRB + lgT);
#pragma unroll
      for (int m = 0; m < 16; ++m) nxt[m] = ld_f2<FMCW_NT_SPEC_LD>(p + (size_t)m * S);
    } else {
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const uint32_t c = (uint32_t)(tq + P2 * m);
        nxt[m] = ld_f2<FMCW_NT_SPEC_LD>(src + (((((rbase + (c >> lgT)) << lgRB) + rin) << lgT) | (c & (uint32_t)(T - 1))));
      }
    }
  };

  // K1 prefetch registers: the next K1 item's raw samples, loaded during the current one
  typename LD::Raw in[8];
  float cw_n = 1.f;
  auto load_group = [&](int g) {
    const int fr = g / ncb;
    const int cb = g - fr * ncb;
    const size_t chirp = (size_t)fr * NC + (size_t)cb * T + q;
    const int t = opaque(t10);
#pragma unroll
    for (int m = 0; m < 8; ++m) in[m] = LD::fetch(a.cube, chirp * N + 2 * t + (N / 8) * m);
    if (a.chirp_w) cw_n = a.chirp_w[cw_index(cb * T + q)];
  };

  const int Gd = (int)gridDim.x;
  const int b = (int)blockIdx.x;
  if (b < a.n_groups) load_group(b);
  // half the workgroups of each XCD (ids b, b + 8, ... land on XCD b % 8) start with K2
  const int first = (b >> 3) & 1;
  const int jmax = max((a.n_groups + Gd - 1) / Gd, (n_units + Gd - 1) / Gd);
  bool have_tile = false;  // nxt holds this workgroup's next K2 unit

  for (int h = 0; h < 2 * jmax; ++h) {
    const int i = (h >> 1) * Gd + b;
    if (((h + first) & 1) == 0) {
      // ======================= K1 item: chirp group i =======================
      if (i >= a.n_groups) continue;  // uniform
      const int fr = i / ncb;
      const int cb = i - fr * ncb;
      const int t = opaque(t10);
      float2* buf = lds1 + q * REG;
      const float cw = cw_n;
      // range window re-read per item (L1 / L2 hits): held across the K2 items it would cost
      // 16 VGPRs at the register peak
      float2 wh[8];
#pragma unroll
      for (int m = 0; m < 8; ++m) wh[m] = *reinterpret_cast<const float2*>(a.win_r + 2 * t + (N / 8) * m);
      __syncthreads();  // the previous item's LDS reads (K1 tiles, K2 wave regions) are done
      float4 ax[8];
#pragma unroll
      for (int m = 0; m < 8; ++m) ax[m] = LD::expand(in[m]);
      // the K2 unit that follows this item streams in behind it (issued after the wait for this
      // item's samples: vmcnt counts in issue order)
      {
        const int i2 = ((h + 1) >> 1) * Gd + b;
        if (FMCW_PAIR_K2PF && !have_tile && h + 1 < 2 * jmax && i2 < n_units) {
          load_tile(i2);
          have_tile = true;
        }
      }
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        float2 v[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          const float we = (e ? wh[m].y : wh[m].x) * cw;
          v[m] = e ? make_float2(ax[m].z * we, ax[m].w * we) : make_float2(ax[m].x * we, ax[m].y * we);
        }
        Dft<8>::run(v);
        float2* d = buf + pad16((2 * t + e) * 8);
#pragma unroll
        for (int m = 0; m < 8; ++m) d[m] = v[m];
      }
      if (i + Gd < a.n_groups) load_group(i + Gd);
      pass_sync<false>();
      stockham_from<N, 8, P1, false>(buf, t);
      __syncthreads();
      const float2* rd0 = lds1 + opaque(rd0_off);
      const size_t dbase = (size_t)fr * N * NC + ((size_t)chunk0 * ncb + cb) * (RB * T) + win0;
      float2* dst = a.inter_w + dbase;
      const size_t dstep = (size_t)CI * ncb * (RB * T);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float2 v0, v1;
        if constexpr ((N / 8) % 16 == 0) {
          v0 = rd0[padoff(k * (N / 8))];
          v1 = rd0[REG + padoff(k * (N / 8))];
        } else {
          v0 = lds1[c0 * REG + pad16(r0c + k * (N / 8))];
          v1 = lds1[(c0 + 1) * REG + pad16(r0c + k * (N / 8))];
        }
        st_f4<FMCW_NT_SPEC_ST>(dst + k * dstep, make_float4(v0.x, v0.y, v1.x, v1.y));
      }
      __syncthreads();  // K2's wave regions overlap these chirp rows
    } else {
      // ======================= K2 item: unit i (one wave tile per wave) =======================
      if (i >= n_units) continue;  // uniform
      if (!have_tile) load_tile(i);
      have_tile = false;
      int f, lt;
      unit_tile(i, f, lt);
      const int t = opaque(t20);
      const int r0 = lt * WR;
      float2* buf = wreg + rr * REGD;
      float2 v[16];
#pragma unroll
      for (int m = 0; m < 16; ++m) v[m] = nxt[m];
      Dft<16>::run(v);  // pass 1: L = 1, no twiddles
      {
        float2* d = buf + pad16(16 * t);
#pragma unroll
        for (int m = 0; m < 16; ++m) d[m] = v[m];
      }
      pass_sync<false>();
      float2 X[LG][LR];
      if constexpr (TWH) stockham_last_tw<NC, 16, P2>(buf, t, X, twh);
      else stockham_to_regs<NC, 16, P2, false>(buf, t, X);
      float acc[LG][LR];
#pragma unroll
      for (int g = 0; g < LG; ++g)
#pragma unroll
        for (int m = 0; m < LR; ++m) acc[g][m] = cabs2(X[g][m]);
      pass_sync<false>();  // every read of the last pass is issued: the rows may be rewritten
      float* mrow = mags + rr * REGM;
#pragma unroll
      for (int g = 0; g < LG; ++g) {
        float* m0 = mrow + midx(t + P2 * g);
#pragma unroll
        for (int m = 0; m < LR; ++m) m0[mpadoff(m * (NC / LR))] = mag_sqrt(acc[g][m]);
      }
      pass_sync<false>();
      if (a.cf.enabled) {
        fill_halo<NC, P2>(mrow, t);
        pass_sync<false>();
      }
      if (a.lin_map) {
        constexpr int Q = WR * NC / 4 / 64;
        const size_t mbase = ((size_t)f * N + r0) * NC;
        const int lane = opaque(lane0);
#pragma unroll
        for (int k = 0; k < Q; ++k) {
          const int e = 4 * (lane + 64 * k);
          const int rl = e / NC, d = e - rl * NC;
          st_f4<FMCW_NT_MAP>(a.lin_map + mbase + e, *reinterpret_cast<const float4*>(mags + rl * REGM + midx(d)));
        }
      }
      if (a.cf.enabled)
        cfar1d_wave<NC, 8, 2, true>(mags, list, rr, t, r0, a.frame0 + f, a.tile0 + f * TPF + lt, a.cf, a.sink);
      pass_sync<false>();
    }
  }
}
