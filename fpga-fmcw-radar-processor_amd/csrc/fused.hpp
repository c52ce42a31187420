// fused.hpp -- K12 k_fused: window + range FFT + corner turn + Doppler FFT + |X| + map + 1-D
// OS-CFAR in ONE persistent launch, with the corner-turned spectrum kept in the XCD's L2.
// Included from inside namespace fmcw by kernels.hpp (uses k_range's and k_doppler's building
// blocks, RangeGeom / DopplerGeom, DetSink, cfar1d_dispatch).
//
// Why.  K1 -> HBM -> K2 moves 7 MiB per config-2 frame (2 MiB cube in, 2 MiB spectrum out,
// 2 MiB spectrum back in, 1 MiB map out); only 3 MiB are compulsory.  The reference keeps the
// corner turn on chip in a ping-pong BRAM (rtl/src/corner_turner.vhd:98-166).  The MI355X
// analogue: one frame's spectrum (2 MiB) fits one XCD's 4 MiB L2, which is write-back for
// plain stores (tools/l2_probe.hip, profiles/r02/l2_probe_pmc.json: 32 rewrites of a 2 MiB
// region per XCD leave L2 once, at the end of the kernel).
//
// Structure.  The launch is 8 independent frame engines, one per XCD.  Each workgroup reads
// its XCD id from the hardware (HW_REG_XCC_ID) and claims a slot in its XCD's group, so the
// grouping is a hardware fact, never an assumption about dispatch order.  Frames f = x, x + 8,
// ... (local index k) go to XCD x through a ring of kRing spectrum slots S[x][k % kRing]:
//   role A (range, n_a workgroups): k_range's body on chirp groups u = slot, slot + n_a, ...
//          of each frame; before its first store of frame k into slot k % kRing it waits until
//          every Doppler wave has loaded frame k - kRing from that slot; after its last store:
//          s_waitcnt vmcnt, barrier, ready[slot] += 1.
//   role B (Doppler, n_b workgroups of 4 independent waves): wave w takes wave tile
//          (w + 37 k) mod (4 n_b) of frame k (a rotation, so the tiles that hold targets and
//          take longest visit every wave), loads its 16 points per lane from S with
//          L1-bypassing (nt) loads as soon as ready[slot] says the frame is stored -- normally
//          while it is still computing frame k - 1, into its prefetch registers -- then
//          s_waitcnt, freed[slot] += 1, and runs k_doppler's body (FFT, |X|, map, CFAR).
// The ring lets the range side run kRing frames ahead of the Doppler side, so the two roles
// overlap like independent kernels (HBM-streaming range work beside VALU-heavy Doppler work
// on the same CUs) instead of alternating.  A slot is written and read on ONE XCD: the
// spectrum lives in that XCD's L2 (and, once evicted, as write-backs in the Infinity Cache,
// 8 x kRing x 2 MiB = 64 MiB at config 2), never needing a cross-XCD release.
// Hand-off (MI355X_MICROARCH.md, workgroup visibility): producer plain stores -> every storing
// wave's s_waitcnt vmcnt -> workgroup barrier -> one relaxed agent-scope atomic add; consumer:
// relaxed agent-scope atomic-load poll -> nt loads, which are served by the (shared) L2 and
// never by the reading CU's L1.  Producer and consumer share the L2 by construction (same XCC
// id), and a line the L2 evicts is written back before anyone can miss on it.
// Every wait is bounded; a timeout sets the error word and every workgroup drains
// (fmcw_process reports it and re-runs the batch on K1 + K2).
#pragma once

#ifndef FMCW_RING
#define FMCW_RING 4
#endif
constexpr int kRing = FMCW_RING;  // spectrum slots per XCD

struct FusedCtl {  // word offsets in the control block (zeroed before every launch)
  static constexpr int kLine = 32;  // uint32 per 128-B line: every counter on its own line
  static constexpr int kPerX = 2 + 2 * kRing;
  __host__ __device__ static constexpr int join(int x) { return x * kPerX * kLine; }
  __host__ __device__ static constexpr int claim(int x) { return (x * kPerX + 1 + 2 * kRing) * kLine; }
  __host__ __device__ static constexpr int ready(int x, int s) { return (x * kPerX + 1 + s) * kLine; }
  __host__ __device__ static constexpr int freed(int x, int s) { return (x * kPerX + 1 + kRing + s) * kLine; }
  static constexpr int kErr = 8 * kPerX * kLine;
  static constexpr int kWords = kErr + kLine;
};

struct FusedArgs {
  const void* cube;        // [n_frames][NC][N] complex samples
  float2* spec;            // 8 x kRing frame slots S[x][s], k_range's tiled corner-turn layout
  const float* win_r;      // range window [N]
  const float* chirp_w;    // Doppler window [NC], folded into the range stage (linearity)
  float* lin_map;          // [n_frames][N][NC] or null
  float* db_map;           // or null
  uint32_t* ctl;           // FusedCtl
  int n_frames, frame0, tile0;
  int per_xcd, n_a, n_b;   // workgroups per XCD group; range (A) and Doppler (B) roles
  int mag_mode;
  int census;              // 1: only join, check the group sizes and co-residency, exit
  uint32_t spin_limit;     // polls before a wait gives up (sets the error word)
  Cfar1DArgs cf;
  DetSink sink;
  uint64_t* trace;         // diagnostics (FMCW_FUSED_TRACE): [x][k < kTraceFrames][8] timestamps
};
constexpr int kTraceFrames = 64;

// 100 MHz real-time counter; trace slot (x, k, e) written by thread 0 of the tracing workgroup
__device__ __forceinline__ void fused_trace(const FusedArgs& a, int x, int k, int e) {
  if (a.trace && k < kTraceFrames && threadIdx.x == 0)
    a.trace[((size_t)x * kTraceFrames + k) * 8 + e] = __builtin_amdgcn_s_memrealtime();
}

__device__ __forceinline__ int xcc_id() {
  int x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 7;
}

__device__ __forceinline__ uint32_t ctl_load(const uint32_t* ctl, int w) {
  return __hip_atomic_load(ctl + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ctl_add(uint32_t* ctl, int w, uint32_t v) {
  __hip_atomic_fetch_add(ctl + w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One lane polls ctl[w] >= target.  Returns false on the error word or on timeout (which then
// sets the error word, so every other waiter leaves too).
__device__ __forceinline__ bool fused_wait(uint32_t* ctl, int w, uint32_t target, uint32_t limit) {
  for (uint32_t spins = 0;; ++spins) {
    if (ctl_load(ctl, w) >= target) return true;
    if (ctl_load(ctl, FusedCtl::kErr)) return false;
    if (spins >= limit) {
      __hip_atomic_store(ctl + FusedCtl::kErr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

template <int N, int NC> struct FusedGeom {
  using RG = RangeGeom<N>;
  using DG = DopplerGeom<NC>;
  static constexpr int UPF = NC / RG::T;      // range units (T chirps) per frame
  static constexpr int WTPF = N / DG::WR;     // Doppler wave tiles per frame
  static constexpr int LDS_A = RG::T * RG::REG * 2;
  static constexpr int LDS_B = DG::WPB * DG::WFL;
  static constexpr int LDS = LDS_A > LDS_B ? LDS_A : LDS_B;  // floats
  static constexpr bool OK = RG::NT == 256 && DG::NT == 256 && (size_t)N * NC * 8 <= (2u << 20);
};

// ---- role A: k_range's body over this workgroup's chirp groups of each frame ------------
template <int N, int NC, typename LD>
__device__ __forceinline__ void fused_range_role(const FusedArgs& a, int x, int ai, int nk, float* ldsf,
                                                 int* s_fail) {
  using Gm = RangeGeom<N>;
  constexpr int P = Gm::P, T = Gm::T, RB = Gm::RB, REG = Gm::REG;
  constexpr int UPF = NC / T, ncb = NC / T;
  float2* const lds = reinterpret_cast<float2*>(ldsf);
  const int tid = threadIdx.x;
  const int q = tid / P;
  const int t0 = tid % P;
  const int e0 = 2 * tid;
  const int chunk0 = e0 / (RB * T);
  const int win0 = e0 - chunk0 * (RB * T);
  const int r0 = chunk0 * RB + win0 / T;
  const int c0 = win0 % T;
  constexpr int CI = T * N / 1024;
  const int rd0_off = c0 * REG + pad16(r0);
  constexpr uint32_t WTPF = N / DopplerGeom<NC>::WR;  // Doppler wave tiles: one freed count each

  float4 in[8];
  auto load_job = [&](int k, int u) {
    const size_t chirp = (size_t)(x + 8 * k) * NC + (size_t)u * T + q;
    const int t = opaque(t0);
#pragma unroll
    for (int m = 0; m < 8; ++m) in[m] = LD::load2(a.cube, chirp * N + 2 * t + (N / 8) * m);
  };
  if (ai < UPF && nk > 0) load_job(0, ai);
  const bool tr = ai == 0, tr_last = ai == a.n_a - 1;
  for (int k = 0; k < nk; ++k) {
    if (tr) fused_trace(a, x, k, 0);
    const int sl = k % kRing;
    float2* const S = a.spec + ((size_t)x * kRing + sl) * N * NC;
    for (int u = ai; u < UPF; u += a.n_a) {
      const int t = opaque(t0);
      float2* buf = lds + q * REG;
      const float cw = a.chirp_w ? a.chirp_w[u * T + q] : 1.f;
      float2 w[8];
#pragma unroll
      for (int m = 0; m < 8; ++m) w[m] = *reinterpret_cast<const float2*>(a.win_r + 2 * t + (N / 8) * m);
      __syncthreads();  // the previous unit's transposed reads are done with lds
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        float2 v[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          const float we = (e ? w[m].y : w[m].x) * cw;
          v[m] = e ? make_float2(in[m].z * we, in[m].w * we) : make_float2(in[m].x * we, in[m].y * we);
        }
        Dft<8>::run(v);
        float2* d = buf + pad16((2 * t + e) * 8);
#pragma unroll
        for (int m = 0; m < 8; ++m) d[m] = v[m];
      }
      const bool last = u + a.n_a >= UPF;  // last unit of this frame for this workgroup
      if (!last) load_job(k, u + a.n_a);   // prefetch within the frame, behind the FFT
      pass_sync<Gm::WG_SYNC>();
      stockham_from<N, 8, P, Gm::WG_SYNC>(buf, t);
      __syncthreads();
      if (u == ai && k >= kRing) {  // first store of frame k: every wave has read frame k - kRing
        if (tid == 0 && !fused_wait(a.ctl, FusedCtl::freed(x, sl), WTPF * (uint32_t)(k / kRing), a.spin_limit))
          *s_fail = 1;
        __syncthreads();
        if (*s_fail) return;
      }
      if (tr && u == ai) fused_trace(a, x, k, 1);
      // tiled corner turn into S[x]: plain stores, resident in this XCD's L2
      const float2* rd0 = lds + opaque(rd0_off);
      float2* dst = S + ((size_t)chunk0 * ncb + u) * (RB * T) + win0;
      const size_t dstep = (size_t)CI * ncb * (RB * T);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float2 v0, v1;
        if constexpr ((N / 8) % 16 == 0) {
          v0 = rd0[padoff(i * (N / 8))];
          v1 = rd0[REG + padoff(i * (N / 8))];
        } else {
          v0 = lds[c0 * REG + pad16(r0 + i * (N / 8))];
          v1 = lds[(c0 + 1) * REG + pad16(r0 + i * (N / 8))];
        }
        st_f4<false>(dst + i * dstep, make_float4(v0.x, v0.y, v1.x, v1.y));
      }
      if (last) {
        // the next frame's first unit is loaded AFTER the stores, so vmcnt (in order for loads
        // and stores) can wait for the stores alone while those loads stay in flight
        asm volatile("" ::: "memory");
        if (k + 1 < nk) {
          load_job(k + 1, ai);
          asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        if (tid == 0) ctl_add(a.ctl, FusedCtl::ready(x, sl), 1u);
        if (tr) fused_trace(a, x, k, 2);
        if (tr_last) fused_trace(a, x, k, 7);
      }
    }
  }
}

// ---- role B: k_doppler's body (MTI off, one rx), waves independent, rotating wave tiles ---
template <int N, int NC>
__device__ __forceinline__ void fused_doppler_role(const FusedArgs& a, int x, int bi, int nk, float* ldsf) {
  using Gm = DopplerGeom<NC>;
  using RG = RangeGeom<N>;
  constexpr int P = Gm::P, WR = Gm::WR, REGD = Gm::REGD, REGM = Gm::REGM;
  constexpr int LR = Gm::LR, LG = Gm::LG;
  constexpr int WTPF = N / WR;
  constexpr int T = RG::T, RB = RG::RB;
  constexpr int lgT = __builtin_ctz(T), lgRB = __builtin_ctz(RB), lgncb = __builtin_ctz(NC) - lgT;
  const int tid = threadIdx.x;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane0 = tid & 63;
  const int rr = lane0 / P;
  const int t0 = lane0 % P;
  float* const mags = ldsf + wv * Gm::WFL;
  float2* const wreg = reinterpret_cast<float2*>(mags);
  uint32_t* const list = reinterpret_cast<uint32_t*>(mags + Gm::LIST);
  constexpr bool TWH = NC / 16 <= 16 && P % 16 == 0;
  GroupTwiddles<NC / 16, NC> twh;
  if constexpr (TWH) twh.init(t0 & 15);
  // this wave's 16 points of tile vt of frame k: chirps c = t + P m of row r
  auto load_tile = [&](int k, int vt, float2 (&dst)[16]) {
    const float2* S = a.spec + ((size_t)x * kRing + k % kRing) * N * NC;
    const int r = vt * WR + rr;
    const uint32_t rbase = (uint32_t)(r >> lgRB) << lgncb;
    const uint32_t rin = (uint32_t)(r & ((1 << lgRB) - 1));
    const int tq = opaque(t0);
    if constexpr ((P & (T - 1)) == 0) {
      const float2* p = S + ((((rbase + ((uint32_t)tq >> lgT)) << lgRB) + rin) << lgT) +
                        ((uint32_t)tq & (uint32_t)(T - 1));
      constexpr uint32_t SM = (uint32_t)(P >> lgT) << (lgRB + lgT);
#pragma unroll
      for (int m = 0; m < 16; ++m) dst[m] = ld_f2<true>(p + (size_t)m * SM);
    } else {
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const uint32_t c = (uint32_t)(tq + P * m);
        dst[m] = ld_f2<true>(S + (((((rbase + (c >> lgT)) << lgRB) + rin) << lgT) | (c & (uint32_t)(T - 1))));
      }
    }
  };
  auto ready_target = [&](int k) { return (uint32_t)a.n_a * (uint32_t)(k / kRing + 1); };
  auto signal_freed = [&](int k) {
    if (lane0 == 0) ctl_add(a.ctl, FusedCtl::freed(x, k % kRing), 1u);
  };
  // Doppler work queue of this XCD: tile id = k * WTPF + wave tile, claimed in order by
  // whichever wave is free (one returning atomic per tile), so a wave that drew a slow tile
  // (targets: many CFAR survivors) never holds the others back
  auto claim = [&]() -> uint32_t {
    uint32_t v = 0;
    if (lane0 == 0) v = __hip_atomic_fetch_add(a.ctl + FusedCtl::claim(x), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
  };
  const bool tr = bi == 0 && wv == 0;
  const uint32_t n_tiles = (uint32_t)nk * WTPF;

  float2 nxt[16];
  bool have_next = false;                 // nxt holds tile `tc`'s points, loads issued
  uint32_t tc = claim();
  while (tc < n_tiles) {
    const int k = (int)(tc / WTPF);
    const int vt = (int)(tc % WTPF);
    const int f = x + 8 * k;
    if (tr) fused_trace(a, x, k, 3);
    if (have_next) {
      // prefetched during the previous tile: reading the registers makes the compiler wait for
      // exactly these loads (not for the map / detection stores issued after them); then the
      // slot is released
#pragma unroll
      for (int m = 0; m < 16; ++m) asm volatile("" ::"v"(nxt[m].x), "v"(nxt[m].y));
      signal_freed(k);
    } else {                              // not prefetched: wait for the frame, load, signal
      bool ok = true;
      if (lane0 == 0) ok = fused_wait(a.ctl, FusedCtl::ready(x, k % kRing), ready_target(k), a.spin_limit);
      if (!__builtin_amdgcn_readfirstlane((int)ok)) return;
      load_tile(k, vt, nxt);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      signal_freed(k);
    }
    if (tr) fused_trace(a, x, k, 4);
    float2 v[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = nxt[m];
    // the next tile: claimed now, its frame's ready word read after pass 1, prefetched if stored
    const uint32_t tn = claim();
    const bool more = tn < n_tiles;
    const int kn = (int)(tn / WTPF);
    uint32_t rdy = 0;
    if (more) rdy = ctl_load(a.ctl, FusedCtl::ready(x, kn % kRing));
    const int t = opaque(t0);
    const int r0 = vt * WR;
    float2* buf = wreg + rr * REGD;
    {
      Dft<16>::run(v);                    // pass 1: L = 1, no twiddles
      float2* d = buf + pad16(16 * t);
#pragma unroll
      for (int m = 0; m < 16; ++m) d[m] = v[m];
    }
    have_next = false;
    if (more && (uint32_t)__builtin_amdgcn_readfirstlane((int)rdy) >= ready_target(kn)) {
      load_tile(kn, (int)(tn % WTPF), nxt);   // in flight through this tile's compute
      have_next = true;
    }
    if (tr) fused_trace(a, x, k, 5);
    {
      pass_sync<false>();
      float2 X[LG][LR];
      if constexpr (TWH) stockham_last_tw<NC, 16, P>(buf, t, X, twh);
      else stockham_to_regs<NC, 16, P, false>(buf, t, X);
      float acc[LG][LR];
      const bool ambm = a.mag_mode == FMCW_MAG_AMBM;
      if (ambm) {
#pragma unroll
        for (int g = 0; g < LG; ++g)
#pragma unroll
          for (int m = 0; m < LR; ++m) {
            const float ai = fabsf(X[g][m].x), aq = fabsf(X[g][m].y);
            const float mx = fmaxf(ai, aq), mn = fminf(ai, aq);
            acc[g][m] = mx + floorf(mn * 0.25f) + floorf(mn * 0.125f);
          }
      } else {
#pragma unroll
        for (int g = 0; g < LG; ++g)
#pragma unroll
          for (int m = 0; m < LR; ++m) acc[g][m] = cabs2(X[g][m]);
      }
      pass_sync<false>();
      float* mrow = mags + rr * REGM;
#pragma unroll
      for (int g = 0; g < LG; ++g) {
        float* m0 = mrow + midx(t + P * g);
#pragma unroll
        for (int m = 0; m < LR; ++m) m0[mpadoff(m * (NC / LR))] = ambm ? acc[g][m] : mag_sqrt(acc[g][m]);
      }
      pass_sync<false>();
      if (a.cf.enabled) {
        fill_halo<NC, P>(mrow, t);
        pass_sync<false>();
      }
      {
        constexpr int Q = WR * NC / 4 / 64;
        const size_t mbase = ((size_t)f * N + r0) * NC;
        const int lane = opaque(lane0);
#pragma unroll
        for (int i = 0; i < Q; ++i) {
          const int e = 4 * (lane + 64 * i);
          const int rl = e / NC, d = e - rl * NC;
          const float4 mv = *reinterpret_cast<const float4*>(mags + rl * REGM + midx(d));
          if (a.lin_map) st_f4<FMCW_NT_MAP>(a.lin_map + mbase + e, mv);
          if (a.db_map) {
            const float kdb = 6.0205999132796239f;  // 20 / log2(10)
            *reinterpret_cast<float4*>(a.db_map + mbase + e) =
                make_float4(kdb * __log2f(mv.x + 1.f), kdb * __log2f(mv.y + 1.f), kdb * __log2f(mv.z + 1.f),
                            kdb * __log2f(mv.w + 1.f));
          }
        }
      }
      if (a.cf.enabled)
        cfar1d_dispatch<NC>(mags, list, rr, t, r0, a.frame0 + f, a.tile0 + f * WTPF + vt, a.cf, a.sink);
      pass_sync<false>();  // the region is reused by the next frame
    }
    if (tr) fused_trace(a, x, k, 6);
    tc = tn;
  }
}

#ifndef FMCW_FUSED_WAVES  // waves per SIMD asked of the register allocator (4 = 4 workgroups per CU)
#define FMCW_FUSED_WAVES 3
#endif
template <int N, int NC, typename LD>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FMCW_FUSED_WAVES)))
k_fused(FusedArgs a) {
  using G = FusedGeom<N, NC>;
  static_assert(G::OK, "fused geometry");
  __shared__ __attribute__((aligned(16))) float lds[G::LDS];
  __shared__ int s_slot, s_fail;
  const int x = xcc_id();
  if (threadIdx.x == 0) {
    s_slot = (int)__hip_atomic_fetch_add(a.ctl + FusedCtl::join(x), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_fail = 0;
  }
  __syncthreads();
  const int slot = s_slot;
  if (slot >= a.per_xcd) {  // more workgroups on this XCD than the group expects
    if (threadIdx.x == 0) __hip_atomic_store(a.ctl + FusedCtl::kErr, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  if (a.census) {  // group size and co-residency check: every member must arrive in time
    if (threadIdx.x == 0) (void)fused_wait(a.ctl, FusedCtl::join(x), (uint32_t)a.per_xcd, a.spin_limit);
    return;
  }
  const int nk = a.n_frames > x ? (a.n_frames - x + 7) / 8 : 0;
  // roles: [0, n_a) range, [n_a, n_a + n_b) Doppler, the rest of the group idles (n_a <= the
  // frame's chirp groups, so every range workgroup has work in every frame and the ready count
  // n_a * (k + 1) means "frame k stored")
  if (slot < a.n_a) fused_range_role<N, NC, LD>(a, x, slot, nk, lds, &s_fail);
  else if (slot < a.n_a + a.n_b) fused_doppler_role<N, NC>(a, x, slot - a.n_a, nk, lds);
}
