// kernels.hpp -- HIP kernels of the FMCW hot path for gfx950.
//
//  K1 k_range     window + range FFT + corner turn        (radar_core.vhd:267-327)
//  K2 k_doppler   Doppler window + FFT + |X| / NCI + map + 1-D OS-CFAR, one wave per tile
//                                                        (radar_core.vhd:340-374, os_cfar.vhd)
//  K3 k_cfar2d    2-D OS-CFAR over the magnitude map       (os_cfar_2d.vhd:83-230)
//     k_det_list (fmcw_api.hip)          deterministic detection list (radar_core.vhd:396-418)
//
// Intermediate (corner-turned range spectrum) layout in HBM, per (frame, rx):
//     inter[rb][cb][RB][T]  complex fp32,  rb = r / RB, cb = c / T
// where T = chirps per K1 workgroup and RB = 128 / T range bins, so K1 writes whole 1 KiB
// chunks and K2 reads runs of (rows per wave) x T x 8 B; element (r, c) sits at
//     ((rb * NCB + cb) * RB + r % RB) * T + c % T.
// This is the corner turner's [range][chirp] order (corner_turner.vhd:80,
// rd_addr = range + doppler * N_RANGE) tiled so both sides stream full lines.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#include "../../include/fmcw.h"
#include "fft_device.hpp"

namespace fmcw {

// K1 spectrum stores at N <= 4096 are write-through (sc1): measured at config 2 (two boxes) K1
// 62.2 -> 60.5 us per 96-frame launch, 756 -> 768 k frames/s; config 3 neutral; config 5 (N = 8192)
// K1 64.9 -> 68.5 us per launch with them, so k_range_px stores write-back.  K2's map stores stay
// non-temporal write-back (write-through: K2 55.5 -> 59.5 us per launch at config 2).  Every other
// alternative measured in rounds 1-4 ("removed after measurement") is gone
// from the sources; the numbers stay in DESIGN.md and the lab builds in git history.
constexpr bool kK1WriteThrough = true;

// --------------------------------------------------------------------------------------
// Input loaders: two consecutive complex samples -> float4 (re0, im0, re1, im1).
// ADC word {Q[31:16], I[15:0]} (rtl/src/tb_radar_core.vhd:115-118) = little-endian short2(I,Q).
// fetch() issues the load and returns the raw bits; expand() converts them.  K1 prefetches the
// raw bits and expands them only when it consumes them: a conversion next to the load would
// make the prefetch wait for its data at once (fp16 / int16 input, config 5).
// --------------------------------------------------------------------------------------
// fetch1 / expand1: one complex sample per lane (k_range_sq's radix-16 first pass).
template <bool NT>
__device__ __forceinline__ uint32_t ld_u1(const void* p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(p));
  else return *reinterpret_cast<const uint32_t*>(p);
}
struct LoadF32 {
  static constexpr int bytes = 8;
  using Raw = float4;
  using Raw1 = float2;
  __device__ __forceinline__ static Raw fetch(const void* base, size_t idx) {
    return ld_f4<kNtCube>(reinterpret_cast<const float2*>(base) + idx);
  }
  __device__ __forceinline__ static float4 expand(Raw r) { return r; }
  __device__ __forceinline__ static float4 load2(const void* base, size_t idx) { return fetch(base, idx); }
  __device__ __forceinline__ static Raw1 fetch1(const void* base, size_t idx) {
    return ld_f2<kNtCube>(reinterpret_cast<const float2*>(base) + idx);
  }
  __device__ __forceinline__ static float2 expand1(Raw1 r) { return r; }
  __device__ __forceinline__ static float2 expand1_scaled(Raw1 r, float s) { return make_float2(r.x * s, r.y * s); }
};
struct LoadF16 {
  static constexpr int bytes = 4;
  using Raw = fmcw_u2v;
  using Raw1 = uint32_t;
  __device__ __forceinline__ static Raw fetch(const void* base, size_t idx) {
    return ld_u2<kNtCube>(reinterpret_cast<const uint32_t*>(base) + idx);
  }
  __device__ __forceinline__ static float4 expand(Raw u) {
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    const h4 h = __builtin_bit_cast(h4, u);
    return make_float4((float)h[0], (float)h[1], (float)h[2], (float)h[3]);
  }
  __device__ __forceinline__ static float4 load2(const void* base, size_t idx) { return expand(fetch(base, idx)); }
  __device__ __forceinline__ static Raw1 fetch1(const void* base, size_t idx) {
    return ld_u1<kNtCube>(reinterpret_cast<const uint32_t*>(base) + idx);
  }
  __device__ __forceinline__ static float2 expand1(Raw1 u) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const h2 h = __builtin_bit_cast(h2, u);
    return make_float2((float)h[0], (float)h[1]);
  }
  // (I, Q) * s: v_fma_mix_f32 converts the half and multiplies in one instruction (fma(x, s, 0) =
  // fl(x s): the fp16 -> fp32 conversion is exact)
  __device__ __forceinline__ static float2 expand1_scaled(Raw1 u, float s) {
    float re, im;
    asm("v_fma_mix_f32 %0, %1, %2, 0 op_sel_hi:[1,0,0]" : "=v"(re) : "v"(u), "v"(s));
    asm("v_fma_mix_f32 %0, %1, %2, 0 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(im) : "v"(u), "v"(s));
    return make_float2(re, im);
  }
};
struct LoadI16 {
  static constexpr int bytes = 4;
  using Raw = fmcw_u2v;
  using Raw1 = uint32_t;
  __device__ __forceinline__ static Raw fetch(const void* base, size_t idx) {
    return ld_u2<kNtCube>(reinterpret_cast<const uint32_t*>(base) + idx);
  }
  __device__ __forceinline__ static float4 expand(Raw u) {
    typedef short s4 __attribute__((ext_vector_type(4)));
    const s4 s = __builtin_bit_cast(s4, u);
    return make_float4((float)s[0], (float)s[1], (float)s[2], (float)s[3]);
  }
  __device__ __forceinline__ static float4 load2(const void* base, size_t idx) { return expand(fetch(base, idx)); }
  __device__ __forceinline__ static Raw1 fetch1(const void* base, size_t idx) {
    return ld_u1<kNtCube>(reinterpret_cast<const uint32_t*>(base) + idx);
  }
  __device__ __forceinline__ static float2 expand1(Raw1 u) {
    typedef short s2 __attribute__((ext_vector_type(2)));
    const s2 s = __builtin_bit_cast(s2, u);
    return make_float2((float)s[0], (float)s[1]);
  }
  __device__ __forceinline__ static float2 expand1_scaled(Raw1 u, float w) {
    const float2 x = expand1(u);
    return make_float2(x.x * w, x.y * w);
  }
};

// Corner-turned spectrum element: complex fp32 (8 B) or, with FMCW_SPEC_F16, a half2 (4 B)
// holding X / N_range (|X| <= N max|x| would overflow fp16 for ADC-scale input; the 2^-log2 N
// scale is exact and K2 undoes it at load).
// Spectrum formats (fmcw.h fmcw_spectrum_dtype): SP_F32 float2 (8 B), SP_F16 half2 of X / N (4 B),
// S48 (6 B, below) in its quad (SP_S48, T >= 8), strided-quad (SP_S48S, T = 4) or strided-pair
// (SP_S48PS, T = 2) form; K1 and K2 are instantiated per form.  (Value 3 was round 5's first pair
// form -- adjacent chirps, each K2 lane loading the pair's element and decoding one point; the
// strided pair replaced it: config 3 23.9-24.5 k -> 24.4-24.5 k frames/s.)
constexpr int SP_F32 = 0, SP_F16 = 1, SP_S48 = 2, SP_S48S = 4, SP_S48PS = 5;
// strided S48 forms: the chirps a K1 group holds (and shares an exponent over) are the ones a K2
// lane holds, p = n_doppler / 16 apart (section 3 of DESIGN.md)
template <int SP> constexpr int s48_strided_g() { return SP == SP_S48S ? 4 : SP == SP_S48PS ? 2 : 0; }
struct __attribute__((packed)) S48 { uint16_t h[3]; };  // one S48 point: pointer steps of 6 B
template <int SP> struct SpecEl { using T = float2; };
template <> struct SpecEl<SP_F16> { using T = uint32_t; };
template <> struct SpecEl<SP_S48> { using T = S48; };
template <> struct SpecEl<SP_S48S> { using T = S48; };
template <> struct SpecEl<SP_S48PS> { using T = S48; };
typedef _Float16 fmcw_h2 __attribute__((ext_vector_type(2)));

// ---- S48: the corner-turned spectrum in 6 bytes per point, one exponent per chirp group --------
// The G chirps Gk .. Gk + G - 1 of one range bin (contiguous in a tile row) share one exponent
// E = max frexp exponent of their 2G components (|x| < 2^E), clamped to >= -95; each component is
// stored as q = rint(x 2^(W - 1 - E)), a W-bit two's-complement significand (clamped to
// 2^(W-1) - 1), so |x - q 2^(E - W + 1)| <= 2^(E - W): 2^-W of the group's largest component (or
// of 2^-95), where fp32 keeps 2^-24 of each.  By K1's tile width T:
//   quad (T >= 8, n_range <= 512): G = 4 adjacent chirps, W = 23, 2 exponent bits per point;
//   strided quad (T = 4, n_range = 1024): G = 4 chirps p apart (p = n_doppler / 16), W = 23;
//   strided pair (T = 2, n_range >= 2048): G = 2 chirps p apart, W = 22, 4 exponent bits per point.
// Point record (48 bits, little-endian, point q of the group at bytes 6q .. 6q + 5): bits 0 .. W-1
// re, then the 8/G bits (8/G) q .. of e8 = E + 127, then im in the top W bits.
// K1 lanes hold chirp pairs (c0, c0 + 1) of the group, c0 even; in the quad forms they exchange the
// pair maximum with the lane of the other pair (lane ^ 1).  K2: adjacent quads sit in lanes
// t .. t + 3 (P % 4 == 0), which OR their exponent pieces together (DPP); a strided group sits in
// one lane (the points t + p m it transforms), decoded from its whole element.  Measured on the
// CPU model (fp64 oracle, per-bin error on bins >= 1e-3 of the frame peak): quad <= 3.3e-5 over 48
// config-2 frames, pair 3.7e-8 at config 5 and 2.5e-8 at config 3, against 1e-4 allowed; one
// exponent per point with 20-bit significands reached 1.9e-4 at config 2.
typedef uint32_t fmcw_u3v __attribute__((ext_vector_type(3)));
template <int G>
__device__ __forceinline__ fmcw_u3v s48_pack(float2 v0, float2 v1, int q0) {
  static_assert(G == 2 || G == 4, "pair or quad");
  constexpr int W = G == 4 ? 23 : 22, PB = 8 / G;
  // the largest |component| by an integer max of the sign-cleared bits (finite values): fmaxf's
  // operand canonicalisation became a late `v_max_f32 vX, |vY|, |vY|` that hipcc (ROCm 7.2) placed
  // right after the previous element's dwordx3 store, overwriting that store's data VGPRs without
  // the 2 wait states the hazard needs -- intermittently corrupt tiles (tools/store_hazard_scan.py)
  constexpr uint32_t AB = 0x7fffffffu;
  const uint32_t mb = max(max(__float_as_uint(v0.x) & AB, __float_as_uint(v0.y) & AB),
                          max(__float_as_uint(v1.x) & AB, __float_as_uint(v1.y) & AB));
  // E from the largest |component| m raised by 2^-(W-1) relative: m (1 + 2^-(W-1)) < 2^E gives
  // m < 2^E (1 - 2^-W), so rint(|x| 2^(W-1-E)) <= 2^(W-1) - 1 and no significand needs a clamp (a
  // group within 2^-W of a power of two takes the next exponent: one bit less, still within 2^-W)
  int el = __builtin_amdgcn_frexp_expf(__uint_as_float(mb) * (1.0f + 1.0f / (1 << (W - 1))));
  if constexpr (G == 4) el = max(el, __builtin_amdgcn_mov_dpp(el, 0xB1 /* quad_perm [1,0,3,2]: lane ^ 1 */, 0xf, 0xf, false));
  const int E = max(el, -95);  // K2's scale 2^(E - 31) stays a normal float
  const uint32_t e8 = (uint32_t)(E + 127);
  // 2^(W-1-E) as a float (W-1-E in [-8, 117]: normal): one packed multiply scales re and im
  const float sc = __uint_as_float((uint32_t)(W - 1 - E + 127) << 23);
  typedef float f2v __attribute__((ext_vector_type(2)));
  const f2v s0 = f2v{v0.x, v0.y} * f2v{sc, sc}, s1 = f2v{v1.x, v1.y} * f2v{sc, sc};
  auto sig = [](float x) -> uint32_t { return (uint32_t)(int)__builtin_rintf(x); };
  const uint32_t r0 = sig(s0.x), i0 = sig(s0.y), r1 = sig(s1.x), i1 = sig(s1.y);
  constexpr uint32_t PM = (1u << PB) - 1;
  const uint32_t b0 = (e8 >> (PB * q0)) & PM, b1 = (e8 >> (PB * q0 + PB)) & PM;
  constexpr uint32_t MW = (1u << W) - 1;
  fmcw_u3v w;
  w.x = (r0 & MW) | (b0 << W) | (i0 << (W + PB));                                   // P0 bits 0-31
  w.y = ((i0 >> (32 - W - PB)) & 0xffffu) | (r1 << 16);                             // P0 32-47, P1 0-15
  w.z = ((r1 >> 16) & ((1u << (W - 16)) - 1)) | (b1 << (W - 16)) | (i1 << (W - 16 + PB));  // P1 16-47
  return w;
}
// Strided-quad form (SP_S48S): K2 lane t holds the 4 points of a quad (chirps t + 4 p k + p j,
// j = 0..3, as K1 grouped them) in one 24-byte element, loaded as two 12-byte halves w0 (points 0,
// 1) and w1 (points 2, 3): the exponent is assembled from the 4 records' 2-bit pieces in the lane,
// no exchange; record j's bits 0-31 / 16-47 are byte-aligned slices of the 6 words.
__device__ __forceinline__ void s48s_unpack4(fmcw_u3v w0, fmcw_u3v w1, float2 (&out)[4]) {
  const uint32_t lo[4] = {w0.x, __builtin_amdgcn_alignbyte(w0.z, w0.y, 2), w1.x, __builtin_amdgcn_alignbyte(w1.z, w1.y, 2)};
  const uint32_t hi[4] = {__builtin_amdgcn_alignbyte(w0.y, w0.x, 2), w0.z, __builtin_amdgcn_alignbyte(w1.y, w1.x, 2), w1.z};
  uint32_t e = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) e |= __builtin_amdgcn_ubfe(lo[j], 23, 2) << (2 * j);
  const float sc = __uint_as_float((e - 31) << 23);  // 2^(E - 31)
  typedef float f2v __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f2v r = f2v{(float)(int)(lo[j] << 9), (float)(int)(hi[j] & 0xfffffe00u)} * f2v{sc, sc};
    out[j] = make_float2(r.x, r.y);
  }
}
// Strided-pair form (SP_S48PS): a lane's points 2k, 2k + 1 (chirps t + 2 p k + p j) in one 12-byte
// element, both decoded in the lane
__device__ __forceinline__ void s48ps_unpack2(fmcw_u3v w, float2 (&out)[2]) {
  constexpr int W = 22;
  const uint32_t lo[2] = {w.x, __builtin_amdgcn_alignbyte(w.z, w.y, 2)};
  const uint32_t hi[2] = {__builtin_amdgcn_alignbyte(w.y, w.x, 2), w.z};
  const uint32_t e = __builtin_amdgcn_ubfe(w.x, W, 4) | (__builtin_amdgcn_ubfe(w.z, W - 16, 4) << 4);
  const float sc = __uint_as_float((e - 31) << 23);  // 2^(E - 31)
  typedef float f2v __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const f2v r = f2v{(float)(int)(lo[j] << (32 - W)), (float)(int)(hi[j] & ~((1u << (32 - W)) - 1))} * f2v{sc, sc};
    out[j] = make_float2(r.x, r.y);
  }
}
// A 12-byte S48 store, padded: a VALU write of a wide store's data VGPRs within 2 wait states of
// the store corrupts the stored data under load, and hipcc (ROCm 7.2, gfx950) pads that hazard
// only for stores whose soffset is not an SGPR -- k_range_px's S48 tile stores (SGPR soffset) came
// out with the next element's packing writing into the previous store's data VGPRs at once, and
// the first frame of multi-group launches read back wrong under load (tools/store_hazard_scan.py
// finds such sequences in a .s).  The two wait states are placed here, fenced against scheduling.
// (k_range / k_range_sq store with soffset 0, which hipcc pads itself: they use the plain store,
// config-2 K1 74.3-74.7 against 74.6-75.2 us per launch with the fenced one.)
template <int AUX>
__device__ __forceinline__ void store_b96_padded(fmcw_u3v w, __amdgpu_buffer_rsrc_t rs, uint32_t vo, uint32_t so) {
  __builtin_amdgcn_raw_buffer_store_b96(w, rs, vo, so, AUX);
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 1");
  __builtin_amdgcn_sched_barrier(0);
}
// One point from the 8 bytes loaded at its record's byte offset rounded down to 4 (odd = its point
// index is odd: the record starts at byte 2 of them); qs = (8/G) (c % G), the shift of its exponent
// piece.  Every lane of the group must call it together.  Two byte permutes give the record's bits
// 0-31 and 16-47; the significands land in the top W bits of a word (low bits zero), so
// v_cvt_f32_i32 reads q 2^(32-W) exactly and one packed multiply by 2^(E - 31) scales both.
template <int G>
__device__ __forceinline__ float2 s48_unpack(fmcw_u2v raw, uint32_t odd, uint32_t qs) {
  constexpr int W = G == 4 ? 23 : 22, PB = 8 / G;
  const uint32_t so = odd * 0x02020202u;
  const uint32_t w0 = __builtin_amdgcn_perm(raw.y, raw.x, 0x03020100u + so);  // record bits 0-31
  const uint32_t w1 = __builtin_amdgcn_perm(raw.y, raw.x, 0x05040302u + so);  // record bits 16-47
  const float re = (float)(int)(w0 << (32 - W)), im = (float)(int)(w1 & ~((1u << (32 - W)) - 1));
  int e = (int)(__builtin_amdgcn_ubfe(w0, W, PB) << qs);
  e |= __builtin_amdgcn_mov_dpp(e, 0xB1 /* lane ^ 1 */, 0xf, 0xf, false);
  if constexpr (G == 4) e |= __builtin_amdgcn_mov_dpp(e, 0x4E /* quad_perm [2,3,0,1]: lane ^ 2 */, 0xf, 0xf, false);
  const float sc = __uint_as_float((uint32_t)(e - 31) << 23);  // 2^(E - 31), E = e - 127 >= -95
  typedef float f2v __attribute__((ext_vector_type(2)));
  const f2v r = f2v{re, im} * f2v{sc, sc};
  return make_float2(r.x, r.y);
}
// The raw 8 bytes of point p (record at 6 p bytes from the S48 array's start): loaded from the
// 4-aligned byte 6 p - 2 (p & 1)
template <bool NT>
__device__ __forceinline__ fmcw_u2v ld_s48_raw(const S48* p, uint32_t odd) {
  return ld_u2<NT>(reinterpret_cast<const char*>(p) - 2 * odd);
}
__device__ __forceinline__ uint32_t pack_h2(float x, float y) {
  return __builtin_bit_cast(uint32_t, fmcw_h2{(_Float16)x, (_Float16)y});
}
template <bool NT>
__device__ __forceinline__ float2 ld_spec(const float2* p, float) { return ld_f2<NT>(p); }
template <bool NT>
__device__ __forceinline__ float2 ld_spec(const uint32_t* p, float scale) {
  uint32_t u;
  if constexpr (NT) u = __builtin_nontemporal_load(p);
  else u = *p;
  const fmcw_h2 h = __builtin_bit_cast(fmcw_h2, u);
  return make_float2((float)h[0] * scale, (float)h[1] * scale);
}

// Per-call status counters (fmcw.h: status words 2 / 3 of fmcw_enqueue): a thread's count, summed
// over its wave by shuffles, one atomic per wave that saw any event.  Called once per kernel, by
// every lane of the wave (after the grid-stride loop).
__device__ __forceinline__ void status_add(uint32_t* word, uint32_t n) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) n += (uint32_t)__shfl_xor((int)n, d, 64);
  if (word && n && (threadIdx.x & 63) == 0) atomicAdd(word, n);
}

// K1 geometry per range-FFT size: T chirps per workgroup, RB = 128/T (1 KiB chunks).
template <int N> struct RangeGeom {
  static constexpr int P = N / 16;                   // threads per transform
  // Measured on MI355X (config 2, tools/ablate.py over build variants): at N = 1024, T = 4
  // (4 waves, 35 KiB LDS, 3 workgroups per CU at 141 VGPRs) beats T = 8 (8 waves, one
  // workgroup per CU) by 9 % in K1 with K2 unchanged; T = 2 is 3 % faster again in K1 but
  // halves K2's read runs (64 B) and costs more there than it saves.
  static constexpr int T = N <= 128 ? 16 : N <= 512 ? 8 : N == 1024 ? 4 : 2;
  static constexpr int NT = T * P;                   // threads per workgroup
  static constexpr int RB = 128 / T;                 // range bins per 1 KiB chunk
  static constexpr int REG = padded(N) + 4;          // LDS row (complex) per chirp
  static constexpr bool WG_SYNC = P > 64;            // transform spans several waves
};

// --------------------------------------------------------------------------------------
// K1: window + range FFT + corner turn.  One workgroup = T chirps of one (frame, rx),
// grid-stride over all chirp groups.  Each thread: 8 coalesced 16-B loads, windowing,
// radix-8 pass in registers, Stockham passes through LDS, then the tiled transposed store.
// --------------------------------------------------------------------------------------
// Q15 = RTL-compat integer range window (FMCW_WIN_Q15_RTL, int16 input): `win` then holds the
// ROM integers c[n] (exact in fp32) and each sample is windowed as sat16((x c + 2^14) >> 14)
// (window_multiplier.vhd:146-158) before it becomes fp32.
// SP = spectrum format: SP_F16 (FMCW_SPEC_F16) tiles hold half2(X / N) (8-B stores of two chirps),
// SP_S48 (FMCW_SPEC_S48) two 6-B S48 points (12-B stores; the quad form at T >= 4, pair at T = 2).
template <int N, typename LD, bool Q15 = false, int SP = SP_F32>
__global__ void __launch_bounds__(RangeGeom<N>::NT)
__attribute__((amdgpu_waves_per_eu(1)))
k_range(const void* __restrict__ cube, float2* __restrict__ inter, const float* __restrict__ win,
        const float* __restrict__ chirp_w, int nc, int n_groups, float q15_scale, uint32_t* __restrict__ status) {
  using Gm = RangeGeom<N>;
  constexpr int P = Gm::P, T = Gm::T, RB = Gm::RB, REG = Gm::REG;
  __shared__ __attribute__((aligned(16))) float2 lds[T * REG];

  const int tid = threadIdx.x;
  const int q = tid / P;  // chirp within the group
  const int t0 = tid % P;
  const int ncb = nc / T;

  // transposed-store geometry: piece i of this thread is range r0 + i*N/8, chirps c0, c0+1
  const int e0 = 2 * tid;
  const int chunk0 = e0 / (RB * T);
  const int win0 = e0 - chunk0 * (RB * T);
  const int r0 = chunk0 * RB + win0 / T;
  const int c0 = win0 % T;
  constexpr int CI = T * N / 1024;  // chunks advanced per piece
  const int rd0_off = c0 * REG + pad16(r0);

  int g = blockIdx.x;
  uint32_t n_sat = 0;     // Q15: windowed samples this thread saturated
  typename LD::Raw a[8];  // this group's samples, raw (expanded at use)
  // Doppler window of the next chirp, loaded with its samples: a vector load issued after the
  // previous iteration's eight tile stores would make the wait for it (vmcnt counts in issue
  // order) wait for those stores too.  From N = 1024 a wave holds one chirp (P >= 64), so the
  // index is wave-uniform and the load goes through the scalar cache (lgkmcnt, not vmcnt).
  auto cw_index = [](int i) { return P >= 64 ? __builtin_amdgcn_readfirstlane(i) : i; };
  // chirp q of group cb: cb T + q, or (strided S48, T = G) t + T p k + p q, the chirps of K2's lane t
  // (cb = t + p k, p = nc / 16 lanes per Doppler row), whose T points K2 then holds in one lane
  constexpr int SGS = s48_strided_g<SP>();
  static_assert(SGS == 0 || SGS == T, "strided S48: one exponent group per K1 group");
  const int lgp = __builtin_ctz(nc) - 4;
  auto chirp_of = [&](int cb) -> int {
    if constexpr (SGS > 0) return (cb & ((1 << lgp) - 1)) + ((cb >> lgp) << (lgp + __builtin_ctz(T))) + (q << lgp);
    else return cb * T + q;
  };
  float cw_n = 1.f;
  if (g < n_groups) {
    const int fr = g / ncb;
    const int cb = g - fr * ncb;
    const size_t chirp = (size_t)fr * nc + (size_t)chirp_of(cb);
#pragma unroll
    for (int m = 0; m < 8; ++m) a[m] = LD::fetch(cube, chirp * N + 2 * t0 + (N / 8) * m);
    if (chirp_w) cw_n = chirp_w[cw_index(chirp_of(cb))];
  }
  // window coefficients for samples 2t + {0,1} + (N/8) m, held for the whole kernel (round 4:
  // re-reading them every group below N = 4096 measured 845-848 k against 856-857 k frames/s)
  constexpr bool HOLD_W = true;
  float2 wh[HOLD_W ? 8 : 1];
  if constexpr (HOLD_W) {
#pragma unroll
    for (int m = 0; m < 8; ++m) wh[m] = *reinterpret_cast<const float2*>(win + 2 * t0 + (N / 8) * m);
    // complete them here: loads still in flight at the loop header make the compiler's
    // wait there vmcnt(0), i.e. also on the previous iteration's tile stores
#pragma unroll
    for (int m = 0; m < 8; ++m) asm volatile("" ::"v"(wh[m].x), "v"(wh[m].y));
  }
  for (; g < n_groups; g += gridDim.x) {
    const int fr = g / ncb;  // frame*nrx + rx within this chunk
    const int cb = g - fr * ncb;
    const int t = opaque(t0);
    float2* buf = lds + q * REG;
    // Doppler window of this chirp folded in (K2 then skips it; FFT linearity), or 1
    const float cw = cw_n * (SP == SP_F16 ? 1.0f / N : 1.0f);

    float2 w[8];
#pragma unroll
    for (int m = 0; m < 8; ++m)
      w[m] = HOLD_W ? wh[HOLD_W ? m : 0] : *reinterpret_cast<const float2*>(win + 2 * t + (N / 8) * m);

    __syncthreads();  // previous group's transposed reads are done with lds
    float4 ax[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) ax[m] = LD::expand(a[m]);
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      float2 v[8];
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        if constexpr (Q15) {
          const int c = (int)(e ? w[m].y : w[m].x);
          const float xi = e ? ax[m].z : ax[m].x, xq = e ? ax[m].w : ax[m].y;
          uint32_t clip = 0;  // the sample's saturation_flag (I or Q clipped, window_multiplier.vhd:152-158)
          auto win16 = [c, &clip](float x) {
            const int y = ((int)x * c + (1 << 14)) >> 14;  // floor: arithmetic shift
            const int ys = min(max(y, -32768), 32767);
            clip |= (uint32_t)(ys != y);
            return (float)ys;
          };
          // 2^-range_shift (the IP's scaling schedule) applies after the integer window
          v[m] = make_float2(win16(xi) * (cw * q15_scale), win16(xq) * (cw * q15_scale));
          n_sat += clip;
        } else {
          const float we = (e ? w[m].y : w[m].x) * cw;
          v[m] = e ? make_float2(ax[m].z * we, ax[m].w * we) : make_float2(ax[m].x * we, ax[m].y * we);
        }
      }
      Dft<8>::run(v);
      float2* d = buf + pad16((2 * t + e) * 8);
#pragma unroll
      for (int m = 0; m < 8; ++m) d[m] = v[m];
    }
    // prefetch the next group into the (now free) input registers
    {
      const int gn = g + gridDim.x;
      if (gn < n_groups) {
        const int frn = gn / ncb;
        const int cbn = gn - frn * ncb;
        const size_t chirp = (size_t)frn * nc + (size_t)chirp_of(cbn);
#pragma unroll
        for (int m = 0; m < 8; ++m) a[m] = LD::fetch(cube, chirp * N + 2 * t + (N / 8) * m);
        if (chirp_w) cw_n = chirp_w[cw_index(chirp_of(cbn))];
      }
    }
    pass_sync<Gm::WG_SYNC>();
    stockham_from<N, 8, P, Gm::WG_SYNC>(buf, t);
    __syncthreads();

    // tiled corner turn: element (r, c) -> inter[rb][cb][RB][T]
    const float2* rd0 = lds + opaque(rd0_off);
    const size_t dbase = (size_t)fr * N * nc + ((size_t)chunk0 * ncb + cb) * (RB * T) + win0;
    float2* dst = inter + dbase;
    uint2* dst16 = reinterpret_cast<uint2*>(reinterpret_cast<uint32_t*>(inter) + dbase);
    const size_t dstep = (size_t)CI * ncb * (RB * T);
    // write-through stores (the launch's spectrum is < 4 GiB: fmcw_create caps the chunk)
    const __amdgpu_buffer_rsrc_t wrs = wt_rsrc(inter, 0xffffffffu);
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
      if constexpr (SP == SP_F16) dst16[i * dstep / 2] = make_uint2(pack_h2(v0.x, v0.y), pack_h2(v1.x, v1.y));
      else if constexpr (SP == SP_S48 || SGS > 0) {
        // (soffset 0: hipcc pads the store-data hazard itself here, see store_b96_padded)
        __builtin_amdgcn_raw_buffer_store_b96(s48_pack<T >= 4 ? 4 : 2>(v0, v1, c0 & (T >= 4 ? 3 : 0)), wrs,
                                              (uint32_t)((dbase + i * dstep) * sizeof(S48)), 0,
                                              kK1WriteThrough ? 16 /* sc1 */ : 0);
      }
      else if constexpr (kK1WriteThrough && N <= 4096) st_f4_wt(wrs, (uint32_t)((dbase + i * dstep) * sizeof(float2)), make_float4(v0.x, v0.y, v1.x, v1.y));
      else st_f4<kNtSpecSt>(dst + i * dstep, make_float4(v0.x, v0.y, v1.x, v1.y));
    }
  }
  if constexpr (Q15) status_add(status, n_sat);  // status word 2 (status = n_dets_dev + 2): window saturations
}

// --------------------------------------------------------------------------------------
// K1 "sequential pair" k_range_sq<N, LD, V, E> (the default at N = 4096, round 3).  T = 2 tiled
// output (the 16-B (chirp 0, chirp 1) element per range bin), the two chirps of a group going
// through ONE chirp's worth of LDS one after the other: the first chirp's spectrum waits in
// registers (V values per thread) while the second is transformed, then both are stored as 16-B
// pairs straight from registers.  Half the LDS of a two-chirp buffer doubles the workgroups per CU
// (N = 4096: three of 34 KiB), so one workgroup's barriers and LDS passes overlap another's memory
// phases.  (Round 2's "dual" kernel -- both chirps per thread in a two-chirp buffer, one workgroup
// of 8 waves per CU at N = 8192 -- was latency-bound at 0.53 of HBM and is gone since round 4.)
//   V = values per thread (16 or 32), P = N / V threads (one transform per workgroup pass);
//   E = consecutive samples per lane per load: the first pass is a radix-(V/E) Stockham pass on
//   the E groups j = E t + e, v[m] = x[j + m N/(V/E)] (E = 1: radix 16 from 8-B fp32 / 4-B fp16
//   loads, so N = 4096 = 16^3 takes two LDS exchanges instead of three; E = 2: 16-B fp32 / 8-B fp16
//   loads).  Then radix-16 LDS passes while more than V points remain per group, and the last
//   pass into registers: lane t holds X[j + m L] for j = t + P g, whole 1 KiB tiles per store
//   instruction.
// The next chirp's raw input is loaded as soon as this chirp's first pass has consumed its
// registers (one chirp ahead, whatever group it belongs to), so the load overlaps three LDS passes.
// Replaces the Xilinx range FFT (rtl/src/radar_core.vhd:303-316) + corner turner (:318-327).
// --------------------------------------------------------------------------------------
template <int N, int V> struct SqGeom {
  static constexpr int P = N / V;
  static constexpr int T = 2, RB = 64;          // = RangeGeom<N> for N >= 2048
  static constexpr int REG = padded(N);
  static constexpr int WAVES = V == 16 ? 4 : 2;  // per SIMD: 16 (V = 16) or 8 (V = 32) waves per CU
};
template <int N, typename LD, int V, int E, int W = SqGeom<N, V>::WAVES, int SP = SP_F32>
__global__ void __launch_bounds__(N / V) __attribute__((amdgpu_waves_per_eu(W)))
k_range_sq(const void* __restrict__ cube, float2* __restrict__ inter, const float* __restrict__ win,
           const float* __restrict__ chirp_w, int nc, int n_groups, float /* q15_scale */, uint32_t* /* status */) {
  using Gm = SqGeom<N, V>;
  constexpr int P = Gm::P, T = Gm::T, RB = Gm::RB;
  constexpr int M = V / E;                      // first-pass radix
  constexpr int S0 = N / M;                     // its input stride (= P E)
  constexpr int LL = vlast_L<N, M, V>();        // sub-transform size before the last pass
  constexpr int RF = N / LL, GF = V / RF;       // last pass: radix, groups per thread
  static_assert(RangeGeom<N>::T == T && RangeGeom<N>::RB == RB, "tile format of K2");
  static_assert(E == 1 || E == 2, "one or two samples per load");
  static_assert(M <= 16 && (M == 16 || E == 2), "first pass writes whole padded 16-point runs");
  __shared__ __attribute__((aligned(16))) float2 lds[Gm::REG];
  const int t0 = threadIdx.x;
  const int ncb = nc / T;

  // raw input of the next chirp to transform (E = 2: M loads of 2 samples; E = 1: M of 1)
  using RawT = std::conditional_t<E == 2, typename LD::Raw, typename LD::Raw1>;
  RawT a[M];
  float cwn = 1.f;
  // chirp q of group cb: cb T + q, or (SP_S48PS) the strided pair t + 2 p k + p q (k_range's chirp_of)
  const int lgp = __builtin_ctz(nc) - 4;
  auto chirp_of = [&](int cb, int q) -> int {
    if constexpr (SP == SP_S48PS) return (cb & ((1 << lgp) - 1)) + ((cb >> lgp) << (lgp + 1)) + (q << lgp);
    else return cb * T + q;
  };
  auto fetch = [&](int g, int q) {
    const int fr = g / ncb;
    const int cb = g - fr * ncb;
    const int c = chirp_of(cb, q);
    const size_t chirp = (size_t)fr * nc + (size_t)c;
    const int t = opaque(t0);
#pragma unroll
    for (int m = 0; m < M; ++m) {
      if constexpr (E == 2) a[m] = LD::fetch(cube, chirp * N + 2 * t + S0 * m);
      else a[m] = LD::fetch1(cube, chirp * N + t + S0 * m);
    }
    if (chirp_w) cwn = chirp_w[__builtin_amdgcn_readfirstlane(c)];
  };
  // range window of this thread's first-pass samples, held (V floats)
  float wh[V];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    if constexpr (E == 2) {
      const float2 w2 = *reinterpret_cast<const float2*>(win + 2 * t0 + S0 * m);
      wh[2 * m] = w2.x;
      wh[2 * m + 1] = w2.y;
    } else {
      wh[m] = win[t0 + S0 * m];
    }
  }
#pragma unroll
  for (int i = 0; i < V; ++i) asm volatile("" ::"v"(wh[i]));  // complete before the loop (vmcnt order)

  int g = blockIdx.x;
  if (g < n_groups) fetch(g, 0);
  for (; g < n_groups; g += gridDim.x) {
    const int fr = g / ncb;
    const int cb = g - fr * ncb;
    float2 X[2][GF][RF];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int t = opaque(t0);
      const float cw = cwn;
      __syncthreads();  // the previous transform's last-pass reads are done with lds
      // first pass from registers: window (x Doppler weight of the chirp), radix M, E groups
#pragma unroll
      for (int e = 0; e < E; ++e) {
        float2 v[M];
#pragma unroll
        for (int m = 0; m < M; ++m) {
          float2 x;
          if constexpr (E == 2) {
            const float4 x4 = LD::expand(a[m]);
            x = e ? make_float2(x4.z, x4.w) : make_float2(x4.x, x4.y);
          } else {
            x = LD::expand1(a[m]);
          }
          const float we = wh[E * m + e] * cw;
          v[m] = make_float2(x.x * we, x.y * we);
        }
        Dft<M>::run(v);
        float2* d = lds + pad16((E * t + e) * M);
#pragma unroll
        for (int m = 0; m < M; ++m) d[m] = v[m];
      }
      // the next chirp's input: this group's second chirp, or the next group's first
      if (q == 0) fetch(g, 1);
      else if (g + (int)gridDim.x < n_groups) fetch(g + gridDim.x, 0);
      __syncthreads();
      vpasses_mid<N, M, P, V>(lds, t);
      vpass_last<N, LL, P, V>(lds, t, X[q]);
    }
    // tile stores: lane t holds range bins d = t + P gg + LL m of both chirps; write-through (sc1)
    // at N <= 4096 as k_range: no dirty spectrum lines left in L2 for the end-of-kernel release
    // (config 3: K1 58.3-58.7 -> 57.2-57.6 us per launch, 21.7-21.8 k -> 22.0-22.1 k frames/s,
    // profiles/r04/k1/policy/; nt + sc1 7 % slower)
    // (SP_S48: the pair form, 12 B per element, same policy)
    const int t = opaque(t0);
    const size_t fbase = (size_t)fr * N * nc;
    constexpr bool WT = kK1WriteThrough && N <= 4096;
    constexpr bool S48V = SP == SP_S48 || SP == SP_S48PS;  // (S48 names the point struct)
    constexpr size_t EB = S48V ? sizeof(S48) : sizeof(float2);  // bytes per point
    const __amdgpu_buffer_rsrc_t srs =  // one frame's tiles < 4 GiB
        S48V ? wt_rsrc(reinterpret_cast<char*>(inter) + fbase * EB, 0xffffffffu) : wt_rsrc(inter + fbase, 0xffffffffu);
#pragma unroll
    for (int gg = 0; gg < GF; ++gg)
#pragma unroll
      for (int m = 0; m < RF; ++m) {
        const int d = t + P * gg + LL * m;
        const size_t off = ((size_t)(d / RB) * ncb + cb) * (RB * T) + (size_t)(d % RB) * T;
        if constexpr (S48V) {
          __builtin_amdgcn_raw_buffer_store_b96(s48_pack<2>(X[0][gg][m], X[1][gg][m], 0), srs, (uint32_t)(off * EB), 0,
                                                WT ? 16 /* sc1 */ : 0);  // (soffset 0: padded by hipcc)
        } else {
          const float4 x = make_float4(X[0][gg][m].x, X[0][gg][m].y, X[1][gg][m].x, X[1][gg][m].y);
          if constexpr (WT) st_f4_wt(srs, (uint32_t)(off * sizeof(float2)), x);
          else st_f4<kNtSpecSt>(inter + fbase + off, x);
        }
      }
  }
}

// --------------------------------------------------------------------------------------
// K1 "permlane pair" k_range_px<LD> for N = 8192 (round 3): k_range_sq's sequential pair with
// 16 values per thread (512 threads, one 68 KiB transform buffer, two workgroups per CU), but
// 8192 = 16 x 16 x 16 x 2 with two LDS exchanges instead of three:
//   pass A  radix 16 from registers (one fp16/int16/fp32 sample per lane per load, stride 512),
//           window x Doppler weight fused, written to LDS;
//   pass B  radix 16 through LDS (sub-transforms 16 -> 256);
//   pass C  radix 16 read from LDS into registers (256 -> 4096), thread (lane l, wave w) taking
//           j = (l & 31) + 32 w + 256 (l >> 5): the two half-waves hold the two 4096-point
//           halves y0, y1 at the same offsets k + 256 m;
//   pass D  the last radix-2 (4096 -> 8192) between the half-waves: v_permlane32_swap of
//           registers m and m + 8 leaves each lane 8 complete (y0, y1) pairs, p = k + 256 m',
//           m' = m + 8 (1 - h), X[p] = y0 + W^p y1, X[p + 4096] = y0 - W^p y1.
// (Measured and dropped: pass B inside each wave -- lane (w, l) playing pass-A thread u + 32 i and
// pass-B thread 16 u + i, u = 4 w + (l >> 4), i = l & 15, so the A -> B exchange needs no barrier
// -- makes every pass-A load instruction read 16-B runs of 16 lines: 132 us per 3-frame launch
// (105 us with cached loads) against 58 us, profiles/r03/k1px/k1lab_c5_3f_wl.log.)
// The first chirp's 16 outputs wait in registers while the second is transformed, then both go out
// as 16-B (chirp 0, chirp 1) tile elements: lanes 0-31 and 32-63 each write 512 contiguous bytes.
// Replaces the Xilinx range FFT (rtl/src/radar_core.vhd:303-316) + corner turner (:318-327).
// --------------------------------------------------------------------------------------
__device__ __forceinline__ void swap32(float2& a, float2& b) {
  // a, b := [a_lo, b_lo], [a_hi, b_hi] (lo / hi = lanes 0-31 / 32-63)
  const auto rx = __builtin_amdgcn_permlane32_swap(__float_as_uint(a.x), __float_as_uint(b.x), false, false);
  const auto ry = __builtin_amdgcn_permlane32_swap(__float_as_uint(a.y), __float_as_uint(b.y), false, false);
  a = make_float2(__uint_as_float(rx[0]), __uint_as_float(ry[0]));
  b = make_float2(__uint_as_float(rx[1]), __uint_as_float(ry[1]));
}
// (Measured and dropped: an XOR-swizzled unpadded layout in which pass A stores into exactly the
// slots its own lane read in the previous pass C, so the barrier between them goes (3 per chirp):
// 64.9 vs 59.3 us per 3-frame launch, equal at 12 frames -- profiles/r03/k1px/k1lab_c5_sw.log.)
// WS: range-window values per thread kept in LDS instead of VGPRs (the last WS of the 16).  At 128
// VGPRs (4 waves per SIMD) the kernel otherwise spills a window value to scratch, and its reload --
// a vector-memory op issued after the group's 16 tile stores -- makes the next group's pass A wait,
// in vmcnt order, for every one of those stores.  68 + 2 WS KiB of LDS per workgroup: two still fit
// a CU (160 KiB) up to WS = 6.
template <typename LD, int W = 4, int WS = 4, int SP = SP_F32>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(W)))
k_range_px(const void* __restrict__ cube, float2* __restrict__ inter, const float* __restrict__ win,
           const float* __restrict__ chirp_w, int nc, int n_groups, float /* q15_scale */, uint32_t* /* status */) {
  constexpr int N = 8192, T = 2, RB = 64;
  static_assert(RangeGeom<N>::T == T && RangeGeom<N>::RB == RB, "tile format of K2");
  static_assert(WS >= 0 && WS <= 6, "two workgroups per CU");
  __shared__ __attribute__((aligned(16))) float2 lds[padded(N)];
  __shared__ float wlds[WS > 0 ? WS * 512 : 1];
  const int t0 = threadIdx.x;
  const int lane = t0 & 63, wv = t0 >> 6, h = lane >> 5;
  const int ncb = nc / T;

  // loads and stores through buffer descriptors: one lane offset, the m-dependent part in the
  // SGPR offset (no 64-bit address per load / store in VGPRs)
  using Raw1 = typename LD::Raw1;
  constexpr int SB = sizeof(Raw1);  // bytes per sample
  constexpr int NTL = kNtCube ? 2 : 0;  // non-temporal cube loads (read once)
  Raw1 a[16];
  float cwn = 1.f;
  // chirp q of group cb: cb T + q, or (SP_S48PS) the strided pair t + 2 p k + p q (k_range's chirp_of)
  const int lgp = __builtin_ctz(nc) - 4;
  auto chirp_of = [&](int cb, int q) -> int {
    if constexpr (SP == SP_S48PS) return (cb & ((1 << lgp) - 1)) + ((cb >> lgp) << (lgp + 1)) + (q << lgp);
    else return cb * T + q;
  };
  auto fetch = [&](int g, int q) {
    const int fr = g / ncb;
    const int cb = g - fr * ncb;
    const int c = chirp_of(cb, q);
    const size_t chirp = (size_t)fr * nc + (size_t)c;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(reinterpret_cast<const char*>(cube)) + chirp * N * SB, (short)0, N * SB, 0x00020000);
    const int vo = opaque(t0) * SB;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      if constexpr (SB == 4) {
        a[m] = __builtin_bit_cast(Raw1, __builtin_amdgcn_raw_buffer_load_b32(rs, vo, m * 512 * SB, NTL));
      } else {
        a[m] = __builtin_bit_cast(Raw1, __builtin_amdgcn_raw_buffer_load_b64(rs, vo, m * 512 * SB, NTL));
      }
    }
    if (chirp_w) cwn = chirp_w[__builtin_amdgcn_readfirstlane(c)];
  };
  float wh[16 - WS];  // range window of samples t + 512 m, held (m < 16 - WS; the rest in wlds)
#pragma unroll
  for (int m = 0; m < 16 - WS; ++m) wh[m] = win[t0 + 512 * m];
#pragma unroll
  for (int m = 16 - WS; m < 16; ++m) wlds[(m - 16 + WS) * 512 + t0] = win[t0 + 512 * m];
#pragma unroll
  for (int i = 0; i < 16 - WS; ++i) asm volatile("" ::"v"(wh[i]));  // complete before the loop (vmcnt order)

  // pass C's group j = kc + 256 h; the pass-D twiddle base W_8192^(kc + 2048 (1 - h))
  const int kc = (lane & 31) + 32 * wv;
  const float2 cd = twiddle<N>(kc + 2048 * (1 - h));

  int g = blockIdx.x;
  if (g < n_groups) fetch(g, 0);
  for (; g < n_groups; g += gridDim.x) {
    const int fr = g / ncb;
    const int cb = g - fr * ncb;
    float2 X[2][16];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int t = opaque(t0);
      const float cw = cwn;
      __syncthreads();  // the previous transform's pass-C reads are done with lds
      {  // pass A: window, radix 16 over x[t + 512 m]
        float2 v[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) {
          const float w = m < 16 - WS ? wh[m < 16 - WS ? m : 0] : wlds[(m - 16 + WS) * 512 + t];
          v[m] = LD::expand1_scaled(a[m], w * cw);
        }
        Dft<16>::run(v);
        float2* d = lds + pad16(16 * t);
#pragma unroll
        for (int m = 0; m < 16; ++m) d[m] = v[m];
      }
      // the next chirp's input: this group's second chirp, or the next group's first
      if (q == 0) fetch(g, 1);
      else if (g + (int)gridDim.x < n_groups) fetch(g + gridDim.x, 0);
      {  // pass B: radix 16, L = 16 (in place, barriers around the exchange)
        __syncthreads();
        float2 v[16];
        const float2* src = lds + pad16(t);
#pragma unroll
        for (int m = 0; m < 16; ++m) v[m] = src[padoff(m * 512)];
        __syncthreads();
        const int k = t & 15;
        GroupTwiddles<16, 256> tb;
        tb.init(k);
#pragma unroll
        for (int m = 1; m < 16; ++m) v[m] = cmul(v[m], tb.pow(m));
        Dft<16>::run(v);
        float2* dst = lds + pad16((t >> 4) * 256 + k);
#pragma unroll
        for (int m = 0; m < 16; ++m) dst[padoff(m * 16)] = v[m];
        __syncthreads();
      }
      {  // pass C: radix 16, L = 256, into registers; v[m] = y_h[kc + 256 m]
        float2* v = X[q];
        const float2* src = lds + pad16(opaque(kc + 256 * h));
#pragma unroll
        for (int m = 0; m < 16; ++m) v[m] = src[padoff(m * 512)];
        GroupTwiddles<16, 4096> tc;
        tc.init(opaque(kc));
#pragma unroll
        for (int m = 1; m < 16; ++m) v[m] = cmul(v[m], tc.pow(m));
        float2 cdl = cd;  // per chirp: the W_32^m products below must not be hoisted (14 VGPRs)
        asm volatile("" : "+v"(cdl.x), "+v"(cdl.y));
        Dft<16>::run(v);
        // pass D: radix 2 between the half-waves; X[q][m + 8] = y0[p], X[q][m] = y1[p] ->
        // X[q][m + 8] = X[p], X[q][m] = X[p + 4096], p = kc + 256 (m + 8 (1 - h))
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          swap32(v[m + 8], v[m]);
          // W_8192^(p) = cd * W_32^m
          const float2 w32 = make_float2(__builtin_cosf(2.0f * 3.14159265358979323846f * m / 32.f),
                                         -__builtin_sinf(2.0f * 3.14159265358979323846f * m / 32.f));
          const float2 tw = m ? cmul(cdl, w32) : cdl;
          const float2 b = cmul(v[m], tw);
          const float2 a0 = v[m + 8];
          v[m + 8] = cadd(a0, b);
          v[m] = csub(a0, b);
        }
      }
    }
    // tile stores: lane holds X[d] of both chirps for d = p (register m + 8) and p + 4096 (m)
    // d / 64 = (w >> 1) + 4 m' + 64 s, d % 64 = (l & 31) + 32 (w & 1); tile (d / 64, cb) is 1 KiB
    // (SP_S48: the pair form, 12-B elements in 768-B tiles)
    constexpr bool S48V = SP == SP_S48 || SP == SP_S48PS;  // (S48 names the point struct)
    constexpr int EB = S48V ? 2 * (int)sizeof(S48) : 16;  // bytes per (chirp 0, chirp 1) element
    void* const fbase = S48V ? static_cast<void*>(reinterpret_cast<char*>(inter) + (size_t)fr * N * nc * (EB / 2))
                                     : static_cast<void*>(inter + (size_t)fr * N * nc);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(fbase, (short)0, N * nc * (EB / 2), 0x00020000);
    const int t = opaque(t0);
    const int l = t & 63, w = t >> 6;
    const int vo = (((w >> 1) + 32 * (1 - (l >> 5))) * ncb + cb) * (64 * EB) + ((l & 31) + 32 * (w & 1)) * EB;
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int r = s ? m : m + 8;
        if constexpr (S48V) {
          store_b96_padded<0 /* write-back */>(s48_pack<2>(X[0][r], X[1][r], 0), rs, (uint32_t)vo,
                                               (4 * m + 64 * s) * ncb * (64 * EB));
        } else {
          typedef float f4v __attribute__((ext_vector_type(4)));
          const f4v x = {X[0][r].x, X[0][r].y, X[1][r].x, X[1][r].y};
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(fmcw_u4v, x), rs, vo,
                                                 (4 * m + 64 * s) * ncb * (64 * EB), 0 /* write-back */);
        }
      }
  }
}

// --------------------------------------------------------------------------------------
// Detection sink shared by the CFAR kernels.  Tile `wg` (a workgroup's unit: frame, range
// rows) writes its detections, in (range, doppler) order, to its own fixed slot
// scratch[wg * slot_cap ...] -- no atomic, no round trip.  Only a tile with more than
// slot_cap detections reserves room in the overflow region with one atomic (a single global
// counter serialises at ~88 returning atomics/us, MI355X_MICROARCH "dequeue", which is why
// the common path must not touch it).  (wg_base, wg_count) per tile then let
// k_det_list order the list by tile id = (frame, range): deterministic.
// Detections that fit nowhere are counted in counter[1] (reported as FMCW_EDETCAP).
// --------------------------------------------------------------------------------------
struct DetSink {
  fmcw_det* scratch;
  uint32_t cap;        // total scratch entries (slots + overflow)
  uint32_t slot_cap;   // entries per tile slot
  uint32_t ovf_base;   // first entry of the overflow region
  uint32_t* counter;   // [0] overflow entries used, [1] dropped detections
  uint32_t* wg_base;
  uint32_t* wg_count;
};

// Reserve a tile's range in the sink: every thread gets the same base.  `total` is uniform;
// the overflow branch (rare) needs one broadcast through LDS.
__device__ __forceinline__ uint32_t det_reserve(const DetSink& sink, int wg, int total, int* s_bcast) {
  uint32_t base = (uint32_t)wg * sink.slot_cap;
  if ((uint32_t)total > sink.slot_cap) {
    if (threadIdx.x == 0) {
      uint32_t b = sink.ovf_base + atomicAdd(sink.counter, (uint32_t)total);
      if (b + (uint32_t)total > sink.cap) atomicAdd(sink.counter + 1, b + (uint32_t)total - max(b, sink.cap));
      *s_bcast = (int)b;
    }
    __syncthreads();
    base = (uint32_t)*s_bcast;
  }
  if (threadIdx.x == 0) {
    sink.wg_base[wg] = base;
    sink.wg_count[wg] = (uint32_t)total;
  }
  return base;
}

// Exclusive scan of one int per thread over the workgroup (one barrier): wave scans by
// shuffles, each thread then adds the totals of the earlier waves.  s_wave[NT/64] must not
// be rewritten before every thread has passed (callers end the tile with a barrier).
template <int NT>
__device__ __forceinline__ int block_excl_scan1(int v, int* s_wave, int& total) {
  constexpr int NW = NT / 64;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) s_wave[wv] = x;
  __syncthreads();
  int before = 0, all = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const int w = s_wave[i];
    before += i < wv ? w : 0;
    all += w;
  }
  total = all;
  return before + x - v;
}

template <int NT>
__device__ __forceinline__ int block_excl_scan(int v, int* s_wave, int& total) {
  constexpr int NW = NT / 64;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) s_wave[wv] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int i = 0; i < NW; ++i) {
      const int tt = s_wave[i];
      s_wave[i] = acc;
      acc += tt;
    }
    s_wave[NW] = acc;
  }
  __syncthreads();
  total = s_wave[NW];
  const int r = s_wave[wv] + x - v;
  __syncthreads();
  return r;
}

// 1 if x < y, for non-negative finite floats given as bit patterns (their unsigned order is
// the float order and |xb - yb| < 2^31).  CFAR inputs are magnitudes (>= +0), like the
// reference's unsigned magnitude stream (magnitude_calc.vhd).  No VCC / SGPR mask involved.
__device__ __forceinline__ uint32_t lt_bit(uint32_t xb, uint32_t yb) { return (xb - yb) >> 31; }

// Caller-supplied maps (fmcw_cfar) enter the CFAR as the RTL's unsigned magnitude stream:
// negative cells and -0.0 become +0 (integer max on the bit pattern: every pattern with the
// sign bit set is negative as an int32), so the bit-pattern compares above stay exact.
__device__ __forceinline__ float nonneg(float x) { return __int_as_float(max(__float_as_int(x), 0)); }
__device__ __forceinline__ float4 nonneg4(float4 v) {
  return make_float4(nonneg(v.x), nonneg(v.y), nonneg(v.z), nonneg(v.w));
}
// RTL-compat cell (FMCW_COMPAT_CFAR): the 17-bit unsigned CFAR input word (DATA_WIDTH 17,
// os_cfar.vhd:13, os_cfar_2d.vhd:11), q = min(floor(max(x, 0)), 2^17 - 1); exact in fp32.
constexpr uint32_t kQ17Mask = (1u << 17) - 1u;
__device__ __forceinline__ float q17(float x) { return fminf(floorf(nonneg(x)), (float)kQ17Mask); }
__device__ __forceinline__ float4 q17x4(float4 v) { return make_float4(q17(v.x), q17(v.y), q17(v.z), q17(v.w)); }

struct Cfar1DArgs {
  int enabled;
  int ref, guard, rank;
  float alpha;
  int compat;        // FMCW_COMPAT_CFAR: 17-bit integer cells, T = (ranked * alpha) mod 2^17
};

// --------------------------------------------------------------------------------------
// Magnitude rows in LDS (K2, the 1-D CFAR and K3).  A row holds the NC cells plus a 16-cell
// circular halo on each side (cells -16..-1 = NC-16..NC-1, cells NC..NC+15 = 0..15), so a
// CFAR window of reach <= 16 never wraps and its addresses are a per-lane base plus
// immediates.  Every 16 cells are followed by 4 pad floats: each 16-cell block starts 16-B
// aligned (one ds_read_b128 per 4 cells) and 16 lanes reading blocks 16 cells apart touch 16
// disjoint bank quads (20 t mod 64 are distinct).
// --------------------------------------------------------------------------------------
// |X| from |X|^2: the hardware square root (v_sqrt_f32, <= 1 ulp) instead of the correctly
// rounded libm sequence (~15 VALU instructions each: denormal scaling plus two fma fix-ups).
// Magnitudes are specified to 1e-4 relative (BASELINE north_star), the CFAR is exact on
// whatever map is produced, and |X|^2 is never denormal-sensitive at these scales.  Scaling
// the input by 2 still scales the map by exactly 2 (an even exponent shift).
__device__ __forceinline__ float mag_sqrt(float p) { return __builtin_amdgcn_sqrtf(p); }
// |X|^2 with both products rounded before the sum.  Left to -ffp-contract, whether x*x + y*y
// becomes fma(x, x, y*y) depended on the surrounding code, so K2's variants and the paired
// kernel differed in the last bit of 7 % of the cells; with contraction off in this scope every
// kernel that computes a magnitude (K2, the fused and the paired kernels) rounds it identically.
__device__ __forceinline__ float cabs2(float2 X) {
#pragma clang fp contract(off)
  return X.x * X.x + X.y * X.y;
}

constexpr int MH = 16;  // halo cells per side
__host__ __device__ constexpr int midx(int d) { return (d + MH) + (((d + MH) >> 4) << 2); }
// midx(x + o) - midx(x) for x % 16 == 0 and a compile-time o >= -MH
__host__ __device__ constexpr int moff(int o) { return o + 4 * (o >= 0 ? o / 16 : -((15 - o) / 16)); }
// midx(x + o) - midx(x) for o >= 0 when x % 16 + o % 16 < 16 (cf. padoff)
__host__ __device__ constexpr int mpadoff(int o) { return o + 4 * (o / 16); }
template <int NC> constexpr int mrow_floats() { return (((NC + 2 * MH) * 5 / 4) + 3) & ~3; }
__host__ __device__ constexpr int floor4(int x) { return x >= 0 ? x & ~3 : -((-x + 3) & ~3); }

// Fill the circular halos of one magnitude row once its NC cells are written; the P lanes
// that share the row copy cells j = t, t + P, ... of the 32 halo cells.
template <int NC, int P>
__device__ __forceinline__ void fill_halo(float* row, int t) {
  for (int j = t; j < 2 * MH; j += P) {
    const int dst = j < MH ? NC + j : j - 2 * MH;
    const int src = j < MH ? j : NC + j - 2 * MH;
    row[midx(dst)] = row[midx(src)];
  }
}

// Cells [o0, o0 + 4 NV) of a row relative to a 16-cell-aligned lane base (o0 % 4 == 0), as NV
// 16-byte LDS reads.
template <int NV>
__device__ __forceinline__ void load_cells(const float* base, int o0, float (&v)[4 * NV]) {
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const float4 q = *reinterpret_cast<const float4*>(base + moff(o0 + 4 * c));
    v[4 * c] = q.x;
    v[4 * c + 1] = q.y;
    v[4 * c + 2] = q.z;
    v[4 * c + 3] = q.w;
  }
}

// --------------------------------------------------------------------------------------
// Wave tiles.  K2 and the stand-alone 1-D CFAR work on tiles of WR = 64 / P range rows x all
// NC Doppler cells of one frame (P = NC/16 lanes per row, 16 cells per lane), ONE WAVEFRONT
// per tile: a row's Doppler FFT, its magnitudes, its CFAR window and its detection list all
// live in that wave's private LDS region, so no workgroup barrier is ever needed.  The waves
// of a workgroup drift apart freely and one wave's HBM loads overlap another's FFT and CFAR
// arithmetic (a workgroup is only the unit of LDS allocation).  A tile is also the unit of
// detection ordering (DetSink tile = (frame, range rows)).
// --------------------------------------------------------------------------------------
constexpr int cmax(int a, int b) { return a > b ? a : b; }

template <int NC> struct DopplerGeom {
  static constexpr int P = NC / 16;                     // lanes per range row (16 cells each)
  static constexpr int WR = 64 / P;                     // range rows per wave tile
  // waves per workgroup (independent; a workgroup's waves take consecutive row groups of one
  // frame, so together they read WPB x WR x T x 8 B of every 1 KiB spectrum tile)
  static constexpr int WPB = 4;  // (8 at NC = 1024, one workgroup reading whole 128-B lines: 56.5 -> 65.3 us)
  static constexpr int NT = 64 * WPB;
  static constexpr int REGD = padded(NC) + 4;           // complex per range row (FFT)
  static constexpr int REGM = mrow_floats<NC>();        // floats per magnitude row
  static constexpr int LIST = WR * REGM;                // detection cell list (u32) offset
  // floats per wave region: the FFT rows, later the magnitude rows + the cell list
  static constexpr int WFL = cmax(2 * WR * REGD, LIST + WR * NC);
  static constexpr int LR = FinalRadix<NC, 16>::R;      // last pass radix (after pass 1)
  static constexpr int LG = 16 / LR;
  static_assert(WFL % 4 == 0 && REGM % 4 == 0, "16-B aligned rows and regions");
};

// Wave-level exclusive scan; `total` = the wave's sum, uniform.  DPP adds on the VALU (GCN
// row scan: row_shr 1/2/4/8 inside each row of 16 lanes, then row_bcast:15 / row_bcast:31 carry
// the row totals), where the former __shfl_up version took six ds_bpermute round trips through
// LDS plus a lane-mask select per step (SGPR pressure).  Every caller runs it with the whole wave
// active.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ int dpp_add(int x) {
  return x + __builtin_amdgcn_update_dpp(0, x, CTRL, ROW_MASK, 0xf, false);
}
__device__ __forceinline__ int wave_excl_scan(int v, int& total) {
  int x = v;
  x = dpp_add<0x111, 0xf>(x);  // row_shr:1
  x = dpp_add<0x112, 0xf>(x);  // row_shr:2
  x = dpp_add<0x114, 0xf>(x);  // row_shr:4
  x = dpp_add<0x118, 0xf>(x);  // row_shr:8
  x = dpp_add<0x142, 0xa>(x);  // row_bcast:15 -> rows 1, 3
  x = dpp_add<0x143, 0xc>(x);  // row_bcast:31 -> rows 2, 3
  total = __builtin_amdgcn_readlane(x, 63);
  return x - v;
}

// det_reserve for a one-wave tile: its slot, or (rare) a range in the overflow region
// reserved by lane 0 and broadcast by a shuffle.  `total` is wave-uniform.
__device__ __forceinline__ uint32_t det_reserve_wave(const DetSink& sink, int tile, int total) {
  const int lane = threadIdx.x & 63;
  uint32_t base = (uint32_t)tile * sink.slot_cap;
  if ((uint32_t)total > sink.slot_cap) {
    uint32_t b = 0;
    if (lane == 0) {
      b = sink.ovf_base + atomicAdd(sink.counter, (uint32_t)total);
      if (b + (uint32_t)total > sink.cap) atomicAdd(sink.counter + 1, b + (uint32_t)total - max(b, sink.cap));
    }
    base = (uint32_t)__shfl((int)b, 0, 64);
  }
  if (lane == 0) {
    sink.wg_base[tile] = base;
    sink.wg_count[tile] = (uint32_t)total;
  }
  return base;
}

// exact k-th smallest of 2*REF registers: bitonic sort (compile-time indices), then the max of
// the ascending prefix r[0..rank] (a select chain `i == rank ? r[i] : out` is turned by LLVM
// into a private-array lookup, i.e. a scratch store + indexed load per detection).  On the bit
// patterns: CFAR cells are non-negative (unsigned order == value order), and integer min/max need
// none of the NaN-canonicalising v_max_f32 x, x, x that fminf/fmaxf of loaded values cost.
template <int REF, int GUARD>
__device__ __forceinline__ float ranked_of(float (&rf)[2 * REF], int rank) {
  constexpr int N = 2 * REF;
  static_assert((N & (N - 1)) == 0, "power-of-two reference count");
  uint32_t r[N];
#pragma unroll
  for (int i = 0; i < N; ++i) r[i] = __float_as_uint(rf[i]);
#pragma unroll
  for (int k = 2; k <= N; k <<= 1)
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1)
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const int l = i ^ j;
        if (l > i) {
          const uint32_t a = r[i], b = r[l];
          const bool up = (i & k) == 0;
          r[i] = up ? min(a, b) : max(a, b);
          r[l] = up ? max(a, b) : min(a, b);
        }
      }
  uint32_t out = r[0];
#pragma unroll
  for (int i = 1; i < N; ++i) out = max(out, i <= rank ? r[i] : r[0]);
  return __uint_as_float(out);
}

// 1-D OS-CFAR along Doppler (circular) over a wave tile's magnitude rows, plus ordered
// emission.  Lane (rr, t) tests the 16 consecutive cells d0 = 16 t .. d0 + 15 of row rr, so
// emission in lane order is (range, doppler) order.  detect <=> #{refs : fl(alpha*ref) >= cut}
// < n_ref - rank  <=>  #{fl(alpha*ref) < cut} > rank, which is cut > fl(alpha *
// sorted(refs)[rank]) (rtl/old/os_cfar.vhd:117-137) without a sort.  The count is mask-free
// integer arithmetic (lt_bit) so that hundreds of compares do not become SGPR masks.
// REF > 0: compile-time geometry (REF refs + GUARD guards per side) with the window in
// registers, screened (below); REF == 0: runtime geometry read from LDS.
// ONEG: need = n_ref - rank <= 4 known at compile time (the reference's rank 12 of 16), so
// one qualifying group of 4 rejects and the per-cell screen is a 4-way max (no runtime branch
// per cell, which also kept both screens' registers live).
template <int NC, int REF, int GUARD, bool ONEG = false>
__device__ __forceinline__ void cfar1d_wave(const float* mags, uint32_t* list, int rr, int t, int r0,
                                            int frame, int tile, const Cfar1DArgs& cf,
                                            const DetSink& sink) {
  constexpr int CELLS = 16;
  constexpr int RS = DopplerGeom<NC>::REGM;
  const float* mrow = mags + rr * RS;
  const int d0 = t * CELLS;
  const int nref = 2 * cf.ref;
  const int lane = (int)(threadIdx.x & 63);
  uint32_t bits = 0;
  int total = 0;  // detections of the wave tile (uniform), their cells in list[0, total)
  if constexpr (REF > 0) {
    // Screen, then count exactly where needed.  A group of 4 consecutive reference cells
    // whose minimum satisfies fl(alpha*min) >= cut has all 4 refs at or above cut/alpha
    // (fl(alpha*x) is monotone in x), so 4 * #{such groups} is a lower bound on
    // #{refs : fl(alpha*ref) >= cut}; once it reaches need = n_ref - rank the cell cannot
    // detect.  The exact count (16 compares) runs only for the survivors (below) and decides
    // exactly as the unscreened count.
    static_assert(REF % 4 == 0, "reference runs split into groups of 4");
    constexpr int H = REF + GUARD;
    static_assert(H <= MH, "the window stays inside the row halos");
    constexpr int NGS = REF / 4;               // groups of 4 per side
    constexpr int RO = REF + 2 * GUARD + 1;    // first right ref, relative to the first left ref
    // two halves of 8 cells (a 28-value window each) to keep the register peak low
    const float* lb = mrow + midx(d0);
    const int need = nref - cf.rank;
    constexpr bool one_group = ONEG;           // the reference (rank 12 of 16): any group rejects
    // The lane's whole window at once: cells d0 - H .. d0 + 15 + H, group minima g[k] =
    // min(w[k .. k+3]) over it computed once (2 mins per group), not per 8-cell half.
    {
      constexpr int WW = CELLS + 2 * H;        // 36 at the reference geometry
      constexpr int O0 = floor4(-H);
      constexpr int NV = (WW + (-H - O0) + 3) / 4;
      float vf[4 * NV];
      load_cells<NV>(lb, O0, vf);
      // group minima and maxima on the bit patterns (non-negative cells: unsigned order is the
      // float order; v_min/max_u32 need no NaN canonicalisation, v_min3/max3_u32 fold pairs)
      uint32_t v[4 * NV];
#pragma unroll
      for (int k = 0; k < 4 * NV; ++k) v[k] = __float_as_uint(vf[k]);
      uint32_t g[WW - 3];
      {
        uint32_t m2[WW - 1];
#pragma unroll
        for (int k = 0; k < WW - 1; ++k) m2[k] = min(v[-H - O0 + k], v[-H - O0 + k + 1]);
#pragma unroll
        for (int k = 0; k < WW - 3; ++k) g[k] = min(m2[k], m2[k + 2]);
      }
#pragma unroll
      for (int i = 0; i < CELLS; ++i) {
        const float cut = vf[-O0 + i];
        uint32_t sb;
        if (one_group) {
          // reject <=> alpha M >= cut for the largest group minimum M.  fma(alpha, M, -cut) < 0
          // (exact product) survives a few cells the rounded test would reject -- never the
          // reverse (alpha M >= cut exactly implies fl(alpha M) >= cut) -- and the exact count
          // below decides those, so the screen stays conservative.  Sign bit = survival.
          uint32_t M = g[i];
#pragma unroll
          for (int q = 1; q < NGS; ++q) M = max(M, g[i + 4 * q]);
#pragma unroll
          for (int q = 0; q < NGS; ++q) M = max(M, g[i + RO + 4 * q]);
          sb = __float_as_uint(__builtin_fmaf(cf.alpha, __uint_as_float(M), -cut)) >> 31;
        } else {
          const uint32_t cbits = __float_as_uint(cut);
          uint32_t nlt = 0;  // groups with alpha * min < cut
#pragma unroll
          for (int q = 0; q < NGS; ++q)
            nlt += lt_bit(__float_as_uint(cf.alpha * __uint_as_float(g[i + 4 * q])), cbits) +
                   lt_bit(__float_as_uint(cf.alpha * __uint_as_float(g[i + RO + 4 * q])), cbits);
          sb = 4 * (2 * NGS - (int)nlt) < need ? 1u : 0u;
        }
        bits |= sb << i;
      }
    }
    // Exact count for the survivors only, one survivor per lane.  About 12 of a tile's 1024
    // cells survive the screen on noise + targets, but they sit in ~8 of the 16 cell
    // indices, so counting per index for the whole wave (where any lane survived) cost 8 x 16
    // compares per lane; the ordered survivor list costs one 16-compare round per 64.
    int n_surv;
    const int sx = wave_excl_scan(__popc(bits), n_surv);
    if (n_surv != 0) {  // uniform
      {
        int o = sx;
        for (uint32_t m = bits; m; m &= m - 1, ++o) list[o] = ((uint32_t)rr << 16) | (uint32_t)(d0 + __builtin_ctz(m));
      }
      pass_sync<false>();
      for (int i0 = 0; i0 < n_surv; i0 += 64) {
        const int i = i0 + lane;
        bool det = false;
        uint32_t cell = 0;
        if (i < n_surv) {
          cell = list[i];
          const int d = (int)(cell & 0xffffu);
          const float* cp = mags + (int)(cell >> 16) * RS + midx(d);
          // midx(d + o) - midx(d) = o + 4 floor((q + o) / 16), q = (d + MH) % 16, |o| < 16
          const int q = (d + MH) & 15;
          auto ref = [&](int o) { return cp[o + 4 * ((q + o) >> 4)]; };
          const uint32_t cbits = __float_as_uint(cp[0]);
          uint32_t lt = 0;
#pragma unroll
          for (int j = 0; j < REF; ++j)
            lt += lt_bit(__float_as_uint(cf.alpha * ref(-GUARD - 1 - j)), cbits) +
                  lt_bit(__float_as_uint(cf.alpha * ref(GUARD + 1 + j)), cbits);
          det = (int)lt > cf.rank;
        }
        // in-place ordered compaction: every lane has read its entry of this round, and the
        // detections land at positions <= their survivor index
        const uint64_t bal = __ballot(det);
        const int pos = total + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
        if (det) list[pos] = cell;
        total += (int)__popcll(bal);
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < CELLS; ++i) {
      const int d = d0 + i;
      const uint32_t c = __float_as_uint(mrow[midx(d)]);
      uint32_t lt = 0;
      for (int j = 1; j <= cf.ref; ++j) {
        lt += lt_bit(__float_as_uint(cf.alpha * mrow[midx((d - cf.guard - j) & (NC - 1))]), c);
        lt += lt_bit(__float_as_uint(cf.alpha * mrow[midx((d + cf.guard + j) & (NC - 1))]), c);
      }
      bits |= ((int)lt > cf.rank ? 1u : 0u) << i;
    }
    const int excl = wave_excl_scan(__popc(bits), total);
    int o = excl;
    for (uint32_t m = bits; m; m &= m - 1, ++o) list[o] = ((uint32_t)rr << 16) | (uint32_t)(d0 + __builtin_ctz(m));
  }
  const uint32_t base = det_reserve_wave(sink, tile, total);
  if (total == 0) return;  // uniform
  // Detections cluster (a target lights up consecutive cells of one lane), so the ranked
  // value is computed one detection per lane over the whole wave, from the ordered list of
  // detected cells (rr << 16 | d) in `list` (capacity: the tile's cells).
  pass_sync<false>();
  for (int i = lane; i < total; i += 64) {
    const uint32_t cell = list[i];
    const int rl = (int)(cell >> 16), d = (int)(cell & 0xffffu);
    const float* row = mags + rl * RS;
    float ranked = 0.f;
    if constexpr (REF > 0) {
      float r[2 * REF];
#pragma unroll
      for (int j = 0; j < REF; ++j) {
        r[j] = row[midx(d - GUARD - 1 - j)];
        r[REF + j] = row[midx(d + GUARD + 1 + j)];
      }
      ranked = ranked_of<REF, GUARD>(r, cf.rank);
    } else {
      for (int j = 0; j < nref; ++j) {
        const int oj = j < cf.ref ? -(cf.guard + 1 + j) : (cf.guard + 1 + j - cf.ref);
        const float vj = row[midx((d + oj) & (NC - 1))];
        int lt = 0, le = 0;
        for (int i2 = 0; i2 < nref; ++i2) {
          const int o2 = i2 < cf.ref ? -(cf.guard + 1 + i2) : (cf.guard + 1 + i2 - cf.ref);
          const float v2 = row[midx((d + o2) & (NC - 1))];
          lt += v2 < vj;
          le += v2 <= vj;
        }
        if (lt <= cf.rank && cf.rank < le) ranked = vj;
      }
    }
    const uint32_t slot = base + (uint32_t)i;
    if (slot < sink.cap) {
      fmcw_det dd;
      dd.frame = (uint32_t)frame;
      dd.range = (uint16_t)(r0 + rl);
      dd.doppler = (uint16_t)d;
      dd.mag = row[midx(d)];
      dd.threshold = cf.alpha * ranked;
      sink.scratch[slot] = dd;
    }
  }
}

// RTL-compat 1-D threshold of cell d (rtl/old/os_cfar.vhd:117-132): the 2 ref integer cells
// q17(.) around d (circular), the rank-th smallest by counting (lt <= rank < le picks it, ties
// included), T = (ranked * SCALING_MULT / SCALING_DIV) resized to 17 bits = mod 2^17.
template <int NC>
__device__ __forceinline__ uint32_t rtl1d_threshold(const float* mrow, int d, const Cfar1DArgs& cf) {
  const int nref = 2 * cf.ref;
  uint32_t ranked = 0;
  for (int j = 0; j < nref; ++j) {
    const int oj = j < cf.ref ? -(cf.guard + 1 + j) : (cf.guard + 1 + j - cf.ref);
    const float vj = q17(mrow[midx((d + oj) & (NC - 1))]);
    int lt = 0, le = 0;
    for (int i2 = 0; i2 < nref; ++i2) {
      const int o2 = i2 < cf.ref ? -(cf.guard + 1 + i2) : (cf.guard + 1 + i2 - cf.ref);
      const float v2 = q17(mrow[midx((d + o2) & (NC - 1))]);
      lt += v2 < vj;
      le += v2 <= vj;
    }
    if (lt <= cf.rank && cf.rank < le) ranked = (uint32_t)vj;
  }
  return (ranked * (uint32_t)cf.alpha) & kQ17Mask;
}

// 1-D OS-CFAR in RTL-compat arithmetic (FMCW_COMPAT_CFAR) over a wave tile's magnitude rows:
// detect q17(cut) > T with the wrapped 17-bit threshold, which is not monotone in the ranked
// cell, so every cell gets its exact ranked value (no screen).  Same ordered emission as
// cfar1d_wave.
template <int NC>
__device__ __forceinline__ void cfar1d_wave_rtl(const float* mags, uint32_t* list, int rr, int t, int r0,
                                                int frame, int tile, const Cfar1DArgs& cf,
                                                const DetSink& sink) {
  constexpr int RS = DopplerGeom<NC>::REGM;
  const float* mrow = mags + rr * RS;
  const int d0 = t * 16;
  const int lane = (int)(threadIdx.x & 63);
  uint32_t bits = 0;
  for (int i = 0; i < 16; ++i) {
    const int d = d0 + i;
    const uint32_t cut = (uint32_t)q17(mrow[midx(d)]);
    bits |= (cut > rtl1d_threshold<NC>(mrow, d, cf) ? 1u : 0u) << i;
  }
  int total;
  const int excl = wave_excl_scan(__popc(bits), total);
  {
    int o = excl;
    for (uint32_t m = bits; m; m &= m - 1, ++o) list[o] = ((uint32_t)rr << 16) | (uint32_t)(d0 + __builtin_ctz(m));
  }
  const uint32_t base = det_reserve_wave(sink, tile, total);
  if (total == 0) return;  // uniform
  pass_sync<false>();
  for (int i = lane; i < total; i += 64) {
    const uint32_t cell = list[i];
    const int rl = (int)(cell >> 16), d = (int)(cell & 0xffffu);
    const float* row = mags + rl * RS;
    const uint32_t slot = base + (uint32_t)i;
    if (slot < sink.cap) {
      fmcw_det dd;
      dd.frame = (uint32_t)frame;
      dd.range = (uint16_t)(r0 + rl);
      dd.doppler = (uint16_t)d;
      dd.mag = q17(row[midx(d)]);
      dd.threshold = (float)rtl1d_threshold<NC>(row, d, cf);
      sink.scratch[slot] = dd;
    }
  }
}

// Dispatch on the compile-time fast path (the reference geometry REF 8 / GUARD 2).
template <int NC>
__device__ __forceinline__ void cfar1d_dispatch(const float* mags, uint32_t* list, int rr, int t, int r0,
                                                int frame, int tile, const Cfar1DArgs& cf,
                                                const DetSink& sink) {
  if (cf.compat)
    cfar1d_wave_rtl<NC>(mags, list, rr, t, r0, frame, tile, cf, sink);
  else if (cf.ref == 8 && cf.guard == 2 && 2 * cf.ref - cf.rank <= 4)
    cfar1d_wave<NC, 8, 2, true>(mags, list, rr, t, r0, frame, tile, cf, sink);
  else if (cf.ref == 8 && cf.guard == 2)
    cfar1d_wave<NC, 8, 2>(mags, list, rr, t, r0, frame, tile, cf, sink);
  else
    cfar1d_wave<NC, 0, 0>(mags, list, rr, t, r0, frame, tile, cf, sink);
}

// Stand-alone 1-D OS-CFAR over a caller-supplied [frame][range][doppler] map (fmcw_cfar),
// on the same wave tiles as K2 (so tile ids, and the detection order, are the same).
template <int NC>
__global__ void __launch_bounds__(DopplerGeom<NC>::NT)
k_cfar1d(const float* __restrict__ map, int ns, int n_tiles, int frame0, int tile0, Cfar1DArgs cf,
         DetSink sink) {
  using Gm = DopplerGeom<NC>;
  constexpr int P = Gm::P, WR = Gm::WR, WPB = Gm::WPB, REGM = Gm::REGM;
  __shared__ __attribute__((aligned(16))) float lds[WPB * Gm::WFL];
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float* const mags = lds + wv * Gm::WFL;
  uint32_t* const list = reinterpret_cast<uint32_t*>(mags + Gm::LIST);
  const int tiles_per_frame = ns / WR;
  const int nf = n_tiles / tiles_per_frame;
  for (int tile = blockIdx.x * WPB + wv; tile < n_tiles; tile += gridDim.x * WPB) {
    const int lane = opaque(threadIdx.x & 63);
    // frame-minor order: consecutive tiles are the same rows of consecutive frames, so the
    // rows that hold a target (more candidates, more detections) spread over all waves
    const int f = tile % nf;
    const int lt = tile / nf;                    // wave tile within the frame
    const int r0 = lt * WR;
    const float* src = map + ((size_t)f * ns + r0) * NC;
#pragma unroll
    for (int i = 0; i < WR * NC / 4 / 64; ++i) {
      const int e = 4 * (lane + 64 * i);
      const int rl = e / NC, d = e - rl * NC;
      *reinterpret_cast<float4*>(mags + rl * REGM + midx(d)) = nonneg4(*reinterpret_cast<const float4*>(src + e));
    }
    pass_sync<false>();
    fill_halo<NC, P>(mags + (lane / P) * REGM, lane % P);
    pass_sync<false>();
    cfar1d_dispatch<NC>(mags, list, lane / P, lane % P, r0, frame0 + f, tile0 + f * tiles_per_frame + lt, cf,
                        sink);
    pass_sync<false>();  // the region is reused by the next tile
  }
}

// --------------------------------------------------------------------------------------
// K2: Doppler window + FFT + magnitude (+NCI over rx) + map + 1-D OS-CFAR, one wave tile at a
// time (see "Wave tiles" above).  Lane (rr, t) of P = NC/16 owns range row r0 + rr's
// transform.  Pass 1 (radix 16, no twiddles) reads its 16 points c = t + P m straight from
// the tiled spectrum (8-byte loads: two 256-B runs per load instruction across the wave's
// rows and lanes); the Doppler window was already applied by K1 (MTI off) or is applied here
// after the canceller (MTI on); the last pass stays in registers and feeds |X|^2 (summed over
// rx: NCI) directly.
// --------------------------------------------------------------------------------------
// FMCW_COMPAT_MTI word format: round half to even (the IP's convergent rounding) and saturate
// to int16, per component; and the canceller's output saturation (doppler_notch.vhd:75-93).
__device__ __forceinline__ float sat16(float v) { return fminf(fmaxf(v, -32768.f), 32767.f); }
__device__ __forceinline__ float2 sat16c(float2 v) { return make_float2(sat16(v.x), sat16(v.y)); }
__device__ __forceinline__ float2 q16c(float2 v) { return make_float2(sat16(rintf(v.x)), sat16(rintf(v.y))); }
// the same, counting a sample whose I or Q clipped
__device__ __forceinline__ float2 q16c_count(float2 v, uint32_t& n) {
  const float2 r = make_float2(rintf(v.x), rintf(v.y)), q = sat16c(r);
  n += (uint32_t)(q.x != r.x || q.y != r.y);
  return q;
}
__device__ __forceinline__ float2 sat16c_count(float2 v, uint32_t& n) {
  const float2 q = sat16c(v);
  n += (uint32_t)(q.x != v.x || q.y != v.y);
  return q;
}
// RTL-compat Q15 window on an int16 word pair: y = sat16(floor((x c + 2^14) / 2^14)) per
// component (window_multiplier.vhd:126-158), c = the ROM integer; x c < 2^31 for int16 words.
__device__ __forceinline__ float2 win_q15c(float2 x, float c, uint32_t& n) {
  const int ci = (int)c;
  const int yi = ((int)x.x * ci + (1 << 14)) >> 14, yq = ((int)x.y * ci + (1 << 14)) >> 14;
  const int si = min(max(yi, -32768), 32767), sq = min(max(yq, -32768), 32767);
  n += (uint32_t)(si != yi || sq != yq);
  return make_float2((float)si, (float)sq);
}

// Workgroups are dispatched round-robin over the 8 XCDs (XCD = id % 8, MI355X_MICROARCH.md).
// Giving each XCD a contiguous range of logical ids puts neighbouring tiles -- which read the
// two halves of the same 128-B lines of the tiled spectrum when a workgroup covers only 64 B of
// each 1 KiB tile (NC = 1024: 4 range rows x 16 B) -- behind the same L2.
__device__ __forceinline__ int xcd_block_id(int bid, int grid) {
  if (grid & 7) return bid;
  return (bid & 7) * (grid >> 3) + (bid >> 3);
}

// K2's register prefetch of the next (tile, rx) unit (MTI off), points loaded ahead: all 16 up to
// NC = 256; 8 (half a unit) at NC = 512, which fits 165 instead of 178 VGPRs and so 3 waves per
// SIMD (config-3 K2 41.6-41.9 -> 39.0-39.2 us per launch, profiles/r03/k2/k2_pf_ab.log; 16 points
// 42.1, none 42.2-42.5); none at NC = 1024 (8 or 16 points: 61-64 against 56 us).
template <int NC, int MTI>
// (Round 6, config 3: 4 points ahead 38.4-38.9 against 35.8-35.9 us per launch, profiles/r06/k2_c3_ab/.)
constexpr int k2_prefetch() { return MTI != 0 ? 0 : NC <= 256 ? 16 : NC == 512 ? 8 : 0; }
// FAST (below) at NC = 256 fits 128 VGPRs without scratch: 4 waves per SIMD (4 workgroups of
// 39 KiB LDS per CU); measured K2 58.2 -> 56.0 us per 96-frame launch at config 2.  At NC = 512
// / 1024 the fourth wave costs more than it hides (config 3 K2 41.7 -> 55.9 us, config 5 55.5
// -> 74.6 us per launch; gpurun_out bench_libs, round 2).  The S48 FAST K2 at NC = 256: 4 waves
// (128 VGPRs, 16 B of scratch) measured 0.570 us per frame, 3 waves 0.584-0.598, an 8-point
// prefetch 0.571-0.574 (profiles/r05/spec_ab/).
template <int NC, int MTI, bool FAST = false>
constexpr int k2_waves() { return (FAST && MTI == 0 && NC == 256) ? 4 : 2; }
// FAST: the common configuration fixed at compile time -- |X| magnitude (no AMBM), no dB map,
// and the 1-D CFAR, when enabled, at the reference geometry (8 refs / 2 guards per side, need =
// n_ref - rank <= 4, fp32 compare).  The generic kernel keeps those as uniform runtime branches,
// whose other arms held registers and SGPRs (spills to VGPR lanes) across the tile loop.
// SP: the spectrum format K1 wrote (SP_F32, SP_F16, SP_S48 quad form (T >= 8, P % 4 == 0), SP_S48S / SP_S48PS
// pair form (T = 2, P % 2 == 0); S48 with MTI off).
template <int NC, int MTI, int SP = SP_F32, bool FAST = false>
__global__ void __launch_bounds__(DopplerGeom<NC>::NT) __attribute__((amdgpu_waves_per_eu(k2_waves<NC, MTI, FAST>())))
k_doppler(const float2* __restrict__ inter_in, const float* __restrict__ win_d, int ns, int nrx,
          int lgT, int lgRB, int n_tiles, int frame0, int tile0, float* __restrict__ lin_map,
          float* __restrict__ db_map, int mag_mode, int mti_rtl, int q15d, Cfar1DArgs cf, DetSink sink,
          uint32_t* __restrict__ status) {
  using Gm = DopplerGeom<NC>;
  constexpr int P = Gm::P, WR = Gm::WR, WPB = Gm::WPB, REGD = Gm::REGD, REGM = Gm::REGM;
  constexpr int LR = Gm::LR, LG = Gm::LG;
  static_assert(P <= 64, "a Doppler transform must fit one wave");
  __shared__ __attribute__((aligned(16))) float lds[WPB * Gm::WFL];

  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane0 = threadIdx.x & 63;
  using SE = typename SpecEl<SP>::T;
  const SE* const inter = reinterpret_cast<const SE*>(inter_in);
  const float sscale = SP == SP_F16 ? (float)ns : 1.f;  // undoes K1's 1 / N_range of an fp16 spectrum
  constexpr int SGS = s48_strided_g<SP>();  // strided S48: a lane's SGS points per element (no exchange)
  constexpr bool S48S = SGS > 0;
  constexpr bool S48F = SP == SP_S48;  // adjacent quads: exponent pieces ORed over a lane quad
  constexpr int SG = 4;
  static_assert(!S48F || (MTI == 0 && P % SG == 0), "S48: a lane group holds a chirp group");
  static_assert(!S48S || MTI == 0, "S48: MTI off");
  // S48: this lane's chirps c = t + P m all sit at c % G = t % G of their group (t = lane % P);
  // the two lane constants are derived from t where they are used (not held across the loop)
  auto s48_sh = [](int tt) { return (uint32_t)(tt & 1) << 4; };   // byte offset x 8 of the record in its load
  auto s48_qs = [](int tt) { return (uint32_t)(tt & (SG - 1)) * (8 / SG); };  // its exponent piece's shift
  const int rr = lane0 / P;
  const int t0 = lane0 % P;
  float* const mags = lds + wv * Gm::WFL;
  float2* const wreg = reinterpret_cast<float2*>(mags);
  uint32_t* const list = reinterpret_cast<uint32_t*>(mags + Gm::LIST);
  const int tiles_per_frame = ns / WR;
  const int nf = n_tiles / tiles_per_frame;
  const int T = 1 << lgT;
  const int lgncb = __builtin_ctz(NC) - lgT;
  // Doppler window for this lane's chirps c = t + P m.  MTI off: K1 already applied it
  // (chirp_w), so no registers are spent on it here.  MTI on: the canceller must see the
  // unwindowed spectrum (doppler_notch precedes doppler_fft, radar_core.vhd:329-352).
  // q15d (FMCW_WIN_Q15_RTL, generic kernel only): win_d holds the ROM integers c[n] and the
  // window is the RTL's integer arithmetic on the spectrum's int16 words, applied here.
  constexpr bool WIN_K2 = MTI != 0 || !FAST;
  float wv_d[WIN_K2 ? 16 : 1];
  if constexpr (WIN_K2) {
    if (MTI != 0 || q15d) {
#pragma unroll
      for (int m = 0; m < 16; ++m) wv_d[m] = win_d[t0 + P * m];
    }
  }
  uint32_t n_wsat = 0, n_msat = 0;  // saturated samples: integer Doppler window; int16 words / MTI

  // element (r, c) of the tiled spectrum: ((rb*NCB + c/T)*RB + r%RB)*T + c%T
  auto off_of = [&](uint32_t rbase, uint32_t rin, uint32_t c) -> uint32_t {
    return ((((rbase + (c >> lgT)) << lgRB) + rin) << lgT) | (c & (uint32_t)(T - 1));
  };

  // Software pipeline (MTI off): the 16 points of the next (tile, rx) unit are loaded into
  // registers right after this unit's first pass has consumed its own, so a wave keeps 8 KiB
  // of HBM reads in flight through its FFT, magnitude, map store and CFAR phases instead of
  // exposing the full load latency once per unit.
  constexpr int NPF = k2_prefetch<NC, MTI>();  // points loaded ahead
  constexpr bool PF = NPF > 0;
  // Tile order: the WPB waves of a workgroup take WPB consecutive wave tiles (row groups) of one
  // frame, frame-minor over workgroups, so the 4 x WR rows they read from each 1 KiB block of the
  // tiled spectrum are requested together (DRAM page locality; round 1, config 2: K2 0.905 ->
  // 0.874 us/frame against frame-minor over all waves, which remains for frames whose tile count
  // is not a multiple of WPB).
  const bool grp = tiles_per_frame % WPB == 0;
  auto tile_fl = [&](int tl, int& fo, int& lo) {
    if (grp) {
      const int u = tl / WPB;
      fo = u % nf;
      lo = (u / nf) * WPB + (tl % WPB);
    } else {
      fo = tl % nf;
      lo = tl / nf;
    }
  };
  const int tile_step = gridDim.x * WPB;
  auto unit_src = [&](int tl, int rx) -> const SE* {
    int fu, lu;
    tile_fl(tl, fu, lu);
    const int ru = lu * WR + rr;
    return inter + ((size_t)fu * nrx + rx) * (size_t)ns * NC +
           off_of((uint32_t)(ru >> lgRB) << lgncb, (uint32_t)(ru & ((1 << lgRB) - 1)), 0);
  };
  float2 nxt[PF && !S48S ? NPF : 1];  // prefetched points (S48 quads: the raw 8 bytes)
  fmcw_u3v nxq[PF && S48S ? NPF / 2 : 1];  // strided S48: 12-B loads (a quad's halves, or a pair)
  const __amdgpu_buffer_rsrc_t srs = wt_rsrc(const_cast<SE*>(inter), 0xffffffffu);  // the prefetch's buffer loads
  // last-pass twiddle bases, once per lane (NC = 256: pass 1 + one radix-16 pass, k = t)
  constexpr bool TWH = NC / 16 <= 16 && P % 16 == 0;
  GroupTwiddles<NC / 16, NC> twh;
  if constexpr (TWH) twh.init(t0 & 15);
  auto prefetch = [&](int tl, int rx) {
    if constexpr (PF) {
      if (tl < n_tiles) {
        const SE* p = unit_src(tl, rx);
        const int tq = opaque(t0);
        if constexpr (S48S) {
          // group k of lane t: K1 group cb = t + P k of the row block, element j = 0; groups P apart
          const uint32_t vo = (uint32_t)((const char*)(p + (((uint32_t)tq << lgRB) << lgT)) - (const char*)inter);
          const uint32_t sb = (((uint32_t)P << lgRB) << lgT) * (uint32_t)sizeof(S48);
          uint32_t so = 0;
#pragma unroll
          for (int k = 0; k < NPF / SGS; ++k) {
#pragma unroll
            for (int h = 0; h < SGS / 2; ++h)
              nxq[(SGS / 2) * k + h] = __builtin_bit_cast(fmcw_u3v, __builtin_amdgcn_raw_buffer_load_b96(srs, vo, so + 12u * h, 0));
            so += sb;
            asm volatile("" : "+s"(so));
          }
        } else if ((P & (T - 1)) == 0) {  // uniform: chirps t + P m sit a fixed S elements apart
          const SE* pb = p + ((((uint32_t)tq >> lgT) << lgRB) << lgT) + ((uint32_t)tq & (uint32_t)(T - 1));
          const uint32_t S = (uint32_t)(P >> lgT) << (lgRB + lgT);
          // the uniform m S byte offsets, one SGPR advanced per load: left to the compiler, the 16
          // products were hoisted out of the tile loop and held in 16 SGPRs, which pushed 25
          // others into VGPR lanes (a v_readlane per use inside the loop)
          uint32_t so = 0;
          const uint32_t sb = S * (uint32_t)sizeof(SE);
#pragma unroll
          for (int m = 0; m < NPF; ++m) {
            if constexpr (S48F) {
              // the raw 8 bytes at the point's record rounded down to 4 (decoded at use)
              const uint32_t vo = (uint32_t)((const char*)pb - (const char*)inter) - (s48_sh(tq) >> 3);
              typedef float f2v __attribute__((ext_vector_type(2)));
              const f2v r = __builtin_bit_cast(
                  f2v, __builtin_amdgcn_raw_buffer_load_b64(srs, vo, so, kNtSpecLd ? 2 /* nt */ : 0));
              nxt[m] = make_float2(r.x, r.y);
              so += sb;
              asm volatile("" : "+s"(so));
            } else if constexpr (SP == SP_F32) {
              // buffer load: lane offset in a VGPR, the uniform m S in an SGPR (no 64-bit VALU
              // address add per load; the chunk's spectrum is < 4 GiB, fmcw_create caps it)
              const uint32_t vo = (uint32_t)((const char*)pb - (const char*)inter);
              typedef float f2v __attribute__((ext_vector_type(2)));
              const f2v r = __builtin_bit_cast(
                  f2v, __builtin_amdgcn_raw_buffer_load_b64(srs, vo, so, kNtSpecLd ? 2 /* nt */ : 0));
              nxt[m] = make_float2(r.x, r.y);
              so += sb;
              asm volatile("" : "+s"(so));
            } else {
              nxt[m] = ld_spec<kNtSpecLd>(pb + (size_t)m * S, sscale);
            }
          }
        } else {
#pragma unroll
          for (int m = 0; m < NPF; ++m) {
            const uint32_t c = (uint32_t)(tq + P * m);
            const SE* pc = p + ((((c >> lgT) << lgRB) << lgT) | (c & (uint32_t)(T - 1)));
            if constexpr (S48F) {
              const fmcw_u2v r = ld_s48_raw<kNtSpecLd>(pc, (uint32_t)tq & 1u);
              nxt[m] = make_float2(__uint_as_float(r.x), __uint_as_float(r.y));
            } else {
              nxt[m] = ld_spec<kNtSpecLd>(pc, sscale);
            }
          }
        }
      }
    }
  };
  // XCD-contiguous ids only where a workgroup reads less than a 128-B line of each tile
  // (measured: config 5 K2 177 -> 110 us per 4 frames; configs 2 / 3, whose workgroups read
  // whole lines, 2-3 % slower with it)
  // (S48: its 6-B points, so config 3's 96-B reads take the XCD mapping too)
  // (round 6, config 3 with the remap: K2 37.0-37.9 against 35.8-35.9 us per launch, profiles/r06/k2_c3_ab/)
  const bool xcd = ((WPB * WR * (S48F || S48S ? 6 : 8)) << lgT) < 128;
  const int bid = xcd ? xcd_block_id((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
  prefetch(bid * WPB + wv, 0);

  for (int tile = bid * WPB + wv; tile < n_tiles; tile += tile_step) {
    const int t = opaque(t0);
    float2* buf = wreg + rr * REGD;
    // frame-minor order: consecutive tiles are the same rows of consecutive frames, so the
    // rows that hold a target (more candidates, more detections) spread over all waves
    int f, lt;                                   // frame, wave tile within the frame
    tile_fl(tile, f, lt);
    const int r0 = lt * WR;
    const int r = r0 + rr;
    const uint32_t rbase = (uint32_t)(r >> lgRB) << lgncb;
    const uint32_t rin = (uint32_t)(r & ((1 << lgRB) - 1));
    float acc[LG][LR];
#pragma unroll
    for (int g = 0; g < LG; ++g)
#pragma unroll
      for (int m = 0; m < LR; ++m) acc[g][m] = 0.f;

    for (int rx = 0; rx < nrx; ++rx) {
      const SE* src = inter + ((size_t)f * nrx + rx) * (size_t)ns * NC;
      auto at = [&](uint32_t c) -> float2 {
        if constexpr (S48S) return make_float2(0.f, 0.f);  // (unused: the points come from vq)
        else if constexpr (S48F) return s48_unpack<SG>(ld_s48_raw<kNtSpecLd>(src + off_of(rbase, rin, c), c & 1u), (uint32_t)t & 1u, s48_qs(t));
        else return ld_spec<kNtSpecLd>(src + off_of(rbase, rin, c), sscale);
      };
      float2 v[16];
      // strided S48: all 16 points decoded here, SGS per element, prefetched or loaded now
      float2 vq[S48S ? 16 : 1];
      if constexpr (S48S) {
        const uint32_t q_vo = (uint32_t)((const char*)(src + off_of(rbase, rin, (uint32_t)t << lgT)) - (const char*)inter);
        const uint32_t q_sb = (((uint32_t)P << lgRB) << lgT) * (uint32_t)sizeof(S48);
#pragma unroll
        for (int k = 0; k < 16 / SGS; ++k) {
          fmcw_u3v w[SGS / 2];
#pragma unroll
          for (int h = 0; h < SGS / 2; ++h) {
            if (SGS * k < NPF) w[h] = nxq[SGS * k < NPF ? (SGS / 2) * k + h : 0];
            else w[h] = __builtin_bit_cast(fmcw_u3v, __builtin_amdgcn_raw_buffer_load_b96(srs, q_vo, (uint32_t)k * q_sb + 12u * h, 0));
          }
          if constexpr (SGS == 4) {
            float2 o[4];
            s48s_unpack4(w[0], w[SGS / 2 - 1], o);
#pragma unroll
            for (int j = 0; j < 4; ++j) vq[4 * k + j] = o[j];
          } else {
            float2 o[2];
            s48ps_unpack2(w[0], o);
            vq[2 * k] = o[0];
            vq[2 * k + 1] = o[1];
          }
        }
      }
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const int c = t + P * m;
        float2 x;
        if (S48S) {
          x = vq[S48S ? m : 0];
        } else if (m < NPF) {
          x = nxt[m < NPF && !S48S ? m : 0];
          if constexpr (S48F) x = s48_unpack<SG>(fmcw_u2v{__float_as_uint(x.x), __float_as_uint(x.y)}, (uint32_t)t & 1u, s48_qs(t));
        } else {
          x = at((uint32_t)c);
        }
        // RTL-compat words: the corner turner hands the FFT IP's 16-bit output words on
        // (round half to even, saturate; counted in status word 3)
        const bool words = !FAST && (mti_rtl || q15d);
        if (words) x = q16c_count(x, n_msat);
        if constexpr (MTI >= 2) {  // MTI canceller along slow time, zero history (doppler_notch.vhd:72-102)
          float2 x1 = c >= 1 ? at((uint32_t)(c - 1)) : make_float2(0.f, 0.f);
          float2 x2 = make_float2(0.f, 0.f);
          if constexpr (MTI == 3) x2 = c >= 2 ? at((uint32_t)(c - 2)) : make_float2(0.f, 0.f);
          if (words) {  // 16-bit words in (their own clipping was counted at their own chirp)
            x1 = q16c(x1);
            x2 = q16c(x2);
          }
          // integers below 2^18 on words: every step below is exact
          x = MTI == 2 ? csub(x, x1) : cadd(csub(x, cscale(x1, 2.f)), x2);
          if (words) x = sat16c_count(x, n_msat);  // the canceller's saturating output (:76-93)
        }
        if constexpr (WIN_K2) {
          if (!FAST && q15d) x = win_q15c(x, wv_d[m], n_wsat);  // window_multiplier.vhd:146-158
          else if (MTI != 0) x = cscale(x, wv_d[m]);
        }
        v[m] = x;
      }
      Dft<16>::run(v);                       // pass 1: L = 1, no twiddles
      {
        float2* d = buf + pad16(16 * t);     // y[16 t + m]
#pragma unroll
        for (int m = 0; m < 16; ++m) d[m] = v[m];
      }
      pass_sync<false>();
      {
        // one prefetch site: two (one per branch) merged their register results through copies
        // (round 6: issued right after the strided-S48 decode instead, config 2 K2 measured 64.5-67.8
        // against 64.7-65.3 us per launch, profiles/r06/k2_early_pf/)
        const bool same = rx + 1 < nrx;
        prefetch(same ? tile : tile + tile_step, same ? rx + 1 : 0);
      }
      float2 X[LG][LR];
      if constexpr (TWH) stockham_last_tw<NC, 16, P>(buf, t, X, twh);
      else stockham_to_regs<NC, 16, P, false>(buf, t, X);
      if (!FAST && mag_mode == FMCW_MAG_AMBM) {  // uniform: one branch for the whole block
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
          for (int m = 0; m < LR; ++m) acc[g][m] = rx == 0 ? cabs2(X[g][m]) : acc[g][m] + cabs2(X[g][m]);
      }
      pass_sync<false>();  // every read of the last pass is issued: the rows may be rewritten
    }
    // magnitudes -> the wave region (over the dead FFT rows), for the map store and the CFAR
    const bool ambm = !FAST && mag_mode == FMCW_MAG_AMBM;
    float* mrow = mags + rr * REGM;
#pragma unroll
    for (int g = 0; g < LG; ++g) {
      float* m0 = mrow + midx(t + P * g);
#pragma unroll
      for (int m = 0; m < LR; ++m)
        m0[mpadoff(m * (NC / LR))] = ambm ? acc[g][m] : mag_sqrt(acc[g][m]);
    }
    pass_sync<false>();
    if (cf.enabled) {
      fill_halo<NC, P>(mrow, t);
      pass_sync<false>();
    }

    // map store: WR*NC = 1024 floats contiguous at [f][r0][0], 16 B per lane
    {
      constexpr int Q = WR * NC / 4 / 64;
      const size_t mbase = ((size_t)f * ns + r0) * NC;
      const int lane = opaque(lane0);
#pragma unroll
      for (int i = 0; i < Q; ++i) {
        const int e = 4 * (lane + 64 * i);
        const int rl = e / NC, d = e - rl * NC;
        const float4 v = *reinterpret_cast<const float4*>(mags + rl * REGM + midx(d));
        if (lin_map) {
          st_f4<kNtMap>(lin_map + mbase + e, v);
        }
        if (!FAST && db_map) {
          const float k = 6.0205999132796239f;  // 20 / log2(10)
          *reinterpret_cast<float4*>(db_map + mbase + e) =
              make_float4(k * __log2f(v.x + 1.f), k * __log2f(v.y + 1.f), k * __log2f(v.z + 1.f),
                          k * __log2f(v.w + 1.f));
        }
      }
    }
    if (cf.enabled) {
      if constexpr (FAST)
        cfar1d_wave<NC, 8, 2, true>(mags, list, rr, t, r0, frame0 + f, tile0 + f * tiles_per_frame + lt, cf, sink);
      else
        cfar1d_dispatch<NC>(mags, list, rr, t, r0, frame0 + f, tile0 + f * tiles_per_frame + lt, cf, sink);
    }
    pass_sync<false>();  // the region is reused by the next tile
  }
  if constexpr (!FAST) {
    if (mti_rtl || q15d) {  // uniform
      status_add(status, n_wsat);
      status_add(status ? status + 1 : nullptr, n_msat);
    }
  }
}

// --------------------------------------------------------------------------------------
// K3: 2-D OS-CFAR (rtl/src/os_cfar_2d.vhd:140-217) -- see cfar2d.hpp.
// --------------------------------------------------------------------------------------
#include "cfar2d.hpp"

}  // namespace fmcw
