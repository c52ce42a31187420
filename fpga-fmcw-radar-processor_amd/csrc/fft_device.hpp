// fft_device.hpp -- LDS-staged Stockham FFT building blocks for gfx950 (CDNA4, wave64).
//
// Replaces the Xilinx LogiCORE FFT v9.1 instances of the reference
// (rtl/src/radar_core.vhd:303-316 range FFT, :351-364 Doppler FFT; forward transform,
// config word x"0001" at :247; natural-order output, xfft_0.xci:12-27).  The build spec is
// an *unscaled* fp32 forward DFT X[k] = sum_n x[n] exp(-2 pi i k n / N):
// the IP's block-floating-point exponent is discarded by the reference (:310) and is not
// reproduced.
//
// Decomposition (N = 2^n, 64 <= N <= 8192): P = N/16 threads per transform, 16 complex
// values per thread.  Pass 0 is radix-8 over stride N/8 taken straight from registers, so a
// thread's first-pass inputs are the 16-byte pairs (2t, 2t+1) + (N/8) m -- i.e. 16 B/lane
// coalesced loads.  Further passes are radix-16 while >= 16 points remain, then one final
// radix-2/4/8 pass, each a Stockham autosort step through LDS:
//     group j, k = j mod L:  v[m] = x[j + m N/R] * w_{LR}^{m k};  V = DFT_R(v);
//     y[(j/L) L R + k + m L] = V[m]
// LDS rows are padded by one complex per 16 (index i -> i + i/16) against bank conflicts.
// Twiddles: w^1, w^2, w^4, w^8 from v_sin_f32 / v_cos_f32 (argument in revolutions, exact
// k/LR fractions), other powers as products (GroupTwiddles).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fmcw {

// Complex arithmetic on packed fp32 (VOP3P v_pk_*_f32: one instruction per complex add, two
// per complex product).  Left to itself the SLP vectorizer pairs components of *different*
// complex values and then spends v_mov's re-pairing them (about a third of the FFT's VALU
// instructions, round 2); here every butterfly operation is one packed instruction on a (re, im)
// register pair, the -i rotations and the cross terms of the product folded into op_sel / neg
// modifiers.
typedef float fmcw_cf __attribute__((ext_vector_type(2)));
__device__ __forceinline__ fmcw_cf pk(float2 a) { return fmcw_cf{a.x, a.y}; }
__device__ __forceinline__ float2 unpk(fmcw_cf a) { return make_float2(a.x, a.y); }
__device__ __forceinline__ float2 cadd(float2 a, float2 b) {
  fmcw_cf r;
  asm("v_pk_add_f32 %0, %1, %2" : "=v"(r) : "v"(pk(a)), "v"(pk(b)));
  return unpk(r);
}
__device__ __forceinline__ float2 csub(float2 a, float2 b) {
  fmcw_cf r;
  asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(pk(a)), "v"(pk(b)));
  return unpk(r);
}
// a * b = (a.x b.x - a.y b.y, a.x b.y + a.y b.x): t = a.x * (b.x, b.y); r = t + (-a.y b.y, a.y b.x)
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  fmcw_cf t, r;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(pk(a)), "v"(pk(b)));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]"
      : "=v"(r) : "v"(pk(a)), "v"(pk(b)), "v"(t));
  return unpk(r);
}
// a + (-i) d = (a.x + d.y, a.y - d.x)   and   a - (-i) d = (a.x - d.y, a.y + d.x)
__device__ __forceinline__ float2 cadd_negi(float2 a, float2 d) {
  fmcw_cf r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(pk(a)), "v"(pk(d)));
  return unpk(r);
}
__device__ __forceinline__ float2 csub_negi(float2 a, float2 d) {
  fmcw_cf r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(pk(a)), "v"(pk(d)));
  return unpk(r);
}
__device__ __forceinline__ float2 mul_negi(float2 a) { return make_float2(a.y, -a.x); }  // -i a
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }

constexpr int padded(int n) { return n + n / 16; }
__device__ __forceinline__ int pad16(int i) { return i + (i >> 4); }
// pad16(x + o) for a compile-time offset o = m*S (S a power of two) when x % 16 < S or
// S % 16 == 0 -- true for every Stockham read (x = j < N/R) and write (x % 16 = k < L):
// the padded address is then pad16(x) plus an immediate, so ds_read/ds_write use offsets.
constexpr int padoff(int o) { return o + o / 16; }

// Loop-invariant values (lane index, twiddles, LDS addresses) would otherwise be hoisted out of
// the grid-stride loops by LICM and pinned in ~150 VGPRs; an opaque copy per iteration keeps
// them as cheap recomputation instead (occupancy matters more here than a few VALU ops).
__device__ __forceinline__ int opaque(int x) {
  asm volatile("" : "+v"(x));
  return x;
}

// Cache policy of the streamed HBM traffic (measured by tools/ablate.py against variant builds,
// DESIGN.md section 4): non-temporal (`nt`) loads of the input cube (read once; config 2, round 1:
// K1 0.785 -> 0.667 us/frame) and non-temporal stores of the map (written once; round 2: K2 0.761
// -> 0.728 us/frame); the corner-turned spectrum, which K2 reads back from the Infinity Cache, is
// stored and loaded with the default policy (non-temporal spectrum loads: configs 3 / 5 -30 %,
// round 4).
constexpr bool kNtCube = true, kNtSpecSt = false, kNtSpecLd = false, kNtMap = true;
typedef float fmcw_f4v __attribute__((ext_vector_type(4)));
typedef float fmcw_f2v __attribute__((ext_vector_type(2)));
typedef uint32_t fmcw_u2v __attribute__((ext_vector_type(2)));
typedef uint32_t fmcw_u4v __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ float4 ld_f4(const void* p) {
  fmcw_f4v v;
  if constexpr (NT) v = __builtin_nontemporal_load(reinterpret_cast<const fmcw_f4v*>(p));
  else v = *reinterpret_cast<const fmcw_f4v*>(p);
  return make_float4(v.x, v.y, v.z, v.w);
}
template <bool NT>
__device__ __forceinline__ float2 ld_f2(const void* p) {
  fmcw_f2v v;
  if constexpr (NT) v = __builtin_nontemporal_load(reinterpret_cast<const fmcw_f2v*>(p));
  else v = *reinterpret_cast<const fmcw_f2v*>(p);
  return make_float2(v.x, v.y);
}
template <bool NT>
__device__ __forceinline__ fmcw_u2v ld_u2(const void* p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const fmcw_u2v*>(p));
  else return *reinterpret_cast<const fmcw_u2v*>(p);
}
// Write-through (sc1) 16-B store through a buffer descriptor: the XCD L2 forwards the line at
// once instead of holding it dirty until the end-of-kernel write-back, which a dependent launch
// waits for (MI355X_MICROARCH.md "boundary": + dirty bytes / 6 TB/s).  `off` in bytes.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(base, (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void st_f4_wt(__amdgpu_buffer_rsrc_t r, uint32_t off, float4 x) {
  typedef uint32_t u4v __attribute__((ext_vector_type(4)));
  const u4v v = {__float_as_uint(x.x), __float_as_uint(x.y), __float_as_uint(x.z), __float_as_uint(x.w)};
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16 /* sc1 */);
}
template <bool NT>
__device__ __forceinline__ void st_f4(void* p, float4 x) {
  const fmcw_f4v v = {x.x, x.y, x.z, x.w};
  if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<fmcw_f4v*>(p));
  else *reinterpret_cast<fmcw_f4v*>(p) = v;
}

// exp(-2 pi i e / LR), 0 <= e < LR, LR a power of two: argument reduced to (-1/2, 1/2] rev.
template <int LR>
__device__ __forceinline__ float2 twiddle(int e) {
  const float rev = (e > LR / 2) ? (float)(LR - e) * (1.0f / LR) : -(float)e * (1.0f / LR);
  float c = __builtin_amdgcn_cosf(rev), s = __builtin_amdgcn_sinf(rev);
  // v_cos/v_sin are transcendental: a VALU reading their result needs wait states, which the
  // hazard recognizer does not insert ahead of an inline-asm reader (the packed cmul above).
  // Measured: without this, range transforms with twiddles consumed back to back came out
  // wrong (N = 4096); two wait states here make every later reader safe.
  asm volatile("s_nop 1" : "+v"(c), "+v"(s));
  return make_float2(c, s);
}

// Twiddles of one radix-R group, w^m for w = exp(-2 pi i k / LR), m < R: the powers
// w^1, w^2, w^4, w^8 are evaluated directly (v_sin/v_cos), every other power is a product
// of at most log2(R) of them (<= 4 roundings), so a group holds log2(R) complex values.
template <int R, int LR>
struct GroupTwiddles {
  static constexpr int NB = R == 2 ? 1 : R == 4 ? 2 : R == 8 ? 3 : R == 16 ? 4 : 5;
  float2 b[NB];
  __device__ __forceinline__ void init(int k) {
#pragma unroll
    for (int i = 0; i < NB; ++i) b[i] = twiddle<LR>((k << i) & (LR - 1));
  }
  __device__ __forceinline__ float2 pow(int m) const {  // m compile-time after unrolling
    float2 r = make_float2(1.f, 0.f);
    bool first = true;
#pragma unroll
    for (int i = 0; i < NB; ++i)
      if ((m >> i) & 1) {
        r = first ? b[i] : cmul(r, b[i]);
        first = false;
      }
    return r;
  }
};

// ---- small DFTs, natural order in and out -------------------------------------------
__device__ __forceinline__ void dft2(float2& a, float2& b) {
  const float2 t = a;
  a = cadd(t, b);
  b = csub(t, b);
}

__device__ __forceinline__ void dft4(float2& x0, float2& x1, float2& x2, float2& x3) {
  const float2 a0 = cadd(x0, x2), a1 = csub(x0, x2);
  const float2 a2 = cadd(x1, x3), d = csub(x1, x3);
  x0 = cadd(a0, a2);
  x2 = csub(a0, a2);
  x1 = cadd_negi(a1, d);   // a1 + (-i) d
  x3 = csub_negi(a1, d);
}

template <int R> struct Dft;
template <> struct Dft<2> {
  __device__ __forceinline__ static void run(float2* v) { dft2(v[0], v[1]); }
};
template <> struct Dft<4> {
  __device__ __forceinline__ static void run(float2* v) { dft4(v[0], v[1], v[2], v[3]); }
};
template <> struct Dft<8> {
  __device__ __forceinline__ static void run(float2* v) {
    // DIT: E = DFT4(even), O = DFT4(odd), X[k] = E[k] + w8^k O[k], X[k+4] = E[k] - w8^k O[k]
    float2 e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6];
    float2 o0 = v[1], o1 = v[3], o2 = v[5], o3 = v[7];
    dft4(e0, e1, e2, e3);
    dft4(o0, o1, o2, o3);
    const float c = 0.70710678118654752440f;
    const float2 t1 = cscale(cadd_negi(o1, o1), c);     // w8^1 o1 = c (o1.x + o1.y, o1.y - o1.x)
    const float2 t3 = cscale(csub_negi(o3, o3), -c);    // w8^3 o3 = -c (o3.x - o3.y, o3.y + o3.x)
    v[0] = cadd(e0, o0); v[4] = csub(e0, o0);
    v[1] = cadd(e1, t1); v[5] = csub(e1, t1);
    v[2] = cadd_negi(e2, o2); v[6] = csub_negi(e2, o2);  // w8^2 o2 = -i o2
    v[3] = cadd(e3, t3); v[7] = csub(e3, t3);
  }
};
template <> struct Dft<16> {
  __device__ __forceinline__ static void run(float2* v) {
    // N1 = N2 = 4, n = 4 n1 + n2, k = k1 + 4 k2:
    //   Y[n2][k1] = DFT4_{n1}(x[4 n1 + n2]) * w16^{n2 k1};  X[k1 + 4 k2] = DFT4_{n2}(Y[n2][k1])
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) dft4(v[n2], v[n2 + 4], v[n2 + 8], v[n2 + 12]);
    // after this, v[n2 + 4 k1] = Y[n2][k1]
    const float c8 = 0.70710678118654752440f;   // cos(pi/4)
    const float c16 = 0.92387953251128675613f;  // cos(pi/8)
    const float s16 = 0.38268343236508977173f;  // sin(pi/8)
    // w16^e = (cos(2 pi e/16), -sin(2 pi e/16))
    // w8 = c8 (1 - i), w8^3 = -c8 (1 + i): a packed add with a -i operand and a scale
    v[5] = cmul(v[5], make_float2(c16, -s16));      // n2=1,k1=1: e=1
    v[9] = cscale(cadd_negi(v[9], v[9]), c8);       // n2=1,k1=2: e=2
    v[13] = cmul(v[13], make_float2(s16, -c16));    // n2=1,k1=3: e=3
    v[6] = cscale(cadd_negi(v[6], v[6]), c8);       // n2=2,k1=1: e=2
    //                                                 n2=2,k1=2: e=4, -i, folded below
    v[14] = cscale(csub_negi(v[14], v[14]), -c8);   // n2=2,k1=3: e=6
    v[7] = cmul(v[7], make_float2(s16, -c16));      // n2=3,k1=1: e=3
    v[11] = cscale(csub_negi(v[11], v[11]), -c8);   // n2=3,k1=2: e=6
    v[15] = cmul(v[15], make_float2(-c16, s16));    // n2=3,k1=3: e=9
    dft4(v[0], v[1], v[2], v[3]);
    dft4(v[4], v[5], v[6], v[7]);
    {  // dft4(v[8], v[9], -i v[10], v[11])
      const float2 a0 = cadd_negi(v[8], v[10]), a1 = csub_negi(v[8], v[10]);
      const float2 a2 = cadd(v[9], v[11]), d = csub(v[9], v[11]);
      v[8] = cadd(a0, a2);
      v[10] = csub(a0, a2);
      v[9] = cadd_negi(a1, d);
      v[11] = csub_negi(a1, d);
    }
    dft4(v[12], v[13], v[14], v[15]);
    // now v[4 k1 + k2] = X[k1 + 4 k2]; transpose the 4x4 index to natural order
    float2 t[16];
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1)
#pragma unroll
      for (int k2 = 0; k2 < 4; ++k2) t[k1 + 4 * k2] = v[4 * k1 + k2];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = t[i];
  }
};

template <> struct Dft<32> {
  __device__ __forceinline__ static void run(float2* v) {
    // DIT: E = DFT16(even), O = DFT16(odd), X[k] = E[k] + w32^k O[k], X[k+16] = E[k] - w32^k O[k]
    float2 e[16], o[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      e[i] = v[2 * i];
      o[i] = v[2 * i + 1];
    }
    Dft<16>::run(e);
    Dft<16>::run(o);
    const float c8 = 0.70710678118654752440f;
    // w32^k = (cos(2 pi k / 32), -sin(2 pi k / 32)), k = 1..15 (k = 4, 8, 12 folded below)
    constexpr float C[16] = {1.f, 0.98078528040323044913f, 0.92387953251128675613f, 0.83146961230254523708f,
                             0.70710678118654752440f, 0.55557023301960222474f, 0.38268343236508977173f,
                             0.19509032201612826785f, 0.f, -0.19509032201612826785f, -0.38268343236508977173f,
                             -0.55557023301960222474f, -0.70710678118654752440f, -0.83146961230254523708f,
                             -0.92387953251128675613f, -0.98078528040323044913f};
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      float2 t;
      if (k == 0) t = o[0];
      else if (k == 4) t = cscale(cadd_negi(o[4], o[4]), c8);      // c8 (1 - i) o
      else if (k == 12) t = cscale(csub_negi(o[12], o[12]), -c8);  // -c8 (1 + i) o
      else if (k == 8) {                                           // -i o, folded
        v[8] = cadd_negi(e[8], o[8]);
        v[24] = csub_negi(e[8], o[8]);
        continue;
      } else t = cmul(o[k], make_float2(C[k], k < 8 ? C[k + 8] : -C[k - 8]));  // -sin = cos(. + pi/2)
      v[k] = cadd(e[k], t);
      v[k + 16] = csub(e[k], t);
    }
  }
};

// Synchronisation between passes: an FFT that spans several waves needs a workgroup
// barrier; inside one wave, LDS operations issue and complete in program order, and the
// compiler keeps every read of a pass ahead of its (may-alias) writes.
template <bool WG_SYNC>
__device__ __forceinline__ void pass_sync() {
  if constexpr (WG_SYNC) __syncthreads();
  else __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// One Stockham radix-R pass (L = size of the already-combined sub-transforms), in place on
// `buf` (padded layout).  Thread t of P handles groups j = t + P g, g < 16/R.
template <int N, int R, int L, int P, bool WG_SYNC>
__device__ __forceinline__ void stockham_pass(float2* buf, int t) {
  constexpr int G = N / R / P;
  constexpr int S = N / R;
  static_assert(G * R == 16, "16 values per thread");
  float2 v[G][R];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const float2* src = buf + pad16(t + P * g);
#pragma unroll
    for (int m = 0; m < R; ++m) v[g][m] = src[padoff(m * S)];
  }
  pass_sync<WG_SYNC>();
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int j = t + P * g;
    const int k = j & (L - 1);
    if constexpr (L > 1) {
      GroupTwiddles<R, L * R> tw;
      tw.init(k);
#pragma unroll
      for (int m = 1; m < R; ++m) v[g][m] = cmul(v[g][m], tw.pow(m));
    }
    Dft<R>::run(v[g]);
    float2* dst = buf + pad16((j / L) * L * R + k);
#pragma unroll
    for (int m = 0; m < R; ++m) dst[padoff(m * L)] = v[g][m];
  }
  pass_sync<WG_SYNC>();
}

// Passes L, L*R, ... up to N (all from LDS).
template <int N, int L, int P, bool WG_SYNC>
__device__ __forceinline__ void stockham_from(float2* buf, int t) {
  if constexpr (L < N) {
    constexpr int REM = N / L;
    constexpr int R = REM >= 16 ? 16 : REM;
    stockham_pass<N, R, L, P, WG_SYNC>(buf, t);
    stockham_from<N, L * R, P, WG_SYNC>(buf, t);
  }
}

// Radix of the last pass when the passes start at sub-transform size L0.
template <int N, int L0> struct FinalRadix {
  static constexpr int calc() {
    int L = L0;
    while (N / L > 16) L *= 16;
    return N / L;
  }
  static constexpr int R = calc();
  static constexpr int G = 16 / R;
};

// The last pass alone (N / L <= 16) with its twiddle bases supplied by the caller: when
// P % L == 0 every group of a thread has k = t mod L, so a persistent kernel evaluates the
// v_sin / v_cos bases once per thread instead of once per transform.
template <int N, int L, int P>
__device__ __forceinline__ void stockham_last_tw(const float2* buf, int t, float2 (*out)[N / L],
                                                 const GroupTwiddles<N / L, N>& tw) {
  constexpr int R = N / L;
  constexpr int G = N / R / P;
  static_assert(R <= 16 && P % L == 0, "one pass, group-invariant twiddles");
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const float2* src = buf + pad16(t + P * g);
#pragma unroll
    for (int m = 0; m < R; ++m) out[g][m] = src[padoff(m * (N / R))];
#pragma unroll
    for (int m = 1; m < R; ++m) out[g][m] = cmul(out[g][m], tw.pow(m));
    Dft<R>::run(out[g]);
  }
}

// All passes from sub-transform size L except the last, which stays in registers: on
// return out[g][m] holds X[d] for d = (t + P g) + m * (N / R), R = FinalRadix<N, L>::R.
template <int N, int L, int P, bool WG_SYNC>
__device__ __forceinline__ void stockham_to_regs(float2* buf, int t, float2 (*out)[FinalRadix<N, L>::R]) {
  if constexpr (N / L > 16) {
    stockham_pass<N, 16, L, P, WG_SYNC>(buf, t);
    stockham_to_regs<N, L * 16, P, WG_SYNC>(buf, t, out);
  } else {
    constexpr int R = N / L;
    constexpr int G = N / R / P;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int j = t + P * g;
      const float2* src = buf + pad16(j);
#pragma unroll
      for (int m = 0; m < R; ++m) out[g][m] = src[padoff(m * (N / R))];
      GroupTwiddles<R, L * R> tw;
      tw.init(j & (L - 1));
#pragma unroll
      for (int m = 1; m < R; ++m) out[g][m] = cmul(out[g][m], tw.pow(m));
      Dft<R>::run(out[g]);
    }
  }
}

// ---- V values per thread (V = 16 or 32): the passes of the sequential-pair range kernel -------
// One Stockham radix-R pass in place on `buf` (padded), G = V / R groups j = t + P g per thread,
// workgroup barriers around the exchange.
template <int N, int R, int L, int P, int V>
__device__ __forceinline__ void vpass(float2* buf, int t) {
  constexpr int G = V / R, S = N / R;
  static_assert(G * R == V && P * V == N && S % 16 == 0, "V values per thread, immediate read offsets");
  float2 v[G][R];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const float2* src = buf + pad16(t + P * g);
#pragma unroll
    for (int m = 0; m < R; ++m) v[g][m] = src[padoff(m * S)];
  }
  __syncthreads();
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int j = t + P * g;
    const int k = j & (L - 1);
    if constexpr (L > 1) {
      GroupTwiddles<R, L * R> tw;
      tw.init(k);
#pragma unroll
      for (int m = 1; m < R; ++m) v[g][m] = cmul(v[g][m], tw.pow(m));
    }
    Dft<R>::run(v[g]);
    float2* dst = buf + pad16((j / L) * L * R + k);
#pragma unroll
    for (int m = 0; m < R; ++m) dst[padoff(m * L)] = v[g][m];
  }
  __syncthreads();
}

// Radix-16 passes from sub-transform size L while more than V points remain per transform.
template <int N, int L, int P, int V>
__device__ __forceinline__ void vpasses_mid(float2* buf, int t) {
  if constexpr (N / L > V) {
    vpass<N, 16, L, P, V>(buf, t);
    vpasses_mid<N, L * 16, P, V>(buf, t);
  }
}
// Sub-transform size before the last pass when the LDS passes start at L0.
template <int N, int L0, int V> constexpr int vlast_L() {
  int L = L0;
  while (N / L > V) L *= 16;
  return L;
}
// The last pass, into registers: out[g][m] = X[j + m L] for j = t + P g (no barrier after it).
template <int N, int L, int P, int V>
__device__ __forceinline__ void vpass_last(const float2* buf, int t, float2 (*out)[N / L]) {
  constexpr int R = N / L, G = V / R, S = N / R;
  static_assert(G * R == V && S == L, "last pass: one group per output column");
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int j = t + P * g;
    const float2* src = buf + pad16(j);
#pragma unroll
    for (int m = 0; m < R; ++m) out[g][m] = src[padoff(m * S)];
    GroupTwiddles<R, N> tw;
    tw.init(j & (L - 1));
#pragma unroll
    for (int m = 1; m < R; ++m) out[g][m] = cmul(out[g][m], tw.pow(m));
    Dft<R>::run(out[g]);
  }
}

}  // namespace fmcw
