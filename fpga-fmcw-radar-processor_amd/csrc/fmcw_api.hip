// fmcw_api.hip -- host side of libfmcw.so: the C-ABI declared in include/fmcw.h.
//
// The handle replaces the reference's elaborated radar_core instance (rtl/src/radar_core.vhd
// generics :12-19, FFT IP configuration handshake cfg_proc :279-301): it validates the
// configuration once, uploads the window tables (window_multiplier.vhd:34-49, as fp32) and
// allocates every scratch buffer, so fmcw_enqueue only launches kernels (graph-capturable).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/fmcw.h"
#include "kernels.hpp"

using namespace fmcw;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char b[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(b, sizeof b, fmt, ap);
  va_end(ap);
  g_err = b;
  return code;
}

#define HIP_TRY(expr)                                                                    \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess) return fail(FMCW_EHIP, "%s: %s (%s:%d)", #expr,               \
                                      hipGetErrorString(e_), __FILE__, __LINE__);        \
  } while (0)

bool pow2(uint32_t x) { return x && !(x & (x - 1)); }

constexpr int kWavesPerBlock = 4;  // DopplerGeom<NC>::WPB: wave tiles per K2 / 1-D CFAR workgroup
static_assert(kWavesPerBlock == DopplerGeom<256>::WPB, "host and kernel tile geometry");

struct PendingEvent {
  int kid;
  hipEvent_t a, b;
};

}  // namespace

struct fmcw_handle {
  fmcw_config cfg{};
  int n_cu = 256;
  // range kernel geometry (runtime copies of RangeGeom<N>)
  int T = 0, RB = 0, lgT = 0, lgRB = 0;
  bool k1_dual = true;     // K1 may use the dual-chirp kernel (fixed at fmcw_create)
  bool k2_fast = false;    // K2 runs its FAST instantiation (fixed at fmcw_create)
  uint32_t chunk = 1;
  // device buffers
  float* win_r = nullptr;  // [ns]
  float* win_d = nullptr;  // [nc]
  float2* inter = nullptr; // chunk * nrx * ns * nc
  float* lin_scratch = nullptr;  // chunk * ns * nc (2-D CFAR input when the caller wants no linear map)
  fmcw_det* det_scratch = nullptr;
  uint32_t det_scratch_cap = 0;
  uint32_t slot_cap = 32;  // detections per tile slot (sized in fmcw_create; more -> overflow)
  uint32_t ovf_base = 0;   // first overflow entry
  uint32_t* counter = nullptr;  // [0] overflow entries used, [1] dropped
  uint32_t* wg_base = nullptr;
  uint32_t* wg_count = nullptr;
  uint32_t* wg_off = nullptr;
  uint32_t* block_sum = nullptr;  // ceil(n_wg_max / 1024) scan blocks
  uint32_t* n_dets_tmp = nullptr;
  size_t n_wg_max = 0;
  // fmcw_process host-copy staging, grown on demand and kept (no allocator call per frame batch)
  void* stage_cube = nullptr;
  size_t stage_cube_bytes = 0;
  float* stage_map = nullptr;
  size_t stage_map_bytes = 0;
  fmcw_det* stage_dets = nullptr;
  size_t stage_dets_cap = 0;
  // grid sizes
  int grid_range = 0, grid_doppler = 0, grid_cfar = 0;
  size_t cfar2d_smem = 0;
  // two-stream chunk pipeline (K1 of chunk c + 1 beside K2 of chunk c, fmcw_enqueue)
  int pipe_nb = 0;                      // intermediate buffers in the ring (0 = serial chunks)
  size_t inter_bytes = 0;               // h->inter (chunk frames of the K1 -> K2 spectrum)
  int cfar2_steps = 0;                  // 2-D CFAR steps per strip (0 = cost model; FMCW_CFAR2D_STEPS)
  float2* inter_b[3] = {nullptr, nullptr, nullptr};
  float* lin_b[3] = {nullptr, nullptr, nullptr};
  hipStream_t ps[2] = {nullptr, nullptr};
  hipEvent_t ev_k1[3] = {}, ev_free[3] = {}, ev_fork = nullptr, ev_join = nullptr;
  // fused K1 + K2 (fused.hpp)
  bool fused_ok = false;
  void (*fused_fn)(FusedArgs) = nullptr;
  int fused_per_xcd = 0, fused_na = 0, fused_nb = 0;
  float2* fused_spec = nullptr;  // 8 frame spectra, one per XCD (L2-resident)
  uint32_t* fused_ctl = nullptr;
  uint64_t* fused_trace = nullptr;  // FMCW_FUSED_TRACE=1: phase timestamps of every launch
  int64_t fused_fallbacks = 0;
  bool fused_used_last = false;  // the last fmcw_enqueue ran the fused kernel
  // paired K1 + K2 launches (pair.hpp): chunk c's range stage beside chunk c - 1's Doppler stage
  void (*pair_fn)(PairArgs) = nullptr;
  uint32_t pair_chunk = 0;       // frames per chunk; two chunk spectra (h->inter, pair_b) in flight
  float2* pair_b = nullptr;
  int grid_pair = 0;
  // profiling
  bool profiling = false;
  std::vector<PendingEvent> pending;
  std::vector<hipEvent_t> free_events;
  double ms[FMCW_K_COUNT] = {};
  uint64_t launches[FMCW_K_COUNT] = {};
};

namespace {

// ---- kernel dispatch tables ------------------------------------------------------------
using RangeFn = void (*)(const void*, float2*, const float*, const float*, int, int, float);

template <int N, bool H16>
RangeFn range_fn_t(int dtype, bool q15) {
  switch (dtype) {
    case FMCW_IN_F32: return k_range<N, LoadF32, false, H16>;
    case FMCW_IN_F16: return k_range<N, LoadF16, false, H16>;
    case FMCW_IN_I16: return q15 ? k_range<N, LoadI16, true, H16> : k_range<N, LoadI16, false, H16>;
  }
  return nullptr;
}
template <int N>
RangeFn range_fn(int dtype, bool q15, bool h16) {
  return h16 ? range_fn_t<N, true>(dtype, q15) : range_fn_t<N, false>(dtype, q15);
}

struct RangeInfo {
  RangeFn fn;
  int T, RB, NT;
};

template <int N>
RangeFn range2_fn(int dtype) {
  if constexpr (RangeGeom<N>::T == 2 && RangeGeom<N>::P >= 128) {
    switch (dtype) {
      case FMCW_IN_F32: return k_range2<N, LoadF32>;
      case FMCW_IN_F16: return k_range2<N, LoadF16>;
      case FMCW_IN_I16: return k_range2<N, LoadI16>;
    }
  }
  return nullptr;
}

RangeInfo range_info(uint32_t n, int dtype, int window = FMCW_WIN_HAMMING, bool h16 = false, bool dual = true) {
  const bool q15 = window == FMCW_WIN_Q15_RTL;
  // the dual range kernel (kernels.hpp k_range2): T = 2 geometries from FMCW_K1_DUAL up, fp32
  // window, fp32 spectrum; one thread per (16 points of both chirps).  `dual` = the handle's
  // choice at fmcw_create (environment FMCW_K1_SINGLE=1 turns it off for A/B runs)
  if (FMCW_K1_DUAL && dual && n >= (uint32_t)FMCW_K1_DUAL && !q15 && !h16) {
    switch (n) {
#define R2_(N) case N: if (RangeFn f = range2_fn<N>(dtype)) return {f, RangeGeom<N>::T, RangeGeom<N>::RB, RangeGeom<N>::P}; break;
      R2_(2048) R2_(4096) R2_(8192)
#undef R2_
    }
  }
  switch (n) {
#define R_(N) case N: return {range_fn<N>(dtype, q15, h16), RangeGeom<N>::T, RangeGeom<N>::RB, RangeGeom<N>::NT};
    R_(64) R_(128) R_(256) R_(512) R_(1024) R_(2048) R_(4096) R_(8192)
#undef R_
  }
  return {nullptr, 0, 0, 0};
}

using DopplerFn = void (*)(const float2*, const float*, int, int, int, int, int, int, int, float*,
                           float*, int, int, Cfar1DArgs, DetSink);
struct DopplerInfo {
  DopplerFn fn;
  int WR, NT;  // range rows per wave tile, threads per workgroup (DopplerGeom::WPB tiles)
};
template <int N, bool H16>
DopplerFn doppler_fn_t(int mti, bool fast) {
  return mti == FMCW_MTI_2PULSE   ? k_doppler<N, 2, H16>
         : mti == FMCW_MTI_3PULSE ? k_doppler<N, 3, H16>
         : fast                   ? k_doppler<N, 0, H16, true>
                                  : k_doppler<N, 0, H16>;
}
template <int N>
DopplerFn doppler_fn(int mti, bool h16, bool fast) {
  return h16 ? doppler_fn_t<N, true>(mti, fast) : doppler_fn_t<N, false>(mti, fast);
}
// K2's FAST instantiation (kernels.hpp): MTI off, |X| magnitude, no dB map, and the 1-D CFAR
// (if any) at the reference geometry in fp32
bool k2_fast(const fmcw_config& c) {
  const bool cfar_ok = c.cfar_kind != FMCW_CFAR_OS1D ||
                       (c.cfar1d_ref == 8 && c.cfar1d_guard == 2 && (int)(2 * c.cfar1d_ref) - (int)c.cfar1d_rank <= 4 &&
                        !(c.compat_rtl & FMCW_COMPAT_CFAR));
  return c.mti_mode == FMCW_MTI_OFF && c.mag_mode != FMCW_MAG_AMBM && c.map_kind != FMCW_MAP_DB && cfar_ok &&
         !std::getenv("FMCW_K2_GENERIC");
}
DopplerInfo doppler_info(uint32_t nc, int mti = FMCW_MTI_OFF, bool h16 = false, bool fast = false) {
  switch (nc) {
#define D_(N) case N: return {doppler_fn<N>(mti, h16, fast), DopplerGeom<N>::WR, DopplerGeom<N>::NT};
    D_(32) D_(64) D_(128) D_(256) D_(512) D_(1024)
#undef D_
  }
  return {nullptr, 0, 0};
}

using Cfar1Fn = void (*)(const float*, int, int, int, int, Cfar1DArgs, DetSink);
Cfar1Fn cfar1_fn(uint32_t nc) {
  switch (nc) {
#define C_(N) case N: return k_cfar1d<N>;
    C_(32) C_(64) C_(128) C_(256) C_(512) C_(1024)
#undef C_
  }
  return nullptr;
}

using Cfar2Fn = void (*)(const float*, int, int, int, int, int, Cfar2DArgs, DetSink);
struct Cfar2Info {
  Cfar2Fn fn;
  int TR;
};
// the reference window (Doppler half extent 6, guard 2: os_cfar_2d as instantiated at
// radar_core.vhd:376-382) gets the compile-time phase A; any other geometry the generic one
template <int N>
Cfar2Fn cfar2_fn(int hd, int gd) {
  return (hd == 6 && gd == 2) ? k_cfar2d<N, 6, 2> : k_cfar2d<N, 0, 0>;
}
Cfar2Info cfar2_info(uint32_t nc, int hd = 0, int gd = 0) {
  switch (nc) {
#define C_(N) case N: return {cfar2_fn<N>(hd, gd), Cfar2DGeom<N>::TR};
    C_(32) C_(64) C_(128) C_(256) C_(512) C_(1024)
#undef C_
  }
  return {nullptr, 0};
}

// fused K1 + K2 instantiations: the reference core (1024 x 128), BASELINE config 2 (1024 x 256)
// and two more shapes with 256-thread range and Doppler workgroups and <= 2 MiB spectra
using FusedFn = void (*)(FusedArgs);
template <int N, int NC>
FusedFn fused_fn_t(int dtype) {
  switch (dtype) {
    case FMCW_IN_F32: return k_fused<N, NC, LoadF32>;
    case FMCW_IN_F16: return k_fused<N, NC, LoadF16>;
    case FMCW_IN_I16: return k_fused<N, NC, LoadI16>;
  }
  return nullptr;
}
struct FusedInfo {
  FusedFn fn;
  int upf, wtpf;
};
FusedInfo fused_info(uint32_t n, uint32_t nc, int dtype) {
#define F_(N, NC) \
  if (n == N && nc == NC) return {fused_fn_t<N, NC>(dtype), FusedGeom<N, NC>::UPF, FusedGeom<N, NC>::WTPF};
  F_(1024, 256) F_(1024, 128) F_(512, 256) F_(2048, 128)
#undef F_
  return {nullptr, 0, 0};
}

// paired K1 + K2 instantiations: BASELINE config 2 (1024 x 256)
using PairFn = void (*)(PairArgs);
PairFn pair_fn(uint32_t n, uint32_t nc, int dtype) {
  if (n == 1024 && nc == 256) switch (dtype) {
      case FMCW_IN_F32: return k_pair<1024, 256, LoadF32>;
      case FMCW_IN_F16: return k_pair<1024, 256, LoadF16>;
      case FMCW_IN_I16: return k_pair<1024, 256, LoadI16>;
    }
  return nullptr;
}

// 2-D CFAR derived parameters
Cfar2DArgs cfar2_args(const fmcw_config& c) {
  Cfar2DArgs a{};
  a.gr = (int)c.cfar2d_guard_range;
  a.gd = (int)c.cfar2d_guard_doppler;
  a.hr = (int)(c.cfar2d_ref_range + c.cfar2d_guard_range);
  a.hd = (int)(c.cfar2d_ref_doppler + c.cfar2d_guard_doppler);
  a.n_ref = (2 * a.hr + 1) * (2 * a.hd + 1) - (2 * a.gr + 1) * (2 * a.gd + 1);
  // rank_idx = N_REF * RANK_PCT / 100, clamped to N_REF - 1 (os_cfar_2d.vhd:181-182); 64-bit
  a.rank = (int)std::min<int64_t>((int64_t)a.n_ref * c.cfar2d_rank_pct / 100, (int64_t)a.n_ref - 1);
  a.sc_min = (float)c.cfar2d_scale_min;
  a.sc_nom = (float)c.cfar2d_scale_nom;
  a.sc_max = (float)c.cfar2d_scale_max;
  a.override_ = (int)c.cfar2d_scale_override;
  a.compat = (c.compat_rtl & FMCW_COMPAT_CFAR) != 0;
  a.s_min = a.override_ ? (float)a.override_ : std::min(a.sc_min, std::min(a.sc_nom, a.sc_max));
  return a;
}

Cfar1DArgs cfar1_args(const fmcw_config& c) {
  Cfar1DArgs a{};
  a.enabled = c.cfar_kind == FMCW_CFAR_OS1D;
  a.ref = (int)c.cfar1d_ref;
  a.guard = (int)c.cfar1d_guard;
  a.rank = (int)c.cfar1d_rank;
  a.alpha = c.cfar1d_alpha;
  a.compat = (c.compat_rtl & FMCW_COMPAT_CFAR) != 0;
  return a;
}

size_t cfar2_smem(uint32_t nc, int hr) {
  switch (nc) {
    case 32: return cfar2d_smem_bytes<32>(hr);
    case 64: return cfar2d_smem_bytes<64>(hr);
    case 128: return cfar2d_smem_bytes<128>(hr);
    case 256: return cfar2d_smem_bytes<256>(hr);
    case 512: return cfar2d_smem_bytes<512>(hr);
    case 1024: return cfar2d_smem_bytes<1024>(hr);
  }
  return 0;
}

int validate(const fmcw_config& c) {
  if (!pow2(c.n_range) || c.n_range < 64 || c.n_range > 8192)
    return fail(FMCW_EINVAL, "n_range=%u: must be a power of two in [64, 8192]", c.n_range);
  if (!pow2(c.n_doppler) || c.n_doppler < 32 || c.n_doppler > 1024)
    return fail(FMCW_EINVAL, "n_doppler=%u: must be a power of two in [32, 1024]", c.n_doppler);
  if (c.n_rx < 1 || c.n_rx > 64) return fail(FMCW_EINVAL, "n_rx=%u: must be in [1, 64]", c.n_rx);
  if (c.in_dtype < FMCW_IN_F32 || c.in_dtype > FMCW_IN_I16)
    return fail(FMCW_EINVAL, "in_dtype=%d unknown", c.in_dtype);
  if (c.window != FMCW_WIN_NONE && c.window != FMCW_WIN_HAMMING && c.window != FMCW_WIN_Q15_RTL)
    return fail(FMCW_EINVAL, "window=%d unknown", c.window);
  if (c.window == FMCW_WIN_Q15_RTL && c.in_dtype != FMCW_IN_I16)
    return fail(FMCW_EINVAL, "window Q15_RTL windows int16 ADC words: needs in_dtype I16");
  if (c.mag_mode != FMCW_MAG_ABS && c.mag_mode != FMCW_MAG_AMBM)
    return fail(FMCW_EINVAL, "mag_mode=%d unknown", c.mag_mode);
  if (c.mag_mode == FMCW_MAG_AMBM && c.n_rx != 1)
    return fail(FMCW_EINVAL, "mag_mode AMBM is defined for n_rx == 1 only");
  if (c.map_kind != FMCW_MAP_LINEAR && c.map_kind != FMCW_MAP_DB)
    return fail(FMCW_EINVAL, "map_kind=%d unknown", c.map_kind);
  if (c.mti_mode != FMCW_MTI_OFF && c.mti_mode != FMCW_MTI_2PULSE && c.mti_mode != FMCW_MTI_3PULSE)
    return fail(FMCW_EINVAL, "mti_mode=%d unknown (0 off, 2 or 3 pulse)", c.mti_mode);
  if (range_info(c.n_range, c.in_dtype).T > (int)c.n_doppler)
    return fail(FMCW_EINVAL, "n_doppler=%u smaller than the range kernel's chirp group", c.n_doppler);
  if (c.max_frames < 1) return fail(FMCW_EINVAL, "max_frames must be >= 1");
  if (c.cfar_kind == FMCW_CFAR_OS1D) {
    if (c.cfar1d_ref < 1 || c.cfar1d_rank >= 2 * c.cfar1d_ref)
      return fail(FMCW_EINVAL, "1-D CFAR: need ref >= 1 and rank < 2*ref");
    if (2 * (c.cfar1d_ref + c.cfar1d_guard) + 1 > c.n_doppler)
      return fail(FMCW_EINVAL, "1-D CFAR window wider than n_doppler");
    if (!(c.cfar1d_alpha > 0.f)) return fail(FMCW_EINVAL, "1-D CFAR alpha must be > 0");
    if ((c.compat_rtl & FMCW_COMPAT_CFAR) &&
        !(c.cfar1d_alpha == std::floor(c.cfar1d_alpha) && c.cfar1d_alpha <= 16384.f))
      return fail(FMCW_EINVAL, "compat CFAR: alpha is the integer SCALING_MULT (1..16384)");
  } else if (c.cfar_kind == FMCW_CFAR_OS2D) {
    if (c.cfar2d_rank_pct > 100) return fail(FMCW_EINVAL, "2-D CFAR: rank_pct %u > 100", c.cfar2d_rank_pct);
    if (c.cfar2d_ref_range > 64 || c.cfar2d_ref_doppler > 64 || c.cfar2d_guard_range > 64 ||
        c.cfar2d_guard_doppler > 64)
      return fail(FMCW_EINVAL, "2-D CFAR window extents out of range");
    const Cfar2DArgs a = cfar2_args(c);
    if (a.n_ref < 1 || a.n_ref > 128)
      return fail(FMCW_EINVAL, "2-D CFAR: %d reference cells (supported 1..128)", a.n_ref);
    if (2 * a.hd + 1 > (int)c.n_doppler)
      return fail(FMCW_EINVAL, "2-D CFAR window wider than n_doppler");
    if (c.cfar2d_scale_override > 7)
      return fail(FMCW_EINVAL, "scale_override is a 3-bit port (0..7)");
    if (cfar2_smem(c.n_doppler, a.hr) > 160 * 1024)
      return fail(FMCW_EINVAL, "2-D CFAR range extent too large for LDS");
  } else if (c.cfar_kind != FMCW_CFAR_NONE) {
    return fail(FMCW_EINVAL, "cfar_kind=%d unknown", c.cfar_kind);
  }
  if (c.compat_rtl & ~(uint32_t)(FMCW_COMPAT_CFAR | FMCW_COMPAT_MTI))
    return fail(FMCW_EINVAL, "compat_rtl=0x%x: unknown bits", c.compat_rtl);
  if ((c.compat_rtl & FMCW_COMPAT_MTI) && c.mti_mode == FMCW_MTI_OFF)
    return fail(FMCW_EINVAL, "compat MTI needs mti_mode 2 or 3");
  if (c.range_shift > 13) return fail(FMCW_EINVAL, "range_shift=%u: must be in [0, 13]", c.range_shift);
  if (c.spectrum_dtype != FMCW_SPEC_F32 && c.spectrum_dtype != FMCW_SPEC_F16)
    return fail(FMCW_EINVAL, "spectrum_dtype=%d unknown", c.spectrum_dtype);
  if (c.spectrum_dtype == FMCW_SPEC_F16 && (c.compat_rtl & FMCW_COMPAT_MTI))
    return fail(FMCW_EINVAL, "compat MTI is defined on the fp32 spectrum (spectrum_dtype F16)");
  return FMCW_OK;
}

// fp32 window table: Hamming with the RTL's half-ROM mirrored address, computed in fp64
// (window_multiplier.vhd:34-49, :97-102).  WIN_NONE uploads ones.
std::vector<float> window_table(uint32_t n, int kind, uint32_t shift = 0) {
  std::vector<float> w(n, std::ldexp(1.0f, -(int)shift));  // 2^-shift: exact
  if (kind == FMCW_WIN_Q15_RTL) {  // ROM integers c = integer(w * 32767) (:43-46), mirrored
    const uint32_t half = n / 2;
    for (uint32_t i = 0; i < n; ++i) {
      uint32_t a = i < half ? i : n - 1 - i;
      if (a > half - 1) a = half - 1;
      const double wa = 0.54 - 0.46 * std::cos(2.0 * M_PI * (double)a / (double)(n - 1));
      w[i] = (float)std::min(32767.0, std::floor(wa * 32767.0 + 0.5));
    }
  } else if (kind == FMCW_WIN_HAMMING) {
    const uint32_t half = n / 2;
    for (uint32_t i = 0; i < n; ++i) {
      uint32_t a = i < half ? i : n - 1 - i;
      if (a > half - 1) a = half - 1;
      w[i] = std::ldexp((float)(0.54 - 0.46 * std::cos(2.0 * M_PI * (double)a / (double)(n - 1))), -(int)shift);
    }
  }
  return w;
}

template <typename F>
int occupancy_grid(F fn, int nt, size_t smem, int n_cu, int* grid) {
  int per_cu = 0;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(fn),
                                                              nt, smem);
  if (e != hipSuccess || per_cu < 1) per_cu = 1;
  *grid = per_cu * n_cu;
  return FMCW_OK;
}

hipEvent_t take_event(fmcw_handle* h) {
  if (!h->free_events.empty()) {
    hipEvent_t e = h->free_events.back();
    h->free_events.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

struct ProfScope {
  fmcw_handle* h;
  int kid;
  hipStream_t s;
  hipEvent_t a = nullptr;
  ProfScope(fmcw_handle* h_, int kid_, hipStream_t s_) : h(h_), kid(kid_), s(s_) {
    if (h->profiling) {
      a = take_event(h);
      if (a) hipEventRecord(a, s);
    }
  }
  ~ProfScope() {
    if (h->profiling && a) {
      hipEvent_t b = take_event(h);
      if (b) {
        hipEventRecord(b, s);
        h->pending.push_back({kid, a, b});
      }
    }
  }
};

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(FMCW_EHIP, "launch %s: %s", what, hipGetErrorString(e));
  return FMCW_OK;
}

DetSink make_sink(fmcw_handle* h) {
  DetSink s;
  s.scratch = h->det_scratch;
  s.cap = h->det_scratch_cap;
  s.slot_cap = h->slot_cap;
  s.ovf_base = h->ovf_base;
  s.counter = h->counter;
  s.wg_base = h->wg_base;
  s.wg_count = h->wg_count;
  return s;
}

// Detection tiles per frame: K2's wave tiles (WR range rows), shared by the 1-D and 2-D CFAR.
size_t tiles_per_frame(const fmcw_handle* h) {
  const fmcw_config& c = h->cfg;
  return c.n_range / doppler_info(c.n_doppler).WR;
}

// Steps per 2-D CFAR strip.  A strip of S steps loads S*TR + 2*hr rows for S*TR CUT rows; the
// workgroups run ceil(strips / grid) rounds.  Cost model per round, in units of one step's
// compute: S * (1 + 0.5) (a step's TR new rows cost about half its compute) + 0.5 * 2hr / TR for
// the halo rows a strip loads once.  Longer strips: less halo traffic, fewer strips to spread.
int cfar2_steps_model(int nf, int tpf, int grid, int tr, int hr) {
  int best = 1;
  double best_cost = 1e300;
  // S up to 64: config 5 (2048 steps per frame, 16 frames, 512 workgroups) then takes one round
  // of 64-step strips (measured 1,011 -> 976 us per launch) instead of two of 32
  for (int S = 1; S <= std::min(64, tpf); ++S) {
    const long strips = (long)nf * ((tpf + S - 1) / S);
    const long rounds = (strips + grid - 1) / std::max(1, grid);
    const double cost = (double)rounds * (1.5 * S + (double)hr / tr);
    if (cost < best_cost - 1e-9) {
      best_cost = cost;
      best = S;
    }
  }
  return best;
}

constexpr size_t kCfar2Batch = 16;  // frames per 2-D CFAR launch on the caller's map (at least)

// The CFAR launcher shared by fmcw_enqueue (map just produced by K2) and fmcw_cfar.
int launch_cfar(fmcw_handle* h, const float* map_chunk, int nf, int frame0, hipStream_t s) {
  const fmcw_config& c = h->cfg;
  const DetSink sink = make_sink(h);
  const int tile0 = (int)(frame0 * tiles_per_frame(h));
  if (c.cfar_kind == FMCW_CFAR_OS2D) {
    const Cfar2DArgs a = cfar2_args(c);
    const Cfar2Info ci = cfar2_info(c.n_doppler, a.hd, a.gd);
    // workgroup tiles (steps): 4 consecutive wave tiles of one frame; a strip is `steps` of them
    const int tpf = (int)((tiles_per_frame(h) + 3) / 4);
    const int steps = h->cfar2_steps ? std::min(h->cfar2_steps, tpf)
                                     : cfar2_steps_model(nf, tpf, h->grid_cfar, doppler_info(c.n_doppler).WR * 4, a.hr);
    const int n_strips = nf * ((tpf + steps - 1) / steps);
    const int grid = std::min(n_strips, h->grid_cfar);
    ProfScope ps(h, FMCW_K_CFAR2D, s);
    hipLaunchKernelGGL(ci.fn, dim3(grid), dim3(256), h->cfar2d_smem, s, map_chunk, (int)c.n_range,
                       n_strips, steps, frame0, tile0, a, sink);
    return check_launch("k_cfar2d");
  }
  // 1-D on a caller map (fmcw_cfar); inside fmcw_enqueue the 1-D CFAR is fused into K2
  const DopplerInfo di = doppler_info(c.n_doppler);
  const int n_tiles = nf * (int)(c.n_range / di.WR);
  const int grid = std::min((n_tiles + kWavesPerBlock - 1) / kWavesPerBlock, h->grid_doppler);
  ProfScope ps(h, FMCW_K_CFAR2D, s);
  hipLaunchKernelGGL(cfar1_fn(c.n_doppler), dim3(grid), dim3(di.NT), 0, s, map_chunk, (int)c.n_range,
                     n_tiles, frame0, tile0, cfar1_args(c), sink);
  return check_launch("k_cfar1d");
}

int launch_det_finish(fmcw_handle* h, size_t n_frames, fmcw_det* dets, size_t det_cap,
                      uint32_t* n_dets_dev, hipStream_t s) {
  const int n = (int)(n_frames * tiles_per_frame(h));
  const int nb = (n + 1023) / 1024;
  ProfScope ps(h, FMCW_K_COMPACT, s);
  hipLaunchKernelGGL(k_det_scan_blocks, dim3(nb), dim3(1024), 0, s, h->wg_count, h->wg_off, n, h->block_sum);
  hipLaunchKernelGGL(k_det_scan_top, dim3(1), dim3(1024), 0, s, h->block_sum, nb, n_dets_dev,
                     (const uint32_t*)(h->counter + 1),
                     (const uint32_t*)(h->fused_used_last ? h->fused_ctl + FusedCtl::kErr : nullptr));
  int rc = check_launch("k_det_scan");
  if (rc) return rc;
  if (dets && det_cap) {
    // entries past the handle's scratch capacity are never stored: clip to it as well
    const uint32_t cap = (uint32_t)std::min<size_t>(det_cap, h->det_scratch_cap);
    hipLaunchKernelGGL(k_det_copy, dim3((n + 255) / 256), dim3(256), 0, s, h->det_scratch,
                       h->det_scratch_cap, h->wg_base, h->wg_count, h->wg_off, h->block_sum, n, dets, cap);
    rc = check_launch("k_det_copy");
  }
  return rc;
}

// 2^-range_shift for the Q15 window path (the fp32 window tables carry it otherwise)
float q15_scale(const fmcw_config& c) {
  return c.window == FMCW_WIN_Q15_RTL ? std::ldexp(1.0f, -(int)c.range_shift) : 1.0f;
}

size_t cube_bytes(const fmcw_config& c, size_t n_frames) {
  const size_t per = (size_t)c.n_rx * c.n_range * c.n_doppler;
  const size_t eb = c.in_dtype == FMCW_IN_F32 ? 8 : 4;
  return n_frames * per * eb;
}

bool is_device_ptr(const void* p) {
  if (!p) return false;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

// Grow-only device staging owned by the handle (fmcw_process with host buffers).
template <typename T>
int ensure_stage(T** p, size_t* have, size_t need_bytes, const char* what) {
  if (*have >= need_bytes) return FMCW_OK;
  if (*p) hipFree(*p);
  *p = nullptr;
  *have = 0;
  if (hipMalloc(reinterpret_cast<void**>(p), need_bytes) != hipSuccess) {
    (void)hipGetLastError();
    return fail(FMCW_ENOMEM, "hipMalloc(%zu) for the %s staging buffer failed", need_bytes, what);
  }
  *have = need_bytes;
  return FMCW_OK;
}

}  // namespace

// Decide whether this handle runs the fused K1 + K2 kernel and, if so, verify on the device
// that its persistent grid lands as the kernel needs: exactly per_xcd workgroups on every XCD,
// all co-resident (a census launch of the kernel itself: join, wait for the group, exit).
// Placement is never assumed -- a device or runtime that places differently keeps K1 + K2.
void setup_fused(fmcw_handle* h) {
  const fmcw_config& c = h->cfg;
  // opt-in (FMCW_FUSED=1): measured slower than the K1/K2 pipeline at config 2
  const char* env = std::getenv("FMCW_FUSED");
  if (!env || env[0] != '1') return;
  if (c.n_rx != 1 || c.mti_mode != FMCW_MTI_OFF || c.window == FMCW_WIN_Q15_RTL ||
      c.spectrum_dtype != FMCW_SPEC_F32)
    return;
  if (h->n_cu % 8 != 0) return;
  const FusedInfo fi = fused_info(c.n_range, c.n_doppler, c.in_dtype);
  if (!fi.fn) return;
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(fi.fn), 256, 0) !=
          hipSuccess ||
      occ < 1) {
    (void)hipGetLastError();
    return;
  }
  occ = std::min(occ, 4);
  const int per_xcd = occ * h->n_cu / 8;
  // Doppler workgroups (4 waves, at most one wave tile each per frame): 3/4 of the group by
  // default (FMCW_FUSED_NB overrides), at least enough to cover a frame's wave tiles
  const char* nbs = std::getenv("FMCW_FUSED_NB");
  int nb = nbs ? std::atoi(nbs) : per_xcd * 3 / 4;
  nb = std::max(nb, (fi.wtpf + 3) / 4);
  const int na = std::min(per_xcd - nb, fi.upf);  // every range workgroup has a unit per frame
  if (na < 8) return;
  const size_t spec_bytes = 8 * kRing * (size_t)c.n_range * c.n_doppler * sizeof(float2);
  if (hipMalloc(reinterpret_cast<void**>(&h->fused_spec), spec_bytes) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&h->fused_ctl), FusedCtl::kWords * 4) != hipSuccess) {
    (void)hipGetLastError();
    return;
  }
  FusedArgs a{};
  a.ctl = h->fused_ctl;
  a.per_xcd = per_xcd;
  a.n_a = na;
  a.n_b = nb;
  a.census = 1;
  a.spin_limit = 20000;
  std::vector<uint32_t> ctl(FusedCtl::kWords, 0);
  if (hipMemset(h->fused_ctl, 0, FusedCtl::kWords * 4) != hipSuccess) return;
  hipLaunchKernelGGL(fi.fn, dim3(8 * per_xcd), dim3(256), 0, 0, a);
  if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
      hipMemcpy(ctl.data(), h->fused_ctl, FusedCtl::kWords * 4, hipMemcpyDeviceToHost) != hipSuccess) {
    (void)hipGetLastError();
    return;
  }
  if (ctl[FusedCtl::kErr] != 0) return;
  for (int x = 0; x < 8; ++x)
    if (ctl[FusedCtl::join(x)] != (uint32_t)per_xcd) return;
  if (std::getenv("FMCW_FUSED_VERBOSE"))
    std::fprintf(stderr, "fmcw: fused kernel on, %d workgroups per XCD (%d range, %d Doppler)\n", per_xcd, na, nb);
  const char* tr = std::getenv("FMCW_FUSED_TRACE");
  if (tr && tr[0] == '1' && hipMalloc(reinterpret_cast<void**>(&h->fused_trace), 8 * kTraceFrames * 8 * 8) != hipSuccess) {
    (void)hipGetLastError();
    h->fused_trace = nullptr;
  }
  h->fused_fn = fi.fn;
  h->fused_per_xcd = per_xcd;
  h->fused_na = na;
  h->fused_nb = nb;
  h->fused_ok = true;
}

// Paired launches (pair.hpp), default on where instantiated: one rx, MTI off, the FAST K2
// configuration without the 2-D CFAR, fp32 window and spectrum.  Chunk: the largest multiple of
// the frames one round of the persistent grid covers with both chunk spectra (written and read)
// within ~3/4 of the 256 MiB Infinity Cache.  FMCW_PAIR=0 / 1 overrides kPairDefault (A/B runs).
constexpr bool kPairDefault = false;
void setup_pair(fmcw_handle* h, size_t frame_inter) {
  const fmcw_config& c = h->cfg;
  const char* env = std::getenv("FMCW_PAIR");
  if (!(env ? env[0] == '1' : kPairDefault)) return;
  if (c.n_rx != 1 || c.window == FMCW_WIN_Q15_RTL || c.spectrum_dtype != FMCW_SPEC_F32 ||
      c.cfar_kind == FMCW_CFAR_OS2D || !h->k2_fast)
    return;
  const PairFn fn = pair_fn(c.n_range, c.n_doppler, c.in_dtype);
  if (!fn) return;
  occupancy_grid(fn, 256, 0, h->n_cu, &h->grid_pair);
  const size_t tpf = (size_t)c.n_range / doppler_info(c.n_doppler).WR;
  const size_t units_pf = tpf / kWavesPerBlock;  // K2 items per frame (K1: n_doppler / T)
  size_t ch = std::max<size_t>(1, (192u << 20) / (2 * frame_inter));
  if ((size_t)h->grid_pair % units_pf == 0) {
    const size_t unit = (size_t)h->grid_pair / units_pf;
    if (ch >= 2 * unit) ch -= ch % unit;
  }
  if (const char* pc = std::getenv("FMCW_PAIR_CHUNK")) ch = (size_t)std::max(1, std::atoi(pc));
  h->pair_chunk = (uint32_t)std::min<size_t>(ch, c.max_frames);
  if (h->pair_chunk >= c.max_frames) return;  // a batch never spans two chunks: nothing to pair
  h->pair_fn = fn;
}

// the thread-local fmcw_last_error() message, for the other translation units of the library
int fmcw_internal_fail(int code, const char* msg) { return fail(code, "%s", msg); }

// =======================================================================================
extern "C" {

const char* fmcw_version(void) { return "fmcw-mi355x 0.1.0 (gfx950)"; }
int fmcw_abi_version(void) { return FMCW_ABI_VERSION; }
const char* fmcw_last_error(void) { return g_err.c_str(); }

void fmcw_config_default(fmcw_config* c) {
  if (!c) return;
  std::memset(c, 0, sizeof *c);
  c->n_range = 1024;  // radar_core.vhd:13
  c->n_doppler = 128; // :14
  c->n_rx = 1;
  c->in_dtype = FMCW_IN_F32;
  c->window = FMCW_WIN_HAMMING;
  c->mag_mode = FMCW_MAG_ABS;
  c->map_kind = FMCW_MAP_LINEAR;
  c->cfar_kind = FMCW_CFAR_OS2D;
  c->cfar1d_ref = 8;  // rtl/old/radar_core_v3.vhd:376-380
  c->cfar1d_guard = 2;
  c->cfar1d_rank = 12;
  c->cfar1d_alpha = 4.0f;
  c->cfar2d_ref_range = 4;     // radar_core.vhd:16 CFAR_REF_R (rows)
  c->cfar2d_guard_range = 1;   // :19 CFAR_GUARD_D=1 acts on rows (naming swap)
  c->cfar2d_ref_doppler = 4;   // :17 CFAR_REF_D
  c->cfar2d_guard_doppler = 2; // :18 CFAR_GUARD_R=2 acts along Doppler
  c->cfar2d_rank_pct = 75;     // :380
  c->cfar2d_scale_min = 2;
  c->cfar2d_scale_nom = 4;
  c->cfar2d_scale_max = 6;
  c->cfar2d_scale_override = 0;
  c->max_frames = 1;
  c->chunk_frames = 0;
  c->device_id = 0;
}

// Frames per K1 -> K2 chunk when the caller leaves chunk_frames at 0.  The corner-turned
// spectrum of a chunk is written by K1 and read back by K2 right after; kept to ~3/4 of the
// 256 MiB Infinity Cache (MALL), K2's reads hit there.  Measured on config 2 (round 2, 1024
// frames per step, gpurun_out chunk sweep): K2 0.63 us/frame at 128 frames (256 MiB), 0.57 at
// 96, 0.55 at 108-120, 0.81 from 256 frames up (reads from HBM); K1 unchanged.  Within that,
// a multiple of the frames one full round of K2's persistent grid covers (config 2: 3072
// waves / 256 wave tiles = 12 frames, K1 the same), so neither kernel ends on a partial round.
uint32_t auto_chunk(const fmcw_handle* h, size_t frame_inter) {
  const fmcw_config& c = h->cfg;
  constexpr size_t kMallBudget = 192u << 20;
  size_t ch = std::max<size_t>(1, kMallBudget / frame_inter);
  const size_t waves = (size_t)h->grid_doppler * kWavesPerBlock;
  const size_t tpf = (size_t)c.n_range / doppler_info(c.n_doppler).WR;
  if (waves % tpf == 0) {
    const size_t unit = waves / tpf;  // frames per full K2 round
    if (ch >= 2 * unit) ch -= ch % unit;
  }
  return (uint32_t)std::min<size_t>(c.max_frames, ch);
}

int fmcw_create(const fmcw_config* cfg, fmcw_handle** out) {
  if (!cfg || !out) return fail(FMCW_EINVAL, "null argument");
  *out = nullptr;
  int rc = validate(*cfg);
  if (rc) return rc;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
    (void)hipGetLastError();
    return fail(FMCW_ENODEV, "no HIP device");
  }
  if (cfg->device_id < 0 || cfg->device_id >= ndev) return fail(FMCW_ENODEV, "device_id %d out of range", cfg->device_id);
  HIP_TRY(hipSetDevice(cfg->device_id));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, cfg->device_id));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(FMCW_ENODEV, "device %d is %s; this build targets gfx950 (MI355X)", cfg->device_id,
                prop.gcnArchName);

  fmcw_handle* h = new fmcw_handle();
  h->cfg = *cfg;
  const fmcw_config& c = h->cfg;
  h->n_cu = prop.multiProcessorCount;
  h->k1_dual = !std::getenv("FMCW_K1_SINGLE");
  h->k2_fast = k2_fast(c);
  const RangeInfo ri = range_info(c.n_range, c.in_dtype, c.window, c.spectrum_dtype == FMCW_SPEC_F16, h->k1_dual);
  h->T = ri.T;
  h->RB = ri.RB;
  h->lgT = __builtin_ctz(ri.T);
  h->lgRB = __builtin_ctz(ri.RB);
  const size_t frame_inter = (size_t)c.n_rx * c.n_range * c.n_doppler *
                             (c.spectrum_dtype == FMCW_SPEC_F16 ? sizeof(uint32_t) : sizeof(float2));
  occupancy_grid(ri.fn, ri.NT, 0, h->n_cu, &h->grid_range);
#ifdef FMCW_K1_GRID_PER_CU  // tuning switch (tools/build_variants.sh): K1 workgroups per CU
  h->grid_range = std::min(h->grid_range, FMCW_K1_GRID_PER_CU * h->n_cu);
#endif
  const DopplerInfo di = doppler_info(c.n_doppler, c.mti_mode, c.spectrum_dtype == FMCW_SPEC_F16, h->k2_fast);
  occupancy_grid(di.fn, di.NT, 0, h->n_cu, &h->grid_doppler);
  // two-stream pipeline of chunks (FMCW_PIPE=1): ring of FMCW_PIPE_BUFS intermediate buffers of
  // FMCW_PIPE_CHUNK frames, sized so the ring stays in the 256 MiB Infinity Cache
  if (const char* cs = std::getenv("FMCW_CFAR2D_STEPS")) h->cfar2_steps = std::max(0, std::atoi(cs));
  const char* pe = std::getenv("FMCW_PIPE");
  const bool pipe = pe && pe[0] == '1';
  if (pipe) {
    const char* pc = std::getenv("FMCW_PIPE_CHUNK");
    const char* pb = std::getenv("FMCW_PIPE_BUFS");
    h->pipe_nb = std::max(2, std::min(3, pb ? std::atoi(pb) : 2));
    const size_t want = pc ? (size_t)std::max(1, std::atoi(pc)) : std::max<size_t>(1, (64u << 20) / frame_inter);
    h->chunk = (uint32_t)std::max<size_t>(1, std::min<size_t>(c.max_frames, want));
  } else if (c.chunk_frames) {
    h->chunk = std::min<uint32_t>(c.chunk_frames, c.max_frames);
  } else {
    h->chunk = auto_chunk(h, frame_inter);
  }
  auto cleanup = [&](int code) {
    fmcw_destroy(h);
    return code;
  };
#define ALLOC(ptr, bytes)                                                                   \
  do {                                                                                      \
    if (hipMalloc(reinterpret_cast<void**>(&(ptr)), (bytes)) != hipSuccess) {               \
      (void)hipGetLastError();                                                              \
      return cleanup(fail(FMCW_ENOMEM, "hipMalloc(%zu) for %s failed", (size_t)(bytes), #ptr)); \
    }                                                                                       \
  } while (0)
  ALLOC(h->win_r, c.n_range * sizeof(float));
  ALLOC(h->win_d, c.n_doppler * sizeof(float));
  // >= one fp32 frame: fmcw_range_ct writes the fp32 spectrum through it whatever spectrum_dtype
  setup_pair(h, frame_inter);
  // K1 addresses a launch's spectrum with 32-bit byte offsets (write-through buffer stores)
  h->chunk = (uint32_t)std::max<size_t>(1, std::min<size_t>(h->chunk, ((size_t)1 << 32) / frame_inter - 1));
  h->inter_bytes = std::max(std::max<size_t>(h->chunk, h->pair_fn ? h->pair_chunk : 0) * frame_inter,
                            (size_t)c.n_rx * c.n_range * c.n_doppler * sizeof(float2));
  ALLOC(h->inter, h->inter_bytes);
  if (h->pair_fn) ALLOC(h->pair_b, (size_t)h->pair_chunk * frame_inter);
  if (c.cfar_kind == FMCW_CFAR_OS2D) ALLOC(h->lin_scratch, (size_t)h->chunk * c.n_range * c.n_doppler * sizeof(float));
  if (h->pipe_nb) {
    h->inter_b[0] = h->inter;
    h->lin_b[0] = h->lin_scratch;
    for (int b = 1; b < h->pipe_nb; ++b) {
      ALLOC(h->inter_b[b], h->chunk * frame_inter);
      if (c.cfar_kind == FMCW_CFAR_OS2D) ALLOC(h->lin_b[b], (size_t)h->chunk * c.n_range * c.n_doppler * sizeof(float));
    }
    for (int i = 0; i < 2; ++i)
      if (hipStreamCreateWithFlags(&h->ps[i], hipStreamNonBlocking) != hipSuccess)
        return cleanup(fail(FMCW_EHIP, "stream create"));
    for (int b = 0; b < h->pipe_nb; ++b)
      if (hipEventCreateWithFlags(&h->ev_k1[b], hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&h->ev_free[b], hipEventDisableTiming) != hipSuccess)
        return cleanup(fail(FMCW_EHIP, "event create"));
    if (hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming) != hipSuccess)
      return cleanup(fail(FMCW_EHIP, "event create"));
  }
  h->n_wg_max = (size_t)c.max_frames * tiles_per_frame(h);
  {
    // Each tile owns a slot of 1/32 of its cells (a 3 % detection density, far above any
    // sane false-alarm rate; 32 entries for a 1024-cell wave tile); denser tiles spill into
    // a shared overflow region of a further 1/64 of all cells.  Detections beyond both are
    // counted as dropped (FMCW_EDETCAP).
    const size_t cells_frame = (size_t)c.n_range * c.n_doppler;
    const size_t cells_tile = cells_frame / tiles_per_frame(h);
    h->slot_cap = (uint32_t)std::max<size_t>(32, cells_tile / 32);
    const size_t slots = h->n_wg_max * h->slot_cap;
    const size_t ovf = std::max<size_t>((size_t)c.max_frames * cells_frame / 64, 65536);
    if (slots + ovf > 0x7fffffffu) return cleanup(fail(FMCW_EINVAL, "max_frames too large for the detection scratch"));
    h->ovf_base = (uint32_t)slots;
    h->det_scratch_cap = (uint32_t)(slots + ovf);
  }
  ALLOC(h->det_scratch, (size_t)h->det_scratch_cap * sizeof(fmcw_det));
  ALLOC(h->counter, 16);
  ALLOC(h->n_dets_tmp, 16);
  ALLOC(h->wg_base, h->n_wg_max * sizeof(uint32_t));
  ALLOC(h->wg_count, h->n_wg_max * sizeof(uint32_t));
  ALLOC(h->wg_off, h->n_wg_max * sizeof(uint32_t));
  ALLOC(h->block_sum, ((h->n_wg_max + 1023) / 1024 + 1) * sizeof(uint32_t));
#undef ALLOC
  {
    // the range table carries the 2^-range_shift scaling (Q15: applied after the integer window)
    std::vector<float> wr = window_table(c.n_range, c.window, c.window == FMCW_WIN_Q15_RTL ? 0 : c.range_shift),
                       wd = window_table(c.n_doppler, c.window == FMCW_WIN_Q15_RTL ? FMCW_WIN_HAMMING : c.window);
    if (hipMemcpy(h->win_r, wr.data(), wr.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(h->win_d, wd.data(), wd.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(h->wg_count, 0, h->n_wg_max * sizeof(uint32_t)) != hipSuccess)
      return cleanup(fail(FMCW_EHIP, "window upload failed"));
  }
  if (c.cfar_kind == FMCW_CFAR_OS2D) {
    const Cfar2DArgs a = cfar2_args(c);
    h->cfar2d_smem = cfar2_smem(c.n_doppler, a.hr);
    const Cfar2Info ci = cfar2_info(c.n_doppler, a.hd, a.gd);  // the kernel launch_cfar runs
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(ci.fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)h->cfar2d_smem) != hipSuccess)
      (void)hipGetLastError();
    occupancy_grid(ci.fn, 256, h->cfar2d_smem, h->n_cu, &h->grid_cfar);
  }
  setup_fused(h);
  *out = h;
  return FMCW_OK;
}

int fmcw_destroy(fmcw_handle* h) {
  if (!h) return FMCW_OK;
  hipSetDevice(h->cfg.device_id);
  void* ptrs[] = {h->win_r, h->win_d, h->inter, h->lin_scratch, h->det_scratch, h->counter,
                  h->n_dets_tmp, h->wg_base, h->wg_count, h->wg_off, h->block_sum,
                  h->stage_cube, h->stage_map, h->stage_dets, h->fused_spec, h->fused_ctl, h->fused_trace,
                  h->pair_b};
  for (void* p : ptrs)
    if (p) hipFree(p);
  for (auto& pe : h->pending) {
    hipEventDestroy(pe.a);
    hipEventDestroy(pe.b);
  }
  for (auto e : h->free_events) hipEventDestroy(e);
  for (int b = 1; b < 3; ++b) {
    if (h->inter_b[b]) hipFree(h->inter_b[b]);
    if (h->lin_b[b]) hipFree(h->lin_b[b]);
  }
  for (int b = 0; b < 3; ++b) {
    if (h->ev_k1[b]) hipEventDestroy(h->ev_k1[b]);
    if (h->ev_free[b]) hipEventDestroy(h->ev_free[b]);
  }
  if (h->ev_fork) hipEventDestroy(h->ev_fork);
  if (h->ev_join) hipEventDestroy(h->ev_join);
  for (int i = 0; i < 2; ++i)
    if (h->ps[i]) hipStreamDestroy(h->ps[i]);
  delete h;
  return FMCW_OK;
}

int fmcw_enqueue(fmcw_handle* h, const void* cube, size_t n_frames, float* rd_map, fmcw_det* dets,
                 size_t det_cap, uint32_t* n_dets_dev, void* stream) {
  if (!h || !cube) return fail(FMCW_EINVAL, "null handle or cube");
  const fmcw_config& c = h->cfg;
  if (n_frames < 1 || n_frames > c.max_frames)
    return fail(FMCW_EINVAL, "n_frames=%zu outside [1, max_frames=%u]", n_frames, c.max_frames);
  if (c.cfar_kind != FMCW_CFAR_NONE && !n_dets_dev)
    return fail(FMCW_EINVAL, "n_dets_dev is required when a CFAR is configured");
  HIP_TRY(hipSetDevice(c.device_id));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const RangeInfo ri = range_info(c.n_range, c.in_dtype, c.window, c.spectrum_dtype == FMCW_SPEC_F16, h->k1_dual);
  const DopplerInfo di = doppler_info(c.n_doppler, c.mti_mode, c.spectrum_dtype == FMCW_SPEC_F16, h->k2_fast);
  const size_t frame_px = (size_t)c.n_range * c.n_doppler;
  const size_t in_frame_bytes = cube_bytes(c, 1);
  const Cfar1DArgs cf1 = cfar1_args(c);
  const DetSink sink = make_sink(h);
  int rc;
  if (c.cfar_kind != FMCW_CFAR_NONE) HIP_TRY(hipMemsetAsync(h->counter, 0, 2 * sizeof(uint32_t), s));

  // fused K1 + K2: one persistent launch for the whole batch (the 2-D CFAR needs the whole
  // linear map, so it runs on the fused path only when the caller asks for that map)
  const bool fuse = h->fused_ok && (c.cfar_kind != FMCW_CFAR_OS2D || (rd_map && c.map_kind == FMCW_MAP_LINEAR));
  h->fused_used_last = fuse;
  if (fuse) {
    HIP_TRY(hipMemsetAsync(h->fused_ctl, 0, FusedCtl::kWords * 4, s));
    FusedArgs a{};
    a.cube = cube;
    a.spec = h->fused_spec;
    a.win_r = h->win_r;
    a.chirp_w = h->win_d;
    a.lin_map = rd_map && c.map_kind == FMCW_MAP_LINEAR ? rd_map : nullptr;
    a.db_map = rd_map && c.map_kind == FMCW_MAP_DB ? rd_map : nullptr;
    a.ctl = h->fused_ctl;
    a.n_frames = (int)n_frames;
    a.frame0 = 0;
    a.tile0 = 0;
    a.per_xcd = h->fused_per_xcd;
    a.n_a = h->fused_na;
    a.n_b = h->fused_nb;
    a.mag_mode = c.mag_mode;
    a.census = 0;
    a.spin_limit = 2000000;  // ~0.1-1 s of polling: only a broken group ever reaches it
    a.cf = cf1;
    a.sink = sink;
    a.trace = h->fused_trace;
    if (h->fused_trace) HIP_TRY(hipMemsetAsync(h->fused_trace, 0, 8 * kTraceFrames * 8 * 8, s));
    {
      ProfScope ps(h, FMCW_K_FUSED, s);
      hipLaunchKernelGGL(h->fused_fn, dim3(8 * h->fused_per_xcd), dim3(256), 0, s, a);
      if ((rc = check_launch("k_fused"))) return rc;
    }
    if (c.cfar_kind == FMCW_CFAR_OS2D)
      for (size_t f0 = 0; f0 < n_frames; f0 += std::max<size_t>(h->chunk, kCfar2Batch)) {
        const int nf = (int)std::min<size_t>(std::max<size_t>(h->chunk, kCfar2Batch), n_frames - f0);
        if ((rc = launch_cfar(h, rd_map + f0 * frame_px, nf, (int)f0, s))) return rc;
      }
    if (c.cfar_kind != FMCW_CFAR_NONE) return launch_det_finish(h, n_frames, dets, det_cap, n_dets_dev, s);
    return FMCW_OK;
  }

  // Paired launches: launch i runs K1 of chunk i into buffer i % 2 beside K2 of chunk i - 1
  // from buffer (i - 1) % 2; the kernel boundary orders every write before its read
  if (h->pair_fn && n_frames > h->pair_chunk) {
    const size_t C = h->pair_chunk;
    const size_t n_chunks = (n_frames + C - 1) / C;
    const size_t tpf = c.n_range / di.WR;
    float2* bufs[2] = {h->inter, h->pair_b};
    for (size_t i = 0; i <= n_chunks; ++i) {
      PairArgs a{};
      a.win_r = h->win_r;
      a.chirp_w = h->win_d;
      a.cf = cf1;
      a.sink = sink;
      if (i < n_chunks) {
        const size_t f0 = i * C, nf = std::min(C, n_frames - f0);
        a.cube = static_cast<const char*>(cube) + f0 * in_frame_bytes;
        a.inter_w = bufs[i & 1];
        a.n_groups = (int)(nf * (c.n_doppler / ri.T));
      }
      if (i >= 1) {
        const size_t f0 = (i - 1) * C, nf = std::min(C, n_frames - f0);
        a.inter_r = bufs[(i - 1) & 1];
        a.n_tiles = (int)(nf * tpf);
        a.frame0 = (int)f0;
        a.tile0 = (int)(f0 * tpf);
        a.lin_map = rd_map && c.map_kind == FMCW_MAP_LINEAR ? rd_map + f0 * frame_px : nullptr;
      }
      const int items = std::max(a.n_groups, a.n_tiles / kWavesPerBlock);
      ProfScope ps(h, FMCW_K_PAIR, s);
      hipLaunchKernelGGL(h->pair_fn, dim3(std::min(items, h->grid_pair)), dim3(256), 0, s, a);
      if ((rc = check_launch("k_pair"))) return rc;
    }
    if (c.cfar_kind != FMCW_CFAR_NONE) return launch_det_finish(h, n_frames, dets, det_cap, n_dets_dev, s);
    return FMCW_OK;
  }

  // Chunks of h->chunk frames: K1 -> intermediate -> K2 (+ K3).  With the two-stream pipeline
  // (h->pipe_nb buffers) chunk c's K1 runs on ps[0] beside chunk c - 1's K2 on ps[1]; buffer b
  // is rewritten by K1 only after the K2 that read it (ev_free[b]).  Fork from / join to the
  // caller's stream with events, so the call stays stream-ordered (and graph-capturable).
  const size_t n_chunks = (n_frames + h->chunk - 1) / h->chunk;
  const bool piped = h->pipe_nb > 0 && n_chunks > 1;
  hipStream_t sa = s, sb = s;
  if (piped) {
    sa = h->ps[0];
    sb = h->ps[1];
    HIP_TRY(hipEventRecord(h->ev_fork, s));
    HIP_TRY(hipStreamWaitEvent(sa, h->ev_fork, 0));
    HIP_TRY(hipStreamWaitEvent(sb, h->ev_fork, 0));
  }
  size_t k3_f0 = 0;  // first frame of the caller's map not yet through the 2-D CFAR
  for (size_t ci = 0; ci < n_chunks; ++ci) {
    const size_t f0 = ci * h->chunk;
    const int nf = (int)std::min<size_t>(h->chunk, n_frames - f0);
    const void* src = static_cast<const char*>(cube) + f0 * in_frame_bytes;
    const int b = piped ? (int)(ci % h->pipe_nb) : 0;
    float2* inter = piped ? h->inter_b[b] : h->inter;
    if (piped && ci >= (size_t)h->pipe_nb) HIP_TRY(hipStreamWaitEvent(sa, h->ev_free[b], 0));
    {
      const int n_groups = nf * (int)c.n_rx * (int)(c.n_doppler / ri.T);
      ProfScope ps(h, FMCW_K_RANGE, sa);
      // MTI off: K1 applies the Doppler window too (k_doppler<NC, 0> expects it)
      const float* chirp_w = c.mti_mode == FMCW_MTI_OFF ? h->win_d : nullptr;
      hipLaunchKernelGGL(ri.fn, dim3(std::min(n_groups, h->grid_range)), dim3(ri.NT), 0, sa, src, inter,
                         h->win_r, chirp_w, (int)c.n_doppler, n_groups, q15_scale(c));
      if ((rc = check_launch("k_range"))) return rc;
    }
    if (piped) {
      HIP_TRY(hipEventRecord(h->ev_k1[b], sa));
      HIP_TRY(hipStreamWaitEvent(sb, h->ev_k1[b], 0));
    }
    float* lin = nullptr;
    float* db = nullptr;
    if (rd_map && c.map_kind == FMCW_MAP_LINEAR) lin = rd_map + f0 * frame_px;
    if (rd_map && c.map_kind == FMCW_MAP_DB) db = rd_map + f0 * frame_px;
    if (c.cfar_kind == FMCW_CFAR_OS2D && !lin) lin = piped ? h->lin_b[b] : h->lin_scratch;
    {
      const int n_tiles = nf * (int)(c.n_range / di.WR);
      const int grid = std::min((n_tiles + kWavesPerBlock - 1) / kWavesPerBlock, h->grid_doppler);
      ProfScope ps(h, FMCW_K_DOPPLER, sb);
      hipLaunchKernelGGL(di.fn, dim3(grid), dim3(di.NT), 0, sb, inter,
                         h->win_d, (int)c.n_range, (int)c.n_rx, h->lgT, h->lgRB, n_tiles, (int)f0,
                         (int)(f0 * (c.n_range / di.WR)), lin, db, c.mag_mode,
                         (c.compat_rtl & FMCW_COMPAT_MTI) ? 1 : 0, cf1, sink);
      if ((rc = check_launch("k_doppler"))) return rc;
    }
    if (piped) HIP_TRY(hipEventRecord(h->ev_free[b], sb));
    if (c.cfar_kind == FMCW_CFAR_OS2D) {
      // on the caller's map the 2-D CFAR runs over batches of >= kCfar2Batch frames: its
      // strips then cover more rows per workgroup and more frames share one launch
      const size_t done = f0 + (size_t)nf;
      if (!(rd_map && c.map_kind == FMCW_MAP_LINEAR)) {  // chunk scratch: this chunk only
        if ((rc = launch_cfar(h, lin, nf, (int)f0, sb))) return rc;
      } else if (done - k3_f0 >= kCfar2Batch || done == n_frames) {
        if ((rc = launch_cfar(h, rd_map + k3_f0 * frame_px, (int)(done - k3_f0), (int)k3_f0, sb))) return rc;
        k3_f0 = done;
      }
    }
  }
  if (piped) {  // join: everything on ps[0] precedes ps[1]'s last K2, so ps[1] alone is enough
    HIP_TRY(hipEventRecord(h->ev_join, sb));
    HIP_TRY(hipStreamWaitEvent(s, h->ev_join, 0));
  }
  if (c.cfar_kind != FMCW_CFAR_NONE) return launch_det_finish(h, n_frames, dets, det_cap, n_dets_dev, s);
  return FMCW_OK;
}

int fmcw_process(fmcw_handle* h, const void* cube, size_t n_frames, float* rd_map, fmcw_det* dets,
                 size_t det_cap, size_t* n_dets, void* stream) {
  if (!h || !cube) return fail(FMCW_EINVAL, "null handle or cube");
  const fmcw_config& c = h->cfg;
  if (n_frames < 1 || n_frames > c.max_frames)
    return fail(FMCW_EINVAL, "n_frames=%zu outside [1, max_frames=%u]", n_frames, c.max_frames);
  HIP_TRY(hipSetDevice(c.device_id));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const size_t cb = cube_bytes(c, n_frames);
  const size_t map_bytes = n_frames * (size_t)c.n_range * c.n_doppler * sizeof(float);
  const void* d_cube = cube;
  float* d_map = rd_map;
  fmcw_det* d_dets = dets;
  int rc;
  if (!is_device_ptr(cube)) {
    if ((rc = ensure_stage(&h->stage_cube, &h->stage_cube_bytes, cb, "cube"))) return rc;
    HIP_TRY(hipMemcpyAsync(h->stage_cube, cube, cb, hipMemcpyHostToDevice, s));
    d_cube = h->stage_cube;
  }
  if (rd_map && !is_device_ptr(rd_map)) {
    if ((rc = ensure_stage(&h->stage_map, &h->stage_map_bytes, map_bytes, "map"))) return rc;
    d_map = h->stage_map;
  }
  if (dets && det_cap && !is_device_ptr(dets)) {
    size_t have = h->stage_dets_cap * sizeof(fmcw_det);
    if ((rc = ensure_stage(&h->stage_dets, &have, det_cap * sizeof(fmcw_det), "detection"))) return rc;
    h->stage_dets_cap = have / sizeof(fmcw_det);
    d_dets = h->stage_dets;
  }
  if ((rc = fmcw_enqueue(h, d_cube, n_frames, d_map, d_dets, det_cap, h->n_dets_tmp, stream))) return rc;
  uint32_t ndd[2] = {0, 0};  // found, dropped
  hipError_t e = hipSuccess;
  if (c.cfar_kind != FMCW_CFAR_NONE)
    e = hipMemcpyAsync(ndd, h->n_dets_tmp, sizeof ndd, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess && rd_map && d_map != rd_map)
    e = hipMemcpyAsync(rd_map, d_map, map_bytes, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e == hipSuccess && h->fused_used_last) {
    uint32_t ferr = 0;
    e = hipMemcpy(&ferr, h->fused_ctl + FusedCtl::kErr, 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess && ferr) {
      // the fused launch gave up (a bounded wait expired): redo the batch on K1 + K2 and keep
      // this handle there
      h->fused_ok = false;
      h->fused_fallbacks += 1;
      return fmcw_process(h, cube, n_frames, rd_map, dets, det_cap, n_dets, stream);
    }
  }
  const uint32_t nd = ndd[0];
  if (e == hipSuccess && dets && d_dets != dets && nd)
    e = hipMemcpy(dets, d_dets, std::min<size_t>(nd, det_cap) * sizeof(fmcw_det), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return fail(FMCW_EHIP, "fmcw_process: %s", hipGetErrorString(e));
  if (n_dets) *n_dets = nd;
  if (c.cfar_kind != FMCW_CFAR_NONE && (nd > det_cap || ndd[1] > 0))
    return fail(FMCW_EDETCAP, "%u detections, det_cap %zu, %u beyond the handle's scratch", nd, det_cap,
                ndd[1]);
  return FMCW_OK;
}

int fmcw_range_ct(fmcw_handle* h, const void* cube, size_t n_frames, void* spec, void* stream) {
  if (!h || !cube || !spec) return fail(FMCW_EINVAL, "null argument");
  const fmcw_config& c = h->cfg;
  if (n_frames < 1 || n_frames > c.max_frames) return fail(FMCW_EINVAL, "n_frames out of range");
  HIP_TRY(hipSetDevice(c.device_id));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // the stage output is the fp32 spectrum whatever spectrum_dtype the path uses: K1's fp32
  // variant, as many frames per launch as the intermediate buffer holds at 8 B per point
  const RangeInfo ri = range_info(c.n_range, c.in_dtype, c.window, false, h->k1_dual);
  const size_t in_frame_bytes = cube_bytes(c, 1);
  const size_t fr_px = (size_t)c.n_rx * c.n_range * c.n_doppler;
  const size_t rc_chunk = std::max<size_t>(1, h->inter_bytes / (fr_px * sizeof(float2)));
  for (size_t f0 = 0; f0 < n_frames; f0 += rc_chunk) {
    const int nf = (int)std::min<size_t>(rc_chunk, n_frames - f0);
    const int n_groups = nf * (int)c.n_rx * (int)(c.n_doppler / ri.T);
    {
      ProfScope ps(h, FMCW_K_RANGE, s);
      hipLaunchKernelGGL(ri.fn, dim3(std::min(n_groups, h->grid_range)), dim3(ri.NT), 0, s,
                         static_cast<const char*>(cube) + f0 * in_frame_bytes, h->inter, h->win_r,
                         (const float*)nullptr, (int)c.n_doppler, n_groups, q15_scale(c));
      int rc = check_launch("k_range");
      if (rc) return rc;
    }
    const size_t total = (size_t)nf * fr_px;
    hipLaunchKernelGGL(k_unblock, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, h->inter,
                       static_cast<float2*>(spec) + f0 * fr_px, (int)c.n_range, (int)c.n_doppler, h->T,
                       h->RB, total);
    int rc = check_launch("k_unblock");
    if (rc) return rc;
  }
  return FMCW_OK;
}

int fmcw_magnitude(const float* iq, float* out, size_t n, int mag_mode, void* stream) {
  if (!iq || !out) return fail(FMCW_EINVAL, "null argument");
  if (mag_mode != FMCW_MAG_ABS && mag_mode != FMCW_MAG_AMBM) return fail(FMCW_EINVAL, "mag_mode");
  if (!n) return FMCW_OK;
  hipLaunchKernelGGL(k_magnitude, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const float2*>(iq), out, n,
                     mag_mode);
  return check_launch("k_magnitude");
}

int fmcw_cfar(fmcw_handle* h, const float* map, size_t n_frames, fmcw_det* dets, size_t det_cap,
              uint32_t* n_dets_dev, void* stream) {
  if (!h || !map || !n_dets_dev) return fail(FMCW_EINVAL, "null argument");
  const fmcw_config& c = h->cfg;
  if (c.cfar_kind == FMCW_CFAR_NONE) return fail(FMCW_EINVAL, "handle has cfar_kind NONE");
  if (n_frames < 1 || n_frames > c.max_frames) return fail(FMCW_EINVAL, "n_frames out of range");
  HIP_TRY(hipSetDevice(c.device_id));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  h->fused_used_last = false;
  HIP_TRY(hipMemsetAsync(h->counter, 0, 2 * sizeof(uint32_t), s));
  int rc = launch_cfar(h, map, (int)n_frames, 0, s);
  if (rc) return rc;
  return launch_det_finish(h, n_frames, dets, det_cap, n_dets_dev, s);
}

int fmcw_set_profiling(fmcw_handle* h, int enable) {
  if (!h) return fail(FMCW_EINVAL, "null handle");
  h->profiling = enable != 0;
  return FMCW_OK;
}

int fmcw_get_info(fmcw_handle* h, int key, int64_t* value) {
  if (!h || !value) return fail(FMCW_EINVAL, "null argument");
  switch (key) {
    case FMCW_INFO_FUSED: *value = h->fused_ok ? 1 : 0; return FMCW_OK;
    case FMCW_INFO_FUSED_GROUP: *value = h->fused_per_xcd; return FMCW_OK;
    case FMCW_INFO_FUSED_FALLBACKS: *value = h->fused_fallbacks; return FMCW_OK;
    case FMCW_INFO_CHUNK: *value = h->chunk; return FMCW_OK;
    case FMCW_INFO_PAIR_CHUNK: *value = h->pair_fn ? h->pair_chunk : 0; return FMCW_OK;
  }
  return fail(FMCW_EINVAL, "fmcw_get_info: unknown key %d", key);
}

int fmcw_get_fused_trace(fmcw_handle* h, uint64_t* out, size_t n_words) {
  if (!h || !out) return fail(FMCW_EINVAL, "null argument");
  if (!h->fused_trace) return fail(FMCW_EINVAL, "no fused trace (create the handle with FMCW_FUSED_TRACE=1)");
  HIP_TRY(hipSetDevice(h->cfg.device_id));
  HIP_TRY(hipMemcpy(out, h->fused_trace, std::min<size_t>(n_words, 8 * kTraceFrames * 8) * 8, hipMemcpyDeviceToHost));
  return FMCW_OK;
}

int fmcw_kernel_times(fmcw_handle* h, double* ms, uint64_t* launches) {
  if (!h) return fail(FMCW_EINVAL, "null handle");
  HIP_TRY(hipSetDevice(h->cfg.device_id));
  for (auto& pe : h->pending) {
    HIP_TRY(hipEventSynchronize(pe.b));
    float t = 0.f;
    HIP_TRY(hipEventElapsedTime(&t, pe.a, pe.b));
    h->ms[pe.kid] += t;
    h->launches[pe.kid] += 1;
    h->free_events.push_back(pe.a);
    h->free_events.push_back(pe.b);
  }
  h->pending.clear();
  for (int k = 0; k < FMCW_K_COUNT; ++k) {
    if (ms) ms[k] = h->ms[k];
    if (launches) launches[k] = h->launches[k];
  }
  return FMCW_OK;
}

int fmcw_reset_kernel_times(fmcw_handle* h) {
  if (!h) return fail(FMCW_EINVAL, "null handle");
  int rc = fmcw_kernel_times(h, nullptr, nullptr);
  for (int k = 0; k < FMCW_K_COUNT; ++k) {
    h->ms[k] = 0;
    h->launches[k] = 0;
  }
  return rc;
}

int fmcw_device_alloc(size_t bytes, void** ptr, int device_id) {
  if (!ptr) return fail(FMCW_EINVAL, "null ptr");
  HIP_TRY(hipSetDevice(device_id));
  if (hipMalloc(ptr, bytes) != hipSuccess) {
    (void)hipGetLastError();
    return fail(FMCW_ENOMEM, "hipMalloc(%zu)", bytes);
  }
  return FMCW_OK;
}

int fmcw_device_free(void* ptr) {
  if (ptr) HIP_TRY(hipFree(ptr));
  return FMCW_OK;
}

int fmcw_memcpy(void* dst, const void* src, size_t bytes, int kind) {
  const hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : kind == 1 ? hipMemcpyDeviceToHost
                                                                        : hipMemcpyDeviceToDevice;
  HIP_TRY(hipMemcpy(dst, src, bytes, k));
  return FMCW_OK;
}

int fmcw_device_count(int* n) {
  if (!n) return fail(FMCW_EINVAL, "null");
  *n = 0;
  if (hipGetDeviceCount(n) != hipSuccess) {
    (void)hipGetLastError();
    *n = 0;
  }
  return FMCW_OK;
}

}  // extern "C"
