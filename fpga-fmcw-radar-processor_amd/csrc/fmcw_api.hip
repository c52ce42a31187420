// fmcw_api.hip -- host side of libfmcw.so: the C-ABI declared in include/fmcw.h.
//
// The handle replaces the reference's elaborated radar_core instance (rtl/src/radar_core.vhd
// generics :12-19, FFT IP configuration handshake cfg_proc :279-301): it validates the
// configuration once, uploads the window tables (window_multiplier.vhd:34-49, as fp32) and
// allocates every scratch buffer, so fmcw_enqueue only launches kernels (graph-capturable).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/fmcw.h"
#include "dispatch.hpp"

using namespace fmcw;

// The host side's own small kernels (one translation unit: no instantiation tables).
namespace fmcw {
// --------------------------------------------------------------------------------------
// Detection ordering: one pass over the per-tile counts (in tile = (frame, range) order) that
// scans them and copies each tile's run to its final place.
// --------------------------------------------------------------------------------------
// Zeroing of up to three word arrays in one launch (two hipMemsetAsync fills cost ~12 us): the
// caller's status words of a call without a CFAR, and the handle's per-call counters when the
// previous call did not re-arm them (k_det_list).
__global__ void k_zero_words(uint32_t* __restrict__ a, int na, uint32_t* __restrict__ b, int nb,
                             uint32_t* __restrict__ c, int nc) {
  for (int i = threadIdx.x; i < max(na, max(nb, nc)); i += blockDim.x) {
    if (a && i < na) a[i] = 0u;
    if (b && i < nb) b[i] = 0u;
    if (c && i < nc) c[i] = 0u;
  }
}

// Look-back status word of workgroup w: high half = this call's epoch << 2 | error << 1 |
// inclusive, low half = w's detection count (aggregate) or, once inclusive, the count of tiles
// 0 .. kDetTiles (w + 1) - 1.  One 64-bit store / load at agent scope: coherent across the XCDs' L2s.
// The epoch lives in device memory (ep[0], 1 .. 2^30 - 1; ep[1] counts the workgroups that have
// published their inclusive word): every workgroup reads it once at its start, and the last one
// to publish -- when every workgroup of the launch has read it -- advances it and re-arms ep[1].
// So a launch captured into a hipGraph tags its words afresh on every replay (a host-chosen epoch
// would be baked into the graph, and a replay could take a previous replay's word for its own).
constexpr uint32_t kLbIncl = 1u, kLbErr = 2u;
// tiles (= threads) per k_det_list workgroup (256-tile workgroups: 10.7-10.9 / 6.0 / 8.9-9.1 us per
// step at configs 2 / 3 / 5 against 7.4-7.6 / 5.2-5.3 / 7.2-7.3, profiles/r04/detlist/)
constexpr int kDetTiles = 1024;
constexpr uint32_t kLbMaxPolls = 1u << 20;  // >> any real wait (one poll ~1 us): a safety net only

__device__ __forceinline__ void lb_publish(uint64_t* st, uint32_t hi, uint32_t v) {
  __hip_atomic_store(st, ((uint64_t)hi << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Round 4: one launch instead of a level-1 scan launch plus a level-2 / copy launch.  Workgroup
// w owns tiles kDetTiles w .. kDetTiles (w + 1) - 1, one per thread: it scans their counts, publishes its aggregate, and takes
// its offset by decoupled look-back -- wave 0 reads the status words of the 64 nearest
// predecessors at once and sums back to the nearest inclusive one.  A workgroup only waits for
// lower ids, which the dispatcher started before it, so the chain drains; the wait is bounded
// all the same, and a workgroup that gives up marks its word (and so every later one) with an
// error the last workgroup reports as every detection lost.  One lane per tile copies the
// tile's records; a tile with more than 8 (a target's row) is copied by the whole wave, 64
// records per step, so one hot tile does not serialise the kernel.  The last workgroup writes
// the status words -- [0] every detection found, [1] of which not stored, [2] / [3] the
// saturation counts the call's K1 / K2 accumulated in the handle's `sat` -- and re-arms the
// handle's per-call counters (overflow use, drops, saturations, the 2-D CFAR launches'
// candidate counters) for the next call: every kernel that uses them ran before this one.
__global__ void __launch_bounds__(kDetTiles)
k_det_list(const fmcw_det* __restrict__ scratch, uint32_t scratch_cap, const uint32_t* __restrict__ wg_base,
           const uint32_t* __restrict__ wg_count, int n, fmcw_det* __restrict__ out, uint32_t cap,
           uint64_t* __restrict__ lb, uint32_t* __restrict__ ep, uint32_t* __restrict__ n_dets,
           uint32_t* __restrict__ counter, uint32_t* __restrict__ sat, uint32_t* __restrict__ k3_ctr, int n_k3) {
  __shared__ int s_wave[kDetTiles / 64 + 1];
  __shared__ uint32_t s_pre, s_err;
  const int lane = threadIdx.x & 63;
  const int w = blockIdx.x;
  const int i = w * kDetTiles + threadIdx.x;
  const uint32_t c = i < n ? wg_count[i] : 0u;
  int agg;
  const uint32_t e = (uint32_t)block_excl_scan<kDetTiles>((int)c, s_wave, agg);
  if (threadIdx.x < 64) {
    // this launch's epoch (set by the previous launch's last publisher: visible at launch start)
    const uint32_t epoch = __builtin_amdgcn_readfirstlane(
        __hip_atomic_load(ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const uint32_t tag = epoch << 2;
    uint32_t pre = 0, err = 0;
    if (w > 0) {
      if (lane == 0) lb_publish(lb + w, tag, (uint32_t)agg);
      int top = w - 1;  // nearest predecessor not yet summed
      uint32_t polls = 0;
      for (;;) {
        const int k = top - lane;
        uint32_t hi = tag | kLbIncl, v = 0;  // below workgroup 0: an inclusive zero
        if (k >= 0) {
          const uint64_t x = __hip_atomic_load(lb + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          hi = (uint32_t)(x >> 32);
          v = (uint32_t)x;
        }
        const bool ready = (hi >> 2) == epoch;
        const uint64_t rdy = __ballot(ready), inc = __ballot(ready && (hi & kLbIncl));
        const int f = inc ? __builtin_ctzll(inc) : 63;            // nearest inclusive lane
        const uint64_t need = f == 63 ? ~0ull : (2ull << f) - 1;  // lanes 0 .. f
        if ((rdy & need) == need) {
          uint32_t t = lane <= f ? v : 0u, te = lane <= f ? (hi & kLbErr) : 0u;
#pragma unroll
          for (int x = 32; x >= 1; x >>= 1) {
            t += (uint32_t)__shfl_xor((int)t, x, 64);
            te |= (uint32_t)__shfl_xor((int)te, x, 64);
          }
          pre += t;
          err |= te;
          if (inc) break;
          top -= 64;
          polls = 0;
        } else if (++polls > kLbMaxPolls) {
          err = kLbErr;
          break;
        }
      }
    }
    if (lane == 0) {
      lb_publish(lb + w, tag | kLbIncl | err, pre + (uint32_t)agg);
      s_pre = pre;
      s_err = err;
      // the last workgroup to get here: every other one has read `epoch` (it did so before
      // publishing), so the next launch's epoch can be set, and the count re-armed
      if (__hip_atomic_fetch_add(ep + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
        const uint32_t nx = (epoch + 1u) & 0x3fffffffu;
        __hip_atomic_store(ep + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ep, nx ? nx : 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  __syncthreads();
  const uint32_t P = s_pre;
  if (w == (int)gridDim.x - 1) {
    if (threadIdx.x == 0) {
      n_dets[0] = P + (uint32_t)agg;
      n_dets[1] = s_err ? 0xffffffffu : counter[1];
      n_dets[2] = sat ? sat[0] : 0u;
      n_dets[3] = sat ? sat[1] : 0u;
      counter[0] = 0u;
      counter[1] = 0u;
      if (sat) sat[0] = sat[1] = 0u;
    }
    for (int k = threadIdx.x; k < n_k3; k += kDetTiles) k3_ctr[k] = 0u;
  }
  if (!out) return;
  const uint32_t b = c ? wg_base[i] : 0u, o = P + e;
  if (c <= 8)
    for (uint32_t k = 0; k < c; ++k)
      if (b + k < scratch_cap && o + k < cap) out[o + k] = scratch[b + k];
  uint64_t big = __ballot(c > 8);
  while (big) {
    const int l = __builtin_ctzll(big);
    big &= big - 1;
    const uint32_t cl = (uint32_t)__shfl((int)c, l, 64), bl = (uint32_t)__shfl((int)b, l, 64);
    const uint32_t ol = (uint32_t)__shfl((int)o, l, 64);
    for (uint32_t k = lane; k < cl; k += 64)
      if (bl + k < scratch_cap && ol + k < cap) out[ol + k] = scratch[bl + k];
  }
}

// --------------------------------------------------------------------------------------
// Kernels of the stage entry points.
// --------------------------------------------------------------------------------------
// inter (tiled) -> spec[fr][r][c] canonical corner-turner order.
__global__ void k_unblock(const float2* __restrict__ inter, float2* __restrict__ spec, int ns, int nc,
                          int T, int RB, size_t total) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const size_t per = (size_t)ns * nc;
  const size_t fr = i / per;
  const int rem = (int)(i - fr * per);
  const int r = rem / nc, c = rem - r * nc;
  const int ncb = nc / T;
  const size_t off = ((size_t)((r / RB) * ncb + c / T) * RB + (r % RB)) * T + (c % T);
  spec[i] = inter[fr * per + off];
}

__global__ void k_magnitude(const float2* __restrict__ iq, float* __restrict__ out, size_t n, int mode) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float2 X = iq[i];
  if (mode == FMCW_MAG_AMBM) {
    const float ai = fabsf(X.x), aq = fabsf(X.y);
    const float mx = fmaxf(ai, aq), mn = fminf(ai, aq);
    out[i] = mx + floorf(mn * 0.25f) + floorf(mn * 0.125f);
  } else {
    out[i] = mag_sqrt(X.x * X.x + X.y * X.y);
  }
}

}  // namespace fmcw

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
  int k1_want = kRangePx;   // preferred K1 family (FMCW_LAB builds: environment FMCW_K1)
  int k1_kind = kRangeSingle;  // the family the handle runs
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
  uint32_t* sat = nullptr;      // [0] window, [1] word saturations of the current call (status words 2, 3)
  // the per-call device counters (counter[0..1], sat, k3_ctr) are zero: re-armed by the previous
  // call's k_det_list (or at fmcw_create); a call that stopped early leaves this false and the
  // next one zeroes them first
  bool counters_armed = false;
  uint32_t* wg_base = nullptr;
  uint32_t* wg_count = nullptr;
  uint64_t* lb_status = nullptr;  // k_det_list look-back words, one per kDetTiles tiles
  uint32_t* det_epoch = nullptr;   // k_det_list's device-resident call tag and publish count (2 words)
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
  int grid_k3b = 0, grid_k3c = 0;       // K3b / K3c grids (kCfar2DecideGrid / kCfar2EmitGrid)
  size_t cfar2d_smem = 0;
  size_t inter_bytes = 0;               // h->inter (chunk frames of the K1 -> K2 spectrum)
  int cfar2_steps = 0;                  // 2-D CFAR steps per strip (0 = cost model; FMCW_PARAM_CFAR2D_STEPS)
  int cfar2_steps_last = 0;             // the strip length of the last 2-D CFAR launch (FMCW_INFO_CFAR2D_STEPS)
  // 2-D CFAR candidate lists (cfar2d.hpp Cfar2Cands): room for every cell of k3_frames frames, and
  // a counter pair per K3 launch of a call (k3_launches of them, zeroed with the status words)
  uint32_t* cand_cell = nullptr;
  float* cand_thr = nullptr;
  uint32_t* cand_tiles = nullptr;
  uint32_t* cand_pcell = nullptr;   // k_cfar2d_lv's strip-private spill regions (Cfar2Cands pcell / ptile)
  uint32_t* cand_ptile = nullptr;
  uint32_t* k3_ctr = nullptr;
  int k3_frames = 0, k3_launches = 0;
  int k3_launch_idx = 0;                // launches of the current call so far
  uint32_t last_status[2] = {0, 0};     // fmcw_process: status words 2, 3 of its last call
  // profiling
  bool profiling = false;
  std::vector<PendingEvent> pending;
  std::vector<hipEvent_t> free_events;
  double ms[FMCW_K_COUNT] = {};
  uint64_t launches[FMCW_K_COUNT] = {};
};

namespace {

// K2's FAST instantiation (kernels.hpp): MTI off, |X| magnitude, no dB map, fp32 windows, and the
// 1-D CFAR (if any) at the reference geometry in fp32
bool k2_fast(const fmcw_config& c) {
  const bool cfar_ok = c.cfar_kind != FMCW_CFAR_OS1D ||
                       (c.cfar1d_ref == 8 && c.cfar1d_guard == 2 && (int)(2 * c.cfar1d_ref) - (int)c.cfar1d_rank <= 4 &&
                        !(c.compat_rtl & FMCW_COMPAT_CFAR));
  return c.mti_mode == FMCW_MTI_OFF && c.mag_mode != FMCW_MAG_AMBM && c.map_kind != FMCW_MAP_DB &&
         c.window != FMCW_WIN_Q15_RTL && cfar_ok
#if FMCW_LAB  // A/B builds only (tools/build_variants.sh): the generic kernel on a FAST configuration
         && !std::getenv("FMCW_K2_GENERIC")
#endif
      ;
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
  if (range_info(c.n_range, c.in_dtype, c.window, FMCW_SPEC_F32, kRangePx).T > (int)c.n_doppler)
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
    if (cfar2_info(c.n_doppler, a.hd, a.gd, a.hr, a.gr, a.compat != 0).smem > 160 * 1024)
      return fail(FMCW_EINVAL, "2-D CFAR range extent too large for LDS");
  } else if (c.cfar_kind != FMCW_CFAR_NONE) {
    return fail(FMCW_EINVAL, "cfar_kind=%d unknown", c.cfar_kind);
  }
  if (c.compat_rtl & ~(uint32_t)(FMCW_COMPAT_CFAR | FMCW_COMPAT_MTI))
    return fail(FMCW_EINVAL, "compat_rtl=0x%x: unknown bits", c.compat_rtl);
  if ((c.compat_rtl & FMCW_COMPAT_MTI) && c.mti_mode == FMCW_MTI_OFF)
    return fail(FMCW_EINVAL, "compat MTI needs mti_mode 2 or 3");
  if (c.range_shift > 13) return fail(FMCW_EINVAL, "range_shift=%u: must be in [0, 13]", c.range_shift);
  if (c.spectrum_dtype != FMCW_SPEC_F32 && c.spectrum_dtype != FMCW_SPEC_F16 && c.spectrum_dtype != FMCW_SPEC_S48)
    return fail(FMCW_EINVAL, "spectrum_dtype=%d unknown", c.spectrum_dtype);
  if (c.spectrum_dtype == FMCW_SPEC_S48) {
    // one exponent per chirp group of a range bin (a quad of a K1 tile row at n_range <= 1024, a
    // pair above): the group must be one K2 lane group (n_doppler >= 64), and no MTI (the
    // canceller reads neighbouring chirps from other lanes of the group)
    if (c.n_doppler < 64) return fail(FMCW_EINVAL, "spectrum_dtype S48 needs n_doppler >= 64");
    if (c.mti_mode != FMCW_MTI_OFF || c.window == FMCW_WIN_Q15_RTL)
      return fail(FMCW_EINVAL, "spectrum_dtype S48 is defined with MTI off and an fp32 window (not Q15_RTL)");
  }
  if (c.spectrum_dtype == FMCW_SPEC_F16 && (c.compat_rtl & FMCW_COMPAT_MTI))
    return fail(FMCW_EINVAL, "compat MTI is defined on the fp32 spectrum (spectrum_dtype F16)");
  // the Q15 path rounds the corner-turned spectrum to int16 words (and windows them in K2): an fp16
  // spectrum has 11 significant bits, so words above 2048 would already be quantised
  if (c.spectrum_dtype == FMCW_SPEC_F16 && c.window == FMCW_WIN_Q15_RTL)
    return fail(FMCW_EINVAL, "window Q15_RTL is defined on the fp32 spectrum (spectrum_dtype F16)");
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

// Per-kernel timing (fmcw_set_profiling): the scope's first launch takes the start event and its
// last launch the stop event through hipExtLaunchKernelGGL, so the events carry the dispatches'
// own begin / end timestamps -- the kernels' span, as rocprofv3's kernel trace reports it, without
// the event marker packets (and their dispatch gaps) that hipEventRecord around a launch adds.
struct ProfScope {
  fmcw_handle* h;
  int kid;
  hipEvent_t a = nullptr, b = nullptr;
  bool started = false;
  ProfScope(fmcw_handle* h_, int kid_) : h(h_), kid(kid_) {
    if (h->profiling) {
      a = take_event(h);
      b = a ? take_event(h) : nullptr;
      if (!b && a) h->free_events.push_back(a), a = nullptr;
    }
  }
  // events for one launch of the scope: start on the first, stop on the one flagged last
  hipEvent_t start() {
    if (started) return nullptr;
    started = true;
    return a;
  }
  hipEvent_t stop(bool last) const { return last ? b : nullptr; }
  ~ProfScope() {
    if (a && b && started) h->pending.push_back({kid, a, b});
    else if (a && b) h->free_events.push_back(a), h->free_events.push_back(b);
  }
};
// hipLaunchKernelGGL with the scope's events (none outside profiling)
template <typename F, typename... Args>
void launch_k(ProfScope& ps, bool last, F fn, dim3 grid, dim3 block, uint32_t smem, hipStream_t s, Args... args) {
  if (ps.a) hipExtLaunchKernelGGL(fn, grid, block, smem, s, ps.start(), ps.stop(last), 0u, args...);
  else hipLaunchKernelGGL(fn, grid, block, smem, s, args...);
}

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

// true while `s` is being captured into a hipGraph (nothing the call enqueues runs now)
bool capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return st == hipStreamCaptureStatusActive;
}

// Zero the per-call counters unless the previous call's k_det_list left them armed; the flag
// drops until this call's k_det_list is enqueued.  A call captured into a graph always zeroes
// them (a replay may follow any call, including one that stopped early) and leaves the flag as
// it was: capturing runs nothing, so the device state is still the one the flag describes.
int arm_counters(fmcw_handle* h, hipStream_t s, bool cap) {
  if (!h->counters_armed || cap) {
    hipLaunchKernelGGL(k_zero_words, dim3(1), dim3(256), 0, s, h->counter, 2, h->sat, 2, h->k3_ctr,
                       2 * h->k3_launches);
    if (int rc = check_launch("k_zero_words")) return rc;
  }
  if (!cap) h->counters_armed = false;
  return FMCW_OK;
}

constexpr size_t kCfar2Batch = 16;  // frames per 2-D CFAR launch on the caller's map (at least)
// K3b / K3c grids (4 waves per workgroup; K3b one candidate per wave at a time, K3c one wave tile).
// Round 5, with k_cfar2d_lv's ~10^5 candidates per 16-frame launch at config 5 (tools/cfar2d_bench.py,
// profiles/r05/k3_rules/): 1024 / 256 workgroups 336 us per launch, 2048 / 256 323, 2048 / 1024
// 302, 4096 / 2048 297; with round 4's few thousand candidates the grid was measured neutral.
// After K3b's software pipeline (later in round 5; tools/k3_grid_ab.sh, profiles/r05/k3_grid/, two
// interleaved passes, us per K3 batch, config 5 / config 3): 2048 / 1024 workgroups 261, 252 /
// 75.6, 75.1; 1024 / 1024 258, 250 / 73.3, 72.3; 4096 / 1024 253, 255 / 81.7, 81.4; emit grids 256 /
// 512 within noise.  With k_cfar2d_lv's later levels (8x fewer candidates at config 5) 2048 / 1024 /
// 512 decide workgroups and emit grids 1024 / 256 all measured 222-231 us (k3grid2, noise): 1024.
constexpr int kCfar2DecideGrid = 1024;
constexpr int kCfar2EmitGrid = 1024;

// The CFAR launcher shared by fmcw_enqueue (map just produced by K2) and fmcw_cfar.
int launch_cfar(fmcw_handle* h, const float* map_chunk, int nf, int frame0, hipStream_t s) {
  const fmcw_config& c = h->cfg;
  const DetSink sink = make_sink(h);
  const int tile0 = (int)(frame0 * tiles_per_frame(h));
  if (c.cfar_kind == FMCW_CFAR_OS2D) {
    const Cfar2DArgs a = cfar2_args(c);
    const Cfar2Info ci = cfar2_info(c.n_doppler, a.hd, a.gd, a.hr, a.gr, a.compat != 0);
    const size_t frame_px = (size_t)c.n_range * c.n_doppler;
    // pieces of at most k3_frames frames (the candidate lists' capacity), each its own K3a/b/c
    for (int p0 = 0; p0 < nf; p0 += h->k3_frames) {
      const int np = std::min(h->k3_frames, nf - p0);
      if (h->k3_launch_idx >= h->k3_launches) return fail(FMCW_EINVAL, "2-D CFAR: launch counter slots exhausted");
      Cfar2Cands cands{h->cand_cell, h->cand_thr, h->cand_tiles, h->k3_ctr + 2 * h->k3_launch_idx++,
                       h->cand_pcell, h->cand_ptile};
      const float* mp = map_chunk + (size_t)p0 * frame_px;
      // workgroup tiles (steps): 4 consecutive wave tiles of one frame; a strip is `steps` of them
      const int tpf = (int)((tiles_per_frame(h) + 3) / 4);
      const int steps = h->cfar2_steps ? std::min(h->cfar2_steps, tpf)
                                       : cfar2_steps_model(np, tpf, h->grid_cfar, doppler_info(c.n_doppler).WR * 4, a.hr);
      const int n_strips = np * ((tpf + steps - 1) / steps);
      const int grid = std::min(n_strips, h->grid_cfar);
      h->cfar2_steps_last = steps;
      ProfScope ps(h, FMCW_K_CFAR2D);
      launch_k(ps, false, ci.fn, dim3(grid), dim3(256), (uint32_t)h->cfar2d_smem, s, mp, (int)c.n_range, n_strips,
               steps, frame0 + p0, tile0 + (int)(p0 * tiles_per_frame(h)), a, sink, cands);
      if (int rc = check_launch("k_cfar2d")) return rc;
      // K3b / K3c: fixed grids that read the candidate counts on the device (no host round trip)
      launch_k(ps, false, ci.decide, dim3(h->grid_k3b), dim3(256), 0u, s, mp, (int)c.n_range, a, cands);
      launch_k(ps, true, ci.emit, dim3(h->grid_k3c), dim3(256), 0u, s, mp, (int)c.n_range, frame0 + p0, a, cands,
               sink);
      if (int rc = check_launch("k_cfar2d_decide / _emit")) return rc;
    }
    return FMCW_OK;
  }
  // 1-D on a caller map (fmcw_cfar); inside fmcw_enqueue the 1-D CFAR is fused into K2
  const DopplerInfo di = doppler_info(c.n_doppler);
  const int n_tiles = nf * (int)(c.n_range / di.WR);
  const int wpb = di.NT / 64;  // DopplerGeom<NC>::WPB: wave tiles per workgroup
  const int grid = std::min((n_tiles + wpb - 1) / wpb, h->grid_doppler);
  ProfScope ps(h, FMCW_K_CFAR2D);
  launch_k(ps, true, cfar1_fn(c.n_doppler), dim3(grid), dim3(di.NT), 0u, s, map_chunk, (int)c.n_range, n_tiles,
           frame0, tile0, cfar1_args(c), sink);
  return check_launch("k_cfar1d");
}

int launch_det_finish(fmcw_handle* h, size_t n_frames, fmcw_det* dets, size_t det_cap,
                      uint32_t* n_dets_dev, uint32_t* sat, hipStream_t s) {
  const int n = (int)(n_frames * tiles_per_frame(h));
  if (n < 1 || (size_t)n > h->n_wg_max) return fail(FMCW_EINVAL, "detection list over %d tiles", n);
  ProfScope ps(h, FMCW_K_COMPACT);
  // entries past the handle's scratch capacity are never stored: clip to it as well
  const bool copy = dets && det_cap;
  const uint32_t cap = copy ? (uint32_t)std::min<size_t>(det_cap, h->det_scratch_cap) : 0u;
  launch_k(ps, true, k_det_list, dim3((n + kDetTiles - 1) / kDetTiles), dim3(kDetTiles), 0u, s, (const fmcw_det*)h->det_scratch,
           h->det_scratch_cap, (const uint32_t*)h->wg_base, (const uint32_t*)h->wg_count, n,
           copy ? dets : (fmcw_det*)nullptr, cap, h->lb_status, h->det_epoch, n_dets_dev, h->counter, sat, h->k3_ctr,
           2 * h->k3_launches);
  return check_launch("k_det_list");
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
// spectrum of a chunk is written by K1 and read back by K2 right after; kept to ~13/16 of the
// 256 MiB Infinity Cache (MALL), K2's reads hit there.  Measured on config 2 (round 2, 1024
// frames per step): K2 0.63 us/frame at 128 frames (256 MiB), 0.57 at 96, 0.55 at 108-120, 0.81
// from 256 frames up (reads from HBM).  Round 4, same box, 3 runs each
// (profiles/r04/chunk/): 96 frames 807.7-809.6 k frames/s, 104 frames 814.8-820.0 k, 112 frames
// 810.3-819.5 k -- so 208 MiB, without round 2's rounding down to whole rounds of K2's grid
// (96 frames), which no longer paid.  Configs 3 / 5 (64 MiB per frame) keep 3 frames.
uint32_t auto_chunk(const fmcw_handle* h, size_t frame_inter) {
  const fmcw_config& c = h->cfg;
  constexpr size_t kMallBudget = 208u << 20;
  const size_t ch = std::max<size_t>(1, kMallBudget / frame_inter);
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
  // K1 family: k_range_px at N = 8192, the sequential-pair kernel at N = 4096, else k_range.
  // The release library reads no environment; FMCW_LAB builds (tools/build_variants.sh) take
  // FMCW_K1=single|seq|px for A/B runs.
#if FMCW_LAB
  if (const char* k1 = std::getenv("FMCW_K1"))
    h->k1_want = !std::strcmp(k1, "single") ? kRangeSingle : !std::strcmp(k1, "seq") ? kRangeSeq : kRangePx;
#endif
  h->k2_fast = k2_fast(c);
  const RangeInfo ri = range_info(c.n_range, c.in_dtype, c.window, c.spectrum_dtype, h->k1_want);
  h->k1_kind = ri.kind;
  h->T = ri.T;
  h->RB = ri.RB;
  h->lgT = __builtin_ctz(ri.T);
  h->lgRB = __builtin_ctz(ri.RB);
  const size_t frame_inter = (size_t)c.n_rx * c.n_range * c.n_doppler *
                             (c.spectrum_dtype == FMCW_SPEC_F16   ? sizeof(uint32_t)
                              : c.spectrum_dtype == FMCW_SPEC_S48 ? sizeof(S48)
                                                                  : sizeof(float2));
  occupancy_grid(ri.fn, ri.NT, 0, h->n_cu, &h->grid_range);
  const DopplerInfo di = doppler_info(c.n_doppler, c.mti_mode, c.spectrum_dtype, h->k2_fast, false, ri.T);
  if (!ri.fn || !di.fn) {
    delete h;
    return fail(FMCW_EINVAL, "no kernel for this configuration (spectrum_dtype %d)", c.spectrum_dtype);
  }
  occupancy_grid(di.fn, di.NT, 0, h->n_cu, &h->grid_doppler);
#if FMCW_LAB
  if (const char* cs = std::getenv("FMCW_CFAR2D_STEPS")) h->cfar2_steps = std::max(0, std::atoi(cs));
#endif
  h->chunk = c.chunk_frames ? std::min<uint32_t>(c.chunk_frames, c.max_frames) : auto_chunk(h, frame_inter);
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
  // K1 / K2 address a launch's spectrum with 32-bit byte offsets (buffer loads and stores)
  h->chunk = (uint32_t)std::max<size_t>(1, std::min<size_t>(h->chunk, ((size_t)1 << 32) / frame_inter - 1));
  // >= one fp32 frame: fmcw_range_ct writes the fp32 spectrum through it whatever spectrum_dtype
  // (+16 B: an S48 point is read as the 8 bytes from its record rounded down to 4)
  h->inter_bytes = std::max((size_t)h->chunk * frame_inter, (size_t)c.n_rx * c.n_range * c.n_doppler * sizeof(float2)) + 16;
  ALLOC(h->inter, h->inter_bytes);
  if (c.cfar_kind == FMCW_CFAR_OS2D) {
    ALLOC(h->lin_scratch, (size_t)h->chunk * c.n_range * c.n_doppler * sizeof(float));
    // candidate lists for K3 launches of up to k3_frames frames (fmcw_enqueue's batches: >= 16
    // frames, ending on a chunk boundary, so at most 16 + chunk - 1
    // frames): every cell may be a candidate, so they cannot overflow.  8 B per cell: at 8192 x
    // 1024 with the auto chunk (3 frames) 19 frames, 1.2 GiB.  A K3 launch addresses its cells with
    // 32-bit indices, so k3_frames is also capped at 2^32 cells (launch_cfar splits longer
    // batches into pieces of k3_frames).
    const size_t frame_cells = (size_t)c.n_range * c.n_doppler;
    h->k3_frames = (int)std::max<size_t>(1, std::min<size_t>({(size_t)c.max_frames, kCfar2Batch + h->chunk,
                                                              (size_t)0xffffffffu / frame_cells}));
    const size_t cells = (size_t)h->k3_frames * frame_cells;
    // K3 launches per call: one per chunk at most (map-less calls run it on each chunk's scratch),
    // else one per >= 16-frame batch, or one per k3_frames piece (fmcw_cfar)
    const size_t minb = std::min<size_t>(h->chunk, kCfar2Batch);
    h->k3_launches = (int)((c.max_frames + minb - 1) / minb + (c.max_frames + h->k3_frames - 1) / h->k3_frames + 2);
    ALLOC(h->cand_cell, cells * sizeof(uint32_t));
    ALLOC(h->cand_thr, cells * sizeof(float));
    ALLOC(h->cand_tiles, (size_t)h->k3_frames * tiles_per_frame(h) * sizeof(uint32_t));
    {
      const Cfar2DArgs a = cfar2_args(c);
      if (cfar2_info(c.n_doppler, a.hd, a.gd, a.hr, a.gr, a.compat != 0).spill) {
        ALLOC(h->cand_pcell, cells * sizeof(uint32_t));
        ALLOC(h->cand_ptile, (size_t)h->k3_frames * tiles_per_frame(h) * 2 * sizeof(uint32_t));
      }
    }
    ALLOC(h->k3_ctr, (size_t)2 * h->k3_launches * sizeof(uint32_t));
  }
  h->n_wg_max = (size_t)c.max_frames * tiles_per_frame(h);
  {
    // Round 6 (verdict r5 item 1): by default (det_capacity 0) each wave tile owns a slot of ALL
    // its cells, so the detection count a call reports is always backed by stored records, det_cap
    // is the only bound on the list, and no tile ever takes an atomic to store its run -- the
    // reference emits every non-zero CFAR output (radar_core.vhd:413-418), and its own
    // cfar_scale_ovr = 1 (os_cfar_2d.vhd:191-192) detects ~25 % of Rayleigh cells.  Round 5's
    // scratch (slots of 1/32 of a tile, a shared overflow region of 1/64 of the cells) lost 21,199
    // of 86,735 records on a ::3 lattice, and its dense tiles serialised on the region's counter.
    // The memory (16 B per cell) is only reserved: untouched pages cost no bandwidth.  With
    // det_capacity N > 0 a slot holds 1/32 of its tile (32 entries for a 1024-cell tile) and a
    // denser tile moves its whole run to a shared overflow region of N records (one atomic per such
    // tile).
    const size_t cells_frame = (size_t)c.n_range * c.n_doppler;
    const size_t cells_tile = cells_frame / tiles_per_frame(h);
    h->slot_cap = (uint32_t)(c.det_capacity ? std::max<size_t>(32, cells_tile / 32) : cells_tile);
    const size_t slots = h->n_wg_max * h->slot_cap;
    const size_t cells = (size_t)c.max_frames * cells_frame;
    const size_t ovf = c.det_capacity ? std::min<size_t>(c.det_capacity, cells) : 0;
    // 32-bit record indices; the overflow counter may run up to `cells` past ovf_base
    if (slots + cells >= 0xffffffffu)
      return cleanup(fail(FMCW_EINVAL, "max_frames %u: %zu cells exceed the 2^32 detection records of one call",
                          c.max_frames, cells));
    h->ovf_base = (uint32_t)slots;
    h->det_scratch_cap = (uint32_t)(slots + ovf);
  }
  ALLOC(h->det_scratch, (size_t)h->det_scratch_cap * sizeof(fmcw_det));
  ALLOC(h->counter, 16);
  ALLOC(h->sat, 8);
  ALLOC(h->n_dets_tmp, 16);
  ALLOC(h->wg_base, h->n_wg_max * sizeof(uint32_t));
  ALLOC(h->wg_count, h->n_wg_max * sizeof(uint32_t));
  ALLOC(h->lb_status, ((h->n_wg_max + kDetTiles - 1) / kDetTiles) * sizeof(uint64_t));
  ALLOC(h->det_epoch, 2 * sizeof(uint32_t));
#undef ALLOC
  {
    static const uint32_t kEpoch0[2] = {1u, 0u};  // first epoch 1 (the look-back words start at 0)
    // the range table carries the 2^-range_shift scaling (Q15: applied after the integer window)
    std::vector<float> wr = window_table(c.n_range, c.window, c.window == FMCW_WIN_Q15_RTL ? 0 : c.range_shift),
                       wd = window_table(c.n_doppler, c.window);  // Q15: the ROM integers, applied by K2
    if (hipMemcpy(h->win_r, wr.data(), wr.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(h->win_d, wd.data(), wd.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(h->wg_count, 0, h->n_wg_max * sizeof(uint32_t)) != hipSuccess ||
        hipMemset(h->lb_status, 0, ((h->n_wg_max + kDetTiles - 1) / kDetTiles) * sizeof(uint64_t)) != hipSuccess ||
        hipMemcpy(h->det_epoch, kEpoch0, sizeof kEpoch0, hipMemcpyHostToDevice) != hipSuccess)
      return cleanup(fail(FMCW_EHIP, "window upload failed"));
  }
  if (c.cfar_kind == FMCW_CFAR_OS2D) {
    const Cfar2DArgs a = cfar2_args(c);
    const Cfar2Info ci = cfar2_info(c.n_doppler, a.hd, a.gd, a.hr, a.gr, a.compat != 0);  // the kernel launch_cfar runs
    h->cfar2d_smem = ci.smem;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(ci.fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)h->cfar2d_smem) != hipSuccess)
      (void)hipGetLastError();
    occupancy_grid(ci.fn, 256, h->cfar2d_smem, h->n_cu, &h->grid_cfar);
  }
  h->grid_k3b = kCfar2DecideGrid;
  h->grid_k3c = kCfar2EmitGrid;
#if FMCW_LAB
  // experiment knobs (tools/overlap_lab.py): cap a persistent grid so that another stream's
  // kernels find free CU slots beside it
  auto cap_grid = [](const char* name, int* g) {
    if (const char* v = std::getenv(name)) {
      const int n = std::atoi(v);
      if (n > 0) *g = std::min(*g, n);
    }
  };
  cap_grid("FMCW_GRID_RANGE", &h->grid_range);
  cap_grid("FMCW_GRID_DOPPLER", &h->grid_doppler);
  cap_grid("FMCW_GRID_CFAR", &h->grid_cfar);
  for (auto [name, g] : {std::pair<const char*, int*>{"FMCW_GRID_K3B", &h->grid_k3b}, {"FMCW_GRID_K3C", &h->grid_k3c}})
    if (const char* v = std::getenv(name))
      if (std::atoi(v) > 0) *g = std::atoi(v);
#endif
  *out = h;
  return FMCW_OK;
}

int fmcw_destroy(fmcw_handle* h) {
  if (!h) return FMCW_OK;
  hipSetDevice(h->cfg.device_id);
  void* ptrs[] = {h->win_r, h->win_d, h->inter, h->lin_scratch, h->det_scratch, h->counter, h->sat,
                  h->n_dets_tmp, h->wg_base, h->wg_count, h->lb_status, h->det_epoch,
                  h->stage_cube, h->stage_map, h->stage_dets, h->cand_cell, h->cand_thr,
                  h->cand_tiles, h->cand_pcell, h->cand_ptile, h->k3_ctr};
  for (void* p : ptrs)
    if (p) hipFree(p);
  for (auto& pe : h->pending) {
    hipEventDestroy(pe.a);
    hipEventDestroy(pe.b);
  }
  for (auto e : h->free_events) hipEventDestroy(e);
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
  const RangeInfo ri = range_info(c.n_range, c.in_dtype, c.window, c.spectrum_dtype, h->k1_want);
  const DopplerInfo di = doppler_info(c.n_doppler, c.mti_mode, c.spectrum_dtype, h->k2_fast, false, ri.T);
  const size_t frame_px = (size_t)c.n_range * c.n_doppler;
  const size_t in_frame_bytes = cube_bytes(c, 1);
  const Cfar1DArgs cf1 = cfar1_args(c);
  const bool q15 = c.window == FMCW_WIN_Q15_RTL;
  // status words 2 / 3 (saturations) are counted atomically by the kernels that can saturate: into
  // the handle's `sat` words, which the call's last kernel (k_det_list) reports and re-arms
  // with the other per-call counters; without a CFAR there is no such kernel, and the caller's
  // words are zeroed and counted into directly
  const bool cfar = c.cfar_kind != FMCW_CFAR_NONE;
  uint32_t* const status = cfar ? h->sat : n_dets_dev ? n_dets_dev + 2 : nullptr;
  int rc;
  if (!cfar && n_dets_dev) {
    hipLaunchKernelGGL(k_zero_words, dim3(1), dim3(256), 0, s, nullptr, 0, n_dets_dev, FMCW_STATUS_WORDS, nullptr, 0);
    if ((rc = check_launch("k_zero_words"))) return rc;
  }
  const bool cap = capturing(s);
  if (cap && h->profiling) return fail(FMCW_EINVAL, "profiling events cannot be captured into a graph");
  if (cfar && (rc = arm_counters(h, s, cap))) return rc;
  h->k3_launch_idx = 0;

  // Chunks of h->chunk frames: K1 -> corner-turned spectrum -> K2 (+ K3)
  const size_t n_chunks = (n_frames + h->chunk - 1) / h->chunk;
  size_t k3_f0 = 0;  // first frame of the caller's map not yet through the 2-D CFAR
  for (size_t ci = 0; ci < n_chunks; ++ci) {
    // (Measured and dropped: the same number of chunks balanced in whole K2 rounds -- config 5's
    // 16 frames as 3,3,3,3,2,2 instead of 3,3,3,3,3,1: K2 59 -> 61 us per launch, configs 3 / 5
    // 1 % slower, profiles/r03/s2/ab_c*_b*.log.)
    const size_t f0 = ci * h->chunk;
    const int nf = (int)std::min<size_t>(h->chunk, n_frames - f0);
    const void* src = static_cast<const char*>(cube) + f0 * in_frame_bytes;
    {
      const int n_groups = nf * (int)c.n_rx * (int)(c.n_doppler / ri.T);
      ProfScope ps(h, FMCW_K_RANGE);
      // MTI off, fp32 window: K1 applies the Doppler window too (FFT linearity; K2 then skips
      // it); with MTI or the RTL-compat integer window K2 applies it after the canceller
      const float* chirp_w = c.mti_mode == FMCW_MTI_OFF && !q15 ? h->win_d : nullptr;
      launch_k(ps, true, ri.fn, dim3(std::min(n_groups, h->grid_range)), dim3(ri.NT), 0u, s, src, h->inter,
               (const float*)h->win_r, chirp_w, (int)c.n_doppler, n_groups, q15_scale(c), status);
      if ((rc = check_launch("k_range"))) return rc;
    }
    float* lin = nullptr;
    float* db = nullptr;
    if (rd_map && c.map_kind == FMCW_MAP_LINEAR) lin = rd_map + f0 * frame_px;
    if (rd_map && c.map_kind == FMCW_MAP_DB) db = rd_map + f0 * frame_px;
    if (c.cfar_kind == FMCW_CFAR_OS2D && !lin) lin = h->lin_scratch;
    {
      const int n_tiles = nf * (int)(c.n_range / di.WR);
      const int wpb = di.NT / 64;  // DopplerGeom<NC>::WPB
      const int grid = std::min((n_tiles + wpb - 1) / wpb, h->grid_doppler);
      ProfScope ps(h, FMCW_K_DOPPLER);
      launch_k(ps, true, di.fn, dim3(grid), dim3(di.NT), 0u, s, (const float2*)h->inter, (const float*)h->win_d,
               (int)c.n_range, (int)c.n_rx, h->lgT, h->lgRB, n_tiles, (int)f0, (int)(f0 * (c.n_range / di.WR)), lin,
               db, c.mag_mode, (c.compat_rtl & FMCW_COMPAT_MTI) ? 1 : 0, q15 ? 1 : 0, cf1, make_sink(h), status);
      if ((rc = check_launch("k_doppler"))) return rc;
    }
    if (c.cfar_kind == FMCW_CFAR_OS2D) {
      // on the caller's map the 2-D CFAR runs over batches of >= kCfar2Batch frames: its
      // strips then cover more rows per workgroup and more frames share one launch
      const size_t done = f0 + (size_t)nf;
      if (!(rd_map && c.map_kind == FMCW_MAP_LINEAR)) {  // chunk scratch: this chunk only
        if ((rc = launch_cfar(h, lin, nf, (int)f0, s))) return rc;
      } else if (done - k3_f0 >= kCfar2Batch || done == n_frames) {
        if ((rc = launch_cfar(h, rd_map + k3_f0 * frame_px, (int)(done - k3_f0), (int)k3_f0, s))) return rc;
        k3_f0 = done;
      }
    }
  }
  if (cfar) {
    if ((rc = launch_det_finish(h, n_frames, dets, det_cap, n_dets_dev, h->sat, s))) return rc;
    if (!cap) h->counters_armed = true;  // k_det_list re-arms them on the device, in stream order
  }
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
  uint32_t ndd[FMCW_STATUS_WORDS] = {0, 0, 0, 0};  // found, dropped, window / word saturations
  hipError_t e = hipMemcpyAsync(ndd, h->n_dets_tmp, sizeof ndd, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess && rd_map && d_map != rd_map)
    e = hipMemcpyAsync(rd_map, d_map, map_bytes, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  h->last_status[0] = ndd[2];
  h->last_status[1] = ndd[3];
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
  const RangeInfo ri = range_info(c.n_range, c.in_dtype, c.window, FMCW_SPEC_F32, h->k1_want);
  const size_t in_frame_bytes = cube_bytes(c, 1);
  const size_t fr_px = (size_t)c.n_rx * c.n_range * c.n_doppler;
  const size_t rc_chunk = std::max<size_t>(1, h->inter_bytes / (fr_px * sizeof(float2)));
  for (size_t f0 = 0; f0 < n_frames; f0 += rc_chunk) {
    const int nf = (int)std::min<size_t>(rc_chunk, n_frames - f0);
    const int n_groups = nf * (int)c.n_rx * (int)(c.n_doppler / ri.T);
    {
      ProfScope ps(h, FMCW_K_RANGE);
      launch_k(ps, true, ri.fn, dim3(std::min(n_groups, h->grid_range)), dim3(ri.NT), 0u, s,
               static_cast<const void*>(static_cast<const char*>(cube) + f0 * in_frame_bytes), h->inter,
               (const float*)h->win_r, (const float*)nullptr, (int)c.n_doppler, n_groups, q15_scale(c),
               (uint32_t*)nullptr);
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
  const bool cap = capturing(s);
  if (cap && h->profiling) return fail(FMCW_EINVAL, "profiling events cannot be captured into a graph");
  if (int rc0 = arm_counters(h, s, cap)) return rc0;
  h->k3_launch_idx = 0;
  int rc = launch_cfar(h, map, (int)n_frames, 0, s);
  if (rc) return rc;
  if ((rc = launch_det_finish(h, n_frames, dets, det_cap, n_dets_dev, nullptr, s))) return rc;
  if (!cap) h->counters_armed = true;
  return FMCW_OK;
}

int fmcw_set_profiling(fmcw_handle* h, int enable) {
  if (!h) return fail(FMCW_EINVAL, "null handle");
  h->profiling = enable != 0;
  return FMCW_OK;
}

int fmcw_set_param(fmcw_handle* h, int key, int64_t value) {
  if (!h) return fail(FMCW_EINVAL, "null handle");
  switch (key) {
    case FMCW_PARAM_CFAR2D_STEPS:
      if (value < 0 || value > (1 << 20)) return fail(FMCW_EINVAL, "cfar2d steps %lld (0 = cost model)", (long long)value);
      h->cfar2_steps = (int)value;
      return FMCW_OK;
  }
  return fail(FMCW_EINVAL, "fmcw_set_param: unknown key %d", key);
}

int fmcw_get_info(fmcw_handle* h, int key, int64_t* value) {
  if (!h || !value) return fail(FMCW_EINVAL, "null argument");
  switch (key) {
    case FMCW_INFO_CHUNK: *value = h->chunk; return FMCW_OK;
    case FMCW_INFO_RANGE_KERNEL: *value = h->k1_kind; return FMCW_OK;
    case FMCW_INFO_WINDOW_SATURATIONS: *value = h->last_status[0]; return FMCW_OK;
    case FMCW_INFO_WORD_SATURATIONS: *value = h->last_status[1]; return FMCW_OK;
    case FMCW_INFO_CFAR2D_STEPS: *value = h->cfar2_steps_last; return FMCW_OK;
  }
  return fail(FMCW_EINVAL, "fmcw_get_info: unknown key %d", key);
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
