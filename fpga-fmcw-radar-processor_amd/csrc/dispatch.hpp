// dispatch.hpp -- kernel selection tables of libfmcw.so.  Each table lives in its own
// translation unit (inst_*.hip) so the template instantiations compile in parallel; the host
// logic (fmcw_api.hip) sees only these function-pointer factories.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "kernels.hpp"

namespace fmcw {

// ---- K1: window + range FFT + corner turn -------------------------------------------------
using RangeFn = void (*)(const void*, float2*, const float*, const float*, int, int, float, uint32_t*);
// which range kernel family a handle runs (fmcw.h FMCW_INFO_RANGE_KERNEL)
// (1 was round 2's dual kernel k_range2, removed in round 4; the id stays retired)
enum RangeKind { kRangeSingle = 0, kRangeSeq = 2, kRangePx = 3 };
struct RangeInfo {
  RangeFn fn;
  int T, RB, NT;   // chirps per group, range bins per 1 KiB tile, threads per workgroup
  int kind;        // RangeKind actually selected
};
// want = the preferred family (kRangePx: k_range_px at N = 8192, kRangeSeq: k_range_sq at N = 4096,
// else k_range); window FMCW_WIN_Q15_RTL and spec (fmcw_spectrum_dtype) FMCW_SPEC_F16 run k_range;
// FMCW_SPEC_S48 runs the same family as fp32 (quad form at T >= 8, strided quads at T = 4, pair
// form at T = 2)
RangeInfo range_info(uint32_t n, int dtype, int window, int spec, int want);

// ---- K2: Doppler window + FFT + |X| / NCI + map + 1-D CFAR --------------------------------
using DopplerFn = void (*)(const float2*, const float*, int, int, int, int, int, int, int, float*,
                           float*, int, int, int, Cfar1DArgs, DetSink, uint32_t*);
struct DopplerInfo {
  DopplerFn fn;
  int WR, NT;  // range rows per wave tile, threads per workgroup (DopplerGeom::WPB tiles)
};
DopplerFn doppler_fn_f32(uint32_t nc, int mti, bool fast, bool q15);  // inst_doppler.hip
DopplerFn doppler_fn_f16(uint32_t nc, int mti, bool fast);            // inst_doppler_h16.hip
// inst_doppler_s48.hip (nullptr: unsupported); form: the S48 form K1 wrote, by its tile width T
enum S48Form { kS48Quad = 0, kS48Pair = 1, kS48Strided = 2 };
inline int s48_form(int range_T) { return range_T == 2 ? kS48Pair : range_T == 4 ? kS48Strided : kS48Quad; }
DopplerFn doppler_fn_s48(uint32_t nc, int mti, bool fast, int form);
inline DopplerInfo doppler_info(uint32_t nc, int mti = FMCW_MTI_OFF, int spec = FMCW_SPEC_F32, bool fast = false,
                                bool q15 = false, int range_T = 4) {
  DopplerFn fn = spec == FMCW_SPEC_F16   ? doppler_fn_f16(nc, mti, fast)
                 : spec == FMCW_SPEC_S48 ? doppler_fn_s48(nc, mti, fast, s48_form(range_T))
                                         : doppler_fn_f32(nc, mti, fast, q15);
  switch (nc) {
#define D_(N) case N: return {fn, DopplerGeom<N>::WR, DopplerGeom<N>::NT};
    D_(32) D_(64) D_(128) D_(256) D_(512) D_(1024)
#undef D_
  }
  return {nullptr, 0, 0};
}

// ---- stand-alone 1-D CFAR (fmcw_cfar) and K3 2-D CFAR ---------------------------------------
using Cfar1Fn = void (*)(const float*, int, int, int, int, Cfar1DArgs, DetSink);
Cfar1Fn cfar1_fn(uint32_t nc);  // inst_doppler.hip
using Cfar2Fn = void (*)(const float*, int, int, int, int, int, Cfar2DArgs, DetSink, Cfar2Cands);
using Cfar2DecideFn = void (*)(const float*, int, Cfar2DArgs, Cfar2Cands);
using Cfar2EmitFn = void (*)(const float*, int, int, Cfar2DArgs, Cfar2Cands, DetSink);
struct Cfar2Info {
  Cfar2Fn fn;           // K3a k_cfar2d_lv (reference window) / k_cfar2d (any other): screen, the candidate list
  int TR;
  Cfar2DecideFn decide; // K3b k_cfar2d_decide
  Cfar2EmitFn emit;     // K3c k_cfar2d_emit
  size_t smem;          // K3a's dynamic LDS bytes
  bool spill;           // K3a writes strip-private spill regions (Cfar2Cands pcell / ptile: k_cfar2d_lv)
};
Cfar2Info cfar2_info(uint32_t nc, int hd, int gd, int hr, int gr, bool compat);  // inst_cfar2.hip

}  // namespace fmcw
