// inst_range.hip -- K1 instantiations (window + range FFT + corner turn), see dispatch.hpp.
#include "dispatch.hpp"

namespace fmcw {
namespace {

template <int N, int SP>
RangeFn range_fn_t(int dtype, bool q15) {
  switch (dtype) {
    case FMCW_IN_F32: return k_range<N, LoadF32, false, SP>;
    case FMCW_IN_F16: return k_range<N, LoadF16, false, SP>;
    case FMCW_IN_I16: return q15 ? k_range<N, LoadI16, true, SP> : k_range<N, LoadI16, false, SP>;
  }
  return nullptr;
}
template <int N>
RangeFn range_fn(int dtype, bool q15, int spec) {
  // S48: the strided-quad form at T = 4 (N = 1024), else quad (T >= 8) / pair (N = 2048); above
  // N = 2048 the pair kernels (range_sq / range_px)
  if constexpr (RangeGeom<N>::T == 4) {
    if (spec == FMCW_SPEC_S48) return q15 ? nullptr : range_fn_t<N, SP_S48S>(dtype, false);
  } else if constexpr (RangeGeom<N>::T == 2 && N <= 2048) {
    if (spec == FMCW_SPEC_S48) return q15 ? nullptr : range_fn_t<N, SP_S48PS>(dtype, false);
  } else if constexpr (N <= 2048) {
    if (spec == FMCW_SPEC_S48) return q15 ? nullptr : range_fn_t<N, SP_S48>(dtype, false);
  }
  return spec == FMCW_SPEC_F16 ? range_fn_t<N, SP_F16>(dtype, q15) : spec == FMCW_SPEC_F32 ? range_fn_t<N, SP_F32>(dtype, q15)
                                                                                          : nullptr;
}

// k_range_sq (sequential pair, round 3): N = 4096, the measured-fastest values per thread V,
// samples per load E and waves per SIMD W (tools/k1_lab.hip; at N = 8192 k_range_px is faster)
template <int N> struct SqPick;
template <> struct SqPick<4096> { static constexpr int V = 16, E = 1, W = 3; };
template <int N, int SP>
RangeFn range_sq_t(int dtype) {
  using S = SqPick<N>;
  switch (dtype) {
    case FMCW_IN_F32: return k_range_sq<N, LoadF32, S::V, S::E, S::W, SP>;
    case FMCW_IN_F16: return k_range_sq<N, LoadF16, S::V, S::E, S::W, SP>;
    case FMCW_IN_I16: return k_range_sq<N, LoadI16, S::V, S::E, S::W, SP>;
  }
  return nullptr;
}
template <int N>
RangeInfo range_sq(int dtype, int spec) {
  using S = SqPick<N>;
  constexpr int NT = N / S::V;
  RangeFn fn = spec == FMCW_SPEC_S48 ? range_sq_t<N, SP_S48PS>(dtype) : range_sq_t<N, SP_F32>(dtype);
  return {fn, SqGeom<N, S::V>::T, SqGeom<N, S::V>::RB, NT, kRangeSeq};
}

// k_range_px (round 3): N = 8192, two LDS exchanges + a permlane radix-2 (kernels.hpp).  The S48
// instantiation keeps 6 of its 16 range-window values in LDS (fp32: 4): with 4 the S48 packing
// spills 12 B per lane at 128 VGPRs, with 6 none (fp16 / int16 input)
template <int SP>
RangeFn range_px_t(int dtype) {
  switch (dtype) {
    case FMCW_IN_F32: return k_range_px<LoadF32, 4, SP == SP_S48PS ? 6 : 4, SP>;
    case FMCW_IN_F16: return k_range_px<LoadF16, 4, SP == SP_S48PS ? 6 : 4, SP>;
    case FMCW_IN_I16: return k_range_px<LoadI16, 4, SP == SP_S48PS ? 6 : 4, SP>;
  }
  return nullptr;
}
RangeInfo range_px(int dtype, int spec) {
  return {spec == FMCW_SPEC_S48 ? range_px_t<SP_S48PS>(dtype) : range_px_t<SP_F32>(dtype), 2, 64, 512, kRangePx};
}

}  // namespace

RangeInfo range_info(uint32_t n, int dtype, int window, int spec, int want) {
  const bool q15 = window == FMCW_WIN_Q15_RTL;
  // the pair kernels: fp32 window, fp32 or S48 spectrum (the Q15 / fp16-spectrum paths run k_range)
  if (!q15 && (spec == FMCW_SPEC_F32 || spec == FMCW_SPEC_S48)) {
    if (want >= kRangePx && n == 8192) return range_px(dtype, spec);
    if (want >= kRangeSeq && n == 4096) return range_sq<4096>(dtype, spec);
  }
  switch (n) {
#define R_(N) case N: return {range_fn<N>(dtype, q15, spec), RangeGeom<N>::T, RangeGeom<N>::RB, RangeGeom<N>::NT, kRangeSingle};
    R_(64) R_(128) R_(256) R_(512) R_(1024) R_(2048) R_(4096) R_(8192)
#undef R_
  }
  return {nullptr, 0, 0, 0, kRangeSingle};
}

}  // namespace fmcw
