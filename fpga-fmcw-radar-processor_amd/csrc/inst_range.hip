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
  if constexpr (RangeGeom<N>::T >= 4) {  // S48 shares its exponent over 4 chirps of a tile row
    if (spec == FMCW_SPEC_S48) return q15 ? nullptr : range_fn_t<N, SP_S48>(dtype, false);
  }
  return spec == FMCW_SPEC_F16 ? range_fn_t<N, SP_F16>(dtype, q15) : spec == FMCW_SPEC_F32 ? range_fn_t<N, SP_F32>(dtype, q15)
                                                                                          : nullptr;
}

// k_range_sq (sequential pair, round 3): N = 4096, the measured-fastest values per thread V,
// samples per load E and waves per SIMD W (tools/k1_lab.hip; at N = 8192 k_range_px is faster)
template <int N> struct SqPick;
template <> struct SqPick<4096> { static constexpr int V = 16, E = 1, W = 3; };
template <int N>
RangeInfo range_sq(int dtype) {
  using S = SqPick<N>;
  constexpr int NT = N / S::V;
  RangeFn fn = nullptr;
  switch (dtype) {
    case FMCW_IN_F32: fn = k_range_sq<N, LoadF32, S::V, S::E, S::W>; break;
    case FMCW_IN_F16: fn = k_range_sq<N, LoadF16, S::V, S::E, S::W>; break;
    case FMCW_IN_I16: fn = k_range_sq<N, LoadI16, S::V, S::E, S::W>; break;
  }
  return {fn, SqGeom<N, S::V>::T, SqGeom<N, S::V>::RB, NT, kRangeSeq};
}

// k_range_px (round 3): N = 8192, two LDS exchanges + a permlane radix-2 (kernels.hpp)
RangeInfo range_px(int dtype) {
  RangeFn fn = nullptr;
  switch (dtype) {
    case FMCW_IN_F32: fn = k_range_px<LoadF32>; break;
    case FMCW_IN_F16: fn = k_range_px<LoadF16>; break;
    case FMCW_IN_I16: fn = k_range_px<LoadI16>; break;
  }
  return {fn, 2, 64, 512, kRangePx};
}

}  // namespace

RangeInfo range_info(uint32_t n, int dtype, int window, int spec, int want) {
  const bool q15 = window == FMCW_WIN_Q15_RTL;
  // the pair kernels: fp32 window, fp32 spectrum (the Q15 / fp16 / S48-spectrum paths run k_range)
  if (!q15 && spec == FMCW_SPEC_F32) {
    if (want >= kRangePx && n == 8192) return range_px(dtype);
    if (want >= kRangeSeq && n == 4096) return range_sq<4096>(dtype);
  }
  switch (n) {
#define R_(N) case N: return {range_fn<N>(dtype, q15, spec), RangeGeom<N>::T, RangeGeom<N>::RB, RangeGeom<N>::NT, kRangeSingle};
    R_(64) R_(128) R_(256) R_(512) R_(1024) R_(2048) R_(4096) R_(8192)
#undef R_
  }
  return {nullptr, 0, 0, 0, kRangeSingle};
}

}  // namespace fmcw
