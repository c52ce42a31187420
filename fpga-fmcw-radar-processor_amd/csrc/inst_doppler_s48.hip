// inst_doppler_s48.hip -- K2 instantiations on the S48 corner-turned spectrum (FMCW_SPEC_S48,
// kernels.hpp s48_pack / s48_unpack), quad (T >= 8), strided-quad (T = 4) or pair (T = 2) form,
// see dispatch.hpp.
// MTI off only (its neighbours in slow time belong to other lanes of the exponent group);
// n_doppler >= 64.
#include "dispatch.hpp"

namespace fmcw {
namespace {
template <int N, int SP>
DopplerFn dfn_t(int mti, bool fast) {
  if constexpr (N >= 64) {
    if (mti == FMCW_MTI_OFF) return fast ? k_doppler<N, 0, SP, true> : k_doppler<N, 0, SP>;
  }
  return nullptr;
}
template <int N>
DopplerFn dfn(int mti, bool fast, int form) {
  return form == kS48Pair ? dfn_t<N, SP_S48PS>(mti, fast) : form == kS48Strided ? dfn_t<N, SP_S48S>(mti, fast)
                                                                                : dfn_t<N, SP_S48>(mti, fast);
}
}  // namespace

DopplerFn doppler_fn_s48(uint32_t nc, int mti, bool fast, int form) {
  switch (nc) {
#define D_(N) case N: return dfn<N>(mti, fast, form);
    D_(32) D_(64) D_(128) D_(256) D_(512) D_(1024)
#undef D_
  }
  return nullptr;
}
}  // namespace fmcw
