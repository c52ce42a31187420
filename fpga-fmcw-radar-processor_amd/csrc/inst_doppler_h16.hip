// inst_doppler_h16.hip -- K2 instantiations on the fp16 corner-turned spectrum
// (FMCW_SPEC_F16), see dispatch.hpp.
#include "dispatch.hpp"

namespace fmcw {
namespace {
template <int N>
DopplerFn dfn(int mti, bool fast) {
  return mti == FMCW_MTI_2PULSE   ? k_doppler<N, 2, SP_F16>
         : mti == FMCW_MTI_3PULSE ? k_doppler<N, 3, SP_F16>
         : fast                   ? k_doppler<N, 0, SP_F16, true>
                                  : k_doppler<N, 0, SP_F16>;
}
}  // namespace

DopplerFn doppler_fn_f16(uint32_t nc, int mti, bool fast) {
  switch (nc) {
#define D_(N) case N: return dfn<N>(mti, fast);
    D_(32) D_(64) D_(128) D_(256) D_(512) D_(1024)
#undef D_
  }
  return nullptr;
}

}  // namespace fmcw
