// inst_doppler.hip -- K2 instantiations on the fp32 spectrum, and the stand-alone 1-D CFAR
// (see dispatch.hpp).
#include "dispatch.hpp"

namespace fmcw {
namespace {
template <int N>
DopplerFn dfn(int mti, bool fast) {
  return mti == FMCW_MTI_2PULSE   ? k_doppler<N, 2, SP_F32>
         : mti == FMCW_MTI_3PULSE ? k_doppler<N, 3, SP_F32>
         : fast                   ? k_doppler<N, 0, SP_F32, true>
                                  : k_doppler<N, 0, SP_F32>;
}
}  // namespace

DopplerFn doppler_fn_f32(uint32_t nc, int mti, bool fast, bool /* q15: runtime flag of the generic kernel */) {
  switch (nc) {
#define D_(N) case N: return dfn<N>(mti, fast);
    D_(32) D_(64) D_(128) D_(256) D_(512) D_(1024)
#undef D_
  }
  return nullptr;
}

Cfar1Fn cfar1_fn(uint32_t nc) {
  switch (nc) {
#define C_(N) case N: return k_cfar1d<N>;
    C_(32) C_(64) C_(128) C_(256) C_(512) C_(1024)
#undef C_
  }
  return nullptr;
}

}  // namespace fmcw
