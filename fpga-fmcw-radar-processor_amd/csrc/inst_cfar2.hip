// inst_cfar2.hip -- K3 (2-D OS-CFAR) instantiations, see dispatch.hpp.
#include "dispatch.hpp"

namespace fmcw {

// the reference window (range half extent 5, guard 1; Doppler half extent 6, guard 2: os_cfar_2d
// as instantiated at radar_core.vhd:376-382) gets the compile-time level screen; any other
// geometry the generic kernel (runtime window, pair screen)
template <int N>
static Cfar2Fn cfar2_fn(int hd, int gd, int hr, int gr) {
  return (hd == 6 && gd == 2 && hr == 5 && gr == 1) ? k_cfar2d<N, 6, 2, 5, 1> : k_cfar2d<N, 0, 0>;
}

Cfar2Info cfar2_info(uint32_t nc, int hd, int gd, int hr, int gr) {
  switch (nc) {
#define C_(N) case N: return {cfar2_fn<N>(hd, gd, hr, gr), Cfar2DGeom<N>::TR, k_cfar2d_decide<N>, k_cfar2d_emit<N>};
    C_(32) C_(64) C_(128) C_(256) C_(512) C_(1024)
#undef C_
  }
  return {nullptr, 0};
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

}  // namespace fmcw
