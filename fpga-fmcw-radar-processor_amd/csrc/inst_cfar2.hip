// inst_cfar2.hip -- K3 (2-D OS-CFAR) instantiations, see dispatch.hpp.
#include "dispatch.hpp"

namespace fmcw {

// The reference window (range half extent 5, guard 1; Doppler half extent 6, guard 2: os_cfar_2d
// as instantiated at radar_core.vhd:376-382) gets a level screen; any other geometry the generic
// kernel (runtime window, pair screen, candidate test).  Of the two level-screen kernels, k_cfar2d
// (key16 rows + in-launch candidate test) runs where its ring fits 4 workgroups per CU (<= 40 KB of
// LDS: NC <= 512), k_cfar2d_lv (scale rules, 2.5 B per cell, no candidate test) where it does not
// (NC = 1024: 46.7 KB, 3 workgroups per CU; k_cfar2d_lv 40.7 KB, 4).  Measured (tools/cfar2d_bench.py, 16 frames, us per
// launch, profiles/r05/k3_rules/): config 5 k_cfar2d 350, k_cfar2d_lv 297-302; config 3 k_cfar2d
// 73, k_cfar2d_lv 95-100 (its 4-rx NCI cells pass the s_min screen rarely: the rules' extra screen
// work buys nothing there).
static bool lv_window(int hd, int gd, int hr, int gr) { return hd == 6 && gd == 2 && hr == 5 && gr == 1; }
template <int N>
constexpr bool rules_kernel() { return cfar2d_smem_bytes<N>(5) > 40 * 1024; }

template <int N>
static Cfar2Info info_t(bool lv, int hr, bool compat) {
  Cfar2Fn fn = k_cfar2d<N, 0, 0>;
  size_t smem = cfar2d_smem_bytes<N>(hr);
  bool spill = false;
  if (lv) {
    if constexpr (rules_kernel<N>()) {
      static_assert(N == 1024, "k_cfar2d_lv stages one 4-cell column per thread (NC = 1024)");
      fn = compat ? k_cfar2d_lv<N, 5, 1, true> : k_cfar2d_lv<N, 5, 1, false>;
      smem = cfar2d_lv_smem_bytes<N, 5, 1>();
      spill = true;
    } else {
      fn = k_cfar2d<N, 6, 2, 5, 1>;
      smem = cfar2d_smem_bytes<N>(5);
    }
  }
  return {fn, Cfar2DGeom<N>::TR, k_cfar2d_decide<N>, k_cfar2d_emit<N>, smem, spill};
}

Cfar2Info cfar2_info(uint32_t nc, int hd, int gd, int hr, int gr, bool compat) {
  const bool lv = lv_window(hd, gd, hr, gr);
  switch (nc) {
#define C_(N) case N: return info_t<N>(lv, hr, compat);
    C_(32) C_(64) C_(128) C_(256) C_(512) C_(1024)
#undef C_
  }
  return {nullptr, 0, nullptr, nullptr, 0, false};
}

}  // namespace fmcw
