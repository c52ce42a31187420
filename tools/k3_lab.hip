// NOTE (round 5): the kernel sources no longer carry build-time switches or ablation blocks
// (csrc/*.hpp, DESIGN.md section 4 "Build-time constants").  This lab program still builds and
// times the shipped kernels; its -D variants (FMCW_K3_ABLATE, FMCW_K1_ABLATE, FMCW_K3_KEY_*, ...)
// refer to the sources at commit 72a93dd, where the measurements in profiles/r03-r04 were taken.
// k3_lab.hip -- stand-alone timing / exactness harness for the 2-D OS-CFAR (K3) variants at
// BASELINE config 5's map geometry (8192 range x 1024 Doppler, 2-D CFAR with the reference
// window of rtl/src/os_cfar_2d.vhd as instantiated at radar_core.vhd:376-382).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/k3_lab tools/k3_lab.hip
// Run:   tools/k3_lab [frames=16] [reps=5] [ns=8192] [nc=1024] [nrx=1] [steps=0 (cost model)] [wg_per_cu=0 (occupancy)]   (nc 1024 / 512 / 256; nrx > 1:
//        the cells are the non-coherent sum over nrx complex-Gaussian channels, as config 3's NCI map)
// Synthetic map: Rayleigh noise (|complex Gaussian|) plus point targets with Hamming-like
// sidelobes; every variant's detection list (per tile: count + records) must equal the
// production kernel's, and each variant's average launch time is reported.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <functional>

#include "../fpga-fmcw-radar-processor_amd/csrc/kernels.hpp"
#ifdef K3_LAB_PREV  // the previous K3 (tools/cfar2d_prev.hpp, e.g. git show HEAD~:.../cfar2d.hpp) for A/B
namespace fmcw {
namespace prev {
#include "cfar2d_prev.hpp"
}
}  // namespace fmcw
#endif

using namespace fmcw;

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__);     \
      std::exit(3);                                                                        \
    }                                                                                      \
  } while (0)

__device__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
// Rayleigh magnitude (sigma 1000; nrx > 1: sqrt of the sum of nrx squared Rayleigh cells, the NCI
// map) + targets: every 512th range row has a target at Doppler (row * 37) % nc of amplitude 1e6
// with a 3 x 5 neighbourhood at 1e4
__global__ void k_fill_map(float* m, int ns, int nc, int nrx, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float p = 0.f;
    for (int x = 0; x < nrx; ++x) {
      const uint32_t h1 = hash32((uint32_t)i * 8u + 2u * x + 1u);
      const float u1 = ((float)(h1 >> 8) + 0.5f) / 16777216.f;
      p += -2.f * logf(u1);  // |N(0,1) + i N(0,1)|^2
    }
    float v = 1000.f * sqrtf(p);
    const int d = (int)(i % nc);
    const size_t rr = i / nc;
    const int r = (int)(rr % ns);
    const int rt = (r + 2) / 512 * 512;  // nearest target row
    const int dt = (rt * 37) % nc;
    const int dr = r - rt, dd = ((d - dt + nc + nc / 2) % nc) - nc / 2;
    if (rt > 0 && rt < ns && abs(dr) <= 1 && abs(dd) <= 2) v = (dr == 0 && dd == 0) ? 1e6f : 1e4f;
    m[i] = v;
  }
}

struct Var {
  std::string name;
  const void* fn;
  size_t smem;
  std::function<void(int grid, size_t smem, int n_strips, int steps, DetSink sink, Cfar2Cands cands)> launch;
};

int steps_model(int nf, int tpf, int grid, int tr, int hr) {  // = fmcw_api.hip cfar2_steps_model
  int best = 1;
  double best_cost = 1e300;
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

static int g_steps = 0;   // strip length (argv[6]; 0 = the library's cost model)
static int g_per_cu = 0;  // workgroups per CU at most (argv[7]; 0 = occupancy)

template <int NC>
int run(int nf, int reps, int ns, int nrx) {
  const float* map = nullptr;
  Cfar2DArgs a{};
  // the reference core's 2-D CFAR parameters (fmcw_api.hip cfar2_args with the defaults)
  a.gr = 1;
  a.gd = 2;
  a.hr = 5;
  a.hd = 6;
  a.n_ref = 11 * 13 - 3 * 5;
  a.rank = a.n_ref * 75 / 100;
  a.sc_min = 2.f;
  a.sc_nom = 4.f;
  a.sc_max = 6.f;
  a.override_ = 0;
  a.compat = 0;
  a.s_min = 2.f;
  std::vector<Var> vars;
  vars.push_back({"k_cfar2d + decide + emit (production)", reinterpret_cast<const void*>(k_cfar2d<NC, 6, 2, 5, 1>),
                  cfar2d_smem_bytes<NC>(a.hr), [&](int grid, size_t smem, int n_strips, int steps, DetSink sink,
                                                   Cfar2Cands cands) {
                    hipMemsetAsync(cands.ctr, 0, 16, 0);
                    hipLaunchKernelGGL((k_cfar2d<NC, 6, 2, 5, 1>), dim3(grid), dim3(256), smem, 0, map, ns, n_strips,
                                       steps, 0, 0, a, sink, cands);
                    hipLaunchKernelGGL(k_cfar2d_decide<NC>, dim3(1024), dim3(256), 0, 0, map, ns, a, cands);
                    hipLaunchKernelGGL(k_cfar2d_emit<NC>, dim3(256), dim3(256), 0, 0, map, ns, 0, a, cands, sink);
                  }});
#ifdef K3_LAB_PREV  // the previous three-launch K3 (same arguments, its own types)
  vars.push_back({"k_cfar2d + decide + emit (previous)", reinterpret_cast<const void*>(prev::k_cfar2d<NC, 6, 2, 5, 1>),
                  prev::cfar2d_smem_bytes<NC>(a.hr), [&](int grid, size_t smem, int n_strips, int steps, DetSink sink,
                                                         Cfar2Cands cands) {
                    prev::Cfar2DArgs pa;
                    static_assert(sizeof(pa) == sizeof(a), "same argument layout");
                    std::memcpy(&pa, &a, sizeof(a));
                    prev::Cfar2Cands pc;
                    static_assert(sizeof(pc) == sizeof(cands), "same candidate-list layout");
                    std::memcpy(&pc, &cands, sizeof(cands));
                    hipMemsetAsync(cands.ctr, 0, 8, 0);
                    hipLaunchKernelGGL((prev::k_cfar2d<NC, 6, 2, 5, 1>), dim3(grid), dim3(256), smem, 0, map, ns,
                                       n_strips, steps, 0, 0, pa, sink, pc);
                    hipLaunchKernelGGL(prev::k_cfar2d_decide<NC>, dim3(1024), dim3(256), 0, 0, map, ns, pa, pc);
                    hipLaunchKernelGGL(prev::k_cfar2d_emit<NC>, dim3(256), dim3(256), 0, 0, map, ns, 0, pa, pc, sink);
                  }});
#endif
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int n_cu = prop.multiProcessorCount;
  const size_t cells = (size_t)nf * ns * NC;
  {
    float* m;
    CK(hipMalloc(&m, cells * 4));
    hipLaunchKernelGGL(k_fill_map, dim3(8192), dim3(256), 0, 0, m, ns, NC, nrx, cells);
    map = m;
  }
  const int WR = DopplerGeom<NC>::WR;
  const int tiles = nf * ns / WR;
  const uint32_t slot_cap = 32;
  const uint32_t ovf = (uint32_t)std::max<size_t>(cells / 64, 65536);
  const uint32_t cap = (uint32_t)tiles * slot_cap + ovf;
  DetSink sink{};
  CK(hipMalloc(&sink.scratch, (size_t)cap * sizeof(fmcw_det)));
  CK(hipMalloc(&sink.counter, 16));
  CK(hipMalloc(&sink.wg_base, tiles * 4));
  CK(hipMalloc(&sink.wg_count, tiles * 4));
  sink.cap = cap;
  sink.slot_cap = slot_cap;
  sink.ovf_base = (uint32_t)tiles * slot_cap;
  Cfar2Cands cands{};
  CK(hipMalloc(&cands.cell, cells * 4));
  CK(hipMalloc(&cands.thr, cells * 4));
  CK(hipMalloc(&cands.tiles, (size_t)tiles * 4));
  CK(hipMalloc(&cands.ctr, 16));
  std::vector<uint32_t> ref_cnt, ref_base;
  std::vector<fmcw_det> ref_sc;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::printf("map %d frames x %d x %d, %d rx\n", nf, ns, NC, nrx);
  for (size_t vi = 0; vi < vars.size(); ++vi) {
    const Var& v = vars[vi];
    const size_t smem = v.smem;
    CK(hipFuncSetAttribute(v.fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
    int per_cu = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, v.fn, 256, smem));
    if (g_per_cu > 0) per_cu = std::min(per_cu, g_per_cu);
    const int grid_max = std::max(1, per_cu) * n_cu;
    const int tpf = (ns / WR + 3) / 4;
    const int steps = g_steps > 0 ? std::min(g_steps, tpf) : steps_model(nf, tpf, grid_max, WR * 4, a.hr);
    const int n_strips = nf * ((tpf + steps - 1) / steps);
    const int grid = std::min(n_strips, grid_max);
    CK(hipMemset(sink.counter, 0, 16));
    CK(hipMemset(sink.wg_count, 0, tiles * 4));
    v.launch(grid, smem, n_strips, steps, sink, cands);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> cnt(tiles), base(tiles), ctr(4);
    std::vector<fmcw_det> sc(cap);
    CK(hipMemcpy(cnt.data(), sink.wg_count, tiles * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(base.data(), sink.wg_base, tiles * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(sc.data(), sink.scratch, (size_t)cap * sizeof(fmcw_det), hipMemcpyDeviceToHost));
    CK(hipMemcpy(ctr.data(), sink.counter, 16, hipMemcpyDeviceToHost));
    size_t ndet = 0;
    for (int t = 0; t < tiles; ++t) ndet += cnt[t];
    bool same = true;
    if (vi == 0) {
      ref_cnt = cnt;
      ref_base = base;
      ref_sc = sc;
    } else {
      for (int t = 0; t < tiles && same; ++t) {
        if (cnt[t] != ref_cnt[t]) {
          std::printf("  tile %d: %u detections vs %u\n", t, cnt[t], ref_cnt[t]);
          same = false;
          break;
        }
        for (uint32_t k = 0; k < cnt[t]; ++k)
          if (std::memcmp(&sc[base[t] + k], &ref_sc[ref_base[t] + k], sizeof(fmcw_det)) != 0) {
            std::printf("  tile %d record %u differs\n", t, k);
            same = false;
            break;
          }
      }
    }
    float tot = 0;
    for (int r = 0; r < reps; ++r) {
      CK(hipMemset(sink.counter, 0, 16));
      CK(hipEventRecord(e0, 0));
      v.launch(grid, smem, n_strips, steps, sink, cands);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      tot += ms;
    }
    std::printf("%-34s smem %6zu grid %5d (%d/CU) steps %2d  %8.1f us per launch (%.1f us/frame)  dets %zu dropped %u  %s  [survivors %u candidates %u]\n",
                v.name.c_str(), smem, grid, per_cu, steps, tot / reps * 1e3, tot / reps * 1e3 / nf, ndet, ctr[1],
                vi == 0 ? "(reference)" : same ? "IDENTICAL" : "DIFFERENT", ctr[2], ctr[3]);
    std::fflush(stdout);
  }
  return 0;
}

int main(int argc, char** argv) {
  const int nf = argc > 1 ? std::atoi(argv[1]) : 16;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
  const int ns = argc > 3 ? std::atoi(argv[3]) : 8192;
  const int nc = argc > 4 ? std::atoi(argv[4]) : 1024;
  const int nrx = argc > 5 ? std::atoi(argv[5]) : 1;
  g_steps = argc > 6 ? std::atoi(argv[6]) : 0;
  g_per_cu = argc > 7 ? std::atoi(argv[7]) : 0;
  switch (nc) {
    case 1024: return run<1024>(nf, reps, ns, nrx);
    case 512: return run<512>(nf, reps, ns, nrx);
    case 256: return run<256>(nf, reps, ns, nrx);
  }
  std::fprintf(stderr, "nc %d not instantiated\n", nc);
  return 2;
}
