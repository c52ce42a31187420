// NOTE (round 5): the kernel sources no longer carry build-time switches or ablation blocks
// (csrc/*.hpp, DESIGN.md section 4 "Build-time constants").  This lab program still builds and
// times the shipped kernels; its -D variants (FMCW_K3_ABLATE, FMCW_K1_ABLATE, FMCW_K3_KEY_*, ...)
// refer to the sources at commit 72a93dd, where the measurements in profiles/r03-r04 were taken.
// k1_lab.hip -- stand-alone timing / agreement harness for the range-stage (K1) variants.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/k1_lab tools/k1_lab.hip
// Run:   tools/k1_lab <N> <n_chirps> <n_rx> <frames> <f16:0|1> [reps]
// Fills a deterministic cube on the device, runs every K1 variant instantiated for N over the
// same frames, reports each one's average launch time (HIP events), its algorithmic HBM rate
// (cube in + fp32 tiled spectrum out), and its max |diff| / max |ref| against k_range (the first
// variant; round 2's dual kernel k_range2, the former reference, left the library in round 4).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../fpga-fmcw-radar-processor_amd/csrc/kernels.hpp"

using namespace fmcw;

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__);     \
      std::exit(3);                                                                        \
    }                                                                                      \
  } while (0)

using RangeFn = void (*)(const void*, float2*, const float*, const float*, int, int, float, uint32_t*);

__device__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
// complex samples in [-1000, 1000) (fp32) or [-1, 1) (fp16 pairs)
__global__ void k_fill(uint32_t* p, size_t n_words, int f16) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_words; i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t h = hash32((uint32_t)i * 2654435761U + 12345U);
    if (f16) {
      typedef _Float16 h2 __attribute__((ext_vector_type(2)));
      const h2 v = {(_Float16)((float)(h & 0xffff) / 32768.f - 1.f), (_Float16)((float)(h >> 16) / 32768.f - 1.f)};
      p[i] = __builtin_bit_cast(uint32_t, v);
    } else {
      p[i] = __float_as_uint((float)(h >> 8) / 8388.608f - 1000.f);
    }
  }
}
__global__ void k_cmp(const float* a, const float* b, size_t n, uint32_t* out) {
  uint32_t md = 0, mr = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    md = max(md, __float_as_uint(fabsf(a[i] - b[i])));
    mr = max(mr, __float_as_uint(fabsf(a[i])));
  }
  atomicMax(out, md);
  atomicMax(out + 1, mr);
}

struct Var {
  std::string name;
  RangeFn fn;
  int nt;
};

template <int N, typename LD>
void add_vars(std::vector<Var>& v) {
  v.push_back({"k_range", k_range<N, LD>, RangeGeom<N>::NT});
  v.push_back({"sq_v16_e1", k_range_sq<N, LD, 16, 1>, N / 16});
  v.push_back({"sq_v16_e2", k_range_sq<N, LD, 16, 2>, N / 16});
  v.push_back({"sq_v16_e1_w3", k_range_sq<N, LD, 16, 1, 3>, N / 16});
  v.push_back({"sq_v16_e2_w3", k_range_sq<N, LD, 16, 2, 3>, N / 16});
  v.push_back({"sq_v32_e2", k_range_sq<N, LD, 32, 2>, N / 32});
  if constexpr (N == 8192) {
    v.push_back({"px", k_range_px<LD>, 512});
    v.push_back({"px_ws0", k_range_px<LD, 4, 0>, 512});
    v.push_back({"px_ws2", k_range_px<LD, 4, 2>, 512});
    v.push_back({"px_ws6", k_range_px<LD, 4, 6>, 512});
  }
}

int main(int argc, char** argv) {
  if (argc < 6) {
    std::fprintf(stderr, "usage: k1_lab N n_chirps n_rx frames f16 [reps]\n");
    return 2;
  }
  const int N = std::atoi(argv[1]), nc = std::atoi(argv[2]), nrx = std::atoi(argv[3]), frames = std::atoi(argv[4]);
  const int f16 = std::atoi(argv[5]);
  const int reps = argc > 6 ? std::atoi(argv[6]) : 20;
  std::vector<Var> vars;
  if (N == 8192 && f16) add_vars<8192, LoadF16>(vars);
  else if (N == 8192) add_vars<8192, LoadF32>(vars);
  else if (N == 4096 && f16) add_vars<4096, LoadF16>(vars);
  else if (N == 4096) add_vars<4096, LoadF32>(vars);
  else if (N == 2048) add_vars<2048, LoadF32>(vars);
  else {
    std::fprintf(stderr, "N %d not instantiated\n", N);
    return 2;
  }
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int n_cu = prop.multiProcessorCount;
  const size_t px = (size_t)frames * nrx * nc * N;
  const size_t b_in = f16 ? 4 : 8;
  void* cube;
  float2 *ref, *out;
  float *win, *cw;
  uint32_t* cmp;
  CK(hipMalloc(&cube, px * b_in));
  CK(hipMalloc(&ref, px * 8));
  CK(hipMalloc(&out, px * 8));
  CK(hipMalloc(&win, N * 4));
  CK(hipMalloc(&cw, nc * 4));
  CK(hipMalloc(&cmp, 8));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint32_t*)cube, px * b_in / 4, f16);
  {
    std::vector<float> w(N), c(nc);
    for (int i = 0; i < N; ++i) w[i] = (float)(0.54 - 0.46 * std::cos(2 * M_PI * i / (N - 1)));
    for (int i = 0; i < nc; ++i) c[i] = (float)(0.54 - 0.46 * std::cos(2 * M_PI * i / (nc - 1)));
    CK(hipMemcpy(win, w.data(), N * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(cw, c.data(), nc * 4, hipMemcpyHostToDevice));
  }
  const int n_groups = frames * nrx * nc / 2;
  const double bytes = (double)px * (b_in + 8);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::printf("N=%d nc=%d nrx=%d frames=%d %s: %d groups, %.1f MB per launch\n", N, nc, nrx, frames,
              f16 ? "fp16" : "fp32", n_groups, bytes / 1e6);
  for (size_t vi = 0; vi < vars.size(); ++vi) {
    const Var& v = vars[vi];
    int per_cu = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(v.fn), v.nt, 0));
    const int grid = std::min(n_groups, std::max(1, per_cu) * n_cu);
    float2* dst = vi == 0 ? ref : out;
    CK(hipMemset(dst, 0, px * 8));
    hipLaunchKernelGGL(v.fn, dim3(grid), dim3(v.nt), 0, 0, cube, dst, win, cw, nc, n_groups, 1.f, (uint32_t*)nullptr);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    double diff = 0;
    if (vi > 0) {
      CK(hipMemset(cmp, 0, 8));
      hipLaunchKernelGGL(k_cmp, dim3(2048), dim3(256), 0, 0, (const float*)ref, (const float*)out, px * 2, cmp);
      uint32_t h[2];
      CK(hipMemcpy(h, cmp, 8, hipMemcpyDeviceToHost));
      float d, r;
      std::memcpy(&d, &h[0], 4);
      std::memcpy(&r, &h[1], 4);
      diff = r > 0 ? d / r : -1;
    }
    float tot = 0;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(v.fn, dim3(grid), dim3(v.nt), 0, 0, cube, dst, win, cw, nc, n_groups, 1.f, (uint32_t*)nullptr);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0) tot += ms;
    }
    const double us = tot / (reps - 1) * 1e3;
    // the same launches timed by the dispatch's own start / end (hipExtLaunchKernelGGL events): the
    // kernel's span without the marker packets around it
    float tot_x = 0;
    for (int r = 0; r < reps; ++r) {
      hipExtLaunchKernelGGL(v.fn, dim3(grid), dim3(v.nt), 0, 0, e0, e1, 0, cube, dst, (const float*)win,
                            (const float*)cw, nc, n_groups, 1.f, (uint32_t*)nullptr);
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0) tot_x += ms;
    }
    const double us_x = tot_x / (reps - 1) * 1e3;
    std::printf("%-12s %4d thr x %2d WG/CU  %8.1f us  %6.3f TB/s  frac %.3f  (kernel span %8.1f us, frac %.3f)  rel diff %.2e\n",
                v.name.c_str(), v.nt, per_cu, us, bytes / us / 1e6, bytes / us / 1e6 / 8.0, us_x, bytes / us_x / 1e6 / 8.0, diff);
    std::fflush(stdout);
  }
  return 0;
}
