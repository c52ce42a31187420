// launch_probe.hip -- what a dependent kernel boundary costs on one stream (round 4): K back-to-back
// launches of (a) an empty 1-workgroup kernel, (b) an empty kernel with a bench-sized grid, (c) a
// grid that writes 64 MiB with plain stores, (d) the same with non-temporal stores; each timed as a
// plain stream, with hipEventRecord between launches, and as one captured hipGraph.
// usage: tools/launch_probe [K=200]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::printf("%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__);      \
      std::exit(3);                                                                \
    }                                                                              \
  } while (0)

__global__ void k_empty(float* p) {
  if (p && threadIdx.x == 1024) p[0] = 1.f;  // never
}
template <bool NT>
__global__ void k_write(float4* p, size_t n4) {
  const float4 v = make_float4(1.f, 2.f, 3.f, (float)blockIdx.x);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    if constexpr (NT) __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v*>(p + i));
    else p[i] = v;
  }
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? std::atoi(argv[1]) : 200;
  const size_t bytes = 64u << 20, n4 = bytes / 16;
  float4* buf;
  CK(hipMalloc(&buf, bytes));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1, em;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&em));
  struct Case {
    const char* name;
    int kind, grid, nt;
  } cases[] = {{"empty_1wg", 0, 1, 64},       {"empty_512x512", 0, 512, 512}, {"empty_2048x256", 0, 2048, 256},
               {"write64M_wb", 1, 2048, 256}, {"write64M_nt", 2, 2048, 256}};
  auto launch = [&](const Case& c) {
    if (c.kind == 0) hipLaunchKernelGGL(k_empty, dim3(c.grid), dim3(c.nt), 0, s, (float*)nullptr);
    if (c.kind == 1) hipLaunchKernelGGL(k_write<false>, dim3(c.grid), dim3(c.nt), 0, s, buf, n4);
    if (c.kind == 2) hipLaunchKernelGGL(k_write<true>, dim3(c.grid), dim3(c.nt), 0, s, buf, n4);
  };
  for (const Case& c : cases) {
    for (int i = 0; i < 20; ++i) launch(c);
    CK(hipStreamSynchronize(s));
    // (1) plain stream
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < K; ++i) launch(c);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms_plain = 0.f;
    CK(hipEventElapsedTime(&ms_plain, e0, e1));
    // (2) an event marker between launches
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < K; ++i) {
      launch(c);
      CK(hipEventRecord(em, s));
    }
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms_ev = 0.f;
    CK(hipEventElapsedTime(&ms_ev, e0, e1));
    // (3) one captured graph of K launches
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < K; ++i) launch(c);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms_graph = 0.f;
    CK(hipEventElapsedTime(&ms_graph, e0, e1));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    std::printf("%-16s per launch: stream %7.2f us   +event marker %7.2f us   graph %7.2f us\n", c.name,
                1e3 * ms_plain / K, 1e3 * ms_ev / K, 1e3 * ms_graph / K);
    std::fflush(stdout);
  }
  CK(hipFree(buf));
  return 0;
}
