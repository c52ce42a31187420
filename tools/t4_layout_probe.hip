// t4_layout_probe.hip -- would T = 4 tiles (32 range bins x 4 chirps per 1 KiB) serve config 5
// better than the T = 2 tiles K1 writes at N = 8192?  (round-3 verdict item 3)
// Store side: K1 k_range_px's pattern -- one 512-thread workgroup per chirp pair, 16 B (the pair's
// two chirps at one range bin) per lane, 16 stores per lane of lanes' consecutive range bins --
// into the T = 2 layout (whole 1 KiB tiles per store) or the T = 4 layout (16 B of every 32-B
// element: the other half is the partner pair's, ideally written from the same XCD's L2).
// Read side: K2's pattern at NC = 1024 (one range row per wave, lane t reads chirps t + 64 m,
// 8 B each; 4 waves = 4 consecutive rows per workgroup) on either layout.
// No arithmetic: stores write the lane id, loads fold into one float.
// usage: tools/t4_layout_probe [frames=3] [reps=20]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int NS = 8192, NC = 1024;

__device__ __forceinline__ int xcd_id(int b, int g) { return (g & 7) ? b : (b % 8) * (g / 8) + b / 8; }

// element (r, c) in float2 units: T = 2: ((r / 64 * NC/2 + c / 2) * 64 + r % 64) * 2 + c % 2
//                                 T = 4: ((r / 32 * NC/4 + c / 4) * 32 + r % 32) * 4 + c % 4
template <int T>
__device__ __forceinline__ size_t off_of(int r, int c) {
  constexpr int RB = 128 / T;
  return ((size_t)((r / RB) * (NC / T) + c / T) * RB + (r % RB)) * T + (c % T);
}

// K1 store pattern: group g = (frame, pair); lane (l, w) stores range bins
// d = 64 ((w >> 1) + 4 m + 64 s) + (l & 31) + 32 (w & 1), m < 8, s < 2 (k_range_px's order)
// X = 1: logical group ids XCD-contiguous, so pairs 2j, 2j + 1 (the halves of T = 4 elements)
// run behind the same L2
template <int T, int X>
__global__ void __launch_bounds__(512) k1_store(float2* __restrict__ s, int groups) {
  const int g = X ? xcd_id(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  if (g >= groups) return;
  const int fr = g / (NC / 2), cp = g % (NC / 2);
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  float2* p = s + (size_t)fr * NS * NC;
  const float4 v = make_float4((float)l, (float)w, (float)g, 1.f);
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int d = 64 * ((w >> 1) + 4 * m + 64 * q) + (l & 31) + 32 * (w & 1);
      *reinterpret_cast<float4*>(p + off_of<T>(d, 2 * cp)) = v;
    }
}

// K2 read pattern: row = 4 b + wave; X = 1: XCD-contiguous ids (K2 uses them at T = 2)
template <int T, int X>
__global__ void __launch_bounds__(256) k2_read(const float2* __restrict__ s, int rows, float* __restrict__ sink) {
  const int b = X ? xcd_id(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
  const int row = b * 4 + w;
  if (row >= rows) return;
  const int f = row / NS, r = row % NS;
  const float2* p = s + (size_t)f * NS * NC;
  float acc = 0.f;
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const float2 v = p[off_of<T>(r, t + 64 * m)];
    acc += v.x + v.y;
  }
  sink[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main(int argc, char** argv) {
  const int frames = argc > 1 ? atoi(argv[1]) : 3;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const size_t bytes = (size_t)frames * NS * NC * sizeof(float2);
  const int rows = frames * NS, groups = frames * NC / 2;
  float2* s;
  float* sink;
  CHECK(hipMalloc(&s, bytes));
  CHECK(hipMemset(s, 0, bytes));
  CHECK(hipMalloc(&sink, (size_t)rows * 64 * sizeof(float)));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1e3 * ms / reps;
    printf("%-14s %8.1f us per pass over %zu MiB  = %6.0f GB/s\n", name, us, bytes >> 20, bytes / us * 1e-3);
  };
  const int gr = rows / 4;
  run("store_t2", [&] { hipLaunchKernelGGL((k1_store<2, 0>), dim3(groups), dim3(512), 0, 0, s, groups); });
  run("store_t4", [&] { hipLaunchKernelGGL((k1_store<4, 0>), dim3(groups), dim3(512), 0, 0, s, groups); });
  run("store_t4_xcd", [&] { hipLaunchKernelGGL((k1_store<4, 1>), dim3(groups), dim3(512), 0, 0, s, groups); });
  run("read_t2_xcd", [&] { hipLaunchKernelGGL((k2_read<2, 1>), dim3(gr), dim3(256), 0, 0, s, rows, sink); });
  run("read_t4", [&] { hipLaunchKernelGGL((k2_read<4, 0>), dim3(gr), dim3(256), 0, 0, s, rows, sink); });
  run("read_t4_xcd", [&] { hipLaunchKernelGGL((k2_read<4, 1>), dim3(gr), dim3(256), 0, 0, s, rows, sink); });
  CHECK(hipGetLastError());
  CHECK(hipFree(s));
  CHECK(hipFree(sink));
  return 0;
}
