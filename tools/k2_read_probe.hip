// k2_read_probe.hip -- how fast can the tiled corner-turned spectrum be READ in K2's order at
// config 5 (N = 8192 range rows, NC = 1024 chirps, T = 2 chirps x RB = 64 rows per 1 KiB tile),
// with no FFT work at all?  Decides whether K2's ~0.59 of HBM at config 5 is its access pattern
// or its compute.  Loads only; each thread folds what it loaded into one float.
//
//   k2_rows8   K2's pattern: one range row per wave, lane t loads chirps t + 64 m (m < 16), 8 B
//              each; the 4 waves of a workgroup take 4 consecutive rows; XCD-contiguous ids
//   rows8_w*   k2_rows8 with 8 / 2 waves (rows) per workgroup, and without the XCD remap
//   k2_rows16  16-B loads: lane t loads both chirps of tile (t & 31) + 32 m (m < 16) of row
//              2 * wave + (t >> 5), i.e. 2 rows per wave, 16 loads per lane
//   pairs32    2 rows per wave, lanes 2k / 2k + 1 load rows r / r + 1 of one tile: 32 contiguous
//              bytes per tile and instruction (a K2 that would hold chirp pairs per lane)
//   linear16   the same bytes front to back, 16 B per lane (the streaming ceiling)
//   s48_*      the S48 pair form (6-B points, 12-B chirp-pair elements, 768-B tiles), K2's rows8
//              order over as many frames as fill the same bytes (4 for 3 fp32 frames):
//              s48_x2 = 8 B per lane from the point's record rounded down to 4 (the quad form's
//              load), s48_x3 = the pair's whole 12 B per lane, s48_2x1 = two aligned dword loads
//              per lane, s48_x3w8 = s48_x3 with 8 waves (rows) per workgroup
// usage: tools/k2_read_probe [frames=3] [reps=20]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int NS = 8192, NC = 1024, T = 2, RB = 64, NCB = NC / T;

__device__ __forceinline__ int xcd_id(int b, int g) { return (b % 8) * (g / 8) + b / 8; }

// element (r, c) of one frame: ((r / RB * NCB + c / T) * RB + r % RB) * T + c % T  (float2 units)
__device__ __forceinline__ size_t off_of(int r, int c) {
  return ((size_t)((r / RB) * NCB + c / T) * RB + (r % RB)) * T + (c % T);
}

__global__ void __launch_bounds__(256) k2_rows8(const float2* __restrict__ s, int rows, float* __restrict__ sink) {
  const int b = xcd_id(blockIdx.x, gridDim.x);
  const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
  const int row = b * 4 + w;  // global row over all frames
  if (row >= rows) return;
  const int f = row / NS, r = row % NS;
  const float2* p = s + (size_t)f * NS * NC;
  float acc = 0.f;
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const float2 v = p[off_of(r, t + 64 * m)];
    acc += v.x + v.y;
  }
  sink[blockIdx.x * 256 + threadIdx.x] = acc;
}

// as k2_rows8 with W waves per workgroup (W consecutive rows: W = 8 reads whole 128-B lines of
// each tile) and the XCD-contiguous id remap on (X = 1) or off
template <int W, int X>
__global__ void __launch_bounds__(64 * W) k2_rows8w(const float2* __restrict__ s, int rows, float* __restrict__ sink) {
  const int b = X ? xcd_id(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
  const int row = b * W + w;
  if (row >= rows) return;
  const int f = row / NS, r = row % NS;
  const float2* p = s + (size_t)f * NS * NC;
  float acc = 0.f;
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const float2 v = p[off_of(r, t + 64 * m)];
    acc += v.x + v.y;
  }
  sink[blockIdx.x * 64 * W + threadIdx.x] = acc;
}

__global__ void __launch_bounds__(256) k2_rows16(const float4* __restrict__ s, int rows, float* __restrict__ sink) {
  const int b = xcd_id(blockIdx.x, gridDim.x);
  const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
  const int row = b * 8 + 2 * w + (t >> 5);  // 8 rows per workgroup, 2 per wave
  if (row >= rows) return;
  const int f = row / NS, r = row % NS;
  const float2* p = reinterpret_cast<const float2*>(s) + (size_t)f * NS * NC;
  float acc = 0.f;
#pragma unroll
  for (int m = 0; m < 16; ++m) {  // tiles (t & 31) + 32 m: both chirps of the tile row, 16 B
    const int c = 2 * ((t & 31) + 32 * m);
    const float4 v = *reinterpret_cast<const float4*>(p + off_of(r, c));
    acc += v.x + v.y + v.z + v.w;
  }
  sink[blockIdx.x * 256 + threadIdx.x] = acc;
}

// two rows per wave with 32 contiguous bytes per tile and instruction: lanes 2k and 2k + 1 load
// rows r and r + 1 (adjacent in the tile) of tile k + 32 m, both chirps (16 B) each
__global__ void __launch_bounds__(256) k2_pairs32(const float4* __restrict__ s, int rows, float* __restrict__ sink) {
  const int b = xcd_id(blockIdx.x, gridDim.x);
  const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
  const int row = b * 8 + 2 * w + (t & 1);
  if (row >= rows) return;
  const int f = row / NS, r = row % NS;
  const float2* p = reinterpret_cast<const float2*>(s) + (size_t)f * NS * NC;
  float acc = 0.f;
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const int c = 2 * ((t >> 1) + 32 * m);
    const float4 v = *reinterpret_cast<const float4*>(p + off_of(r, c));
    acc += v.x + v.y + v.z + v.w;
  }
  sink[blockIdx.x * 256 + threadIdx.x] = acc;
}

// S48 pair form: element (r, c) of one frame at byte 6 * off_of(r, c)
template <int MODE, int W = 4>
__global__ void __launch_bounds__(64 * W) k2_s48(const char* __restrict__ s, int rows, float* __restrict__ sink) {
  const int b = xcd_id(blockIdx.x, gridDim.x);
  const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
  const int row = b * W + w;
  if (row >= rows) return;
  const int f = row / NS, r = row % NS;
  const char* p = s + (size_t)f * NS * NC * 6;
  const int odd = t & 1;
  uint32_t acc = 0;
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const char* e = p + 6 * off_of(r, t + 64 * m);
    if constexpr (MODE == 0) {
      const uint2 v = *reinterpret_cast<const uint2*>(e - 2 * odd);
      acc += v.x ^ v.y;
    } else if constexpr (MODE == 1) {
      const uint32_t* q = reinterpret_cast<const uint32_t*>(e - 6 * odd);
      acc += q[0] ^ q[1] ^ q[2];
    } else {
      const uint32_t* q = reinterpret_cast<const uint32_t*>(e - 2 * odd);
      acc += q[0] ^ __builtin_nontemporal_load(q + 1);
    }
  }
  sink[blockIdx.x * 64 * W + threadIdx.x] = (float)acc;
}

__global__ void __launch_bounds__(256) linear16(const float4* __restrict__ s, size_t n4, float* __restrict__ sink) {
  float acc = 0.f;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    const float4 v = s[i];
    acc += v.x + v.y + v.z + v.w;
  }
  sink[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main(int argc, char** argv) {
  const int frames = argc > 1 ? atoi(argv[1]) : 3;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const size_t bytes = (size_t)frames * NS * NC * sizeof(float2);
  const int rows = frames * NS;
  float2* s;
  float* sink;
  CHECK(hipMalloc(&s, bytes));
  CHECK(hipMemset(s, 0, bytes));
  const int g8 = rows / 4, g16 = rows / 8, glin = 256 * 8;
  CHECK(hipMalloc(&sink, (size_t)rows * 64 * sizeof(float) + (size_t)glin * 256 * sizeof(float)));
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
    printf("%-10s %8.1f us per pass over %zu MiB  = %6.0f GB/s\n", name, us, bytes >> 20, bytes / us * 1e-3);
  };
  run("k2_rows8", [&] { hipLaunchKernelGGL(k2_rows8, dim3(g8), dim3(256), 0, 0, s, rows, sink); });
  run("rows8_w8", [&] { hipLaunchKernelGGL((k2_rows8w<8, 1>), dim3(rows / 8), dim3(512), 0, 0, s, rows, sink); });
  run("rows8_w2", [&] { hipLaunchKernelGGL((k2_rows8w<2, 1>), dim3(rows / 2), dim3(128), 0, 0, s, rows, sink); });
  run("rows8_nox", [&] { hipLaunchKernelGGL((k2_rows8w<4, 0>), dim3(rows / 4), dim3(256), 0, 0, s, rows, sink); });
  run("rows8_w8nx", [&] { hipLaunchKernelGGL((k2_rows8w<8, 0>), dim3(rows / 8), dim3(512), 0, 0, s, rows, sink); });
  run("k2_rows16", [&] { hipLaunchKernelGGL(k2_rows16, dim3(g16), dim3(256), 0, 0, reinterpret_cast<const float4*>(s), rows, sink); });
  run("pairs32", [&] { hipLaunchKernelGGL(k2_pairs32, dim3(g16), dim3(256), 0, 0, reinterpret_cast<const float4*>(s), rows, sink); });
  {
    const int rows48 = (int)(bytes / (NS * NC * 6)) * NS;  // same bytes: 4 S48 frames per 3 fp32
    const char* c = reinterpret_cast<const char*>(s);
    run("s48_x2", [&] { hipLaunchKernelGGL((k2_s48<0>), dim3(rows48 / 4), dim3(256), 0, 0, c, rows48, sink); });
    run("s48_x3", [&] { hipLaunchKernelGGL((k2_s48<1>), dim3(rows48 / 4), dim3(256), 0, 0, c, rows48, sink); });
    run("s48_2x1", [&] { hipLaunchKernelGGL((k2_s48<2>), dim3(rows48 / 4), dim3(256), 0, 0, c, rows48, sink); });
    run("s48_x3w8", [&] { hipLaunchKernelGGL((k2_s48<1, 8>), dim3(rows48 / 8), dim3(512), 0, 0, c, rows48, sink); });
  }
  run("linear16", [&] { hipLaunchKernelGGL(linear16, dim3(glin), dim3(256), 0, 0, reinterpret_cast<const float4*>(s), bytes / 16, sink); });
  CHECK(hipGetLastError());
  CHECK(hipFree(s));
  CHECK(hipFree(sink));
  return 0;
}
