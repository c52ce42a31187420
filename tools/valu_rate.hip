// valu_rate.hip -- issue rate of 32-bit integer vs fp32 VALU instructions on gfx950 (wave64):
// 8 independent chains per lane, 4096 iterations, 4 waves per SIMD (1024 threads per CU), all CUs.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/valu_rate tools/valu_rate.hip ; Run: tools/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITER 4096
__global__ void __launch_bounds__(256) k_int(uint32_t* out, uint32_t s) {
  uint32_t a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i + s;
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // 4 integer VALU ops per chain per iteration
      uint32_t t;
      asm volatile("v_sub_u32 %0, %1, %2" : "=v"(t) : "v"(a[i]), "v"(s));
      asm volatile("v_lshrrev_b32 %0, 7, %1" : "=v"(t) : "v"(t));
      asm volatile("v_and_b32 %0, 0x1010101, %1" : "=v"(t) : "v"(t));
      asm volatile("v_add_u32 %0, %1, %2" : "=v"(a[i]) : "v"(a[i]), "v"(t));
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r ^= a[i];
  if (r == 0x12345678u) out[0] = r;
}
__global__ void __launch_bounds__(256) k_fp(float* out, float s) {
  float a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 0.001f + i;
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // 4 fp32 VALU ops per chain per iteration
      float t;
      asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(t) : "v"(a[i]), "v"(s), "v"(s));
      asm volatile("v_add_f32 %0, %1, %2" : "=v"(t) : "v"(t), "v"(s));
      asm volatile("v_mul_f32 %0, %1, %2" : "=v"(t) : "v"(t), "v"(s));
      asm volatile("v_add_f32 %0, %1, %2" : "=v"(a[i]) : "v"(a[i]), "v"(t));
    }
  }
  float r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r += a[i];
  if (r == 1234.5f) out[0] = r;
}
__global__ void __launch_bounds__(256) k_align(uint32_t* out, uint32_t s) {
  uint32_t a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i + s;
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // alignbyte + add3 + sub + and
      uint32_t t;
      asm volatile("v_alignbyte_b32 %0, %1, %2, 2" : "=v"(t) : "v"(a[i]), "v"(s));
      asm volatile("v_sub_u32 %0, %1, %2" : "=v"(t) : "v"(t), "v"(s));
      asm volatile("v_and_b32 %0, 0x1010101, %1" : "=v"(t) : "v"(t));
      asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(a[i]) : "v"(a[i]), "v"(t), "v"(s));
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r ^= a[i];
  if (r == 0x12345678u) out[0] = r;
}
int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int n_cu = p.multiProcessorCount;
  void* buf;
  hipMalloc(&buf, 64);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int waves_per_simd : {1, 2, 4}) {
    const int grid = n_cu * waves_per_simd;  // 256 threads = 4 waves = one per SIMD per workgroup
    const double instr = (double)grid * 4 /*waves*/ * ITER * 8 * 4;
    for (int k = 0; k < 3; ++k) {
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        if (k == 0) hipLaunchKernelGGL(k_int, dim3(grid), dim3(256), 0, 0, (uint32_t*)buf, 3u);
        else if (k == 1) hipLaunchKernelGGL(k_fp, dim3(grid), dim3(256), 0, 0, (float*)buf, 0.999f);
        else hipLaunchKernelGGL(k_align, dim3(grid), dim3(256), 0, 0, (uint32_t*)buf, 3u);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (rep == 1)
          std::printf("%-6s waves/SIMD %d: %.1f us, %.3f wave-instr per CU per ns (%.2f per CU per 2.4-GHz clock)\n",
                      k == 0 ? "int" : k == 1 ? "fp32" : "align", waves_per_simd, ms * 1e3,
                      instr / n_cu / (ms * 1e6), instr / n_cu / (ms * 1e6) / 2.4);
      }
    }
  }
  return 0;
}
