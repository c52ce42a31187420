// valu_rate.hip -- issue rate of single VALU opcodes on gfx950 (wave64): 8 independent chains
// per lane of one opcode, 4 waves per SIMD on every CU; reports wave-instructions per CU per
// 2.4-GHz clock (the chip runs under DVFS, so absolute rates read ~10-15 % low; compare rows).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/valu_rate tools/valu_rate.hip ; Run: tools/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITER 2048
#define CH 8
#define KERNEL(NAME, T, INIT, ...)                                                      \
  __global__ void __launch_bounds__(256) NAME(T* out, uint32_t s) {                      \
    T a[CH];                                                                             \
    _Pragma("unroll") for (int i = 0; i < CH; ++i) a[i] = INIT;                          \
    for (int it = 0; it < ITER; ++it) {                                                  \
      _Pragma("unroll") for (int i = 0; i < CH; ++i) { __VA_ARGS__; }                           \
    }                                                                                    \
    T r = a[0];                                                                          \
    _Pragma("unroll") for (int i = 1; i < CH; ++i) r = r + a[i];                         \
    if (sink(r)) out[0] = r;                                                             \
  }
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ bool sink(uint32_t r) { return r == 12345u; }
__device__ bool sink(uint64_t r) { return r == 12345u; }
__device__ bool sink(float r) { return r == 12345.f; }
__device__ bool sink(f2 r) { return r.x == 12345.f; }
KERNEL(k_add_u32, uint32_t, threadIdx.x + i, asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(s)))
KERNEL(k_and, uint32_t, threadIdx.x + i, asm volatile("v_and_b32 %0, 0x1010101, %0" : "+v"(a[i])))
KERNEL(k_lshr, uint32_t, threadIdx.x + i, asm volatile("v_lshrrev_b32 %0, 1, %0" : "+v"(a[i])))
KERNEL(k_add3, uint32_t, threadIdx.x + i, asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(s)))
KERNEL(k_align, uint32_t, threadIdx.x + i, asm volatile("v_alignbyte_b32 %0, %0, %1, 2" : "+v"(a[i]) : "v"(s)))
KERNEL(k_perm, uint32_t, threadIdx.x + i, asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(s)))
KERNEL(k_bitop3, uint32_t, threadIdx.x + i, asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(a[i]) : "v"(s)))
KERNEL(k_fma, float, threadIdx.x * 0.001f + i, asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"((float)s)))
KERNEL(k_add_f32, float, threadIdx.x * 0.001f + i, asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"((float)s)))
KERNEL(k_pk_add, f2, (f2{threadIdx.x * 0.001f + i, 1.f}), asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(f2{(float)s, 1.f})))
KERNEL(k_pk_fma, f2, (f2{threadIdx.x * 0.001f + i, 1.f}), asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(f2{(float)s, 1.f})))
KERNEL(k_pk_mul, f2, (f2{threadIdx.x * 0.001f + i, 1.f}), asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(a[i]) : "v"(f2{(float)s, 1.f})))
KERNEL(k_fmac, float, threadIdx.x * 0.001f + i, asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a[i]) : "v"((float)s), "v"((float)(s + 1))))
KERNEL(k_mul_f32, float, threadIdx.x * 0.001f + i, asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[i]) : "v"((float)s)))
KERNEL(k_sub_f32, float, threadIdx.x * 0.001f + i, asm volatile("v_sub_f32 %0, %0, %1" : "+v"(a[i]) : "v"((float)s)))
KERNEL(k_lshl_add64, uint64_t, threadIdx.x + i, asm volatile("v_lshl_add_u64 %0, %0, 0, %0" : "+v"(a[i])))
KERNEL(k_lshr64, uint64_t, threadIdx.x + i, asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(a[i])))
KERNEL(k_sqrt, float, threadIdx.x * 0.001f + i + 1.f, asm volatile("v_sqrt_f32 %0, %0" : "+v"(a[i])))
KERNEL(k_cndmask, uint32_t, threadIdx.x + i, asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(s) : "vcc"))
// (round 6) integer multiply and the cndmask forms the K3 screen compiles to; the mask set once
// outside the chains (the row above declares vcc clobbered, so every instance waits on a VALU write)
KERNEL(k_mul_lo, uint32_t, threadIdx.x + i, asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(s)))
KERNEL(k_mul_u24, uint32_t, threadIdx.x + i, asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(s)))
KERNEL(k_lshl_add, uint32_t, threadIdx.x + i, asm volatile("v_lshl_add_u32 %0, %0, 8, %0" : "+v"(a[i])))
KERNEL(k_cnd_sgpr, uint32_t, threadIdx.x + i, asm volatile("v_cndmask_b32_e64 %0, 0, %0, %1" : "+v"(a[i]) : "s"((uint64_t)s * 0x5555u)))
KERNEL(k_cmp_cnd, uint32_t, threadIdx.x + i, asm volatile("v_cmp_gt_u32_e64 s[40:41], 33, %0\n\tv_cndmask_b32_e64 %0, 0, %0, s[40:41]" : "+v"(a[i]) :: "s40", "s41"))

struct K { const char* name; void* fn; };
int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int n_cu = p.multiProcessorCount;
  void* buf;
  (void)hipMalloc(&buf, 64);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  K ks[] = {{"v_add_u32", (void*)k_add_u32}, {"v_and_b32 lit", (void*)k_and}, {"v_lshrrev_b32", (void*)k_lshr},
            {"v_add3_u32", (void*)k_add3}, {"v_alignbyte_b32", (void*)k_align}, {"v_perm_b32", (void*)k_perm},
            {"v_bitop3_b32", (void*)k_bitop3}, {"v_fma_f32", (void*)k_fma}, {"v_add_f32", (void*)k_add_f32},
            {"v_pk_add_f32", (void*)k_pk_add}, {"v_pk_fma_f32", (void*)k_pk_fma}, {"v_pk_mul_f32", (void*)k_pk_mul},
            {"v_fmac_f32", (void*)k_fmac}, {"v_mul_f32", (void*)k_mul_f32}, {"v_sub_f32", (void*)k_sub_f32}, {"v_lshl_add_u64", (void*)k_lshl_add64},
            {"v_lshrrev_b64", (void*)k_lshr64}, {"v_sqrt_f32", (void*)k_sqrt}, {"v_cndmask_b32", (void*)k_cndmask},
            {"v_mul_lo_u32", (void*)k_mul_lo}, {"v_mul_u32_u24", (void*)k_mul_u24}, {"v_lshl_add_u32", (void*)k_lshl_add},
            {"v_cndmask sgpr", (void*)k_cnd_sgpr}, {"v_cmp+v_cndmask", (void*)k_cmp_cnd}};
  const int grid = n_cu * 4;  // 256 threads = one wave per SIMD per workgroup -> 4 waves per SIMD
  const double instr = (double)grid * 4 * ITER * CH;
  for (const K& k : ks) {
    float best = 1e9f;
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(reinterpret_cast<void (*)(void*, uint32_t)>(k.fn), dim3(grid), dim3(256), 0, 0, buf, 3u);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep > 0 && ms < best) best = ms;
    }
    std::printf("%-16s %8.1f us  %.2f wave-instr per CU per 2.4-GHz clock\n", k.name, best * 1e3,
                instr / n_cu / (best * 1e6) / 2.4);
  }
  return 0;
}
