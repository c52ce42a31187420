// l2_probe.hip -- does a 2 MiB per-XCD working set written with plain stores stay in the
// XCD's L2 (write-back), so that a same-XCD reader never touches HBM?  Decides the design of
// the fused range+Doppler kernel.  Run under rocprofv3 --pmc WRITE_SIZE / FETCH_SIZE.
//
//   store_rep   every workgroup rewrites its slice of its XCD's region REPS times
//   store_load  write the slice once, then REPS times read it back (L1-bypassing nt loads)
//   cross_read  write the slice, XCD-local arrival counter, then read ANOTHER workgroup's
//               slice of the same XCD (the fused kernel's hand-off), REPS times
// Region per XCD: 1, 2, 4, 8 MiB.  Grid = 4 workgroups of 256 threads per CU (1024).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ int xcc_id() {
  int x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 0xf;
}

typedef float f4v __attribute__((ext_vector_type(4)));

// slot of this workgroup within its XCD: claimed with an atomic per XCD (placement-independent)
__device__ int claim_slot(int* slot_ctr, int xcc) {
  __shared__ int s;
  if (threadIdx.x == 0) s = atomicAdd(slot_ctr + xcc, 1);
  __syncthreads();
  return s;
}

__global__ void __launch_bounds__(256) store_rep(f4v* buf, size_t region_f4, int per_xcd, int reps, int* slot_ctr) {
  const int xcc = xcc_id();
  const int slot = claim_slot(slot_ctr, xcc);
  if (slot >= per_xcd) return;
  const size_t slice = region_f4 / per_xcd;
  f4v* p = buf + (size_t)xcc * region_f4 + (size_t)slot * slice;
  for (int r = 0; r < reps; ++r)
    for (size_t i = threadIdx.x; i < slice; i += 256) p[i] = f4v{(float)r, (float)i, 1.f, 2.f};
}

__global__ void __launch_bounds__(256) store_load(f4v* buf, size_t region_f4, int per_xcd, int reps, int* slot_ctr,
                                                  float* sink) {
  const int xcc = xcc_id();
  const int slot = claim_slot(slot_ctr, xcc);
  if (slot >= per_xcd) return;
  const size_t slice = region_f4 / per_xcd;
  f4v* p = buf + (size_t)xcc * region_f4 + (size_t)slot * slice;
  for (size_t i = threadIdx.x; i < slice; i += 256) p[i] = f4v{1.f, (float)i, 1.f, 2.f};
  __syncthreads();
  float acc = 0.f;
  for (int r = 0; r < reps; ++r)
    for (size_t i = threadIdx.x; i < slice; i += 256) {
      f4v v = __builtin_nontemporal_load(p + i);
      acc += v.x + v.y * (float)r;
    }
  if (acc == 1234.5f) sink[0] = acc;
}

__global__ void __launch_bounds__(256) cross_read(f4v* buf, size_t region_f4, int per_xcd, int reps, int* slot_ctr,
                                                  int* arrive, float* sink) {
  const int xcc = xcc_id();
  const int slot = claim_slot(slot_ctr, xcc);
  if (slot >= per_xcd) return;
  const size_t slice = region_f4 / per_xcd;
  f4v* base = buf + (size_t)xcc * region_f4;
  f4v* p = base + (size_t)slot * slice;
  for (size_t i = threadIdx.x; i < slice; i += 256) p[i] = f4v{(float)slot, (float)i, 1.f, 2.f};
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(arrive + xcc, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int spins = 0;
    while (__hip_atomic_load(arrive + xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < per_xcd && spins < (1 << 22)) {
      __builtin_amdgcn_s_sleep(2);
      ++spins;
    }
  }
  __syncthreads();
  float acc = 0.f;
  int bad = 0;
  for (int r = 0; r < reps; ++r) {
    const int other = (slot + 1 + r) % per_xcd;
    const f4v* q = base + (size_t)other * slice;
    for (size_t i = threadIdx.x; i < slice; i += 256) {
      f4v v = __builtin_nontemporal_load(q + i);
      bad += (v.x != (float)other) | (v.y != (float)i);
      acc += v.z;
    }
  }
  if (bad) atomicAdd(reinterpret_cast<int*>(sink) + 1, bad);
  if (acc == 1234.5f) sink[0] = acc;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 32;
  const int per_xcd = 128;  // 4 WGs per CU x 32 CUs
  const int grid = 8 * per_xcd;
  const size_t max_region = (size_t)8 << 20;
  f4v* buf;
  int *slot_ctr, *arrive;
  float* sink;
  CHECK(hipMalloc(&buf, 8 * max_region));
  CHECK(hipMalloc(&slot_ctr, 64));
  CHECK(hipMalloc(&arrive, 64));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMemset(sink, 0, 64));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (size_t mib : {1, 2, 4, 8}) {
    const size_t region_f4 = (mib << 20) / 16;
    for (int v = 0; v < 3; ++v) {
      for (int it = 0; it < 3; ++it) {
        CHECK(hipMemset(slot_ctr, 0, 64));
        CHECK(hipMemset(arrive, 0, 64));
        CHECK(hipEventRecord(a));
        if (v == 0) hipLaunchKernelGGL(store_rep, dim3(grid), dim3(256), 0, 0, buf, region_f4, per_xcd, reps, slot_ctr);
        if (v == 1) hipLaunchKernelGGL(store_load, dim3(grid), dim3(256), 0, 0, buf, region_f4, per_xcd, reps, slot_ctr, sink);
        if (v == 2) hipLaunchKernelGGL(cross_read, dim3(grid), dim3(256), 0, 0, buf, region_f4, per_xcd, reps, slot_ctr, arrive, sink);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        const double bytes = (double)reps * 8 * (mib << 20);
        if (it == 2)
          printf("%-10s region %zu MiB/XCD reps %d: %8.1f us  %7.2f TB/s (reps x 8 regions)\n",
                 v == 0 ? "store_rep" : v == 1 ? "store_load" : "cross_read", mib, reps, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
      }
    }
  }
  int bad[2];
  CHECK(hipMemcpy(bad, sink, 8, hipMemcpyDeviceToHost));
  printf("cross_read mismatches: %d\n", bad[1]);
  return 0;
}
