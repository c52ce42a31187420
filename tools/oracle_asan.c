/* oracle_asan.c -- the CPU restatement (oracle/fmcw_cpu.c, test infrastructure) under
 * AddressSanitizer + UndefinedBehaviorSanitizer on the host: whole path with the 1-D and 2-D
 * CFAR on seeded random cubes at several geometries (power-of-two ns / nc, 1-4 rx, detection
 * capacities smaller than the list), then the CFAR alone.  A sanitizer report aborts with a
 * non-zero status.  Build and run: tools/oracle_asan.sh */
#include "../oracle/fmcw_cpu.c"

#include <stdio.h>

static uint32_t rng = 12345u;
static float urand(void) {
  rng = rng * 1664525u + 1013904223u;
  return (float)(rng >> 8) / 16777216.0f - 0.5f;
}

int main(void) {
  const int geo[][4] = {{64, 32, 1, 2}, {256, 64, 2, 3}, {1024, 128, 1, 2}, {512, 256, 4, 1}, {128, 16, 1, 4}};
  size_t total = 0;
  for (size_t g = 0; g < sizeof geo / sizeof geo[0]; ++g) {
    const int ns = geo[g][0], nc = geo[g][1], nrx = geo[g][2], F = geo[g][3];
    const size_t n = (size_t)F * nrx * nc * ns * 2;
    float* cube = malloc(n * sizeof(float));
    float* map = malloc((size_t)F * ns * nc * sizeof(float));
    for (size_t i = 0; i < n; ++i) cube[i] = urand();
    for (int f = 0; f < F; ++f)                        /* a tone per frame: detections exist */
      for (int c = 0; c < nc; ++c)
        for (int i = 0; i < ns; ++i) {
          float* x = cube + (((size_t)f * nrx) * nc + c) * ns * 2 + 2 * i;
          x[0] += 40.f * cosf(0.37f * i + 0.9f * c);
          x[1] += 40.f * sinf(0.37f * i + 0.9f * c);
        }
    for (int kind = 1; kind <= 2; ++kind) {
      cpu_cfar p = {0};
      p.kind = kind;
      p.ref1 = 8, p.guard1 = 2, p.rank1 = 12, p.alpha = 3.0f;
      p.ref_r = 5, p.guard_r = 1, p.ref_d = 6, p.guard_d = 2, p.rank_pct = 75, p.smin = 2, p.snom = 4, p.smax = 6;
      if (kind == 2 && (ns < 2 * p.ref_r + 1 || nc < 2 * p.ref_d + 1)) continue;
      for (size_t cap = 4; cap <= 1u << 16; cap *= 64) {   /* list longer than cap, then not */
        cpu_det* d = malloc(cap * sizeof(cpu_det));
        const size_t k = fmcw_cpu_process(cube, F, ns, nc, nrx, &p, map, d, cap, 4);
        const size_t k2 = fmcw_cpu_cfar(map, F, ns, nc, &p, d, cap, 4);
        if (k != k2) {
          printf("mismatch ns %d nc %d kind %d: %zu vs %zu\n", ns, nc, kind, k, k2);
          return 1;
        }
        total += k;
        free(d);
      }
    }
    free(cube);
    free(map);
  }
  printf("oracle under ASan/UBSan: ok (%zu detections over all runs)\n", total);
  return 0;
}
