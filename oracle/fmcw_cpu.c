/*
 * fmcw_cpu.c -- TEST/BENCH INFRASTRUCTURE ONLY: a multithreaded C restatement of the oracle
 * (oracle/fmcw_oracle.py) used as bench.py's CPU baseline and cross-checked against the
 * NumPy oracle by tests/test_cpu_backend.py.  Never linked or loaded by the product path.
 *
 * Stages (reference = Aurellia-Beam/fpga-fmcw-radar-processor, VHDL):
 *   window (Hamming, half-ROM mirrored)   rtl/src/window_multiplier.vhd:34-49, :97-102
 *   range FFT, forward, natural order     rtl/src/radar_core.vhd:247, :303-316
 *   corner turn out[r][c] = in[c][r]      rtl/src/corner_turner.vhd:79-80
 *   Doppler window + FFT                  rtl/src/radar_core.vhd:340-364
 *   |X| (sqrt of the sum over rx: NCI)    SURVEY.md 8a-R7
 *   1-D OS-CFAR 16/4 (circular)           rtl/old/os_cfar.vhd:98-144
 *   2-D OS-CFAR 128 refs, adaptive scale  rtl/src/os_cfar_2d.vhd:152-217
 * Arithmetic: fp32 throughout (the FFT is a radix-2 Stockham transform with a fp64-built
 * twiddle table); the CFAR follows the oracle's fp32 definitions exactly (ranked value by
 * selection, fl(alpha * ranked), the 2-D mean as the oracle's tree_sum_f32), so detections on
 * a given map are bit-identical to fmcw_oracle.cfar_os1d / cfar_os2d on that map.
 * Threads: OpenMP inside each frame (chirps, range rows, CFAR rows).
 *
 * Build: oracle/Makefile (gcc -O3 -march=x86-64-v3 -fopenmp -shared).
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { float re, im; } cf;

typedef struct {
  uint32_t frame;
  uint16_t range, doppler;
  float mag, threshold;
} cpu_det;

static void hamming(int n, float* w) {
  const int half = n / 2;
  for (int i = 0; i < n; ++i) {
    int a = i < half ? i : n - 1 - i;
    if (a > half - 1) a = half - 1;
    w[i] = (float)(0.54 - 0.46 * cos(2.0 * M_PI * (double)a / (double)(n - 1)));
  }
}

static void twiddles(int n, cf* w) {
  for (int k = 0; k < n / 2; ++k) {
    w[k].re = (float)cos(-2.0 * M_PI * k / n);
    w[k].im = (float)sin(-2.0 * M_PI * k / n);
  }
}

/* Stockham autosort radix-2 DIF, out of place with ping-pong; result in x. */
static void fft(int n, cf* restrict x, cf* restrict y, const cf* restrict w) {
  cf* a = x;
  cf* b = y;
  for (int l = n / 2, m = 1; l >= 1; l /= 2, m *= 2) {
    for (int j = 0; j < l; ++j) {
      const cf wj = w[j * m];
      const cf* a0 = a + j * m;
      const cf* a1 = a + j * m + l * m;
      cf* b0 = b + 2 * j * m;
      cf* b1 = b0 + m;
      for (int k = 0; k < m; ++k) {
        const float dr = a0[k].re - a1[k].re, di = a0[k].im - a1[k].im;
        b0[k].re = a0[k].re + a1[k].re;
        b0[k].im = a0[k].im + a1[k].im;
        b1[k].re = wj.re * dr - wj.im * di;
        b1[k].im = wj.re * di + wj.im * dr;
      }
    }
    cf* t = a;
    a = b;
    b = t;
  }
  if (a != x) memcpy(x, a, sizeof(cf) * (size_t)n);
}

/* k-th smallest of v[0..n) (v is clobbered): quickselect */
static float select_k(float* v, int n, int k) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const float p = v[(lo + hi) / 2];
    int i = lo, j = hi;
    while (i <= j) {
      while (v[i] < p) ++i;
      while (v[j] > p) --j;
      if (i <= j) {
        const float t = v[i];
        v[i] = v[j];
        v[j] = t;
        ++i;
        --j;
      }
    }
    if (k <= j) hi = j;
    else if (k >= i) lo = i;
    else return v[k];
  }
  return v[k];
}

/* oracle tree_sum_f32: pad to 128 with zeros, halve s[i] = s[i] + s[i + n/2] */
static float tree_sum_128(const float* refs, int n) {
  float s[128];
  for (int i = 0; i < 128; ++i) s[i] = i < n ? refs[i] : 0.f;
  for (int h = 64; h >= 1; h >>= 1)
    for (int i = 0; i < h; ++i) s[i] = s[i] + s[i + h];
  return s[0];
}

typedef struct {
  int kind;                    /* 0 none, 1 OS 1-D, 2 OS 2-D */
  int ref1, guard1, rank1;     /* 1-D */
  float alpha;
  int ref_r, guard_r, ref_d, guard_d, rank_pct, smin, snom, smax, override_;  /* 2-D */
} cpu_cfar;

/* one frame's map -> detections appended to out (returns count; stores at most cap - *n) */
static size_t cfar_frame(const float* map, int ns, int nc, const cpu_cfar* p, uint32_t frame, cpu_det* out,
                         size_t cap, size_t n0) {
  size_t n = n0;
  if (p->kind == 1) {
    /* detect <=> #{refs : fl(alpha * ref) < cut} > rank (fl(alpha x) is monotone), the same
     * decision as cut > fl(alpha * sorted(refs)[rank]); the threshold is selected only for
     * detections */
    const int nref = 2 * p->ref1;
    for (int r = 0; r < ns; ++r) {
      const float* row = map + (size_t)r * nc;
      for (int d = 0; d < nc; ++d) {
        const float cut = row[d];
        float v[64];
        int lt = 0;
        for (int j = 0; j < p->ref1; ++j) {
          v[j] = row[(d - p->guard1 - 1 - j) & (nc - 1)];
          v[p->ref1 + j] = row[(d + p->guard1 + 1 + j) & (nc - 1)];
        }
        for (int j = 0; j < nref; ++j) lt += p->alpha * v[j] < cut;
        if (lt > p->rank1) {
          const float thr = p->alpha * select_k(v, nref, p->rank1);
          if (out && n < cap) out[n] = (cpu_det){frame, (uint16_t)r, (uint16_t)d, cut, thr};
          ++n;
        }
      }
    }
  } else if (p->kind == 2) {
    const int hr = p->ref_r + p->guard_r, hd = p->ref_d + p->guard_d;
    int offs[256][2], nref = 0;
    for (int dr = -hr; dr <= hr; ++dr)
      for (int dd = -hd; dd <= hd; ++dd) {
        if (abs(dr) <= p->guard_r && abs(dd) <= p->guard_d) continue;
        offs[nref][0] = dr;
        offs[nref][1] = dd;
        ++nref;
      }
    long long kk = (long long)nref * p->rank_pct / 100;
    const int rank = (int)(kk < nref - 1 ? kk : nref - 1);
    for (int r = hr; r < ns - hr; ++r) {
      for (int d = 0; d < nc; ++d) {
        float v[256], s[256];
        for (int j = 0; j < nref; ++j) {
          v[j] = map[(size_t)(r + offs[j][0]) * nc + ((d + offs[j][1]) & (nc - 1))];
          s[j] = v[j];
        }
        const float mean = tree_sum_128(s, nref) / (float)nref;
        const int need = nref - rank;          /* ranked > M <=> #{ref > M} >= nref - rank */
        float scale;
        if (p->override_) scale = (float)p->override_;
        else {
          const float half = mean * 0.5f, hi = mean + half;
          int n_hi = 0, n_lo = 0;
          for (int j = 0; j < nref; ++j) {
            n_hi += v[j] > hi;
            n_lo += v[j] < half;
          }
          scale = n_hi >= need ? (float)p->smax : n_lo >= rank + 1 ? (float)p->smin : (float)p->snom;
        }
        const float cut = map[(size_t)r * nc + d];
        int n_ge = 0;                          /* detect <=> #{fl(scale ref) >= cut} < need */
        for (int j = 0; j < nref; ++j) n_ge += scale * v[j] >= cut;
        if (n_ge < need) {
          const float thr = select_k(v, nref, rank) * scale;
          if (out && n < cap) out[n] = (cpu_det){frame, (uint16_t)r, (uint16_t)d, cut, thr};
          ++n;
        }
      }
    }
  }
  return n;
}

/* CFAR of one frame's map, rows split over the OpenMP threads, results concatenated in range
 * order (deterministic); appends to dets from index n, returns the new count */
static size_t cfar_rows_parallel(const float* m, int ns, int nc, const cpu_cfar* cfar, uint32_t f, cpu_det* dets,
                                 size_t cap, size_t n) {
  /* rows in parallel chunks, then concatenated in range order (deterministic) */
  const int nt = omp_get_max_threads();
  size_t* cnt = calloc((size_t)nt + 1, sizeof(size_t));
  cpu_det** part = calloc((size_t)nt, sizeof(cpu_det*));
  size_t* pcap = calloc((size_t)nt, sizeof(size_t));
#pragma omp parallel num_threads(nt)
  {
    const int t = omp_get_thread_num(), T = omp_get_num_threads();
    const int r0 = (int)((long long)ns * t / T), r1 = (int)((long long)ns * (t + 1) / T);
    /* a sub-map view would change the 2-D edge rule: run the full-frame CFAR on a row band */
    cpu_cfar pc = *cfar;
    size_t c = 0, cp = 1024;
    cpu_det* buf = malloc(sizeof(cpu_det) * cp);
    for (int r = r0; r < r1; ++r) {
      /* single-row pass: reuse cfar_frame on a one-row window with the range context */
      if (pc.kind == 1) {
        size_t got = cfar_frame(m + (size_t)r * nc, 1, nc, &pc, f, NULL, 0, 0);
        if (got) {
          if (c + got > cp) {
            while (c + got > cp) cp *= 2;
            buf = realloc(buf, sizeof(cpu_det) * cp);
          }
          cfar_frame(m + (size_t)r * nc, 1, nc, &pc, f, buf + c, got, 0);
          for (size_t i = 0; i < got; ++i) buf[c + i].range = (uint16_t)r;
          c += got;
        }
      } else {
        const int hr = pc.ref_r + pc.guard_r;
        if (r < hr || r >= ns - hr) continue;
        /* rows r-hr .. r+hr as a (2hr+1)-row map whose only tested row is hr */
        size_t got = cfar_frame(m + (size_t)(r - hr) * nc, 2 * hr + 1, nc, &pc, f, NULL, 0, 0);
        if (got) {
          if (c + got > cp) {
            while (c + got > cp) cp *= 2;
            buf = realloc(buf, sizeof(cpu_det) * cp);
          }
          cfar_frame(m + (size_t)(r - hr) * nc, 2 * hr + 1, nc, &pc, f, buf + c, got, 0);
          for (size_t i = 0; i < got; ++i) buf[c + i].range = (uint16_t)r;
          c += got;
        }
      }
    }
    cnt[t] = c;
    part[t] = buf;
    pcap[t] = cp;
  }
  for (int t = 0; t < nt; ++t) {
    for (size_t i = 0; i < cnt[t]; ++i, ++n)
      if (dets && n < cap) dets[n] = part[t][i];
    free(part[t]);
  }
  free(cnt);
  free(part);
  free(pcap);
  return n;
}

/*
 * cube [F][nrx][nc][ns] complex fp32 -> map [F][ns][nc] fp32 (may be NULL) and detections.
 * Returns the number of detections found (entries beyond cap are not stored).
 * threads <= 0: OpenMP default.
 */
/* nc (Doppler bins) is a power of two, as the library requires (circular index = mask) */
size_t fmcw_cpu_process(const float* cube, int F, int ns, int nc, int nrx, const cpu_cfar* cfar, float* map_out,
                        cpu_det* dets, size_t cap, int threads) {
  if (threads > 0) omp_set_num_threads(threads);
  float* wr = malloc(sizeof(float) * ns);
  float* wd = malloc(sizeof(float) * nc);
  cf* twr = malloc(sizeof(cf) * (ns / 2 + 1));
  cf* twd = malloc(sizeof(cf) * (nc / 2 + 1));
  cf* spec = malloc(sizeof(cf) * (size_t)ns * nc);          /* one rx: [range][chirp] */
  float* pw = malloc(sizeof(float) * (size_t)ns * nc);       /* sum over rx of |X|^2 */
  float* mapf = malloc(sizeof(float) * (size_t)ns * nc);
  hamming(ns, wr);
  hamming(nc, wd);
  twiddles(ns, twr);
  twiddles(nc, twd);
  size_t n = 0;
  for (int f = 0; f < F; ++f) {
    for (int rx = 0; rx < nrx; ++rx) {
      const cf* x = (const cf*)cube + ((size_t)f * nrx + rx) * (size_t)nc * ns;
#pragma omp parallel
      {
        cf* a = malloc(sizeof(cf) * (ns > nc ? ns : nc));
        cf* b = malloc(sizeof(cf) * (ns > nc ? ns : nc));
#pragma omp for schedule(static)
        for (int c = 0; c < nc; ++c) {                        /* window + range FFT */
          const cf* xc = x + (size_t)c * ns;
          for (int i = 0; i < ns; ++i) {
            a[i].re = xc[i].re * wr[i];
            a[i].im = xc[i].im * wr[i];
          }
          fft(ns, a, b, twr);
          for (int r = 0; r < ns; ++r) spec[(size_t)r * nc + c] = a[r];   /* corner turn */
        }
#pragma omp for schedule(static)
        for (int r = 0; r < ns; ++r) {                        /* Doppler window + FFT + |X|^2 */
          cf* row = spec + (size_t)r * nc;
          for (int c = 0; c < nc; ++c) {
            a[c].re = row[c].re * wd[c];
            a[c].im = row[c].im * wd[c];
          }
          fft(nc, a, b, twd);
          float* pr = pw + (size_t)r * nc;
          for (int d = 0; d < nc; ++d) {
            const float p = a[d].re * a[d].re + a[d].im * a[d].im;
            pr[d] = rx ? pr[d] + p : p;
          }
        }
        free(a);
        free(b);
      }
    }
    float* m = map_out ? map_out + (size_t)f * ns * nc : mapf;
#pragma omp parallel for schedule(static)
    for (size_t i = 0; i < (size_t)ns * nc; ++i) m[i] = sqrtf(pw[i]);
    if (cfar && cfar->kind) {
      n = cfar_rows_parallel(m, ns, nc, cfar, (uint32_t)f, dets, cap, n);
    }
  }
  free(wr);
  free(wd);
  free(twr);
  free(twd);
  free(spec);
  free(pw);
  free(mapf);
  return n;
}

/* CFAR alone on caller maps [F][ns][nc] (the checker of the large GPU parity tests) */
size_t fmcw_cpu_cfar(const float* map, int F, int ns, int nc, const cpu_cfar* cfar, cpu_det* dets, size_t cap,
                     int threads) {
  if (threads > 0) omp_set_num_threads(threads);
  size_t n = 0;
  for (int f = 0; f < F; ++f) n = cfar_rows_parallel(map + (size_t)f * ns * nc, ns, nc, cfar, (uint32_t)f, dets, cap, n);
  return n;
}

int fmcw_cpu_max_threads(void) { return omp_get_max_threads(); }
