/*
 * fmcw.h -- C-ABI of libfmcw.so, the MI355X (gfx950) FMCW range-Doppler + OS-CFAR
 * hot path.  Plain C types only: pointers, sizes, enums.  No torch, no C++.
 *
 * What this boundary replaces in the reference (Aurellia-Beam/fpga-fmcw-radar-processor):
 *
 *   fmcw_config            radar_core generics  rtl/src/radar_core.vhd:12-19 and control
 *                          ports mti_bypass / cfar_scale_ovr :47-49; FFT IP parameters
 *                          vivado_proj/.../ip/xfft_0_1/xfft_0.xci:12-27 (size, direction,
 *                          natural order); 1-D CFAR generics rtl/old/radar_core_v3.vhd:373-381
 *   fmcw_create            the FFT-IP config handshake cfg_proc radar_core.vhd:279-301
 *                          (config word x"0001" = forward, :247) -- done once per handle
 *   fmcw_enqueue /         the radar_core AXI4-Stream entity radar_core.vhd:21-56: ADC words
 *   fmcw_process           {Q[31:16], I[15:0]} in (:25-29), the Vivado IP calls
 *                          u_range_fft / u_doppler_fft (:303-316, :351-364) and every stage
 *                          between them (:267-390), detections out (:31-35, :396-418)
 *   fmcw_det               det_tdata[16:0] / det_range_bin[9:0] / det_doppler_bin[6:0]
 *                          (radar_core.vhd:31-35) + frame index + threshold (dbg_threshold,
 *                          rtl/src/os_cfar_2d.vhd:34, :219)
 *   status words 2, 3     the sticky status_overflow flag (radar_core.vhd:447-456), as counts:
 *   of fmcw_enqueue        samples saturated by the RTL-compat integer windows (win1 / win2
 *                          saturation, window_multiplier.vhd:152-158) and int16 spectrum words /
 *                          canceller outputs clipped (doppler_notch.vhd:75-93).  The fp32 build
 *                          spec never saturates; FMCW_EDETCAP reports a detection list overflow
 *   fmcw_range_ct          window_multiplier -> xfft_range -> corner_turner (:267-327),
 *                          corner-turned spectrum as the CT emits it (corner_turner.vhd:80)
 *   fmcw_magnitude         magnitude_calc (rtl/src/magnitude_calc.vhd:45-88)
 *   fmcw_cfar              os_cfar_2d / os_cfar on a caller-supplied magnitude map
 *                          (rtl/src/os_cfar_2d.vhd:83-230, rtl/old/os_cfar.vhd:98-137)
 *
 * Conventions
 *   - Return value: 0 (FMCW_OK) or a negative fmcw_status.  fmcw_last_error() returns a
 *     thread-local message for the last failure on the calling thread.
 *   - fmcw_enqueue and the stage functions take DEVICE pointers only, are stream-ordered
 *     and asynchronous (nothing synchronises, nothing allocates).  fmcw_enqueue and fmcw_cfar
 *     can be captured into a hipGraph (stream capture) and the graph replayed any number of
 *     times, interleaved with direct calls on the same handle: the detection ordering pass keeps
 *     its call tag in device memory, and a captured call always re-zeroes the per-call counters
 *     first.  Replays of one handle's graphs must not overlap each other or other calls (one
 *     stream at a time, below); profiling (fmcw_set_profiling) must be off while capturing.
 *   - fmcw_process accepts host or device pointers (detected with hipPointerGetAttributes),
 *     and returns after the results are in the caller's buffers.
 *   - A handle is not thread-safe: one handle per host thread, and one stream at a time
 *     (its scratch -- intermediate spectrum, detection slots, counters -- is shared by its
 *     calls, so two calls in flight on different streams race).  Every entry point selects
 *     the handle's device itself.  All kernel scratch is allocated at fmcw_create for up to
 *     cfg.max_frames frames per call; fmcw_process keeps its host-copy staging in the handle.
 *   - Layouts (row-major, complex = interleaved re,im):
 *       cube   [frame][rx][chirp][sample]       in_dtype (f32 / f16 / int16 complex)
 *       map    [frame][range][doppler]          float32 (range-major, as radar_output.txt)
 *       spec   [frame][rx][range][chirp]        complex float32 (fmcw_range_ct)
 *     Doppler bin 0 is zero Doppler (natural FFT order, no fftshift).
 */
#ifndef FMCW_H_
#define FMCW_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FMCW_ABI_VERSION 8  /* 2: fmcw_config grew compat_rtl, range_shift (27 words, 108 B);
                               3: + spectrum_dtype (28 words, 112 B);
                               4: FMCW_K_COUNT 5 -> 6, FMCW_INFO_PAIR_CHUNK;
                               5: n_dets_dev holds FMCW_STATUS_WORDS (4) words (saturation
                                  counts); the fused / paired kernels are gone (FMCW_K_COUNT 4,
                                  info keys 1-3 and 5 retired, fmcw_get_fused_trace removed);
                                  FMCW_WIN_Q15_RTL also windows slow time in integers;
                                  fmcw_comm_create takes wire_cap, fmcw_gather_dets det_cap;
                               6: fmcw_set_param (FMCW_PARAM_CFAR2D_STEPS), FMCW_INFO_CFAR2D_STEPS;
                                  range-kernel id 1 (k_range2) retired; the library reads no
                                  environment variable;
                               7: fmcw_enqueue / fmcw_cfar graph-capturable (device-resident
                                  ordering tag); fmcw_comm_fail_next_alloc_for_test,
                                  fmcw_comm_check_decide_for_test; FMCW_SPEC_S48;
                               8: fmcw_config grew det_capacity (29 words, 116 B): the detection
                                  scratch holds every cell by default, so a call loses no detection
                                  its det_cap has room for; fmcw_comm_info */

typedef enum {
  FMCW_OK = 0,
  FMCW_EINVAL = -1,       /* bad argument / unsupported configuration */
  FMCW_ENOMEM = -2,       /* device allocation failed */
  FMCW_EHIP = -3,         /* HIP runtime error (message in fmcw_last_error) */
  FMCW_EDETCAP = -4,      /* detection list longer than det_cap; *n_dets = required count */
  FMCW_ENODEV = -5        /* no usable gfx950 device */
} fmcw_status;

typedef enum { FMCW_IN_F32 = 0, FMCW_IN_F16 = 1, FMCW_IN_I16 = 2 } fmcw_in_dtype;
/* FMCW_WIN_Q15_RTL (RTL-compat, in_dtype I16 only): both windows in the RTL's integer
 * arithmetic, y = sat16((x * c[n] + 2^14) >> 14) with the ROM c = round(32767 w) on the
 * mirrored half address (window_multiplier.vhd:43-46, :97-102, :146-158) -- a 2x gain with a
 * +1 LSB bias, so a zero word windows to 1.  Fast time: on the ADC words (u_range_window,
 * radar_core.vhd:267-276).  Slow time (u_doppler_window, :340-349): on the corner-turned
 * spectrum's 16-bit words -- the range spectrum scaled by 2^-range_shift (the IP's fixed
 * scaling schedule; pick range_shift so it fits 16 bits), rounded half-to-even and saturated
 * to int16 -- after the MTI canceller when it is on.  The FFTs stay unscaled fp32.  Saturated
 * samples are counted in status words 2 (windows) and 3 (spectrum words, canceller). */
typedef enum { FMCW_WIN_NONE = 0, FMCW_WIN_HAMMING = 1, FMCW_WIN_Q15_RTL = 2 } fmcw_window;
/* FMCW_MAG_ABS: |X| = sqrt(re^2 + im^2) (with n_rx > 1: sqrt(sum_rx |X_rx|^2), NCI).
 * FMCW_MAG_AMBM: max(|re|,|im|) + floor(min/4) + floor(min/8) (magnitude_calc.vhd:78-81). */
typedef enum { FMCW_MAG_ABS = 0, FMCW_MAG_AMBM = 1 } fmcw_mag_mode;
/* What fmcw_enqueue writes into rd_map: linear magnitude, or 20*log10(mag + 1). */
typedef enum { FMCW_MAP_LINEAR = 1, FMCW_MAP_DB = 2 } fmcw_map_kind;
typedef enum { FMCW_CFAR_NONE = 0, FMCW_CFAR_OS1D = 1, FMCW_CFAR_OS2D = 2 } fmcw_cfar_kind;
/* MTI / Doppler notch on the corner-turned spectrum, along slow time per range bin, delay
 * line zeroed at each range bin's first chirp (rtl/src/doppler_notch.vhd:72-102):
 * 2-pulse y[c] = x[c] - x[c-1];  3-pulse y[c] = x[c] - 2 x[c-1] + x[c-2].  OFF = bypass. */
typedef enum { FMCW_MTI_OFF = 0, FMCW_MTI_2PULSE = 2, FMCW_MTI_3PULSE = 3 } fmcw_mti_mode;

typedef struct fmcw_config {
  uint32_t n_range;        /* Ns: samples per chirp = range bins (N_RANGE); power of 2, 64..8192 */
  uint32_t n_doppler;      /* Nc: chirps per frame = Doppler bins (N_DOPPLER); power of 2, 32..1024 */
  uint32_t n_rx;           /* receive channels, >= 1; > 1 => non-coherent integration */
  int32_t in_dtype;        /* fmcw_in_dtype */
  int32_t window;          /* fmcw_window, applied on both fast and slow time */
  int32_t mag_mode;        /* fmcw_mag_mode */
  int32_t map_kind;        /* fmcw_map_kind */
  int32_t cfar_kind;       /* fmcw_cfar_kind */
  int32_t mti_mode;        /* fmcw_mti_mode (mti_bypass port, radar_core.vhd:48) */
  /* 1-D OS-CFAR along Doppler (circular): rtl/old/os_cfar.vhd generics */
  uint32_t cfar1d_ref;     /* reference cells per side (REF_CELLS, 8) */
  uint32_t cfar1d_guard;   /* guard cells per side (GUARD_CELLS, 2) */
  uint32_t cfar1d_rank;    /* 0-based ascending rank k (RANK_IDX, 12) */
  float cfar1d_alpha;      /* threshold multiplier (SCALING_MULT/SCALING_DIV, 4) */
  /* 2-D OS-CFAR (rtl/src/os_cfar_2d.vhd), named by the axis each acts on (the RTL's
   * GUARD_RANGE=2 acts along Doppler, GUARD_DOPPLER=1 along range) */
  uint32_t cfar2d_ref_range;      /* 4 */
  uint32_t cfar2d_guard_range;    /* 1 */
  uint32_t cfar2d_ref_doppler;    /* 4 */
  uint32_t cfar2d_guard_doppler;  /* 2 */
  uint32_t cfar2d_rank_pct;       /* RANK_PCT 75 -> k = floor(n_ref*pct/100) */
  uint32_t cfar2d_scale_min;      /* SCALE_MIN 2 */
  uint32_t cfar2d_scale_nom;      /* SCALE_NOM 4 */
  uint32_t cfar2d_scale_max;      /* SCALE_MAX 6 */
  uint32_t cfar2d_scale_override; /* cfar_scale_ovr port; 0 = adaptive */
  /* resources */
  uint32_t max_frames;     /* largest n_frames per call (scratch is sized for it) */
  uint32_t chunk_frames;   /* frames per internal kernel chunk (0 = auto: a chunk's corner-turned
                            * spectrum within 208 MiB of the 256 MiB Infinity Cache, no rounding;
                            * 104 frames at 1024 x 256 fp32, 3 at 4096 x 512 x 4 rx or 8192 x 1024).
                            * Device memory of a handle: the chunk's spectrum (8 B per point), the
                            * detection scratch (det_capacity below: 16 B per record), and with the
                            * 2-D CFAR a chunk-sized linear map (4 B per cell) and candidate lists of
                            * 8 B per cell for min(max_frames, 16 + chunk, 2^32 cells) frames --
                            * 1.2 GiB at 8192 x 1024 with the auto chunk */
  int32_t device_id;       /* HIP device ordinal */
  /* RTL-compat arithmetic, a bitmask of fmcw_compat; 0 = the fp32 build spec */
  uint32_t compat_rtl;
  /* range FFT output scaled by 2^-range_shift (exact): the Xilinx IP's fixed scaling schedule
   * SCALE_SCH (tb_xfft_128.vhd:480-494), so that spectra fit the IP's 16-bit output word;
   * 0..13 */
  uint32_t range_shift;
  /* fmcw_spectrum_dtype: element type of the internal corner-turned spectrum */
  int32_t spectrum_dtype;
  /* Detection records the handle's scratch holds for one call.  0 (default): a slot of every
   * cell of each detection tile (16 B per cell of max_frames frames: 4 GiB at 1024 frames of
   * 1024 x 256), so no call can lose a detection at any density the CFAR parameters produce --
   * the reference emits every non-zero CFAR output (radar_core.vhd:413-418), and cfar_scale_ovr
   * = 1 or a 1-D alpha of 1 detect ~25 % of noise cells.  N > 0, for callers that bound det_cap:
   * slots of 1/32 of a tile's cells plus a shared region of N records for denser tiles; a call
   * then loses records (status word [1]) only when it finds more than N detections, i.e. never
   * while det_cap <= N would have room for the whole list.  max_frames x cells must stay below
   * 2^32 records. */
  uint32_t det_capacity;
} fmcw_config;

/* fmcw_config.spectrum_dtype.  FMCW_SPEC_F16 stores the corner-turned spectrum (K1 -> K2) as
 * fp16 pairs holding X / n_range: 4 instead of 8 bytes per point written and read back
 * (config 5: 160 -> 128 MiB of HBM traffic per frame).  The map then carries fp16 rounding of
 * the range spectrum: max |map - oracle| <= 2e-3 x max|oracle| per frame (tested), against
 * 1e-4 for FMCW_SPEC_F32; detections stay bit-exact to the oracle CFAR on the map produced.
 * Not with FMCW_COMPAT_MTI (its 16-bit words are defined on the fp32 spectrum).
 * FMCW_SPEC_S48 stores it in 6 bytes per point (config 2: 2 -> 1.5 MiB written and read back per
 * frame; configs 3 / 5: 64 -> 48 MiB, so the auto chunk holds 4 frames instead of 3): a group of
 * G chirps of a range bin (adjacent quads at n_range <= 512; chirps n_doppler / 16 apart at
 * n_range = 1024 (quads) and above (pairs)) shares one 8-bit exponent E (the largest of their 2G components is
 * < 2^E), and every component is a W-bit signed significand of 2^(E - W + 1), i.e. exact to 2^-W
 * of the group's largest component (fp32: 2^-24 of each) -- G = 4, W = 23 at n_range <= 1024;
 * G = 2, W = 22 above.  The map stays within the 1e-4 tolerance of FMCW_SPEC_F32 (per frame and
 * per bin above 1e-3 of the frame peak; tested).  Needs n_doppler >= 64, MTI off and a fp32
 * window. */
typedef enum { FMCW_SPEC_F32 = 0, FMCW_SPEC_F16 = 1, FMCW_SPEC_S48 = 2 } fmcw_spectrum_dtype;

/* fmcw_config.compat_rtl bits.
 * FMCW_COMPAT_CFAR: the CFAR on the RTL's 17-bit unsigned cells (DATA_WIDTH 17): each map
 *   cell enters the CFAR as q = min(floor(max(x, 0)), 2^17 - 1) (the map itself is unchanged).
 *   1-D (rtl/old/os_cfar.vhd:132-137): T = (ranked * alpha) mod 2^17 (resize to DATA_WIDTH),
 *   detect q_cut > T; alpha must be an integer (SCALING_MULT, SCALING_DIV = 1).
 *   2-D (rtl/src/os_cfar_2d.vhd:163, :189-213): mean = floor(sum / n_ref) of the integer refs,
 *   hi = (mean + (mean >> 1)) mod 2^17 (a 17-bit add), lo = mean >> 1, the same brackets,
 *   T = ranked * scale at full width.  fmcw_det.mag / .threshold carry q_cut and T.
 * FMCW_COMPAT_MTI: the MTI canceller on 16-bit words (rtl/src/doppler_notch.vhd:67-93): the
 *   (range_shift-scaled) spectrum is rounded half-to-even and saturated to int16 (the IP's
 *   output word, convergent rounding xfft_0.xci), then y = sat16(x - x1) or
 *   sat16(x - 2 x1 + x2) in integers.  Needs mti_mode != OFF. */
typedef enum { FMCW_COMPAT_CFAR = 1, FMCW_COMPAT_MTI = 2 } fmcw_compat;

/* One detection: 16 bytes, sorted by (frame, range, doppler). */
typedef struct fmcw_det {
  uint32_t frame;
  uint16_t range;
  uint16_t doppler;
  float mag;        /* CUT magnitude (det_tdata) */
  float threshold;  /* scale * ranked reference cell (dbg_threshold) */
} fmcw_det;

typedef struct fmcw_handle fmcw_handle;

/* Kernel ids for fmcw_kernel_times (profiling). */
typedef enum {
  FMCW_K_RANGE = 0,   /* window + range FFT + corner turn */
  FMCW_K_DOPPLER = 1, /* Doppler window + FFT + magnitude (+NCI) (+1-D CFAR) + map */
  FMCW_K_CFAR2D = 2,  /* 2-D OS-CFAR */
  FMCW_K_COMPACT = 3, /* detection list ordering */
  FMCW_K_COUNT = 4
} fmcw_kernel_id;

/* fmcw_get_info keys.  FMCW_INFO_CHUNK: frames per K1 -> K2 chunk.  FMCW_INFO_RANGE_KERNEL: the
 * range-stage kernel the handle runs: 0 k_range (T chirps per workgroup; every N, and the Q15 /
 * fp16-spectrum paths), 2 k_range_sq (two chirps one after the other through one chirp's LDS;
 * N = 4096), 3 k_range_px (as 2 with two LDS exchanges and a cross-lane last pass; N = 8192);
 * 1 (round 2's k_range2) is retired.  FMCW_INFO_WINDOW_SATURATIONS / FMCW_INFO_WORD_SATURATIONS:
 * status words 2 / 3 of the last fmcw_process call (fmcw_enqueue callers read them from
 * n_dets_dev).  FMCW_INFO_CFAR2D_STEPS: the strip length (workgroup steps) of the handle's last
 * 2-D CFAR launch (0 before the first). */
typedef enum { FMCW_INFO_CHUNK = 4, FMCW_INFO_RANGE_KERNEL = 6, FMCW_INFO_WINDOW_SATURATIONS = 7,
               FMCW_INFO_WORD_SATURATIONS = 8, FMCW_INFO_CFAR2D_STEPS = 9 } fmcw_info_key;

/* fmcw_set_param keys (tuning; results never depend on them).  FMCW_PARAM_CFAR2D_STEPS: steps
 * (4-wave-tile workgroup tiles) per 2-D CFAR strip, 0 = the library's cost model (default). */
typedef enum { FMCW_PARAM_CFAR2D_STEPS = 1 } fmcw_param_key;

/* Status words of fmcw_enqueue / fmcw_cfar (n_dets_dev). */
#define FMCW_STATUS_WORDS 4

/* Only the functions below are exported from libfmcw.so (built -fvisibility=hidden). */
#if defined(__GNUC__)
#pragma GCC visibility push(default)
#endif

const char* fmcw_version(void);
int fmcw_abi_version(void);
const char* fmcw_last_error(void);

/* Defaults = the reference core: N_RANGE 1024, N_DOPPLER 128, 1 rx, f32 in, Hamming,
 * |X|, linear map, 2-D OS-CFAR with radar_core.vhd:376-382 parameters. */
void fmcw_config_default(fmcw_config* cfg);

int fmcw_create(const fmcw_config* cfg, fmcw_handle** out);
int fmcw_destroy(fmcw_handle* h);

/* Full hot path on n_frames frames, device pointers, asynchronous on `stream`
 * (hipStream_t; NULL = default stream).  rd_map may be NULL.  dets may be NULL when
 * cfar_kind == NONE.  n_dets_dev points at FMCW_STATUS_WORDS device uint32 words, written by
 * the last kernel of every call that returns FMCW_OK (a call that returns an error may have
 * left them as the previous call wrote them); it may be NULL only when cfar_kind == NONE (then
 * no status):
 *   [0] detections found (may exceed det_cap; entries beyond det_cap are not written),
 *   [1] detections lost because the handle's detection scratch overflowed: only possible with
 *       cfg.det_capacity = N > 0 and more than N detections found (the default scratch holds
 *       every cell).  Non-zero means the list is incomplete; fmcw_process returns FMCW_EDETCAP
 *       then.  0xffffffff: the ordering pass could not complete (a safety net that bounds its
 *       wait; not expected), the whole list is void,
 *   [2] samples saturated by the RTL-compat integer windows (FMCW_WIN_Q15_RTL, either axis;
 *       win1 / win2 saturation_flag, window_multiplier.vhd:152-158),
 *   [3] samples whose int16 spectrum word or canceller output was clipped (FMCW_COMPAT_MTI or
 *       FMCW_WIN_Q15_RTL; doppler_notch.vhd:75-93).
 * [2] and [3] stay 0 on the fp32 build spec, which cannot saturate. */
int fmcw_enqueue(fmcw_handle* h, const void* cube, size_t n_frames, float* rd_map,
                 fmcw_det* dets, size_t det_cap, uint32_t* n_dets_dev, void* stream);

/* Synchronous convenience wrapper; pointers may be host or device memory. */
int fmcw_process(fmcw_handle* h, const void* cube, size_t n_frames, float* rd_map,
                 fmcw_det* dets, size_t det_cap, size_t* n_dets, void* stream);

/* Stage entry points (device pointers, asynchronous).
 * fmcw_cfar reads the map as the RTL's unsigned magnitude stream (magnitude_calc.vhd:45-88):
 * negative cells and -0.0 are taken as +0.  NaN cells are outside the specification (the RTL's
 * magnitudes are integers, and the sorting and counting forms of the OS-CFAR disagree on NaN):
 * a NaN reference never counts, and the 2-D CFAR's level screens (the reference window) take a
 * NaN CUT as below every level and screen it out, so whether a NaN CUT is reported is not
 * specified.  +Inf cells are supported. */
int fmcw_range_ct(fmcw_handle* h, const void* cube, size_t n_frames, void* spec, void* stream);
int fmcw_magnitude(const float* iq, float* out, size_t n, int mag_mode, void* stream);
int fmcw_cfar(fmcw_handle* h, const float* map, size_t n_frames, fmcw_det* dets,
              size_t det_cap, uint32_t* n_dets_dev, void* stream);

/* ---- Multi-GPU detection gather (RCCL over xGMI) ------------------------
 * The reference is one FPGA and has no distributed layer; this is the optional gather of
 * frame-sharded detection lists to one root rank.  One process per GPU.  Rank 0 makes the
 * id (fmcw_comm_unique_id), the caller distributes its FMCW_COMM_ID_BYTES bytes out of band,
 * every rank calls fmcw_comm_create (collective) with the SAME wire_cap (record slots per
 * rank message, 1..2^26; checked with one all-reduce there: FMCW_EINVAL if the ranks differ).
 * fmcw_gather_dets is stream-ordered, allocates nothing and never synchronises with the host:
 * every rank sends a fixed-size message (a 16-B header holding its count, then wire_cap record
 * slots) to `root` with ncclSend/ncclRecv, and the root compacts the lists on the device in
 * rank order (= global frame order for contiguous shards).  A rank sends min(n_dets_dev[0],
 * det_cap, wire_cap) records of dets_dev (det_cap = the capacity of dets_dev, as passed to
 * fmcw_enqueue), each .frame plus `frame_offset` (its first global frame).  On the root:
 * out_dev holds n_ranks * wire_cap records, out_n_dev[0] = records written, out_n_dev[1] =
 * records not sent (beyond det_cap or wire_cap, plus the ranks' n_dets_dev[1] scratch
 * losses).  Other ranks may pass NULL out pointers. */
#define FMCW_COMM_ID_BYTES 128
typedef struct fmcw_comm fmcw_comm;
int fmcw_comm_unique_id(void* id_out);
int fmcw_comm_create(const void* id, int n_ranks, int rank, int device_id, size_t wire_cap,
                     fmcw_comm** out);
int fmcw_comm_destroy(fmcw_comm* c);
/* What RCCL itself reports for the communicator (ncclCommCount / ncclCommUserRank /
 * ncclCommCuDevice), so that a multi-GPU run can show the collective really spans n_ranks GPUs;
 * wire_cap as created.  Any output pointer may be NULL. */
int fmcw_comm_info(const fmcw_comm* c, int* n_ranks, int* rank, int* device, size_t* wire_cap);
int fmcw_gather_dets(fmcw_comm* c, const fmcw_det* dets_dev, size_t det_cap,
                     const uint32_t* n_dets_dev, uint32_t frame_offset, fmcw_det* out_dev,
                     uint32_t* out_n_dev, int root, void* stream);
/* Test hooks of fmcw_comm_create's failure handling: fail_next_alloc makes the process's next
 * fmcw_comm_create treat its buffer allocation as failed (after ncclCommInitRank, before the
 * collective check, which every rank joins whatever failed locally); check_decide returns that
 * check's verdict on the all-reduced words h[3] = max over ranks of {wire_cap, ~wire_cap, failed}
 * (FMCW_ENOMEM if any rank failed, FMCW_EINVAL if wire_cap differs, else FMCW_OK). */
int fmcw_comm_fail_next_alloc_for_test(int enable);
int fmcw_comm_check_decide_for_test(const uint64_t* h, int local_fail, size_t wire_cap);
/* Single-GPU test hooks of the gather's device side (no RCCL): the rank-local pack into one
 * message of (1 + wire_cap) records, and the root's compaction of n_ranks such messages laid
 * end to end in msgs_dev. */
int fmcw_gather_pack_for_test(const fmcw_det* dets_dev, size_t det_cap, const uint32_t* n_dets_dev,
                              size_t wire_cap, uint32_t frame_offset, fmcw_det* msg_dev, void* stream);
int fmcw_gather_compact_for_test(const fmcw_det* msgs_dev, int n_ranks, size_t wire_cap,
                                 fmcw_det* out_dev, uint32_t* out_n_dev, void* stream);

/* Profiling: when enabled, every stage launch carries hipEvents on its stream that take the
 * dispatches' own begin / end timestamps (hipExtLaunchKernelGGL: the first launch of a stage
 * starts the event pair, its last one stops it); fmcw_kernel_times synchronises and returns, per
 * fmcw_kernel_id, the summed milliseconds and the number of stage launches since the last reset. */
int fmcw_set_profiling(fmcw_handle* h, int enable);
int fmcw_set_param(fmcw_handle* h, int key, int64_t value);
int fmcw_get_info(fmcw_handle* h, int key, int64_t* value);
int fmcw_kernel_times(fmcw_handle* h, double* ms, uint64_t* launches);
int fmcw_reset_kernel_times(fmcw_handle* h);

/* Scratch-free helpers so callers without a device allocator can use the library. */
int fmcw_device_alloc(size_t bytes, void** ptr, int device_id);
int fmcw_device_free(void* ptr);
int fmcw_memcpy(void* dst, const void* src, size_t bytes, int kind /*0 H2D,1 D2H,2 D2D*/);
int fmcw_device_count(int* n);

/* ---- Track-while-scan tracker (host side) ----------------------------------------------
 * Replaces rtl/src/tws_tracker.vhd (radar_core.vhd:424-438): MAX_TRACKS alpha-beta tracks in
 * Q2 bins with Q8 gains over the detection list, one scan (= one frame's detections) per
 * fmcw_tws_scan.  CPU code: serial, <= 64 detections x 64 tracks per scan.
 * rtl_compat = 1 is the VHDL bit for bit (wrapping field widths, the signal read of
 * best_distance in ASSOCIATE, the 6-bit detection counter); 0 is the intended tracker (wide
 * integers, nearest-neighbour association).  Output: firm and coasting tracks in track-file
 * order, as ST_OUTPUT streams them (:273-295); *n_out = their count (FMCW_EDETCAP if > cap). */
typedef struct fmcw_tws fmcw_tws;
typedef struct {
  uint32_t max_tracks;   /* MAX_TRACKS (32), <= 64 */
  uint32_t max_dets;     /* detections kept per scan (64, the RTL's MAX_DETS), <= 64 */
  uint32_t init_hits;    /* INIT_HITS (2) */
  uint32_t coast_max;    /* COAST_MAX (5) */
  uint32_t gate_r;       /* ASSOC_GATE_R (10 range bins) */
  uint32_t gate_d;       /* ASSOC_GATE_D (5 Doppler bins) */
  uint32_t alpha_q8;     /* ALPHA_GAIN (128 = 0.5), < 256 */
  uint32_t beta_q8;      /* BETA_GAIN (64 = 0.25), < 256 */
  int32_t rtl_compat;
} fmcw_tws_config;
typedef struct {
  uint16_t id;           /* trk_id: track-file slot */
  uint8_t status;        /* trk_status: 2 FIRM, 3 COAST */
  uint8_t quality;       /* trk_quality 0..15 */
  int32_t range_q2;      /* trk_range: range bin x 4 */
  int32_t doppler_q2;    /* trk_doppler: Doppler bin x 4 */
  int32_t vel_r;         /* trk_vel_r: Q2 range bins per scan */
  int32_t vel_d;         /* trk_vel_d */
  uint32_t last_mag;     /* last associated detection magnitude (rounded) */
  uint32_t age;          /* scans since initiation */
} fmcw_track;
void fmcw_tws_config_default(fmcw_tws_config* cfg);
int fmcw_tws_create(const fmcw_tws_config* cfg, fmcw_tws** out);
int fmcw_tws_destroy(fmcw_tws* t);
int fmcw_tws_scan(fmcw_tws* t, const fmcw_det* dets, size_t n_dets, fmcw_track* out, size_t cap,
                  size_t* n_out, uint32_t* n_active);

#if defined(__GNUC__)
#pragma GCC visibility pop
#endif

#ifdef __cplusplus
}
#endif
#endif /* FMCW_H_ */
