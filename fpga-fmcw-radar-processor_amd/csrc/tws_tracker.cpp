// tws_tracker.cpp -- host-side track-while-scan tracker over the detection lists (fmcw_tws_*).
//
// Replaces rtl/src/tws_tracker.vhd (instantiated at rtl/src/radar_core.vhd:424-438): a track
// file of MAX_TRACKS alpha-beta filters in Q2 range/Doppler bins with Q8 gains, run one scan
// at a time (COLLECT :130-141, PREDICT :143-156, ASSOCIATE :158-177, UPDATE :179-232,
// INITIATE :234-263, MAINTAIN :265-271, OUTPUT :273-295).  Serial and data-dependent over at
// most 64 detections x 32 tracks per scan, so it runs on the CPU after the detection list
// comes back (or after the RCCL gather): it is the consumer of the GPU path, not part of it.
//
// A scan here is one frame (the reference wiring ends a scan per range row).
// rtl_compat = 1 reproduces the VHDL bit for bit, including its quirks (field widths that
// wrap, numeric_std RESIZE truncation, the signal read of best_distance inside ASSOCIATE's
// loop, the 6-bit detection counter); rtl_compat = 0 is the intended tracker (wide integers,
// nearest-neighbour association).  oracle/tws_oracle.py restates both for the tests.
#include <cstdint>
#include <cstdlib>
#include <new>
#include <vector>

#include "../../include/fmcw.h"

namespace {

enum { T_FREE = 0, T_TENT = 1, T_FIRM = 2, T_COAST = 3 };

struct Trk {
  bool active = false;
  int status = T_FREE;
  int64_t range_pos = 0, dopp_pos = 0, range_vel = 0, dopp_vel = 0;
  uint32_t hit = 0, miss = 0, quality = 0, age = 0, last_mag = 0;
};

struct Det {
  int64_t r, d;
  uint32_t mag;
  bool valid, assoc;
};

int64_t wrap(int64_t x, int n) {  // n-bit two's complement
  const uint64_t m = (uint64_t)1 << n;
  uint64_t u = (uint64_t)x & (m - 1);
  return u >= (m >> 1) ? (int64_t)u - (int64_t)m : (int64_t)u;
}
int64_t resize_s(int64_t x, int n) {  // numeric_std RESIZE(signed) shrink: sign + low n-1 bits
  const int64_t low = x & (((int64_t)1 << (n - 1)) - 1);
  return x < 0 ? low - ((int64_t)1 << (n - 1)) : low;
}
int64_t floor_shr8(int64_t x) { return x >= 0 ? x >> 8 : -((-x + 255) >> 8); }  // shift_right(signed, 8)

}  // namespace

struct fmcw_tws {
  fmcw_tws_config cfg{};
  std::vector<Trk> trk;
  uint32_t best_distance = 0xFFFF;  // power-up value; not reset by aresetn (tws_tracker.vhd:92-93)
  uint32_t best_idx = 63;

  int64_t w(int64_t x, int n) const { return cfg.rtl_compat ? wrap(x, n) : x; }
  int64_t rs(int64_t x, int n) const { return cfg.rtl_compat ? resize_s(x, n) : x; }
  uint32_t u(uint64_t x, int n) const { return cfg.rtl_compat ? (uint32_t)(x & ((1ull << n) - 1)) : (uint32_t)x; }
};

extern "C" {

void fmcw_tws_config_default(fmcw_tws_config* c) {
  if (!c) return;
  // radar_core's u_tws generics (radar_core.vhd:424-432; tws_tracker.vhd:11-19)
  c->max_tracks = 32;
  c->max_dets = 64;
  c->init_hits = 2;
  c->coast_max = 5;
  c->gate_r = 10;
  c->gate_d = 5;
  c->alpha_q8 = 128;
  c->beta_q8 = 64;
  c->rtl_compat = 0;
}

int fmcw_tws_create(const fmcw_tws_config* cfg, fmcw_tws** out) {
  if (!cfg || !out) return FMCW_EINVAL;
  *out = nullptr;
  if (cfg->max_tracks < 1 || cfg->max_tracks > 64 || cfg->max_dets < 1 || cfg->max_dets > 64 ||
      cfg->alpha_q8 > 255 || cfg->beta_q8 > 255 || cfg->gate_r > 4096 || cfg->gate_d > 4096)
    return FMCW_EINVAL;  // 6-bit track id and det index (:67-75), 9-bit signed gain operand
  fmcw_tws* t = new (std::nothrow) fmcw_tws;
  if (!t) return FMCW_ENOMEM;
  t->cfg = *cfg;
  t->trk.assign(cfg->max_tracks, Trk{});
  *out = t;
  return FMCW_OK;
}

int fmcw_tws_destroy(fmcw_tws* t) {
  delete t;
  return FMCW_OK;
}

int fmcw_tws_scan(fmcw_tws* t, const fmcw_det* dets, size_t n_dets, fmcw_track* out, size_t cap,
                  size_t* n_out, uint32_t* n_active) {
  if (!t || (n_dets && !dets) || (cap && !out)) return FMCW_EINVAL;
  const fmcw_tws_config& c = t->cfg;
  const bool rtl = c.rtl_compat != 0;

  // ST_COLLECT: the RTL's 6-bit counter admits every detection (det_count < 64 always holds)
  // and wraps, so the 65th overwrites slot 0; the intended tracker keeps the first max_dets.
  std::vector<Det> buf(64, Det{0, 0, 0, false, false});
  uint32_t det_count = 0;
  for (size_t i = 0; i < n_dets; ++i) {
    if (!rtl && det_count >= c.max_dets) break;
    if (rtl && det_count >= c.max_dets) continue;
    const float m = dets[i].mag;
    const uint64_t mi = m <= 0.f ? 0 : m >= 4.0e9f ? 0xFFFFFFFFull : (uint64_t)(m + 0.5f);
    buf[det_count] = Det{(int64_t)t->u(dets[i].range, 10), (int64_t)t->u(dets[i].doppler, 7), t->u(mi, 17),
                         true, false};
    det_count = rtl ? (det_count + 1) & 63 : det_count + 1;
  }

  // ST_PREDICT
  for (Trk& k : t->trk)
    if (k.active) {
      k.range_pos = t->w(k.range_pos + k.range_vel, 12);
      k.dopp_pos = t->w(k.dopp_pos + k.dopp_vel, 9);
      k.age = t->u((uint64_t)k.age + 1, 8);
    }

  // ST_ASSOCIATE + ST_UPDATE, track by track
  for (Trk& k : t->trk) {
    if (!k.active) continue;
    bool hit = false;
    uint32_t bi = 0;
    if (rtl) {
      // best_distance is a signal: every compare in the loop reads the previous track's value
      // and the last qualifying detection wins (tws_tracker.vhd:160-177)
      const uint32_t b_old = t->best_distance;
      uint32_t bd = 0xFFFF;
      bi = 63;
      for (uint32_t i = 0; i < 64; ++i) {
        const Det& e = buf[i];
        if (!e.valid || e.assoc) continue;
        const int64_t dr = std::llabs(k.range_pos - ((e.r << 2) & 0xFFF));
        const int64_t dd = std::llabs(k.dopp_pos - ((e.d << 2) & 0x1FF));
        if (dr < (int64_t)c.gate_r * 4 && dd < (int64_t)c.gate_d * 4) {
          const uint32_t dist = (uint32_t)((dr + dd) & 0xFFFF);
          if (dist < b_old) {
            bd = dist;
            bi = i;
          }
        }
      }
      t->best_distance = bd;
      t->best_idx = bi;
      hit = bi < c.max_dets && bd < 0xFFFF;
    } else {
      int64_t bd = -1;
      for (uint32_t i = 0; i < det_count; ++i) {
        const Det& e = buf[i];
        if (e.assoc) continue;
        const int64_t dr = std::llabs(k.range_pos - 4 * e.r), dd = std::llabs(k.dopp_pos - 4 * e.d);
        if (dr < (int64_t)c.gate_r * 4 && dd < (int64_t)c.gate_d * 4 && (bd < 0 || dr + dd < bd)) {
          bd = dr + dd;
          bi = i;
        }
      }
      hit = bd >= 0;
    }
    if (hit) {
      Det& e = buf[bi];
      e.assoc = true;
      const int64_t ir = t->w(t->w(4 * e.r, 12) - k.range_pos, 12);
      const int64_t id = t->w(t->w(4 * e.d, 9) - k.dopp_pos, 9);
      const uint32_t old_hit = k.hit;
      const int old_status = k.status;
      k.range_pos = t->w(k.range_pos + t->rs(floor_shr8(ir * c.alpha_q8), 12), 12);
      k.dopp_pos = t->w(k.dopp_pos + t->rs(floor_shr8(id * c.alpha_q8), 9), 9);
      k.range_vel = t->w(k.range_vel + t->rs(floor_shr8(ir * c.beta_q8), 10), 10);
      k.dopp_vel = t->w(k.dopp_vel + t->rs(floor_shr8(id * c.beta_q8), 8), 8);
      k.hit = t->u((uint64_t)old_hit + 1, 4);
      k.miss = 0;
      k.last_mag = e.mag;
      if (old_status == T_TENT && old_hit >= c.init_hits) k.status = T_FIRM;
      else if (old_status == T_COAST) k.status = T_FIRM;
      if (k.quality < 15) ++k.quality;
    } else {
      const uint32_t old_miss = k.miss;
      k.miss = t->u((uint64_t)old_miss + 1, 4);
      if (k.status == T_FIRM) k.status = T_COAST;
      if (old_miss >= c.coast_max) {
        k.active = false;
        k.status = T_FREE;
      }
      if (k.quality > 0) --k.quality;
    }
  }

  // ST_INITIATE over detection indices 0 .. det_count-1 (RTL: index 0 even at count 0, :259)
  const uint32_t n_init = (rtl && det_count == 0) ? 1 : det_count;
  for (uint32_t i = 0; i < n_init; ++i) {
    const Det& e = buf[i];
    if (!e.valid || e.assoc) continue;
    for (Trk& k : t->trk)
      if (!k.active) {
        k = Trk{};
        k.active = true;
        k.status = T_TENT;
        k.range_pos = t->w(4 * e.r, 12);
        k.dopp_pos = t->w(4 * e.d, 9);
        k.hit = 1;
        k.quality = 1;
        k.last_mag = e.mag;
        break;
      }
  }

  // ST_MAINTAIN + ST_OUTPUT: firm and coasting tracks in track-file order
  uint32_t active = 0;
  size_t n = 0;
  for (uint32_t i = 0; i < t->trk.size(); ++i) {
    const Trk& k = t->trk[i];
    if (!k.active) continue;
    ++active;
    if (k.status != T_FIRM && k.status != T_COAST) continue;
    if (n < cap) {
      fmcw_track& o = out[n];
      o.id = (uint16_t)i;
      o.status = (uint8_t)k.status;
      o.quality = (uint8_t)k.quality;
      o.range_q2 = (int32_t)k.range_pos;
      o.doppler_q2 = (int32_t)k.dopp_pos;
      o.vel_r = (int32_t)k.range_vel;
      o.vel_d = (int32_t)k.dopp_vel;
      o.last_mag = k.last_mag;
      o.age = k.age;
    }
    ++n;
  }
  if (n_out) *n_out = n;
  if (n_active) *n_active = active;
  return n > cap ? FMCW_EDETCAP : FMCW_OK;
}

}  // extern "C"
