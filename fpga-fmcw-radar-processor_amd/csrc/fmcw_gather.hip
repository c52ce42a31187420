// fmcw_gather.hip -- the optional multi-GPU detection-list gather of include/fmcw.h
// (SURVEY.md 8e): frame-sharded ranks send their ordered lists to one root over RCCL
// (point-to-point over xGMI), and the root compacts them on the device.
//
// The reference is a single FPGA with no distributed layer; this replaces
// nothing in it.  Wire format per rank: one 16-B header record (n found, n lost, 0, 0) and
// `wire_cap` fmcw_det slots.  The message size is fixed, so no rank ever needs another
// rank's count on the host: the whole gather is stream-ordered (pack -> ncclGroupStart /
// ncclSend / ncclRecv / ncclGroupEnd -> compact) and never synchronises with the CPU.
// At config 4 (1024 frames per GPU, ~64 detections per frame) a 128-per-frame wire_cap is
// 2 MiB per rank: tens of microseconds on one 64 GB/s xGMI link, beside a 1.4 ms step.
// wire_cap is part of the communicator (fmcw_comm_create, checked equal on every rank there),
// so the send and receive sizes always match and the gather allocates nothing.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>

#include "../../include/fmcw.h"

int fmcw_internal_fail(int code, const char* msg);  // fmcw_api.hip: sets fmcw_last_error()

namespace {

int gfail(int code, const char* fmt, ...) {
  char b[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(b, sizeof b, fmt, ap);
  va_end(ap);
  return fmcw_internal_fail(code, b);
}

// rank-local: header + min(found, det_cap, wire_cap) records with the frame offset applied.
// n_dets[0] may exceed det_cap (fmcw_enqueue writes at most det_cap records), so the records
// past det_cap are never read: they count as lost, with the scratch losses n_dets[1].
__global__ void k_gather_pack(const fmcw_det* __restrict__ dets, uint32_t det_cap, const uint32_t* __restrict__ n_dets,
                              uint32_t wire_cap, uint32_t frame_offset, fmcw_det* __restrict__ wire) {
  const uint32_t found = n_dets[0], lost_scratch = n_dets[1];
  const uint32_t n = min(found, min(det_cap, wire_cap));
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) {
    uint32_t* hdr = reinterpret_cast<uint32_t*>(wire);
    hdr[0] = n;
    hdr[1] = (found - n) + lost_scratch;
    hdr[2] = 0;
    hdr[3] = 0;
  }
  for (uint32_t k = i; k < n; k += gridDim.x * blockDim.x) {
    fmcw_det d = dets[k];
    d.frame += frame_offset;
    wire[1 + k] = d;
  }
}

// root: exclusive scan of the ranks' counts (one wave; n_ranks <= 64), then every rank's
// records in rank order
__global__ void __launch_bounds__(256) k_gather_compact(const fmcw_det* __restrict__ recv, int n_ranks,
                                                        uint32_t wire_cap, fmcw_det* __restrict__ out,
                                                        uint32_t* __restrict__ out_n) {
  __shared__ uint32_t s_off[65], s_cnt[64];
  const int tid = threadIdx.x;
  if (tid < 64) {
    const uint32_t* hdr = reinterpret_cast<const uint32_t*>(recv + (size_t)tid * (1 + wire_cap));
    const uint32_t c = tid < n_ranks ? min(hdr[0], wire_cap) : 0u, l = tid < n_ranks ? hdr[1] : 0u;
    uint32_t x = c, lx = l;
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d, 64), ly = __shfl_up(lx, d, 64);
      if (tid >= d) {
        x += y;
        lx += ly;
      }
    }
    s_off[tid] = x - c;
    s_cnt[tid] = c;
    if (tid == 63) {
      s_off[64] = x;
      if (blockIdx.x == 0) {
        out_n[0] = x;
        out_n[1] = lx;
      }
    }
  }
  __syncthreads();
  for (int r = 0; r < n_ranks; ++r) {
    const fmcw_det* src = recv + (size_t)r * (1 + wire_cap) + 1;
    fmcw_det* dst = out + s_off[r];
    for (uint32_t k = blockIdx.x * blockDim.x + tid; k < s_cnt[r]; k += gridDim.x * blockDim.x) dst[k] = src[k];
  }
}

// fmcw_comm_create's collective check: 3 words, all-reduced with max over the ranks (wire_cap,
// ~wire_cap, any rank's allocation failure).  A static device array, so that no rank can fail to
// obtain it and skip the collective its peers wait in.
// One lock per device (the array has one instance per device): two ranks of one process on
// different GPUs (a thread each) then never wait on each other's collective.
__device__ uint64_t g_check[3];
constexpr int kMaxCommDevices = 64;
std::mutex g_check_mu[kMaxCommDevices];
bool g_fail_next_alloc = false;  // fmcw_comm_fail_next_alloc_for_test

// The verdict of the check, the same on every rank: the all-reduced words h (or this rank's own,
// n_ranks == 1) against this rank's wire_cap and allocation result.
int comm_check_decide(const uint64_t (&h)[3], bool local_fail, size_t wire_cap, size_t msg) {
  if (h[2])
    return local_fail ? gfail(FMCW_ENOMEM, "gather buffers (%zu B per rank) failed", msg)
                      : gfail(FMCW_ENOMEM, "gather buffers failed on another rank");
  if (h[0] != wire_cap || ~h[1] != wire_cap)
    return gfail(FMCW_EINVAL, "wire_cap differs between ranks (this rank %zu, max %llu, min %llu)", wire_cap,
                 (unsigned long long)h[0], (unsigned long long)~h[1]);
  return FMCW_OK;
}

}  // namespace

struct fmcw_comm {
  ncclComm_t comm = nullptr;
  int n_ranks = 0, rank = 0, device_id = 0;
  fmcw_det* wire = nullptr;   // this rank's outgoing message
  fmcw_det* recv = nullptr;   // root: n_ranks messages
  size_t wire_cap = 0;        // record slots per rank message (equal on every rank)
};

extern "C" {

int fmcw_comm_unique_id(void* id_out) {
  if (!id_out) return gfail(FMCW_EINVAL, "null id");
  static_assert(sizeof(ncclUniqueId) == FMCW_COMM_ID_BYTES, "RCCL unique id size");
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return gfail(FMCW_EHIP, "ncclGetUniqueId: %s", ncclGetErrorString(r));
  std::memcpy(id_out, &id, sizeof id);
  return FMCW_OK;
}

int fmcw_comm_create(const void* id, int n_ranks, int rank, int device_id, size_t wire_cap, fmcw_comm** out) {
  if (!id || !out) return gfail(FMCW_EINVAL, "null argument");
  *out = nullptr;
  if (n_ranks < 1 || n_ranks > 64 || rank < 0 || rank >= n_ranks)
    return gfail(FMCW_EINVAL, "rank %d of %d (1..64 ranks)", rank, n_ranks);
  if (wire_cap < 1 || wire_cap > (1u << 26)) return gfail(FMCW_EINVAL, "wire_cap %zu (1..2^26)", wire_cap);
  if (device_id < 0 || device_id >= kMaxCommDevices) return gfail(FMCW_EINVAL, "device_id %d (0..63)", device_id);
  if (hipSetDevice(device_id) != hipSuccess) {
    (void)hipGetLastError();
    return gfail(FMCW_ENODEV, "device_id %d", device_id);
  }
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof uid);
  fmcw_comm* c = new fmcw_comm();
  c->n_ranks = n_ranks;
  c->rank = rank;
  c->device_id = device_id;
  c->wire_cap = wire_cap;
  const ncclResult_t r = ncclCommInitRank(&c->comm, n_ranks, uid, rank);
  if (r != ncclSuccess) {
    delete c;
    return gfail(FMCW_EHIP, "ncclCommInitRank: %s", ncclGetErrorString(r));
  }
  const size_t msg = (1 + wire_cap) * sizeof(fmcw_det);
  // A failed buffer allocation is not returned at once: every rank still joins the one all-reduce
  // below (with a failure flag), so a local failure fails the whole job instead of hanging the
  // other ranks in their all-reduce.  Nothing before that collective can fail alone: the check
  // words are a static device array (no allocation), and the allocations only set the flag.
  bool local_fail = g_fail_next_alloc;
  g_fail_next_alloc = false;
  if (!local_fail && (hipMalloc(reinterpret_cast<void**>(&c->wire), msg) != hipSuccess ||
                      hipMalloc(reinterpret_cast<void**>(&c->recv), msg * (size_t)n_ranks) != hipSuccess)) {
    (void)hipGetLastError();
    local_fail = true;
  }
  uint64_t h[3] = {(uint64_t)wire_cap, ~(uint64_t)wire_cap, local_fail ? 1u : 0u};  // max: max, ~min, any failed
  if (n_ranks > 1) {
    // every rank must size its message alike (send / recv sizes match) and have its buffers: one
    // collective check here, the only host synchronisation of the communicator's life
    std::lock_guard<std::mutex> lk(g_check_mu[device_id]);  // this device's static check array
    void* v = nullptr;
    ncclResult_t rr = ncclSuccess;
    bool ok = hipGetSymbolAddress(&v, HIP_SYMBOL(g_check)) == hipSuccess;
    if (!ok) {
      // no check word: abort the communicator so that the peers' all-reduce fails rather than waits
      (void)hipGetLastError();
      ncclCommAbort(c->comm);
      c->comm = nullptr;
      fmcw_comm_destroy(c);
      return gfail(FMCW_EHIP, "gather check word: hipGetSymbolAddress failed (communicator aborted)");
    }
    ok = hipMemcpy(v, h, sizeof h, hipMemcpyHostToDevice) == hipSuccess;
    if (!ok) {  // the same: never leave the peers waiting in the collective
      (void)hipGetLastError();
      ncclCommAbort(c->comm);
      c->comm = nullptr;
      fmcw_comm_destroy(c);
      return gfail(FMCW_EHIP, "gather check word: upload failed (communicator aborted)");
    }
    ok = (rr = ncclAllReduce(v, v, 3, ncclUint64, ncclMax, c->comm, nullptr)) == ncclSuccess &&
         hipMemcpy(h, v, sizeof h, hipMemcpyDeviceToHost) == hipSuccess;
    if (!ok) {
      (void)hipGetLastError();
      fmcw_comm_destroy(c);
      return gfail(FMCW_EHIP, "gather check (all-reduce): %s", ncclGetErrorString(rr));
    }
  }
  const int rc = comm_check_decide(h, local_fail, wire_cap, msg);
  if (rc != FMCW_OK) {
    fmcw_comm_destroy(c);
    return rc;
  }
  *out = c;
  return FMCW_OK;
}

int fmcw_comm_destroy(fmcw_comm* c) {
  if (!c) return FMCW_OK;
  hipSetDevice(c->device_id);
  if (c->comm) ncclCommDestroy(c->comm);
  if (c->wire) hipFree(c->wire);
  if (c->recv) hipFree(c->recv);
  delete c;
  return FMCW_OK;
}

int fmcw_comm_info(const fmcw_comm* c, int* n_ranks, int* rank, int* device, size_t* wire_cap) {
  if (!c || !c->comm) return gfail(FMCW_EINVAL, "null communicator");
  int n = 0, r = 0, d = 0;
  ncclResult_t e = ncclCommCount(c->comm, &n);
  if (e == ncclSuccess) e = ncclCommUserRank(c->comm, &r);
  if (e == ncclSuccess) e = ncclCommCuDevice(c->comm, &d);
  if (e != ncclSuccess) return gfail(FMCW_EHIP, "RCCL communicator query: %s", ncclGetErrorString(e));
  if (n_ranks) *n_ranks = n;
  if (rank) *rank = r;
  if (device) *device = d;
  if (wire_cap) *wire_cap = c->wire_cap;
  return FMCW_OK;
}

int fmcw_gather_dets(fmcw_comm* c, const fmcw_det* dets_dev, size_t det_cap, const uint32_t* n_dets_dev,
                     uint32_t frame_offset, fmcw_det* out_dev, uint32_t* out_n_dev, int root, void* stream) {
  if (!c || !dets_dev || !n_dets_dev) return gfail(FMCW_EINVAL, "null argument");
  if (root < 0 || root >= c->n_ranks) return gfail(FMCW_EINVAL, "root %d of %d ranks", root, c->n_ranks);
  if (c->rank == root && (!out_dev || !out_n_dev)) return gfail(FMCW_EINVAL, "root needs out_dev and out_n_dev");
  if (hipSetDevice(c->device_id) != hipSuccess) return gfail(FMCW_EHIP, "hipSetDevice");
  const size_t wire_cap = c->wire_cap;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const size_t msg = (1 + wire_cap) * sizeof(fmcw_det);
  const int pack_blocks = (int)std::min<size_t>(1024, (wire_cap + 255) / 256);
  hipLaunchKernelGGL(k_gather_pack, dim3(pack_blocks), dim3(256), 0, s, dets_dev,
                     (uint32_t)std::min<size_t>(det_cap, 0xffffffffu), n_dets_dev, (uint32_t)wire_cap, frame_offset,
                     c->wire);
  if (hipGetLastError() != hipSuccess) return gfail(FMCW_EHIP, "k_gather_pack launch");
  if (c->rank == root) {
    if (hipMemcpyAsync(reinterpret_cast<char*>(c->recv) + (size_t)root * msg, c->wire, msg, hipMemcpyDeviceToDevice,
                       s) != hipSuccess)
      return gfail(FMCW_EHIP, "root self copy");
  }
  if (c->n_ranks > 1) {
    ncclResult_t r = ncclGroupStart();
    if (c->rank == root) {
      for (int p = 0; p < c->n_ranks && r == ncclSuccess; ++p)
        if (p != root) r = ncclRecv(reinterpret_cast<char*>(c->recv) + (size_t)p * msg, msg, ncclUint8, p, c->comm, s);
    } else if (r == ncclSuccess) {
      r = ncclSend(c->wire, msg, ncclUint8, root, c->comm, s);
    }
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess)
      return gfail(FMCW_EHIP, "RCCL send/recv: %s", ncclGetErrorString(r != ncclSuccess ? r : r2));
  }
  if (c->rank == root) {
    const int blocks = (int)std::min<size_t>(256, (wire_cap + 255) / 256);
    hipLaunchKernelGGL(k_gather_compact, dim3(blocks), dim3(256), 0, s, c->recv, c->n_ranks, (uint32_t)wire_cap,
                       out_dev, out_n_dev);
    if (hipGetLastError() != hipSuccess) return gfail(FMCW_EHIP, "k_gather_compact launch");
  }
  return FMCW_OK;
}

// Test hooks of fmcw_comm_create's failure handling.  fail_next_alloc: the calling process's next
// fmcw_comm_create takes its buffer allocation as failed (after ncclCommInitRank, before the
// collective check).  check_decide: the check's verdict on all-reduced words `h` (max over the
// ranks of {wire_cap, ~wire_cap, failed}), so a CPU-side multi-rank test can all-reduce the words
// with another backend and see every rank return the same error.
int fmcw_comm_fail_next_alloc_for_test(int enable) {
  g_fail_next_alloc = enable != 0;
  return FMCW_OK;
}

int fmcw_comm_check_decide_for_test(const uint64_t* h, int local_fail, size_t wire_cap) {
  if (!h) return gfail(FMCW_EINVAL, "null argument");
  const uint64_t w[3] = {h[0], h[1], h[2]};
  return comm_check_decide(w, local_fail != 0, wire_cap, (1 + wire_cap) * sizeof(fmcw_det));
}

// Single-process test hooks: the pack and compaction kernels without RCCL, so one GPU can check
// N ranks' messages (counts 0, small, over wire_cap, with losses) against a host model.
int fmcw_gather_pack_for_test(const fmcw_det* dets_dev, size_t det_cap, const uint32_t* n_dets_dev,
                              size_t wire_cap, uint32_t frame_offset, fmcw_det* msg_dev, void* stream) {
  if (!dets_dev || !n_dets_dev || !msg_dev || wire_cap < 1 || wire_cap > (1u << 26))
    return gfail(FMCW_EINVAL, "null argument or wire_cap out of 1..2^26");
  const int pack_blocks = (int)std::min<size_t>(1024, (wire_cap + 255) / 256);
  hipLaunchKernelGGL(k_gather_pack, dim3(pack_blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), dets_dev,
                     (uint32_t)std::min<size_t>(det_cap, 0xffffffffu), n_dets_dev, (uint32_t)wire_cap, frame_offset,
                     msg_dev);
  if (hipGetLastError() != hipSuccess) return gfail(FMCW_EHIP, "k_gather_pack launch");
  return FMCW_OK;
}

int fmcw_gather_compact_for_test(const fmcw_det* msgs_dev, int n_ranks, size_t wire_cap, fmcw_det* out_dev,
                                 uint32_t* out_n_dev, void* stream) {
  if (!msgs_dev || !out_dev || !out_n_dev || n_ranks < 1 || n_ranks > 64 || wire_cap < 1 || wire_cap > (1u << 26))
    return gfail(FMCW_EINVAL, "null argument, n_ranks out of 1..64 or wire_cap out of 1..2^26");
  const int blocks = (int)std::min<size_t>(256, (wire_cap + 255) / 256);
  hipLaunchKernelGGL(k_gather_compact, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), msgs_dev,
                     n_ranks, (uint32_t)wire_cap, out_dev, out_n_dev);
  if (hipGetLastError() != hipSuccess) return gfail(FMCW_EHIP, "k_gather_compact launch");
  return FMCW_OK;
}

}  // extern "C"
