"""Frame sharding across GPUs and the optional RCCL detection-list gather.

Frames are independent units: frame f of a batch of F goes to rank floor(f * G / F)
(contiguous blocks), each rank runs the whole hot path on its block with no data-path
collective.  The only exchange is the detection list.  Two implementations:

  RcclGather          the C-ABI gather of libfmcw.so (fmcw_gather_dets): every rank sends a
                      fixed-size message (count header + wire_cap records) to the root with
                      ncclSend/ncclRecv over xGMI, the root compacts on the device.  Stream-
                      ordered, no host synchronisation per step.  What bench.py uses at N > 1.
  gather_detections   torch.distributed: all_gather of the counts, then of the lists padded to
                      the largest count.  Works on any backend (gloo on CPU for the tests);
                      host-synchronising (the counts decide the padded size).

Records carry the global frame index (local frame + the rank's first frame).
The reference has no distributed layer (a single FPGA); this is the MI355X-side addition.
"""
from __future__ import annotations

import ctypes as C
import warnings

from . import _lib as L


def shard_frames(n_frames: int, world: int, rank: int):
    """Contiguous block of frames [lo, hi) for `rank`."""
    lo = (n_frames * rank) // world
    hi = (n_frames * (rank + 1)) // world
    return lo, hi


def gather_detections(dets, n_dets, frame_offset: int, group=None, dropped: int = 0):
    """Gather detection records from every rank (torch.distributed, any backend).

    dets:    uint8/int32 torch tensor holding fmcw_det 16-byte records (device or CPU)
    n_dets:  python int or tensor whose first element is this rank's count of detections
             found (fmcw.h n_dets_dev[0], which may exceed the buffer), and optionally
             second element the detections the library could not store (n_dets_dev[1])
    dropped: records lost upstream, if n_dets carries no second element
    Returns (all_records int32 [total, 4], counts list) on every rank, ordered by rank, i.e.
    by global frame because shards are contiguous.  A rank whose list is incomplete (count
    beyond its buffer, or library-side losses) contributes what it holds and a warning is
    raised, as fmcw_process reports FMCW_EDETCAP.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    dev = dets.device
    rec = dets.view(torch.int32).reshape(-1, 4)
    if hasattr(n_dets, "tolist"):
        v = n_dets.reshape(-1).tolist()
        found = int(v[0])
        lost = int(v[1]) if len(v) > 1 else int(dropped)
    else:
        found, lost = int(n_dets), int(dropped)
    n = min(found, rec.shape[0])
    if lost or n < found:
        warnings.warn(f"rank {dist.get_rank(group)}: detection list incomplete ({found} found, "
                      f"{rec.shape[0]} buffer rows, {lost} lost in the library scratch)")
    mine = rec[:n].clone()
    if frame_offset:
        mine[:, 0] += frame_offset                  # fmcw_det.frame is the first u32
    cnt = torch.tensor([n], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    counts = [int(c.item()) for c in counts]
    m = max(counts) if counts else 0
    if m == 0:
        return rec[:0].clone(), counts
    pad = torch.zeros((m, 4), dtype=torch.int32, device=dev)
    pad[:n] = mine
    outs = [torch.empty((m, 4), dtype=torch.int32, device=dev) for _ in range(world)]
    dist.all_gather(outs, pad, group=group)        # one ring all-gather (RCCL / gloo)
    return torch.cat([outs[r][:counts[r]] for r in range(world)]), counts


class RcclGather:
    """fmcw_comm_* / fmcw_gather_dets of include/fmcw.h: gather-to-root over RCCL.

    ``unique_id`` (FMCW_COMM_ID_BYTES bytes from ``RcclGather.make_id()`` on one rank) must be
    distributed out of band, e.g. with torch.distributed.broadcast_object_list."""

    def __init__(self, unique_id: bytes, n_ranks: int, rank: int, device: int, wire_cap: int):
        """wire_cap: record slots per rank message, the same on every rank (fmcw_comm_create
        checks it with one all-reduce)."""
        lib = L.load()
        if len(unique_id) != L.COMM_ID_BYTES:
            raise ValueError("unique id must be FMCW_COMM_ID_BYTES long")
        buf = C.create_string_buffer(bytes(unique_id), L.COMM_ID_BYTES)
        h = C.c_void_p()
        L.check(lib.fmcw_comm_create(buf, n_ranks, rank, device, wire_cap, C.byref(h)))
        self._h, self._lib = h, lib
        self.n_ranks, self.rank, self.wire_cap = n_ranks, rank, wire_cap

    @staticmethod
    def make_id() -> bytes:
        buf = C.create_string_buffer(L.COMM_ID_BYTES)
        L.check(L.load().fmcw_comm_unique_id(buf))
        return buf.raw

    def info(self) -> dict:
        """fmcw_comm_info: what RCCL reports for the communicator (ncclCommCount /
        ncclCommUserRank / ncclCommCuDevice) and its wire_cap."""
        n, r, d, w = C.c_int(), C.c_int(), C.c_int(), C.c_size_t()
        L.check(self._lib.fmcw_comm_info(self._h, C.byref(n), C.byref(r), C.byref(d), C.byref(w)))
        return {"rccl_ranks": n.value, "rccl_rank": r.value, "rccl_device": d.value, "wire_cap": w.value}

    def gather(self, dets_ptr: int, det_cap: int, n_dets_ptr: int, frame_offset: int,
               out_ptr: int | None, out_n_ptr: int | None, root: int = 0, stream: int = 0):
        """Device pointers; asynchronous on `stream`.  det_cap = the capacity of dets (as given to
        fmcw_enqueue).  On the root, out holds n_ranks * wire_cap records, out_n [0] records
        written, [1] records lost (beyond det_cap or wire_cap, or lost in a rank's scratch)."""
        L.check(self._lib.fmcw_gather_dets(self._h, dets_ptr, det_cap, n_dets_ptr, frame_offset,
                                           out_ptr, out_n_ptr, root, stream or None))

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            self._lib.fmcw_comm_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
