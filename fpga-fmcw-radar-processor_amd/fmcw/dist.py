"""Frame sharding across GPUs and the optional RCCL detection-list gather.

Frames are independent units: frame f of a batch of F goes to rank floor(f * G / F)
(contiguous blocks), each rank runs the whole hot path on its block with no data-path
collective.  The only exchange is the detection list, gathered to every rank (or rank 0)
over RCCL (torch.distributed backend "nccl" on ROCm) in two steps:
  1. all_gather of the per-rank counts (G x 8 B);
  2. all_gather_into_tensor of the lists padded to the largest count (16 B records).
Records carry the global frame index (local frame + the rank's first frame).
The reference has no distributed layer (a single FPGA); this is the MI355X-side addition.
"""
from __future__ import annotations


def shard_frames(n_frames: int, world: int, rank: int):
    """Contiguous block of frames [lo, hi) for `rank`."""
    lo = (n_frames * rank) // world
    hi = (n_frames * (rank + 1)) // world
    return lo, hi


def gather_detections(dets, n_dets, frame_offset: int, group=None):
    """Gather detection records from every rank.

    dets:    uint8/int32 torch tensor holding >= n_dets 16-byte fmcw_det records (device or CPU)
    n_dets:  python int or 1-element tensor with this rank's count
    Returns (all_records int32 [total, 4], counts list) on every rank, ordered by rank, i.e.
    by global frame because shards are contiguous.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    dev = dets.device
    rec = dets.view(torch.int32).reshape(-1, 4)
    n = int(n_dets.item()) if hasattr(n_dets, "item") else int(n_dets)
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
