"""Multi-rank path on CPU: world_size-2 gloo processes exercise frame sharding and the
detection-list gather that bench.py runs over RCCL."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from fmcw.dist import shard_frames, gather_detections  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, frames_per_rank, counts, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = counts[rank]
        cap = max(counts) + 3
        rec = torch.zeros((cap, 4), dtype=torch.int32)
        for i in range(n):                          # local frame i % frames, range 10*rank + i
            rec[i, 0] = i % frames_per_rank
            rec[i, 1] = (10 * rank + i) | ((i % 7) << 16)    # range | doppler << 16
            rec[i, 2] = torch.tensor([float(rank + i)], dtype=torch.float32).view(torch.int32)
            rec[i, 3] = 0
        allr, got_counts = gather_detections(rec, n, frame_offset=rank * frames_per_rank)
        q.put((rank, got_counts, allr.numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("counts", [(5, 3), (0, 4), (0, 0), (6, 6)])
def test_gather_detections_gloo(counts):
    world, frames = 2, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, frames, counts, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda x: x[0])
    for rank, got_counts, allr in res:
        assert got_counts == list(counts)
        assert allr.shape == (sum(counts), 4)
        # ordered by rank = global frame blocks; frame ids offset by rank * frames
        off = 0
        for r, c in enumerate(counts):
            blk = allr[off: off + c]
            assert np.array_equal(blk[:, 0], np.arange(c) % frames + r * frames)
            assert np.array_equal(blk[:, 1] & 0xFFFF, 10 * r + np.arange(c))
            off += c
    assert np.array_equal(res[0][2], res[1][2])


def test_shard_frames_partition():
    for F in (1, 7, 8192):
        for G in (1, 2, 4, 8):
            blocks = [shard_frames(F, G, r) for r in range(G)]
            assert blocks[0][0] == 0 and blocks[-1][1] == F
            assert all(blocks[i][1] == blocks[i + 1][0] for i in range(G - 1))


def _worker_overfull(rank, world, port, q):
    import warnings
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rec = torch.arange(6 * 4, dtype=torch.int32).reshape(6, 4)
        # fmcw.h n_dets_dev: [0] found (beyond this 6-row buffer on rank 0), [1] lost in scratch
        nd = torch.tensor([9, 0] if rank == 0 else [2, 3], dtype=torch.int32)
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            allr, counts = gather_detections(rec, nd, frame_offset=0)
        q.put((rank, counts, allr.shape[0], len(w)))
    finally:
        dist.destroy_process_group()


def test_gather_clamps_to_the_buffer_and_warns():
    """a count beyond the buffer (or library-side losses) must neither crash the
    gather nor pass silently."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_overfull, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, counts, total, n_warn in res:
        assert counts == [6, 2] and total == 8
        assert n_warn == 1            # each rank warns about its own incomplete list
