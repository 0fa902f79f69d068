"""Data-parallel sharding + result gather (yolo_hip.dist) on CPU with gloo, world size 2.

Each rank takes its contiguous shard of a global batch, produces per-image
detections (here with the CPU oracle NMS standing in for the device kernel -
the device NMS itself is pinned against the same oracle in test_gpu_nms.py),
packs them and gathers to rank 0, which must recover exactly the detections of
the whole batch in image order, as the reference's single-process
non_max_suppression (utils/util.py:123-169) would return them.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from yolo_hip import dist
from yolo_hip.synth import synth_head_output

MAX_DET = 300
TOTAL = 5   # ragged on purpose: shards of 3 and 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batch_detections(lo, hi):
    from oracle import nms as onms
    y = np.stack([synth_head_output(anchors=600, nc=8, seed=i).numpy() for i in range(lo, hi)])
    kept = onms.non_max_suppression(y)
    dets = torch.zeros((hi - lo, MAX_DET, 6), dtype=torch.float32)
    counts = torch.zeros((hi - lo,), dtype=torch.int32)
    for i, k in enumerate(kept):
        dets[i, :len(k)] = torch.from_numpy(np.asarray(k, dtype=np.float32))
        counts[i] = len(k)
    return dets, counts


def _worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = dist.shard(TOTAL, rank, world)
        big = dist.shard(TOTAL, 0, world)[1]  # largest shard (rank 0 gets the ceil share)
        dets, counts = _batch_detections(lo, hi)
        if hi - lo < big:  # pad the ragged shard so the collective is uniform
            dets = torch.cat((dets, torch.zeros((big - (hi - lo), MAX_DET, 6))))
            counts = torch.cat((counts, torch.zeros((big - (hi - lo),), dtype=torch.int32)))
        g = dist.Gather(big, MAX_DET, "cpu", rank, world)
        got = g(dets, counts)
        if rank == 0:
            flat = g.detections(got, total=TOTAL)
            torch.save([t.clone() for t in flat], out_path)
    finally:
        torch.distributed.destroy_process_group()


def _worker_pipelined(rank, world, port, out_path):
    """Two batches gathered back to back (as DetectPipeline queues them) before batch 0 is read."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        per = 2
        g = dist.Gather(per, MAX_DET, "cpu", rank, world, slots=2)
        got = []
        for k in range(2):   # batch k covers global images [k*per*world, (k+1)*per*world)
            lo = k * per * world + rank * per
            dets, counts = _batch_detections(lo, lo + per)
            got.append(g(dets, counts))
        if rank == 0:
            torch.save([[t.clone() for t in g.detections(r)] for r in got], out_path)
    finally:
        torch.distributed.destroy_process_group()


def test_shard_covers_every_image_once():
    for total in (0, 1, 7, 32, 256, 257):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                lo, hi = dist.shard(total, r, world)
                assert 0 <= hi - lo <= -(-total // world)
                seen.extend(range(lo, hi))
            assert seen == list(range(total))
    with pytest.raises(ValueError):
        dist.shard(4, 2, 2)


def test_pack_roundtrip():
    dets, counts = _batch_detections(0, 2)
    back = dist.unpack(dist.pack(dets, counts), MAX_DET)
    for i in range(2):
        assert torch.equal(back[i], dets[i, :counts[i]])


def test_gather_world2_gloo(tmp_path):
    out = str(tmp_path / "dets.pt")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    want_d, want_c = _batch_detections(0, TOTAL)
    assert len(got) == TOTAL
    for i in range(TOTAL):
        assert torch.equal(got[i], want_d[i, :want_c[i]]), f"image {i}"


def test_gather_pipelined_batches_keep_their_own_buffers(tmp_path):
    """batch k's gathered rows must survive batch k+1's gather (buffer ring)."""
    out = str(tmp_path / "dets2.pt")
    mp.spawn(_worker_pipelined, args=(2, _free_port(), out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    want_d, want_c = _batch_detections(0, 8)
    assert [len(b) for b in got] == [4, 4]
    for k in range(2):
        for i in range(4):
            j = 4 * k + i
            assert torch.equal(got[k][i], want_d[j, :want_c[j]]), f"batch {k} image {i}"


def test_gather_without_process_group_single_rank():
    dets, counts = _batch_detections(0, 2)
    g = dist.Gather(2, MAX_DET, "cpu", 0, 1, slots=2)
    a = g(dets, counts)
    b = g(torch.zeros_like(dets), torch.zeros_like(counts))
    assert a is not b
    flat = g.detections(a)
    for i in range(2):
        assert torch.equal(flat[i], dets[i, :counts[i]])
    with pytest.raises(RuntimeError):
        dist.Gather(2, MAX_DET, "cpu", 0, 2)(dets, counts)
