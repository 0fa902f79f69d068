"""Data-parallel sharding of the detection path: one process per GPU.

The forward and NMS have no cross-image dependency, so a
global batch is cut into contiguous per-rank shards and each rank runs its own
Engine on its own GPU. The only exchange is the gather of the fixed-size NMS
results to rank 0 - the reference returns `list[Tensor(k, 6)]` per image from
utils/util.py:123-169; here a rank ships its (B, max_det, 6) detection buffer
plus the (B,) counts packed into one float32 tensor, so one collective moves
everything and nothing about it depends on how many boxes survived.

With backend "nccl" (RCCL on ROCm) the gather runs over xGMI on device
tensors; with "gloo" the same code runs on CPU tensors (the tests use that).
"""
import torch


def shard(total, rank, world):
    """Contiguous [lo, hi) image range of `rank` when `total` images are split over `world` ranks.

    Ranks get floor/ceil shares, the larger shares first, so every image is owned exactly once.
    """
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    base, extra = divmod(int(total), world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def pack(dets, counts):
    """(B, max_det, 6) f32 + (B,) int counts -> (B, max_det * 6 + 1) f32.

    Counts are <= max_det (<= 2^24), so they survive the float32 round trip exactly.
    """
    B = dets.shape[0]
    return torch.cat((dets.reshape(B, -1).float(), counts.reshape(B, 1).float()), 1)


def unpack(packed, max_det=300):
    """Inverse of `pack`: list of per-image (k, 6) tensors, the reference's NMS output shape."""
    out = []
    for row in packed:
        k = int(row[-1].item())
        out.append(row[:max_det * 6].view(max_det, 6)[:k].clone())
    return out


class Gather:
    """Preallocated gather of packed detections to rank 0 (one collective per step).

    Every rank must hold the same per-rank batch (the bench's weak-scaling case);
    for ragged shards pad the packed tensor to the largest shard and drop the
    padding rows on rank 0 with `shard()`.
    """

    def __init__(self, batch, max_det, device, rank, world, group=None):
        self.rank, self.world, self.group = rank, world, group
        self.batch, self.max_det = batch, max_det
        self.bufs = ([torch.empty((batch, max_det * 6 + 1), dtype=torch.float32, device=device)
                      for _ in range(world)] if rank == 0 else None)

    def __call__(self, dets, counts):
        """Collective: returns the list of per-rank packed tensors on rank 0, None elsewhere."""
        packed = pack(dets, counts)
        if self.world == 1:
            return [packed]
        torch.distributed.gather(packed, self.bufs, dst=0, group=self.group)
        return self.bufs if self.rank == 0 else None

    def detections(self, gathered, total=None):
        """Rank 0: flatten gathered packed tensors into the global per-image list (rank order)."""
        out = []
        for r, p in enumerate(gathered):
            rows = p
            if total is not None:
                lo, hi = shard(total, r, self.world)
                rows = p[:hi - lo]
            out.extend(unpack(rows, self.max_det))
        return out
