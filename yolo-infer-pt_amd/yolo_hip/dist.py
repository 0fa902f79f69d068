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

    Results land in a ring of `slots` buffer sets, one per call in turn, so a
    pipelined caller (DetectPipeline, up to 2 x lanes batches in flight) can still
    read batch k's gathered rows after batch k+1's gather has been queued; keep
    `slots` at least the number of batches in flight.

    With a torch.distributed process group the gather is always the collective
    (RCCL on device tensors with backend "nccl", also at world size 1); without one
    (plain single-process use) rank 0's own packed rows are returned.
    """

    def __init__(self, batch, max_det, device, rank, world, group=None, slots=8):
        self.rank, self.world, self.group = rank, world, group
        self.batch, self.max_det = batch, max_det
        self.slots = max(1, int(slots))
        self.calls = 0
        self.bufs = ([[torch.empty((batch, max_det * 6 + 1), dtype=torch.float32, device=device)
                       for _ in range(world)] for _ in range(self.slots)] if rank == 0 else None)

    def __call__(self, dets, counts):
        """Collective: returns the list of per-rank packed tensors on rank 0, None elsewhere."""
        packed = pack(dets, counts)
        slot = self.calls % self.slots
        self.calls += 1
        dist = torch.distributed.is_available() and torch.distributed.is_initialized()
        if not dist:
            if self.world != 1:
                raise RuntimeError("Gather over several ranks needs an initialised process group")
            self.bufs[slot][0].copy_(packed)
            return self.bufs[slot]
        out = self.bufs[slot] if self.rank == 0 else None
        torch.distributed.gather(packed, out, dst=0, group=self.group)
        return out

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
