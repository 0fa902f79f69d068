"""Two-stream detection pipeline: the forward of batch k+1 overlaps the NMS of batch k.

The reference's eval loop (main.py:264-273) runs `model(samples)` and then
`util.non_max_suppression(outputs)` back to back for every batch. Both stay
exactly the same computations here; only their scheduling changes:

* the forward (yh_forward, a replayed HIP graph) runs on a lane stream of its own, after an
  event recorded on the caller's stream at submit() (so it sees everything the caller
  queued before, e.g. the copy that filled x);
* the NMS (yh_nms) of the same batch - and, data-parallel, the RCCL gather of
  its fixed-size results - runs on a second stream after an event;
* the head output (B, 4+nc, A) is double-buffered: forward k+2 writes the
  buffer NMS k reads, so it first waits on NMS k's completion event.

nms_image uses one workgroup per image (a few tens of CUs), so it fills CUs
the forward leaves idle at its small 20x20 / 40x40 layers and tail ends.

With several engines ("lanes", each its own workspace and captured graphs),
consecutive batches' forwards also overlap: batch k runs on lane k % L, each
lane on its own stream. The latency-bound 40x40 / 20x20 layers of one forward
then share the chip with the other lane's layers instead of leaving CUs idle.
All NMS calls stay on one stream in submission order (so a data-parallel
gather is issued in the same order on every rank).

Results are identical to the sequential order: every batch gets the full
forward and the full NMS, on its own buffers.
"""
import torch

from .engine import nms


def _tensors(obj):
    if isinstance(obj, torch.Tensor):
        yield obj
    elif isinstance(obj, (list, tuple)):
        for o in obj:
            yield from _tensors(o)


class DetectPipeline:
    """submit(x) -> (dets, counts, extra, done) of that batch; read them on a stream after
    `wait(done)` (or after a device sync).

    `post` (optional) is called on the NMS stream with (dets, counts) - e.g. the
    data-parallel gather - and its return value (`extra`) is kept with the batch.

    Stream safety: dets / counts (and the tensors in `extra`) are allocated on the
    NMS stream; submit() marks them used on the caller's stream (record_stream), so
    once the caller drops them the caching allocator does not hand their blocks to a
    later batch's NMS before the caller's queued reads have run.

    The forward reads x on its lane stream, not on the caller's: nothing the caller queues
    after submit() is ordered after it. x must not be modified in place (nor its storage
    reused) until the returned `done` event has been waited on (wait(done), or a device
    sync); `done` follows the batch's forward, NMS and post. x itself is record_stream'ed on
    the lane stream, so merely dropping the last reference to it is safe.
    """

    def __init__(self, engine, batch, height, width, post=None, depth=2, nms_kwargs=None, nms_on_lane=False,
                 result_ring=False, idle_skip=True):
        # engine: one Engine, or a list of Engines with the same weights (forward lanes)
        self.engs = list(engine) if isinstance(engine, (list, tuple)) else [engine]
        self.eng = self.engs[0]
        dev = self.eng.device
        A = self.eng.num_anchors(height, width)
        depth = max(depth, 2 * len(self.engs))
        self.ys = [torch.empty((batch, 4 + self.eng.num_classes, A), dtype=self.eng.dtype, device=dev)
                   for _ in range(depth)]
        self.free = [None] * depth          # NMS-done event of the batch last held by each buffer
        # result_ring: dets / counts of slot i (and the NMS workspace) are allocated once and reused
        # by batch k + depth; no per-batch allocation or record_stream (see submit())
        self.result_ring = result_ring
        if result_ring:
            from .engine import nms_workspace_bytes
            md = (nms_kwargs or {}).get("max_det", 300)
            self.dets = [torch.empty((batch, md, 6), dtype=torch.float32, device=dev) for _ in range(depth)]
            self.counts = [torch.empty((batch,), dtype=torch.int32, device=dev) for _ in range(depth)]
            nws = len(self.engs) if nms_on_lane else 1   # one per stream the NMS runs on
            wsb = nms_workspace_bytes(batch, self.eng.num_classes, A)
            self.nms_ws = [torch.empty(wsb, dtype=torch.uint8, device=dev) for _ in range(nws)]
        # nms_on_lane: each batch's NMS follows its forward on the lane's stream (one
        # stream fewer: the HIP runtime maps streams onto GPU_MAX_HW_QUEUES = 4 queues)
        # (stream priorities were measured in r06: a high-priority NMS stream or lane cost 1-6 %)
        self.nms_stream = None if nms_on_lane else torch.cuda.Stream(device=dev)
        # every lane on a stream of its own: the caller's stream then holds only the caller's
        # work, so the event a lane waits on before reading x (recorded there at submit) does
        # not also wait for an earlier forward (with lane 0 on the caller's stream every other
        # lane's forward k waited for lane 0's forward k - 1). YH_LANE0_MAIN=1: the old layout.
        import os
        lane0_main = os.environ.get("YH_LANE0_MAIN", "0") == "1" or len(self.engs) == 1
        self.lane_streams = ([None] if lane0_main else [torch.cuda.Stream(device=dev)]) + \
            [torch.cuda.Stream(device=dev) for _ in self.engs[1:]]
        self.post = post
        self.nms_kwargs = nms_kwargs or {}
        # idle_skip: no `ready` marker on the caller's stream when it has no pending work (see submit)
        self.idle_skip = idle_skip
        self.k = 0

    def submit(self, x):
        main = torch.cuda.current_stream(self.eng.device)
        i = self.k % len(self.ys)
        lane = self.k % len(self.engs)
        self.k += 1
        y = self.ys[i]
        fs = main
        if self.lane_streams[lane] is not None:
            fs = self.lane_streams[lane]
            # x (and anything else the caller queued) must be ready before the forward reads it.
            # If the caller's stream has nothing pending, it is already: no marker is queued there.
            # (A marker on the caller's stream sits in whatever hardware queue that stream shares
            # with a lane - GPU_MAX_HW_QUEUES = 4 - behind that lane's queued forwards, which ties
            # every lane's next forward to that one lane's progress.)
            if not (self.idle_skip and main.query()):
                ready = torch.cuda.Event()
                ready.record(main)
                fs.wait_event(ready)
            x.record_stream(fs)
        if self.free[i] is not None:
            fs.wait_event(self.free[i])
        with torch.cuda.stream(fs):
            self.engs[lane].forward(x, out=y)
            fwd_done = torch.cuda.Event()
            fwd_done.record(fs)
        ns = self.nms_stream if self.nms_stream is not None else fs
        with torch.cuda.stream(ns):
            ns.wait_event(fwd_done)
            if self.result_ring:
                # slot i's previous results (batch k - depth) are overwritten here: this NMS runs after
                # fwd_done, which follows `ready`, i.e. everything the caller queued before this
                # submit() (its reads of batch k - depth included)
                dets, counts = nms(y, out=(self.dets[i], self.counts[i]),
                                   workspace=self.nms_ws[lane if self.nms_stream is None else 0], **self.nms_kwargs)
            else:
                dets, counts = nms(y, **self.nms_kwargs)
            extra = self.post(dets, counts) if self.post is not None else None
            done = torch.cuda.Event()
            done.record(ns)
        self.free[i] = done
        # allocated on the NMS stream, read on the caller's: keep the blocks out of the
        # NMS stream's free pool until the caller's work queued after `done` has run
        if ns is not main:
            for t in ((*_tensors(extra),) if self.result_ring else (dets, counts, *_tensors(extra))):
                if t.is_cuda:
                    t.record_stream(main)
        return dets, counts, extra, done

    def wait(self, done):
        """Make the caller's stream wait for one submitted batch's NMS (+ post)."""
        torch.cuda.current_stream(self.eng.device).wait_event(done)

    def drain(self):
        """Make the caller's stream wait for every NMS in flight."""
        main = torch.cuda.current_stream(self.eng.device)
        for fs in self.lane_streams:   # forwards still running on the lane streams
            if fs is not None:
                main.wait_stream(fs)
        for e in self.free:
            if e is not None:
                main.wait_event(e)
