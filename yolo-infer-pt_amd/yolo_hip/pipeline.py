"""Two-stream detection pipeline: the forward of batch k+1 overlaps the NMS of batch k.

The reference's eval loop (main.py:264-273) runs `model(samples)` and then
`util.non_max_suppression(outputs)` back to back for every batch. Both stay
exactly the same computations here; only their scheduling changes:

* the forward (yh_forward, a replayed HIP graph) runs on the caller's stream;
* the NMS (yh_nms) of the same batch - and, data-parallel, the RCCL gather of
  its fixed-size results - runs on a second stream after an event;
* the head output (B, 4+nc, A) is double-buffered: forward k+2 writes the
  buffer NMS k reads, so it first waits on NMS k's completion event.

nms_image uses one workgroup per image (a few tens of CUs), so it fills CUs
the forward leaves idle at its small 20x20 / 40x40 layers and tail ends.
Results are identical to the sequential order: every batch gets the full
forward and the full NMS, on its own buffers.
"""
import torch

from .engine import nms


class DetectPipeline:
    """submit(x) -> (dets, counts) of that batch, valid once `wait(handle)` or a sync has run.

    `post` (optional) is called on the NMS stream with (dets, counts) - e.g. the
    data-parallel gather - and its return value is kept with the batch.
    """

    def __init__(self, engine, batch, height, width, post=None, depth=2, nms_kwargs=None):
        self.eng = engine
        dev = engine.device
        A = engine.num_anchors(height, width)
        self.ys = [torch.empty((batch, 4 + engine.num_classes, A), dtype=engine.dtype, device=dev)
                   for _ in range(depth)]
        self.free = [None] * depth          # NMS-done event of the batch last held by each buffer
        self.nms_stream = torch.cuda.Stream(device=dev)
        self.post = post
        self.nms_kwargs = nms_kwargs or {}
        self.k = 0

    def submit(self, x):
        main = torch.cuda.current_stream(self.eng.device)
        i = self.k % len(self.ys)
        self.k += 1
        y = self.ys[i]
        if self.free[i] is not None:
            main.wait_event(self.free[i])
        self.eng.forward(x, out=y)
        fwd_done = torch.cuda.Event()
        fwd_done.record(main)
        with torch.cuda.stream(self.nms_stream):
            self.nms_stream.wait_event(fwd_done)
            dets, counts = nms(y, **self.nms_kwargs)
            extra = self.post(dets, counts) if self.post is not None else None
            done = torch.cuda.Event()
            done.record(self.nms_stream)
        self.free[i] = done
        # the results were allocated on the NMS stream; the caller reads them after `done`
        return dets, counts, extra, done

    def drain(self):
        """Make the caller's stream wait for every NMS in flight."""
        main = torch.cuda.current_stream(self.eng.device)
        for e in self.free:
            if e is not None:
                main.wait_event(e)
