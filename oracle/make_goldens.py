"""Generate the golden fixtures under tests/golden/ from the reference's own Python.

Runs ONLY in the build/survey container, where the reference is mounted
read-only at /root/reference (it never travels to the GPU box). The reference
imports torchvision at utils/util.py:8, which is not installed, so a stub module
is placed in sys.modules first; its ops.nms is oracle.nms.torchvision_nms
(torchvision's documented contract). utils.util.time is frozen so the
wall-clock cutoff of non_max_suppression (util.py:133-134,166-167) never fires.

Fixtures (inputs are regenerated bit-exactly from yolo_hip.synth; only their
sha256 is stored):
  forward_<variant>_<size>_b<B>.npz  reference output of the fused model
      (YOLO.fuse, nets/nn.py:299-305) evaluated in float64 -> stored as float32,
      plus the deviation of the reference's own float32 / bfloat16 / float16
      CPU forwards from it (the reference's precision noise floor).
  construct_v11_n.json  sha256 of every state_dict tensor of a fresh
      nets.nn.yolo_v11_n() after torch.manual_seed(0) (constructor parity).
  nms_synth.npz       reference non_max_suppression on synthetic head outputs.
  nms_forward_n640.npz  reference non_max_suppression on the v11_n 640 golden output.
  forward_x_1280_b1_sub.npz  (--x1280) v11_x at 1280x1280 (C5's shape, PSA over 1600
      tokens): the float64 output at 4096 seeded anchors, per-row sums, the reference
      NMS detections and the float32 / bfloat16 / float16 deviation statistics.

Usage: PYTHONDONTWRITEBYTECODE=1 python oracle/make_goldens.py
"""
import hashlib
import json
import os
import sys
import time
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
GOLD = os.path.join(ROOT, "tests", "golden")
sys.dont_write_bytecode = True


def import_reference():
    from oracle.nms import torchvision_nms

    tv = types.ModuleType("torchvision")
    tv.ops = types.ModuleType("torchvision.ops")

    def nms(boxes, scores, iou_threshold):
        keep = torchvision_nms(boxes.detach().cpu().numpy(), scores.detach().cpu().numpy(), iou_threshold)
        return torch.from_numpy(keep)

    tv.ops.nms = nms
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.ops"] = tv.ops
    # The reference's nets/ and utils/ are namespace packages (no __init__.py): a
    # regular package of the same name anywhere on sys.path would win, so our own
    # drop-in directory must be off the path while the reference is imported.
    ours = os.path.join(ROOT, "yolo-infer-pt_amd")
    saved = list(sys.path)
    sys.path[:] = [REF] + [p for p in sys.path if os.path.abspath(p or ".") not in (ours, ROOT)]
    for k in [k for k in sys.modules if k.split(".")[0] in ("nets", "utils")]:
        del sys.modules[k]
    from nets import nn as ref_nn  # noqa: E402
    from utils import util as ref_util  # noqa: E402
    ref_util.time = lambda: 0.0  # freeze the NMS wall-clock cutoff
    assert os.path.realpath(ref_nn.__file__).startswith(REF), ref_nn.__file__
    assert os.path.realpath(ref_util.__file__).startswith(REF), ref_util.__file__
    sys.path[:] = saved
    for k in [k for k in sys.modules if k.split(".")[0] in ("nets", "utils")]:
        sys.modules["_ref_" + k] = sys.modules.pop(k)
    return ref_nn, ref_util


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def stats(a, ref):
    d = np.abs(a.astype(np.float64) - ref.astype(np.float64))
    return np.array([d[:, :4].max(), d[:, :4].mean(), d[:, 4:].max(), d[:, 4:].mean()])


def forward_golden(ref_nn, synth, variant, size, batch, seed=5):
    torch.manual_seed(0)
    model = getattr(ref_nn, f"yolo_v11_{variant}")(80)
    model.load_state_dict(synth.synth_state_dict(model.state_dict(), seed=0))
    model.eval().fuse()
    x = synth.synth_scenes(batch, size, size, seed=seed)
    out = {}
    with torch.no_grad():
        import copy
        y64 = copy.deepcopy(model).double()(x.double()).float().numpy()
        torch.set_num_threads(8)
        y32 = model(x).numpy()
        torch.set_num_threads(1)
        y32_1 = model(x).numpy()
        torch.set_num_threads(8)
        yb = copy.deepcopy(model).bfloat16()(x.bfloat16()).float().numpy()
        try:
            yh = copy.deepcopy(model).half()(x.half()).float().numpy()
        except Exception as e:  # noqa: BLE001
            print("  fp16 CPU forward unavailable:", e)
            yh = None
    out["y"] = y64
    out["x_sha256"] = np.array(synth.sha256(x))
    out["dev_fp32_8thr"] = stats(y32, y64)
    out["dev_fp32_1thr"] = stats(y32_1, y64)
    out["dev_bf16"] = stats(yb, y64)
    if yh is not None:
        out["dev_fp16"] = stats(yh, y64)
    out["meta"] = np.array(json.dumps(dict(variant=variant, size=size, batch=batch, input="synth_scenes",
                                           input_seed=seed, weight_seed=0, torch=torch.__version__)))
    path = os.path.join(GOLD, f"forward_{variant}_{size}_b{batch}.npz")
    np.savez_compressed(path, **out)
    print(f"  {os.path.basename(path)}: fp32(8thr) box {out['dev_fp32_8thr'][0]:.2e} cls {out['dev_fp32_8thr'][2]:.2e}; "
          f"bf16 box {out['dev_bf16'][0]:.2e} cls {out['dev_bf16'][2]:.2e}")
    return y64


def forward_golden_sub(ref_nn, ref_util, synth, variant, size, batch, seed=5, n_sub=4096):
    """Large-shape golden kept small: the float64 reference output at n_sub seeded anchors of
    every image (all 4 + nc rows), its per-row sums over all anchors (float64), the
    reference NMS detections of the full float64 output, and the deviation statistics of
    the reference's own float32 / bfloat16 / float16 CPU forwards over the full output."""
    import copy
    torch.manual_seed(0)
    model = getattr(ref_nn, f"yolo_v11_{variant}")(80)
    model.load_state_dict(synth.synth_state_dict(model.state_dict(), seed=0))
    model.eval().fuse()
    x = synth.synth_scenes(batch, size, size, seed=seed)
    t0 = time.time()
    with torch.no_grad():
        y64d = copy.deepcopy(model).double()(x.double())
        y64 = y64d.float().numpy()
        y32 = model(x).numpy()
        yb = copy.deepcopy(model).bfloat16()(x.bfloat16()).float().numpy()
        try:
            yh = copy.deepcopy(model).half()(x.half()).float().numpy()
        except Exception as e:  # noqa: BLE001
            print("  fp16 CPU forward unavailable:", e)
            yh = None
    A = y64.shape[2]
    idx = np.sort(np.random.default_rng(1234).choice(A, size=min(n_sub, A), replace=False)).astype(np.int64)
    dets = ref_util.non_max_suppression(torch.from_numpy(y64), 0.001, 0.65)
    counts, flat = pack_dets(dets)
    out = dict(y_sub=y64[:, :, idx], idx=idx, row_sum=y64d.sum(dim=2).numpy(), anchors=np.array(A),
               dets=flat, counts=counts, x_sha256=np.array(synth.sha256(x)),
               dev_fp32_8thr=stats(y32, y64), dev_bf16=stats(yb, y64))
    if yh is not None:
        out["dev_fp16"] = stats(yh, y64)
    out["meta"] = np.array(json.dumps(dict(variant=variant, size=size, batch=batch, input="synth_scenes",
                                           input_seed=seed, weight_seed=0, torch=torch.__version__,
                                           subsample=int(len(idx)))))
    path = os.path.join(GOLD, f"forward_{variant}_{size}_b{batch}_sub.npz")
    np.savez_compressed(path, **out)
    print(f"  {os.path.basename(path)}: fp32 box {out['dev_fp32_8thr'][0]:.2e}; bf16 box {out['dev_bf16'][0]:.2e} "
          f"cls {out['dev_bf16'][2]:.2e}; kept {counts.tolist()} ({time.time() - t0:.0f}s)")


def construct_golden(ref_nn):
    torch.manual_seed(0)
    m = ref_nn.yolo_v11_n(80)
    d = {k: sha(v.detach().numpy()) for k, v in m.state_dict().items()}
    with open(os.path.join(GOLD, "construct_v11_n.json"), "w") as f:
        json.dump(dict(stride=m.stride.tolist(), tensors=d), f, indent=0, sort_keys=True)
    print(f"  construct_v11_n.json: {len(d)} tensors")


def pack_dets(dets):
    counts = np.array([d.shape[0] for d in dets], dtype=np.int64)
    flat = np.concatenate([d.numpy() if hasattr(d, "numpy") else d for d in dets] + [np.zeros((0, 6), np.float32)])
    return counts, flat.astype(np.float32)


def nms_golden(ref_util, synth):
    cases = [("typical", 0), ("typical", 1), ("dense", 2), ("stress", 3)]
    ys = [synth.synth_head_output(8400, 80, seed=s, mode=m) for m, s in cases]
    y = torch.stack(ys)
    t0 = time.time()
    dets = ref_util.non_max_suppression(y, 0.001, 0.65)
    counts, flat = pack_dets(dets)
    np.savez_compressed(os.path.join(GOLD, "nms_synth.npz"), counts=counts, dets=flat,
                        modes=np.array([m for m, _ in cases]), seeds=np.array([s for _, s in cases]),
                        y_sha256=np.array([synth.sha256(t) for t in ys]))
    print(f"  nms_synth.npz: kept {counts.tolist()} ({time.time() - t0:.1f}s)")


def nms_forward_golden(ref_util, y):
    t = torch.from_numpy(y)
    cand = t[:, 4:][t[:, 4:] > 0.001]
    uniq = np.unique(cand.numpy()).size
    dets = ref_util.non_max_suppression(t, 0.001, 0.65)
    counts, flat = pack_dets(dets)
    np.savez_compressed(os.path.join(GOLD, "nms_forward_n640.npz"), counts=counts, dets=flat,
                        candidates=np.array(cand.numel()), distinct=np.array(uniq))
    print(f"  nms_forward_n640.npz: candidates {cand.numel()} distinct {uniq}, kept {counts.tolist()}")


def main():
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "yolo-infer-pt_amd"))
    from yolo_hip import synth  # our deterministic data (no reference code)
    ref_nn, ref_util = import_reference()
    os.makedirs(GOLD, exist_ok=True)
    torch.set_num_threads(8)
    if "--x1280" in sys.argv:   # the large C5 golden alone (minutes of CPU)
        forward_golden_sub(ref_nn, ref_util, synth, "x", 1280, 1)
        return
    print("constructor parity")
    construct_golden(ref_nn)
    print("forward goldens")
    y640 = forward_golden(ref_nn, synth, "n", 640, 1)
    forward_golden(ref_nn, synth, "n", 320, 2)
    for v in ("t", "s", "m", "l"):
        forward_golden(ref_nn, synth, v, 256, 1)
    forward_golden(ref_nn, synth, "x", 320, 1)
    print("nms goldens")
    nms_golden(ref_util, synth)
    nms_forward_golden(ref_util, y640)


if __name__ == "__main__":
    main()
