"""Python handle around the C ABI: one `Engine` per (device, dtype, variant).

An Engine owns a yh_handle. It is fed the weights of a torch module tree whose
state_dict layout is the reference's (nets/nn.py) - either unfused Conv blocks
(conv + BatchNorm, folded inside the library exactly like fuse_conv,
nets/nn.py:8-25) or already fused ones (conv with bias) - and runs the eval
forward (nets/nn.py:294-297) and the NMS (utils/util.py:123-169) on device.
"""
import ctypes
from ctypes import byref, c_char_p, c_double, c_int, c_size_t, c_void_p

import torch

from . import _lib
from ._lib import YhVariant, check, lib

_DTYPES = {torch.float32: _lib.YH_F32, torch.float16: _lib.YH_F16, torch.bfloat16: _lib.YH_BF16}

OP_CLASSES = ("conv3x3", "conv1x1", "stem", "dwconv", "sppf", "attention", "decode", "head_cls", "box_dfl", "c3k2",
              "c3k", "box_chain", "pw_chain")


def dtype_code(dtype):
    if dtype not in _DTYPES:
        raise TypeError(f"yolo_hip: unsupported dtype {dtype} (float32, float16, bfloat16)")
    return _DTYPES[dtype]


def _stream_ptr(device):
    return c_void_p(torch.cuda.current_stream(device).cuda_stream)


class Engine:
    """HIP inference engine for one YOLOv11 variant on one device in one dtype."""

    def __init__(self, width, depth, csp, num_classes, device, dtype):
        device = torch.device(device)
        if device.type != "cuda":
            raise ValueError("yolo_hip.Engine needs a cuda (HIP) device")
        self.device = device
        self.index = device.index if device.index is not None else torch.cuda.current_device()
        self.dtype = dtype
        self.num_classes = int(num_classes)
        v = YhVariant()
        for i in range(6):
            v.width[i] = int(width[i])
            v.depth[i] = int(depth[i])
        v.csp[0], v.csp[1] = int(bool(csp[0])), int(bool(csp[1]))
        v.num_classes = self.num_classes
        h = c_void_p()
        check(lib().yh_create(byref(v), self.index, dtype_code(dtype), byref(h)), "create")
        self._h = h
        self.convs = []
        n = lib().yh_conv_count(h)
        for i in range(n):
            name, cout, cpg, k, g, hb = c_char_p(), c_int(), c_int(), c_int(), c_int(), c_int()
            check(lib().yh_conv_info(h, i, byref(name), byref(cout), byref(cpg), byref(k), byref(g), byref(hb)))
            self.convs.append((name.value.decode(), cout.value, cpg.value, k.value, g.value, hb.value))
        self.signature = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().yh_destroy(h)
            except Exception:
                pass
            self._h = None

    # ------------------------------------------------------------------ weights
    def load_module(self, model):
        """Upload every conv of a reference-layout module tree (nets.nn.YOLO)."""
        for idx, (name, cout, cpg, k, groups, has_bias) in enumerate(self.convs):
            mod = model.get_submodule(name)
            conv = getattr(mod, "conv", None)
            norm = getattr(mod, "norm", None)
            if not isinstance(conv, torch.nn.Conv2d):  # plain nn.Conv2d (head outputs)
                conv, norm = mod, None
            w = conv.weight.detach()
            if tuple(w.shape) != (cout, cpg, k, k):
                raise ValueError(f"yolo_hip: {name}.weight has shape {tuple(w.shape)}, "
                                 f"expected {(cout, cpg, k, k)}")
            self._load(idx, w, conv.bias, norm)
        self.signature = None

    def load_state_dict(self, sd):
        """Upload from a reference state_dict (`name.conv.weight`, `name.norm.*`, or plain `name.weight`)."""
        for idx, (name, cout, cpg, k, groups, has_bias) in enumerate(self.convs):
            if f"{name}.conv.weight" in sd:
                w = sd[f"{name}.conv.weight"]
                b = sd.get(f"{name}.conv.bias")
                norm = None
                if f"{name}.norm.weight" in sd:
                    norm = _BN(sd[f"{name}.norm.weight"], sd[f"{name}.norm.bias"],
                               sd[f"{name}.norm.running_mean"], sd[f"{name}.norm.running_var"], 1e-3)
            else:
                w, b, norm = sd[f"{name}.weight"], sd.get(f"{name}.bias"), None
            if tuple(w.shape) != (cout, cpg, k, k):
                raise ValueError(f"yolo_hip: {name} weight shape {tuple(w.shape)} != {(cout, cpg, k, k)}")
            self._load(idx, w, b, norm)

    def _load(self, idx, w, b, norm):
        keep = []

        def host(t):
            if t is None:
                return None
            a = t.detach().to(device="cpu", dtype=torch.float32).contiguous()
            keep.append(a)
            return c_void_p(a.data_ptr())

        args = [host(w), host(b)]
        if norm is not None:
            args += [host(norm.weight), host(norm.bias), host(norm.running_mean), host(norm.running_var)]
            eps = float(norm.eps)
        else:
            args += [None, None, None, None]
            eps = 0.0
        check(lib().yh_load_conv(self._h, idx, *args, c_double(eps)), f"load {self.convs[idx][0]}")

    # ------------------------------------------------------------------ compute
    def num_anchors(self, height, width):
        a = c_int()
        check(lib().yh_num_anchors(self._h, int(height), int(width), byref(a)))
        return a.value

    def forward(self, x, out=None):
        """x: (B, 3, H, W) cuda tensor in the engine dtype -> (B, 4 + nc, A).

        x may also be the loader's uint8 image batch: the reference's `x.half() / 255`
        (main.py:265-267, to the engine dtype) then runs inside the stem (yh_forward_u8)."""
        if not x.is_cuda or x.device.index != self.index:
            raise ValueError(f"yolo_hip: input must live on cuda:{self.index}")
        if x.dtype != self.dtype and x.dtype != torch.uint8:
            raise TypeError(f"yolo_hip: input dtype {x.dtype} is neither the engine dtype {self.dtype} nor uint8")
        if x.dim() != 4 or x.shape[1] != 3:
            raise ValueError(f"yolo_hip: expected (B, 3, H, W), got {tuple(x.shape)}")
        x = x.contiguous()
        B, _, H, W = x.shape
        A = self.num_anchors(H, W)
        if out is None:
            out = torch.empty((B, 4 + self.num_classes, A), dtype=self.dtype, device=x.device)
        fwd = lib().yh_forward_u8 if x.dtype == torch.uint8 else lib().yh_forward
        check(fwd(self._h, c_void_p(x.data_ptr()), B, H, W, c_void_p(out.data_ptr()), _stream_ptr(x.device)),
              "forward")
        return out

    def reserve(self, batch, height, width):
        check(lib().yh_reserve(self._h, int(batch), int(height), int(width)), "reserve")

    def set_graph(self, enable):
        check(lib().yh_set_graph(self._h, int(bool(enable))))

    def force_conv_kernel(self, kernel):
        """Run every 16-bit dense conv on candidate plan `kernel` of its layer (clamped to the
        layer's last candidate), or -1 for per-shape autotuning. All plans are bit-identical."""
        check(lib().yh_force_conv_kernel(self._h, int(kernel)), "force_conv_kernel")

    def units(self, batch, height, width):
        """Launch units of the forward at this shape (after a forward), with profiled time."""
        n = lib().yh_unit_count(self._h, int(batch), int(height), int(width))
        if n < 0:
            raise RuntimeError("yolo_hip: no forward has run at this shape yet")
        ops = self.ops(batch, height, width)
        out = []
        for i in range(n):
            f, k, lv, ms, calls = c_int(), c_int(), c_int(), c_double(), c_int()
            check(lib().yh_unit_info(self._h, i, int(batch), int(height), int(width), byref(f), byref(k), byref(lv),
                                     byref(ms), byref(calls)))
            mem = ops[f.value:f.value + k.value]
            out.append(dict(first=f.value, num_ops=k.value, ms=ms.value, calls=calls.value, label=mem[0]["label"],
                            cls=mem[0]["cls"], kernel=mem[0]["kernel"],
                            bytes=sum(o["bytes"] for o in mem), flops=sum(o["flops"] for o in mem), ops=mem))
        return out

    def profile(self, enable):
        check(lib().yh_profile_enable(self._h, int(bool(enable))))

    def profile_reset(self):
        check(lib().yh_profile_reset(self._h))

    def ops(self, batch, height, width):
        """Per-op records: label, class, algorithmic bytes/flops per call, profiled ms, calls."""
        out = []
        for i in range(lib().yh_op_count(self._h)):
            label, cls = c_char_p(), c_int()
            b, f, ms, calls = c_double(), c_double(), c_double(), c_int()
            check(lib().yh_op_info(self._h, i, int(batch), int(height), int(width), byref(label), byref(cls),
                                   byref(b), byref(f), byref(ms), byref(calls)))
            kname = c_char_p()
            rc = lib().yh_op_kernel(self._h, i, int(batch), int(height), int(width), byref(kname))
            out.append(dict(label=label.value.decode(), cls=OP_CLASSES[cls.value], bytes=b.value,
                            flops=f.value, ms=ms.value, calls=calls.value,
                            kernel=kname.value.decode() if rc == 0 else None))
        return out


    # ------------------------------------------------------------------ parity taps (tests)
    def debug_op_desc(self, index, batch, height, width):
        """JSON description of op `index` at this shape (kind, convs, workspace operands)."""
        import json
        buf = ctypes.create_string_buffer(1 << 16)
        rc = lib().yh_debug_op_desc(self._h, int(index), int(batch), int(height), int(width), buf, len(buf))
        if rc < 0:
            check(rc, "debug_op_desc")
        return json.loads(buf.value.decode())

    def debug_run(self, x, y, first, last):
        """Launch the active ops in [first, last) eagerly (after a forward at x's shape)."""
        B, _, H, W = x.shape
        check(lib().yh_debug_run_ops(self._h, c_void_p(x.data_ptr()), int(x.dtype == torch.uint8), B, H, W,
                                     c_void_p(y.data_ptr()), int(first), int(last), _stream_ptr(x.device)),
              "debug_run")

    def debug_operand(self, index, slot, batch, desc):
        """Operand `slot` of op `index` as a dense (batch, H, W, C) tensor of the engine dtype."""
        o = desc["operands"][slot]
        out = torch.empty((batch, o["H"], o["W"], o["C"]), dtype=self.dtype, device=self.device)
        check(lib().yh_debug_operand(self._h, int(index), int(slot), c_void_p(out.data_ptr()),
                                     out.numel() * out.element_size(), _stream_ptr(self.device)), "debug_operand")
        return out


class _BN:
    def __init__(self, weight, bias, mean, var, eps):
        self.weight, self.bias, self.running_mean, self.running_var, self.eps = weight, bias, mean, var, eps


def nms_host(outputs, confidence_threshold=0.001, iou_threshold=0.65, max_det=300, max_nms=30000, max_wh=7680.0,
             threads=0):
    """Host (CPU) batched NMS (yh_nms_host, C++): same contract as `nms` for a CPU tensor.

    Returns (dets (B, max_det, 6) f32, counts (B,) i32) CPU tensors."""
    if outputs.is_cuda:
        raise ValueError("yolo_hip.nms_host needs a CPU tensor")
    y = outputs.detach().contiguous()
    B, no, A = y.shape
    nc = no - 4
    dets = torch.zeros((B, max_det, 6), dtype=torch.float32)
    counts = torch.zeros((B,), dtype=torch.int32)
    check(lib().yh_nms_host(dtype_code(y.dtype), c_void_p(y.data_ptr()), B, nc, A, ctypes.c_float(confidence_threshold),
                            c_double(iou_threshold), int(max_det), int(max_nms), ctypes.c_float(max_wh),
                            c_void_p(dets.data_ptr()), c_void_p(counts.data_ptr()), int(threads)), "nms_host")
    return dets, counts


def nms_workspace_bytes(batch, num_classes, anchors):
    return int(lib().yh_nms_workspace_bytes(int(batch), int(num_classes), int(anchors)))


def nms(outputs, confidence_threshold=0.001, iou_threshold=0.65, max_det=300, max_nms=30000, max_wh=7680.0,
        out=None, workspace=None):
    """On-device batched NMS of a (B, 4 + nc, A) cuda tensor -> (dets (B, max_det, 6) f32, counts (B,) i32).

    out=(dets, counts) and workspace (uint8, >= nms_workspace_bytes) may be given to reuse buffers
    (yolo_hip.pipeline's result ring); otherwise they come from the caching allocator."""
    if not outputs.is_cuda:
        raise ValueError("yolo_hip.nms needs a cuda tensor")
    y = outputs.contiguous()
    B, no, A = y.shape
    nc = no - 4
    dev = y.device
    need = lib().yh_nms_workspace_bytes(B, nc, A)
    if workspace is not None:
        if workspace.dtype != torch.uint8 or workspace.numel() < need or workspace.device != dev:
            raise ValueError(f"yolo_hip.nms: workspace must be a uint8 tensor of >= {need} bytes on {dev}")
        ws = workspace
    else:
        ws = torch.empty(int(need), dtype=torch.uint8, device=dev)  # caching allocator: stream-safe reuse
    if out is not None:
        dets, counts = out
        if (tuple(dets.shape) != (B, max_det, 6) or dets.dtype != torch.float32 or tuple(counts.shape) != (B,)
                or counts.dtype != torch.int32 or dets.device != dev or counts.device != dev
                or not dets.is_contiguous()):
            raise ValueError("yolo_hip.nms: out must be (dets (B, max_det, 6) f32, counts (B,) i32) on the device")
    else:
        dets = torch.empty((B, max_det, 6), dtype=torch.float32, device=dev)
        counts = torch.empty((B,), dtype=torch.int32, device=dev)
    with torch.cuda.device(dev):
        check(lib().yh_nms(dtype_code(y.dtype), c_void_p(y.data_ptr()), B, nc, A, ctypes.c_float(confidence_threshold),
                           c_double(iou_threshold), int(max_det), int(max_nms), ctypes.c_float(max_wh),
                           c_void_p(ws.data_ptr()), c_size_t(ws.numel()), c_void_p(dets.data_ptr()),
                           c_void_p(counts.data_ptr()), _stream_ptr(dev)), "nms")
    return dets, counts
