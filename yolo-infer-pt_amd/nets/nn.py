"""Drop-in for the reference's `nets/nn.py` module API (t0saki/YOLO-Infer-pt).

Every public name of the reference module exists here with the same
constructor signature, attribute names (hence identical state_dict keys and
pickle class paths `nets.nn.*`) and CPU semantics, so `main.py --test`,
`main.py`'s profile() (thop hooks on nn.Conv2d leaves) and pickled
checkpoints keep working.

What changes is the device path: `YOLO.forward(x)` on a CUDA (HIP) tensor in
eval mode does not run the module tree. It hands the whole forward to the
hand-written gfx950 kernels behind the C ABI (include/yolo_hip.h) through
`yolo_hip.Engine`: NHWC implicit-GEMM MFMA convolutions with the BatchNorm
folded in (fuse_conv semantics), zero-copy concat/upsample, fused attention,
fused DFL/anchor decode. If the HIP library is missing this raises; there is
no silent PyTorch fallback on the GPU.

Reference map (file:line into /root/reference):
  fuse_conv 8-25, Conv 28-39, Residual 42-49, CSPModule 52-63, CSP 66-80,
  SPP 83-94, Attention 97-123, PSABlock 126-136, PSA 139-148, DarkNet 151-189,
  DarkFPN 192-209, DFL 212-225, Head 228-279, YOLO 282-305, yolo_v11_* 308-347.
"""
import math

import torch

from utils.util import make_anchors

__all__ = ["fuse_conv", "Conv", "Residual", "CSPModule", "CSP", "SPP", "Attention", "PSABlock", "PSA",
           "DarkNet", "DarkFPN", "DFL", "Head", "YOLO", "yolo_v11_n", "yolo_v11_t", "yolo_v11_s",
           "yolo_v11_m", "yolo_v11_l", "yolo_v11_x"]

_SILU = torch.nn.SiLU
_ID = torch.nn.Identity


@torch.no_grad()
def fuse_conv(conv, norm):
    """Fold an eval BatchNorm into the preceding conv (reference nets/nn.py:8-25).

    scale = gamma / sqrt(eps + var);  W' = scale * W;
    b' = scale * b + (beta - gamma * mean / sqrt(var + eps))   (all fp32 ops, same order)
    """
    out = torch.nn.Conv2d(conv.in_channels, conv.out_channels, conv.kernel_size, conv.stride,
                          conv.padding, groups=conv.groups, bias=True).requires_grad_(False)
    out = out.to(conv.weight.device)
    denom = torch.sqrt(norm.eps + norm.running_var)
    scale = norm.weight.div(denom)
    flat = conv.weight.clone().view(conv.out_channels, -1)
    out.weight.copy_(torch.mm(torch.diag(scale), flat).view(out.weight.size()))
    if conv.bias is None:
        conv_b = torch.zeros(conv.weight.size(0), device=conv.weight.device)
    else:
        conv_b = conv.bias
    shift = norm.bias - norm.weight.mul(norm.running_mean).div(torch.sqrt(norm.running_var + norm.eps))
    out.bias.copy_(torch.mm(torch.diag(scale), conv_b.reshape(-1, 1)).reshape(-1) + shift)
    return out


class Conv(torch.nn.Module):
    """conv(k, s, p, g, no bias) -> BatchNorm(eps 1e-3, momentum 0.03) -> activation."""

    def __init__(self, in_ch, out_ch, activation, k=1, s=1, p=0, g=1):
        super().__init__()
        self.conv = torch.nn.Conv2d(in_ch, out_ch, k, s, p, groups=g, bias=False)
        self.norm = torch.nn.BatchNorm2d(out_ch, eps=0.001, momentum=0.03)
        self.relu = activation

    def forward(self, x):
        return self.relu(self.norm(self.conv(x)))

    def fuse_forward(self, x):
        return self.relu(self.conv(x))


class Residual(torch.nn.Module):
    """x + conv3x3(conv3x3(x)), hidden width int(ch * e)."""

    def __init__(self, ch, e=0.5):
        super().__init__()
        hidden = int(ch * e)
        self.conv1 = Conv(ch, hidden, _SILU(), k=3, p=1)
        self.conv2 = Conv(hidden, ch, _SILU(), k=3, p=1)

    def forward(self, x):
        return x + self.conv2(self.conv1(x))


class CSPModule(torch.nn.Module):
    """C3k: two 1x1 branches, two Residuals on the first, concat, 1x1."""

    def __init__(self, in_ch, out_ch):
        super().__init__()
        half = out_ch // 2
        self.conv1 = Conv(in_ch, half, _SILU())
        self.conv2 = Conv(in_ch, half, _SILU())
        self.conv3 = Conv(2 * half, out_ch, _SILU())
        self.res_m = torch.nn.Sequential(Residual(half, e=1.0), Residual(half, e=1.0))

    def forward(self, x):
        branch = self.res_m(self.conv1(x))
        return self.conv3(torch.cat((branch, self.conv2(x)), dim=1))


class CSP(torch.nn.Module):
    """C3k2: 1x1 split into two halves, n blocks chained on the last, concat all, 1x1."""

    def __init__(self, in_ch, out_ch, n, csp, r):
        super().__init__()
        c = out_ch // r
        self.conv1 = Conv(in_ch, 2 * c, _SILU())
        self.conv2 = Conv((2 + n) * c, out_ch, _SILU())
        blocks = (CSPModule(c, c) if csp else Residual(c) for _ in range(n))
        self.res_m = torch.nn.ModuleList(blocks)

    def forward(self, x):
        parts = list(self.conv1(x).chunk(2, 1))
        for block in self.res_m:
            parts.append(block(parts[-1]))
        return self.conv2(torch.cat(parts, dim=1))


class SPP(torch.nn.Module):
    """SPPF: 1x1, three chained 5x5 max-pools, concat of the four maps, 1x1."""

    def __init__(self, in_ch, out_ch, k=5):
        super().__init__()
        self.conv1 = Conv(in_ch, in_ch // 2, _SILU())
        self.conv2 = Conv(in_ch * 2, out_ch, _SILU())
        self.res_m = torch.nn.MaxPool2d(k, stride=1, padding=k // 2)

    def forward(self, x):
        maps = [self.conv1(x)]
        for _ in range(3):
            maps.append(self.res_m(maps[-1]))
        return self.conv2(torch.cat(tensors=maps, dim=1))


class Attention(torch.nn.Module):
    """Multi-head self-attention over the H*W tokens plus a depthwise positional conv on v."""

    def __init__(self, ch, num_head):
        super().__init__()
        self.num_head = num_head
        self.dim_head = ch // num_head
        self.dim_key = self.dim_head // 2
        self.scale = self.dim_key ** -0.5
        self.qkv = Conv(ch, ch + self.dim_key * num_head * 2, _ID())
        self.conv1 = Conv(ch, ch, _ID(), k=3, p=1, g=ch)
        self.conv2 = Conv(ch, ch, _ID())

    def forward(self, x):
        b, c, h, w = x.shape
        tokens = self.qkv(x).view(b, self.num_head, 2 * self.dim_key + self.dim_head, h * w)
        q, k, v = tokens.split([self.dim_key, self.dim_key, self.dim_head], dim=2)
        weights = ((q.transpose(-2, -1) @ k) * self.scale).softmax(dim=-1)
        mixed = (v @ weights.transpose(-2, -1)).view(b, c, h, w)
        return self.conv2(mixed + self.conv1(v.reshape(b, c, h, w)))


class PSABlock(torch.nn.Module):
    def __init__(self, ch, num_head):
        super().__init__()
        self.conv1 = Attention(ch, num_head)
        self.conv2 = torch.nn.Sequential(Conv(ch, ch * 2, _SILU()), Conv(ch * 2, ch, _ID()))

    def forward(self, x):
        x = x + self.conv1(x)
        return x + self.conv2(x)


class PSA(torch.nn.Module):
    """C2PSA: 1x1 split, PSABlocks on the second half, concat, 1x1."""

    def __init__(self, ch, n):
        super().__init__()
        self.conv1 = Conv(ch, 2 * (ch // 2), _SILU())
        self.conv2 = Conv(2 * (ch // 2), ch, _SILU())
        self.res_m = torch.nn.Sequential(*[PSABlock(ch // 2, ch // 128) for _ in range(n)])

    def forward(self, x):
        keep, attend = self.conv1(x).chunk(2, 1)
        return self.conv2(torch.cat(tensors=(keep, self.res_m(attend)), dim=1))


def _down(cin, cout):
    return Conv(cin, cout, _SILU(), k=3, s=2, p=1)


class DarkNet(torch.nn.Module):
    """Backbone: stem + four stride-2 stages; returns (p3, p4, p5)."""

    def __init__(self, width, depth, csp):
        super().__init__()
        w, d = width, depth
        self.p1 = torch.nn.Sequential(_down(w[0], w[1]))
        self.p2 = torch.nn.Sequential(_down(w[1], w[2]), CSP(w[2], w[3], d[0], csp[0], r=4))
        self.p3 = torch.nn.Sequential(_down(w[3], w[3]), CSP(w[3], w[4], d[1], csp[0], r=4))
        self.p4 = torch.nn.Sequential(_down(w[4], w[4]), CSP(w[4], w[4], d[2], csp[1], r=2))
        self.p5 = torch.nn.Sequential(_down(w[4], w[5]), CSP(w[5], w[5], d[3], csp[1], r=2),
                                      SPP(w[5], w[5]), PSA(w[5], d[4]))

    def forward(self, x):
        p3 = self.p3(self.p2(self.p1(x)))
        p4 = self.p4(p3)
        return p3, p4, self.p5(p4)


class DarkFPN(torch.nn.Module):
    """PAN neck: top-down (upsample + concat + C3k2) then bottom-up (stride-2 conv + concat + C3k2)."""

    def __init__(self, width, depth, csp):
        super().__init__()
        w, n = width, depth[5]
        self.up = torch.nn.Upsample(scale_factor=2)
        self.h1 = CSP(w[4] + w[5], w[4], n, csp[0], r=2)
        self.h2 = CSP(w[4] + w[4], w[3], n, csp[0], r=2)
        self.h3 = _down(w[3], w[3])
        self.h4 = CSP(w[3] + w[4], w[4], n, csp[0], r=2)
        self.h5 = _down(w[4], w[4])
        self.h6 = CSP(w[4] + w[5], w[5], n, csp[1], r=2)

    def forward(self, x):
        p3, p4, p5 = x
        n4 = self.h1(torch.cat(tensors=[self.up(p5), p4], dim=1))
        n3 = self.h2(torch.cat(tensors=[self.up(n4), p3], dim=1))
        n4 = self.h4(torch.cat(tensors=[self.h3(n3), n4], dim=1))
        n5 = self.h6(torch.cat(tensors=[self.h5(n4), p5], dim=1))
        return n3, n4, n5


class DFL(torch.nn.Module):
    """Distribution focal loss integral: softmax over `ch` bins, expectation via a fixed 1x1 conv."""

    def __init__(self, ch=16):
        super().__init__()
        self.ch = ch
        self.conv = torch.nn.Conv2d(ch, out_channels=1, kernel_size=1, bias=False).requires_grad_(False)
        bins = torch.arange(ch, dtype=torch.float).view(1, ch, 1, 1)
        self.conv.weight.data[:] = torch.nn.Parameter(bins)

    def forward(self, x):
        b, _, a = x.shape
        probs = x.view(b, 4, self.ch, a).transpose(2, 1).softmax(1)
        return self.conv(probs).view(b, 4, a)


class Head(torch.nn.Module):
    """Decoupled detect head: box branch (DFL logits) + class branch per pyramid level."""

    anchors = torch.empty(0)
    strides = torch.empty(0)

    def __init__(self, nc=80, filters=()):
        super().__init__()
        self.ch = 16
        self.nc = nc
        self.nl = len(filters)
        self.no = nc + self.ch * 4
        self.stride = torch.zeros(self.nl)
        box = max(64, filters[0] // 4)
        cls = max(80, filters[0], self.nc)
        self.dfl = DFL(self.ch)
        self.box = torch.nn.ModuleList(
            torch.nn.Sequential(Conv(f, box, _SILU(), k=3, p=1), Conv(box, box, _SILU(), k=3, p=1),
                                torch.nn.Conv2d(box, out_channels=4 * self.ch, kernel_size=1))
            for f in filters)
        self.cls = torch.nn.ModuleList(
            torch.nn.Sequential(Conv(f, f, _SILU(), k=3, p=1, g=f), Conv(f, cls, _SILU()),
                                Conv(cls, cls, _SILU(), k=3, p=1, g=cls), Conv(cls, cls, _SILU()),
                                torch.nn.Conv2d(cls, out_channels=self.nc, kernel_size=1))
            for f in filters)

    def forward(self, x):
        for i, (box, cls) in enumerate(zip(self.box, self.cls)):
            x[i] = torch.cat(tensors=(box(x[i]), cls(x[i])), dim=1)
        if self.training:
            return x
        self.anchors, self.strides = (t.transpose(0, 1) for t in make_anchors(x, self.stride))
        flat = torch.cat([t.view(x[0].shape[0], self.no, -1) for t in x], dim=2)
        box, cls = flat.split(split_size=(4 * self.ch, self.nc), dim=1)
        lt, rb = self.dfl(box).chunk(2, 1)
        top_left = self.anchors.unsqueeze(0) - lt
        bottom_right = self.anchors.unsqueeze(0) + rb
        xywh = torch.cat(tensors=((top_left + bottom_right) / 2, bottom_right - top_left), dim=1)
        return torch.cat(tensors=(xywh * self.strides, cls.sigmoid()), dim=1)

    def initialize_biases(self):
        for box, cls, s in zip(self.box, self.cls, self.stride):
            box[-1].bias.data[:] = 1.0
            cls[-1].bias.data[:self.nc] = math.log(5 / self.nc / (640 / s) ** 2)


class YOLO(torch.nn.Module):
    def __init__(self, width, depth, csp, num_classes):
        super().__init__()
        self.net = DarkNet(width, depth, csp)
        self.fpn = DarkFPN(width, depth, csp)
        probe = torch.zeros(1, width[0], 256, 256)
        self.head = Head(num_classes, (width[3], width[4], width[5]))
        # train-mode probe forward, as the reference does (it also primes BN running stats)
        self.head.stride = torch.tensor([256 / t.shape[-2] for t in self.forward(probe)])
        self.stride = self.head.stride
        self.head.initialize_biases()
        self._yh_arch = (tuple(width), tuple(depth), tuple(bool(c) for c in csp), int(num_classes))

    def forward(self, x):
        if x.is_cuda and not self.training:
            return _hip_forward(self, x)
        return self.head(list(self.fpn(self.net(x))))

    def fuse(self):
        for m in self.modules():
            if type(m) is Conv and hasattr(m, "norm"):
                m.conv = fuse_conv(m.conv, m.norm)
                m.forward = m.fuse_forward
                delattr(m, "norm")
        _drop_engines(self)
        return self

    def __setstate__(self, state):
        # checkpoints pickled by the reference have no _yh_arch; rebuild it from the modules
        super().__setstate__(state)
        if "_yh_arch" not in self.__dict__:
            self._yh_arch = _infer_arch(self)


def _infer_arch(model):
    net = model.net
    w1 = net.p1[0].conv.out_channels
    w2 = net.p2[0].conv.out_channels
    w3 = net.p2[1].conv2.conv.out_channels
    w4 = net.p3[1].conv2.conv.out_channels
    w5 = net.p5[0].conv.out_channels
    d = len(net.p2[1].res_m)
    c0 = isinstance(net.p2[1].res_m[0], CSPModule)
    c1 = isinstance(net.p4[1].res_m[0], CSPModule)
    return (3, w1, w2, w3, w4, w5), (d,) * 6, (c0, c1), model.head.nc


def _weights_signature(model):
    tensors = model.__dict__.get("_yh_tensors")
    if tensors is None:
        tensors = list(model.state_dict(keep_vars=True).values())
        model.__dict__["_yh_tensors"] = tensors
    return tuple((t.data_ptr(), t._version, t.dtype) for t in tensors)


def _drop_engines(model):
    model.__dict__.pop("_yh_engines", None)
    model.__dict__.pop("_yh_tensors", None)


def _hip_forward(model, x):
    """Eval forward on the HIP path (include/yolo_hip.h yh_forward)."""
    from yolo_hip.engine import Engine

    engines = model.__dict__.setdefault("_yh_engines", {})
    key = (x.device.index if x.device.index is not None else torch.cuda.current_device(), x.dtype)
    sig = _weights_signature(model)
    eng = engines.get(key)
    if eng is None:
        width, depth, csp, nc = model._yh_arch
        eng = Engine(width, depth, csp, nc, torch.device("cuda", key[0]), x.dtype)
        engines[key] = eng
    if eng.signature != sig:
        eng.load_module(model)
        eng.signature = sig
    return eng.forward(x)


def _build(width, depth, csp, num_classes):
    return YOLO(list(width), list(depth), list(csp), num_classes)


def yolo_v11_n(num_classes: int = 80):
    return _build((3, 16, 32, 64, 128, 256), (1,) * 6, (False, True), num_classes)


def yolo_v11_t(num_classes: int = 80):
    return _build((3, 24, 48, 96, 192, 384), (1,) * 6, (False, True), num_classes)


def yolo_v11_s(num_classes: int = 80):
    return _build((3, 32, 64, 128, 256, 512), (1,) * 6, (False, True), num_classes)


def yolo_v11_m(num_classes: int = 80):
    return _build((3, 64, 128, 256, 512, 512), (1,) * 6, (True, True), num_classes)


def yolo_v11_l(num_classes: int = 80):
    return _build((3, 64, 128, 256, 512, 512), (2,) * 6, (True, True), num_classes)


def yolo_v11_x(num_classes: int = 80):
    return _build((3, 96, 192, 384, 768, 768), (2,) * 6, (True, True), num_classes)
