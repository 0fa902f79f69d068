"""Functional CPU restatement of the reference eval forward (TEST INFRASTRUCTURE ONLY).

Works directly on a reference-layout state_dict (nets/nn.py module tree) with
torch.nn.functional ops, in float32 or float64 (float64 = the "exact" answer of
the reference algorithm). BatchNorm is either folded exactly like fuse_conv
(nets/nn.py:8-25, fp32) or evaluated unfused in eval mode (nets/nn.py:35-36).

Each block cites the reference lines it restates.
"""
import torch
import torch.nn.functional as F

BN_EPS = 1e-3  # nets/nn.py:32


class Oracle:
    def __init__(self, state_dict, width, depth, csp, num_classes=80, dtype=torch.float64, fold_bn=True):
        self.sd = state_dict
        self.w, self.d, self.csp = list(width), list(depth), [bool(c) for c in csp]
        self.nc = num_classes
        self.dtype = dtype
        self.fold = fold_bn
        self._cache = {}

    # -------------------------------------------------------------- parameters
    def _conv_params(self, name):
        """(weight, bias) of conv block `name`, BN folded as fuse_conv does (nets/nn.py:8-25)."""
        key = name
        if key in self._cache:
            return self._cache[key]
        sd = self.sd
        if f"{name}.conv.weight" in sd:
            w = sd[f"{name}.conv.weight"].float()
            b = sd.get(f"{name}.conv.bias")
            if f"{name}.norm.weight" in sd and self.fold:
                g = sd[f"{name}.norm.weight"].float()
                beta = sd[f"{name}.norm.bias"].float()
                mu = sd[f"{name}.norm.running_mean"].float()
                var = sd[f"{name}.norm.running_var"].float()
                scale = g / torch.sqrt(BN_EPS + var)                       # nn.py:17
                w = (scale[:, None] * w.reshape(w.shape[0], -1)).reshape(w.shape)  # nn.py:16-18
                b0 = torch.zeros(w.shape[0]) if b is None else b.float()
                b = scale * b0 + (beta - g * mu / torch.sqrt(var + BN_EPS))       # nn.py:20-23
            elif b is not None:
                b = b.float()
        else:
            w, b = sd[f"{name}.weight"].float(), sd.get(f"{name}.bias")
            b = None if b is None else b.float()
        out = (w.to(self.dtype), None if b is None else b.to(self.dtype))
        self._cache[key] = out
        return out

    def _bn(self, name, y):
        sd = self.sd
        if self.fold or f"{name}.norm.weight" not in sd:
            return y
        t = lambda k: sd[f"{name}.norm.{k}"].to(self.dtype)[None, :, None, None]
        return (y - t("running_mean")) / torch.sqrt(t("running_var") + BN_EPS) * t("weight") + t("bias")

    def conv(self, name, x, act=True, k=1, s=1, g=1):
        """Conv block (nn.py:28-39): act(BN(conv(x))) / fused act(conv'(x)); act = SiLU or identity."""
        w, b = self._conv_params(name)
        y = F.conv2d(x, w, b, stride=s, padding=k // 2, groups=g)
        y = self._bn(name, y)
        return F.silu(y) if act else y

    # -------------------------------------------------------------- blocks
    def residual(self, p, x):                                   # nn.py:42-49
        return x + self.conv(f"{p}.conv2", self.conv(f"{p}.conv1", x, k=3), k=3)

    def c3k(self, p, x):                                        # nn.py:52-63
        y = self.residual(f"{p}.res_m.1", self.residual(f"{p}.res_m.0", self.conv(f"{p}.conv1", x)))
        return self.conv(f"{p}.conv3", torch.cat((y, self.conv(f"{p}.conv2", x)), 1))

    def c3k2(self, p, x, n, use_c3k):                           # nn.py:66-80
        parts = list(self.conv(f"{p}.conv1", x).chunk(2, 1))
        for i in range(n):
            blk = f"{p}.res_m.{i}"
            parts.append(self.c3k(blk, parts[-1]) if use_c3k else self.residual(blk, parts[-1]))
        return self.conv(f"{p}.conv2", torch.cat(parts, 1))

    def sppf(self, p, x):                                       # nn.py:83-94
        maps = [self.conv(f"{p}.conv1", x)]
        for _ in range(3):
            maps.append(F.max_pool2d(maps[-1], 5, 1, 2))
        return self.conv(f"{p}.conv2", torch.cat(maps, 1))

    def attention(self, p, x, heads):                           # nn.py:97-123
        b, c, h, w = x.shape
        dh = c // heads
        dk = dh // 2
        qkv = self.conv(f"{p}.qkv", x, act=False).view(b, heads, 2 * dk + dh, h * w)
        q, k, v = qkv.split([dk, dk, dh], dim=2)
        att = ((q.transpose(-2, -1) @ k) * (dk ** -0.5)).softmax(dim=-1)
        o = (v @ att.transpose(-2, -1)).view(b, c, h, w)
        pe = self.conv(f"{p}.conv1", v.reshape(b, c, h, w), act=False, k=3, g=c)
        return self.conv(f"{p}.conv2", o + pe, act=False)

    def c2psa(self, p, x, n):                                   # nn.py:126-148
        a, y = self.conv(f"{p}.conv1", x).chunk(2, 1)
        ch = y.shape[1]
        for i in range(n):
            blk = f"{p}.res_m.{i}"
            y = y + self.attention(f"{blk}.conv1", y, ch // 64)
            y = y + self.conv(f"{blk}.conv2.1", self.conv(f"{blk}.conv2.0", y), act=False)
        return self.conv(f"{p}.conv2", torch.cat((a, y), 1))

    # -------------------------------------------------------------- network
    def backbone(self, x):                                      # nn.py:151-189
        d, c = self.d, self.csp
        x = self.conv("net.p1.0", x, k=3, s=2)
        x = self.c3k2("net.p2.1", self.conv("net.p2.0", x, k=3, s=2), d[0], c[0])
        p3 = self.c3k2("net.p3.1", self.conv("net.p3.0", x, k=3, s=2), d[1], c[0])
        p4 = self.c3k2("net.p4.1", self.conv("net.p4.0", p3, k=3, s=2), d[2], c[1])
        p5 = self.c3k2("net.p5.1", self.conv("net.p5.0", p4, k=3, s=2), d[3], c[1])
        p5 = self.c2psa("net.p5.3", self.sppf("net.p5.2", p5), d[4])
        return p3, p4, p5

    def neck(self, p3, p4, p5):                                 # nn.py:192-209
        n, c = self.d[5], self.csp
        up = lambda t: F.interpolate(t, scale_factor=2, mode="nearest")
        h1 = self.c3k2("fpn.h1", torch.cat((up(p5), p4), 1), n, c[0])
        h2 = self.c3k2("fpn.h2", torch.cat((up(h1), p3), 1), n, c[0])
        h4 = self.c3k2("fpn.h4", torch.cat((self.conv("fpn.h3", h2, k=3, s=2), h1), 1), n, c[0])
        h6 = self.c3k2("fpn.h6", torch.cat((self.conv("fpn.h5", h4, k=3, s=2), p5), 1), n, c[1])
        return h2, h4, h6

    def head_maps(self, feats):                                 # nn.py:228-257
        out = []
        for i, f in enumerate(feats):
            bx = self.conv(f"head.box.{i}.1", self.conv(f"head.box.{i}.0", f, k=3), k=3)
            bx = self.conv(f"head.box.{i}.2", bx, act=False)
            ch = f.shape[1]
            cl = self.conv(f"head.cls.{i}.0", f, k=3, g=ch)
            cl = self.conv(f"head.cls.{i}.1", cl)
            cl = self.conv(f"head.cls.{i}.2", cl, k=3, g=cl.shape[1])
            cl = self.conv(f"head.cls.{i}.3", cl)
            cl = self.conv(f"head.cls.{i}.4", cl, act=False)
            out.append(torch.cat((bx, cl), 1))
        return out

    def decode(self, maps, strides=(8.0, 16.0, 32.0)):         # nn.py:259-270, util.py:85-96
        b = maps[0].shape[0]
        no = 64 + self.nc
        anchors, stride_col = [], []
        for m, s in zip(maps, strides):
            h, w = m.shape[-2:]
            gy, gx = torch.meshgrid(torch.arange(h, dtype=self.dtype) + 0.5,
                                    torch.arange(w, dtype=self.dtype) + 0.5, indexing="ij")
            anchors.append(torch.stack((gx, gy), -1).view(-1, 2))
            stride_col.append(torch.full((h * w, 1), s, dtype=self.dtype))
        anc = torch.cat(anchors).T                              # (2, A)
        st = torch.cat(stride_col).T                            # (1, A)
        flat = torch.cat([m.reshape(b, no, -1) for m in maps], 2)
        box, cls = flat.split((64, self.nc), 1)
        a = box.shape[-1]
        prob = box.view(b, 4, 16, a).transpose(2, 1).softmax(1)             # nn.py:222-225
        bins = torch.arange(16, dtype=self.dtype).view(1, 16, 1, 1)
        dist = (prob * bins).sum(1)                                          # (b, 4, a)
        lt, rb = dist.chunk(2, 1)
        x1y1, x2y2 = anc[None] - lt, anc[None] + rb
        xywh = torch.cat(((x1y1 + x2y2) / 2, x2y2 - x1y1), 1)
        return torch.cat((xywh * st, cls.sigmoid()), 1)

    @torch.no_grad()
    def __call__(self, x, return_grid_units=False):
        x = x.to(self.dtype)
        maps = self.head_maps(self.neck(*self.backbone(x)))
        return self.decode(maps)


def strides_per_anchor(height, width):
    """Stride of every anchor column of the (B, 4+nc, A) output (8, 16, 32 levels)."""
    out = []
    for s in (8, 16, 32):
        out.append(torch.full(((height // s) * (width // s),), float(s)))
    return torch.cat(out)
