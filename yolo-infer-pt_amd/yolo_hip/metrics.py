"""Detection metrics of the reference's eval loop, on the device.

  compute_metric  utils/util.py:99-120   IoU matching of one image's detections to its labels
  compute_ap      utils/util.py:225-300  PR curves, AP@0.5 and AP@0.5:0.95 over the dataset
  smooth          utils/util.py:172-177  box filter used to pick the max-F1 confidence

main.py:test (264-300) calls them per batch after non_max_suppression. The
reference moves every image's IoU matrix to the host and loops in numpy; here
the matching is vectorised over all IoU thresholds at once on the tensor's
device, and compute_ap's sort / cumulative sums / 1000- and 101-point
interpolations run in float64 torch (device of choice), so the eval loop never
leaves the GPU until the final scalars.

Matching semantics (util.py:108-119), reproduced exactly: a (label, detection)
pair is a candidate at threshold t when IoU >= t and the classes are equal; each
detection keeps its highest-IoU candidate label; then each label keeps, among
the detections that kept it, the one with the LOWEST detection index (the
reference's second numpy.unique runs over matches ordered by detection, not by
IoU). Exact IoU ties between two labels of one detection are ordered by
numpy's unstable argsort in the reference; here the lower label index wins
(parity unpinned for such ties only).
"""
import numpy
import torch


def _iou(target, output):
    """(L, 5) [cls, x1, y1, x2, y2] x (D, >=4) boxes -> (L, D) IoU, util.py:101-105 arithmetic."""
    a1, a2 = target[:, 1:3].unsqueeze(1), target[:, 3:5].unsqueeze(1)
    b1, b2 = output[:, 0:2].unsqueeze(0), output[:, 2:4].unsqueeze(0)
    inter = (torch.min(a2, b2) - torch.max(a1, b1)).clamp(0).prod(2)
    return inter / ((a2 - a1).prod(2) + (b2 - b1).prod(2) - inter + 1e-7)


def compute_metric(output, target, iou_v):
    """output (D, 6) [x1, y1, x2, y2, score, cls], target (L, 5) [cls, x1, y1, x2, y2],
    iou_v (T,) thresholds -> (D, T) bool: detection d is a true positive at threshold t."""
    iou = _iou(target, output)                                   # (L, D)
    same = target[:, 0:1] == output[:, 5]                        # (L, D)
    L, D = iou.shape
    T = iou_v.shape[0]
    if L == 0 or D == 0:
        return torch.zeros((D, T), dtype=torch.bool, device=output.device)
    cand = (iou.unsqueeze(0) >= iou_v.view(T, 1, 1).to(iou.dtype)) & same.unsqueeze(0)   # (T, L, D)
    # per (threshold, detection): the best candidate label (highest IoU, lower label on ties)
    score = torch.where(cand, iou.unsqueeze(0), torch.full_like(iou, -1.0).unsqueeze(0))
    best = score.argmax(dim=1, keepdim=False)                    # (T, D) first max = lowest label
    has = cand.any(dim=1)                                        # (T, D)
    # per (threshold, label): the lowest detection index among the detections that kept it
    big = torch.full((T, L), D, dtype=torch.long, device=iou.device)
    det = torch.arange(D, device=iou.device).expand(T, D)
    best_or_sink = torch.where(has, best, torch.full_like(best, L))   # unmatched detections -> row L (dropped)
    first = torch.cat([big, big[:, :1]], dim=1).scatter_reduce(1, best_or_sink, det, reduce="amin")[:, :L]
    correct = torch.zeros((T, D + 1), dtype=torch.bool, device=iou.device)
    correct.scatter_(1, first, True)
    return correct[:, :D].t().contiguous()


def smooth(y, f=0.1):
    """Box filter of fraction f with edge padding (util.py:172-177); y: 1-D float64 tensor."""
    nf = round(len(y) * f * 2) // 2 + 1
    p = nf // 2
    yp = torch.cat([y[:1].expand(p), y, y[-1:].expand(p)])
    k = torch.full((nf,), 1.0 / nf, dtype=y.dtype, device=y.device)
    return torch.nn.functional.conv1d(yp.view(1, 1, -1), k.view(1, 1, -1)).view(-1)


def _interp(x, xp, fp, left=None):
    """numpy.interp for increasing xp (duplicates allowed), evaluated like numpy's C loop."""
    j = torch.searchsorted(xp, x, right=True) - 1                # last j with xp[j] <= x
    n = xp.shape[0]
    jc = j.clamp(0, max(n - 2, 0))
    if n == 1:
        res = fp[0].expand_as(x).clone()
    else:
        x0, x1, y0, y1 = xp[jc], xp[jc + 1], fp[jc], fp[jc + 1]
        slope = (y1 - y0) / (x1 - x0)
        res = slope * (x - x0) + y0
        bad = torch.isnan(res)
        res = torch.where(bad, slope * (x - x1) + y1, res)
        res = torch.where(torch.isnan(res) & (y0 == y1), y0, res)
    res = torch.where(x >= xp[-1], fp[-1], res)                  # at / past the last point
    res = torch.where(x < xp[0], fp[0] if left is None else torch.as_tensor(left, dtype=fp.dtype,
                                                                             device=fp.device), res)
    return res


def compute_ap(tp, conf, output, target, plot=False, names=(), eps=1e-16, device=None):
    """util.py:225-300 (without the plots): -> (tp, fp, m_pre, m_rec, map50, mean_ap).

    Inputs as the reference takes them (numpy, from the concatenated per-image
    metrics) or tensors; computed in float64 on `device` (default: the tensors'
    device, else CUDA when available)."""
    if plot:
        raise NotImplementedError("PR/F1 curve plotting (util.py:180-222) is not part of this path")
    if device is None:
        device = tp.device if isinstance(tp, torch.Tensor) else ("cuda" if torch.cuda.is_available() else "cpu")
    f64 = dict(dtype=torch.float64, device=device)
    tp = torch.as_tensor(numpy.asarray(tp) if not isinstance(tp, torch.Tensor) else tp).to(**f64)
    conf = torch.as_tensor(numpy.asarray(conf) if not isinstance(conf, torch.Tensor) else conf).to(**f64)
    output = torch.as_tensor(numpy.asarray(output) if not isinstance(output, torch.Tensor) else output).to(**f64)
    target = torch.as_tensor(numpy.asarray(target) if not isinstance(target, torch.Tensor) else target).to(**f64)
    if tp.dim() == 1:
        tp = tp[:, None]
    order = torch.argsort(-conf, stable=True)
    tp, conf, output = tp[order], conf[order], output[order]
    classes, nt = torch.unique(target, return_counts=True)
    nc = classes.shape[0]
    # numpy's linspace grid, bit for bit: the 101 COCO points land exactly on recall
    # steps (0.28, 0.72, ...) where m_pre jumps, so a 1-ulp different grid (torch.linspace
    # fills from both ends) picks the other side of the jump
    px = torch.from_numpy(numpy.linspace(0, 1, 1000)).to(**f64)
    x101 = torch.from_numpy(numpy.linspace(0, 1, 101)).to(**f64)
    p = torch.zeros((nc, 1000), **f64)
    r = torch.zeros((nc, 1000), **f64)
    ap = torch.zeros((nc, tp.shape[1]), **f64)
    for ci in range(nc):
        sel = output == classes[ci]
        nl = nt[ci].item()
        no = int(sel.sum().item())
        if no == 0 or nl == 0:
            continue
        tps = tp[sel]
        fpc = (1 - tps).cumsum(0)
        tpc = tps.cumsum(0)
        recall = tpc / (nl + eps)
        xs = -conf[sel]                                          # increasing (conf sorted descending)
        r[ci] = _interp(-px, xs, recall[:, 0], left=0.0)
        precision = tpc / (tpc + fpc)
        p[ci] = _interp(-px, xs, precision[:, 0], left=1.0)
        one = torch.ones(1, **f64)
        zero = torch.zeros(1, **f64)
        for j in range(tp.shape[1]):
            m_rec = torch.cat([zero, recall[:, j], one])
            m_pre = torch.cat([one, precision[:, j], zero])
            m_pre = torch.flip(torch.cummax(torch.flip(m_pre, [0]), 0).values, [0])
            y = _interp(x101, m_rec, m_pre)
            ap[ci, j] = torch.trapezoid(y, x101)
    f1 = 2 * p * r / (p + r + eps)
    i = int(smooth(f1.mean(0), 0.1).argmax().item())
    p, r, f1 = p[:, i], r[:, i], f1[:, i]
    tp_n = (r * nt.to(torch.float64)).round()
    fp_n = (tp_n / (p + eps) - tp_n).round()
    ap50, apm = ap[:, 0], ap.mean(1)
    return (tp_n.cpu().numpy(), fp_n.cpu().numpy(), p.mean().item(), r.mean().item(),
            ap50.mean().item(), apm.mean().item())
