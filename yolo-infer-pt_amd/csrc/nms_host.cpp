// Host (CPU) batched NMS: the reference's non_max_suppression (utils/util.py:123-169)
// for head outputs that live in host memory, so a GPU-less `main.py --test`
// (main.py:20 picks device "cpu") keeps working through the drop-in. Same contract
// as the device path yh_nms (csrc/nms.hip):
//   * candidates = (anchor, class) pairs with score > threshold, the threshold
//     rounded to the input dtype (torch compares a tensor with a Python float in the
//     tensor's dtype, util.py:130 / 147), row-major (anchor, class) order;
//   * wh2xy corners evaluated in the input dtype (util.py:145), then everything in
//     float32 (util.py:148 torch.cat promotes to float32 through j.float());
//   * score-descending order, ties by the lower (anchor, class) index (the
//     reference's argsort at util.py:157 is unstable: any order of ties is valid
//     there), first max_nms kept;
//   * boxes offset by class * max_wh (util.py:160-161) and the torchvision.ops.nms
//     CPU kernel's greedy loop (IoU = inter / (area_i + area_j - inter) > thr, no
//     +1, in float32), first max_det kept (util.py:163);
//   * no wall-clock cutoff (util.py:133-134, 166-167).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "yolo_hip.h"

namespace {

inline float bf16_to_f(uint16_t h) {
    const uint32_t u = (uint32_t)h << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}
inline float f16_to_f(uint16_t h) {
    const uint32_t s = (uint32_t)(h & 0x8000) << 16, e = (h >> 10) & 0x1f, m = h & 0x3ff;
    uint32_t u;
    if (e == 0) {
        if (m == 0) {
            u = s;
        } else {  // subnormal
            int ee = -1;
            uint32_t mm = m;
            do { ++ee; mm <<= 1; } while (!(mm & 0x400));
            u = s | ((uint32_t)(127 - 15 - ee) << 23) | ((mm & 0x3ff) << 13);
        }
    } else if (e == 31) {
        u = s | 0x7f800000u | (m << 13);
    } else {
        u = s | ((e + 127 - 15) << 23) | (m << 13);
    }
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}
// round a float to the dtype and back (round to nearest even, as torch's casts)
inline float round_bf16(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return f;
    u = (u + 0x7fffu + ((u >> 16) & 1)) & 0xffff0000u;
    float r;
    std::memcpy(&r, &u, 4);
    return r;
}
inline float round_f16(float f) {
    _Float16 h = (_Float16)f;
    return (float)h;
}

struct Cand {
    float score;
    uint32_t idx;   // anchor * nc + class
};

void nms_image(int dtype, const void* y, int nc, int A, float thr, double iou, int max_det, int max_nms,
               float max_wh, float* dets, int* count) {
    auto at = [&](int row, int a) -> float {
        const size_t k = (size_t)row * A + a;
        if (dtype == YH_F32) return static_cast<const float*>(y)[k];
        const uint16_t h = static_cast<const uint16_t*>(y)[k];
        return dtype == YH_BF16 ? bf16_to_f(h) : f16_to_f(h);
    };
    auto rnd = [&](float f) { return dtype == YH_F32 ? f : (dtype == YH_BF16 ? round_bf16(f) : round_f16(f)); };
    std::vector<Cand> c;
    for (int a = 0; a < A; ++a)
        for (int k = 0; k < nc; ++k) {
            const float s = at(4 + k, a);
            if (s > thr) c.push_back({s, (uint32_t)a * (uint32_t)nc + (uint32_t)k});
        }
    std::stable_sort(c.begin(), c.end(), [](const Cand& p, const Cand& q) { return p.score > q.score; });
    if ((int)c.size() > max_nms) c.resize(max_nms);
    const int n = (int)c.size();
    std::vector<float> bx(4 * (size_t)n), area(n), box(4 * (size_t)n);
    for (int i = 0; i < n; ++i) {
        const int a = (int)(c[i].idx / (uint32_t)nc), k = (int)(c[i].idx % (uint32_t)nc);
        const float cx = at(0, a), cy = at(1, a), w = at(2, a), h = at(3, a);
        const float x1 = rnd(cx - w / 2.0f), y1 = rnd(cy - h / 2.0f);
        const float x2 = rnd(cx + w / 2.0f), y2 = rnd(cy + h / 2.0f);
        box[4 * i] = x1; box[4 * i + 1] = y1; box[4 * i + 2] = x2; box[4 * i + 3] = y2;
        const float off = (float)k * max_wh;
        bx[4 * i] = x1 + off; bx[4 * i + 1] = y1 + off; bx[4 * i + 2] = x2 + off; bx[4 * i + 3] = y2 + off;
        area[i] = (bx[4 * i + 2] - bx[4 * i]) * (bx[4 * i + 3] - bx[4 * i + 1]);
    }
    std::vector<char> sup(n, 0);
    int kept = 0;
    for (int i = 0; i < n && kept < max_det; ++i) {
        if (sup[i]) continue;
        const int k = (int)(c[i].idx % (uint32_t)nc);
        float* d = dets + 6 * (size_t)kept;
        d[0] = box[4 * i]; d[1] = box[4 * i + 1]; d[2] = box[4 * i + 2]; d[3] = box[4 * i + 3];
        d[4] = c[i].score; d[5] = (float)k;
        ++kept;
        const float ix1 = bx[4 * i], iy1 = bx[4 * i + 1], ix2 = bx[4 * i + 2], iy2 = bx[4 * i + 3], ia = area[i];
        for (int j = i + 1; j < n; ++j) {
            if (sup[j]) continue;
            const float xx1 = std::max(ix1, bx[4 * j]), yy1 = std::max(iy1, bx[4 * j + 1]);
            const float xx2 = std::min(ix2, bx[4 * j + 2]), yy2 = std::min(iy2, bx[4 * j + 3]);
            const float w = std::max(0.0f, xx2 - xx1), h = std::max(0.0f, yy2 - yy1);
            const float inter = w * h;
            const float ovr = inter / (ia + area[j] - inter);
            if ((double)ovr > iou) sup[j] = 1;   // float ovr vs double threshold, as torchvision
        }
    }
    *count = kept;
}

}  // namespace

extern "C" int yh_nms_host(int dtype, const void* y, int batch, int num_classes, int anchors,
                           float conf_threshold, double iou_threshold, int max_det, int max_nms, float max_wh,
                           float* dets, int* counts, int threads) {
    if (!y || !dets || !counts || batch < 0 || num_classes < 1 || anchors < 0 || max_det < 0 || max_nms < 0)
        return YH_EINVAL;
    if (dtype != YH_F32 && dtype != YH_F16 && dtype != YH_BF16) return YH_EINVAL;
    const float thr = dtype == YH_F32 ? conf_threshold
                                      : (dtype == YH_BF16 ? round_bf16(conf_threshold) : round_f16(conf_threshold));
    const size_t es = dtype == YH_F32 ? 4 : 2;
    const size_t img = (size_t)(4 + num_classes) * anchors * es;
    std::fill(dets, dets + (size_t)batch * max_det * 6, 0.0f);
    auto run = [&](int b) {
        nms_image(dtype, static_cast<const char*>(y) + (size_t)b * img, num_classes, anchors, thr, iou_threshold,
                  max_det, max_nms, max_wh, dets + (size_t)b * max_det * 6, counts + b);
    };
    int nt = threads > 0 ? threads : (int)std::max(1u, std::thread::hardware_concurrency());
    nt = std::min(nt, batch);
    if (nt <= 1) {
        for (int b = 0; b < batch; ++b) run(b);
        return YH_OK;
    }
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; ++t)
        pool.emplace_back([&, t] {
            for (int b = t; b < batch; b += nt) run(b);
        });
    for (auto& th : pool) th.join();
    return YH_OK;
}
