// Eval-mode image preprocessing of the reference's data loader, on the device
// (yh_letterbox) and on the host (yh_letterbox_host, same per-pixel function):
//
//   utils/dataset.py:95-103  load_image: r = input_size / max(h, w); if r != 1
//                            cv2.resize(image, (int(w r), int(h r)), INTER_LINEAR)
//   utils/dataset.py:292-313 resize (augment=False): r <= 1 so no second resize;
//                            zero border (cv2.copyMakeBorder, BORDER_CONSTANT) of
//                            top = round(dh - 0.1), left = round(dw - 0.1) to a
//                            square canvas of input_size
//   utils/dataset.py:86-88   HWC -> CHW and BGR -> RGB
//
// cv2.resize INTER_LINEAR on 8-bit images (OpenCV's published algorithm; cv2 is
// not in this image, so this restatement is parity-unpinned against cv2 itself):
//   scale = 1 / (dst / src) in double; per destination column
//   f = (float)((d + 0.5) * scale - 0.5), s = floor(f), f -= s, with s < 0 -> (0, f 0)
//   and s >= src - 1 -> (src - 1, f 0) on the x axis (rows are clamped instead);
//   11-bit coefficients a0 = rint((1 - f) 2048), a1 = rint(f 2048);
//   horizontal pass in int: H = S[s] a0 + S[s + 1] a1;
//   vertical pass as OpenCV's vector kernel computes it (VResizeLinearVec_32s8u, x86
//   builds with 128-bit universal intrinsics):
//   out = sat_u8((mulhi16(H0 >> 4, b0) + mulhi16(H1 >> 4, b1) + 2) >> 2)
//   over the row's bytes the vector loops cover (16-byte steps while x <= width - 16,
//   then one 8-byte step while x < width - 8, width = 3 nw bytes); the remaining tail
//   bytes take the scalar FixedPtCast: out = sat_u8((H0 b0 + H1 b1 + 2^21) >> 22).
//   Which vector width the cv2 build used is an assumption (parity unpinned vs cv2).
//   Exactly 2x downscales on both axes take INTER_AREA's fast path
//   ((S00 + S01 + S10 + S11 + 2) >> 2), as cv2.resize does.
#include <cmath>
#include <thread>
#include <vector>

#include "common.h"
#include "yolo_hip.h"

namespace yh {

struct LbImage {
    const unsigned char* src;   // HWC BGR uint8, row stride `stride` bytes
    int h, w, stride;
    int nh, nw;                 // resized size
    int top, left;              // border
};

struct LbAxis {
    int s0, s1, a0, a1;
};

// one destination coordinate of the linear resize (see header comment)
__host__ __device__ inline LbAxis lb_axis(int d, int src, double scale, bool clamp_coef) {
#pragma clang fp contract(off)
    const float f0 = (float)(((double)d + 0.5) * scale - 0.5);
    int s = (int)floorf(f0);
    float f = f0 - (float)s;
    if (clamp_coef) {
        if (s < 0) { s = 0; f = 0.f; }
        if (s >= src - 1) { s = src - 1; f = 0.f; }
    }
    LbAxis ax;
    ax.a0 = (int)rintf((1.f - f) * 2048.f);
    ax.a1 = (int)rintf(f * 2048.f);
    ax.s0 = s < 0 ? 0 : (s > src - 1 ? src - 1 : s);
    ax.s1 = s + 1 < 0 ? 0 : (s + 1 > src - 1 ? src - 1 : s + 1);
    return ax;
}

__host__ __device__ inline int lb_mulhi(int a, int b) { return (a * b) >> 16; }

// first byte of a resized row (width = 3 nw bytes) that OpenCV's vertical pass computes
// with its scalar loop instead of VResizeLinearVec_32s8u (see the header comment)
__host__ __device__ inline int lb_vtail(int width) {
    int x = width >= 16 ? ((width - 16) / 16 + 1) * 16 : 0;
    if (x < width - 8) x += 8;
    return x;
}

// Pixel (y, x) of the letterboxed canvas, 3 channels in RGB order.
__host__ __device__ inline void lb_pixel(const LbImage& im, int y, int x, unsigned char rgb[3]) {
    rgb[0] = rgb[1] = rgb[2] = 0;
    const int dy = y - im.top, dx = x - im.left;
    if (dy < 0 || dy >= im.nh || dx < 0 || dx >= im.nw) return;
    const unsigned char* S = im.src;
    if (im.nh == im.h && im.nw == im.w) {   // r == 1: no resize (load_image skips it)
        const unsigned char* p = S + (size_t)dy * im.stride + (size_t)dx * 3;
        rgb[0] = p[2]; rgb[1] = p[1]; rgb[2] = p[0];
        return;
    }
    if (im.h == 2 * im.nh && im.w == 2 * im.nw) {   // INTER_AREA fast path
        const unsigned char* p0 = S + (size_t)(2 * dy) * im.stride + (size_t)(2 * dx) * 3;
        const unsigned char* p1 = p0 + im.stride;
        for (int c = 0; c < 3; ++c) rgb[2 - c] = (unsigned char)((p0[c] + p0[c + 3] + p1[c] + p1[c + 3] + 2) >> 2);
        return;
    }
    const double sx = 1.0 / ((double)im.nw / (double)im.w);
    const double sy = 1.0 / ((double)im.nh / (double)im.h);
    const LbAxis ax = lb_axis(dx, im.w, sx, true);
    const LbAxis ay = lb_axis(dy, im.h, sy, false);
    const unsigned char* r0 = S + (size_t)ay.s0 * im.stride;
    const unsigned char* r1 = S + (size_t)ay.s1 * im.stride;
    const int tail = lb_vtail(3 * im.nw);
    for (int c = 0; c < 3; ++c) {
        const int h0 = r0[ax.s0 * 3 + c] * ax.a0 + r0[ax.s1 * 3 + c] * ax.a1;
        const int h1 = r1[ax.s0 * 3 + c] * ax.a0 + r1[ax.s1 * 3 + c] * ax.a1;
        int v = dx * 3 + c < tail ? (lb_mulhi(h0 >> 4, ay.a0) + lb_mulhi(h1 >> 4, ay.a1) + 2) >> 2
                                  : (h0 * ay.a0 + h1 * ay.a1 + (1 << 21)) >> 22;
        v = v < 0 ? 0 : (v > 255 ? 255 : v);
        rgb[2 - c] = (unsigned char)v;
    }
}

// resized pixel (dy, dx) of an image, 3 channels in the source's (BGR) order
__host__ __device__ inline void lb_resized(const LbImage& im, int dy, int dx, unsigned char bgr[3]) {
    LbImage t = im;
    t.top = 0; t.left = 0;
    unsigned char rgb[3];
    lb_pixel(t, dy, dx, rgb);
    bgr[0] = rgb[2]; bgr[1] = rgb[1]; bgr[2] = rgb[0];
}

// geometry of one image (dataset.py:95-103, 292-313), in the reference's double arithmetic
inline int lb_geometry(int h, int w, int size, LbImage& im) {
    if (h <= 0 || w <= 0 || size <= 0) return YH_EINVAL;
    const double r = (double)size / (double)(h > w ? h : w);
    int nh = h, nw = w;
    if (r != 1.0) { nw = (int)(w * r); nh = (int)(h * r); }
    if (nh < 1 || nw < 1 || nh > size || nw > size) return YH_EINVAL;
    const double dw = (size - nw) / 2.0, dh = (size - nh) / 2.0;
    im.h = h; im.w = w; im.nh = nh; im.nw = nw;
    im.top = (int)std::nearbyint(dh - 0.1);
    im.left = (int)std::nearbyint(dw - 0.1);
    return YH_OK;
}

constexpr int LB_MAX = 32;   // images per launch (kernarg-resident descriptors)
struct LbBatch {
    LbImage im[LB_MAX];
    unsigned char* dst;      // (n, 3, size, size) uint8
    int size, n;
};

__global__ __launch_bounds__(256) void letterbox_u8(const LbBatch b) {
    const int i = blockIdx.y;
    const int px = blockIdx.x * 256 + threadIdx.x;
    const int plane = b.size * b.size;
    if (px >= plane) return;
    unsigned char rgb[3];
    lb_pixel(b.im[i], px / b.size, px - (px / b.size) * b.size, rgb);
    unsigned char* o = b.dst + (size_t)i * 3 * plane + px;
    o[0] = rgb[0];
    o[plane] = rgb[1];
    o[2 * (size_t)plane] = rgb[2];
}

}  // namespace yh

using namespace yh;

extern "C" int yh_letterbox_geometry(int height, int width, int size, int* new_h, int* new_w, int* top,
                                     int* left) {
    LbImage im{};
    const int rc = lb_geometry(height, width, size, im);
    if (rc) return rc;
    if (new_h) *new_h = im.nh;
    if (new_w) *new_w = im.nw;
    if (top) *top = im.top;
    if (left) *left = im.left;
    return YH_OK;
}

extern "C" int yh_letterbox(const void* const* srcs, const int* heights, const int* widths, const int* strides,
                            int batch, int size, void* dst, void* stream) {
    if (batch < 0 || size <= 0 || (batch > 0 && (!srcs || !heights || !widths || !dst))) return YH_EINVAL;
    for (int b0 = 0; b0 < batch; b0 += LB_MAX) {
        LbBatch lb{};
        lb.n = batch - b0 < LB_MAX ? batch - b0 : LB_MAX;
        lb.size = size;
        lb.dst = static_cast<unsigned char*>(dst) + (size_t)b0 * 3 * size * size;
        for (int k = 0; k < lb.n; ++k) {
            LbImage& im = lb.im[k];
            const int rc = lb_geometry(heights[b0 + k], widths[b0 + k], size, im);
            if (rc) return rc;
            im.src = static_cast<const unsigned char*>(srcs[b0 + k]);
            im.stride = strides ? strides[b0 + k] : 3 * widths[b0 + k];
            if (!im.src || im.stride < 3 * im.w) return YH_EINVAL;
        }
        const dim3 g((unsigned)((size * size + 255) / 256), (unsigned)lb.n);
        hipLaunchKernelGGL(letterbox_u8, g, dim3(256), 0, (hipStream_t)stream, lb);
        if (hipGetLastError() != hipSuccess) return YH_EHIP;
    }
    return YH_OK;
}

extern "C" int yh_letterbox_host(const void* src, int height, int width, int stride, int size, void* dst,
                                 int threads) {
    LbImage im{};
    const int rc = lb_geometry(height, width, size, im);
    if (rc) return rc;
    if (!src || !dst) return YH_EINVAL;
    im.src = static_cast<const unsigned char*>(src);
    im.stride = stride > 0 ? stride : 3 * width;
    if (im.stride < 3 * width) return YH_EINVAL;
    unsigned char* o = static_cast<unsigned char*>(dst);
    const size_t plane = (size_t)size * size;
    auto rows = [&](int y0, int y1) {
        for (int y = y0; y < y1; ++y)
            for (int x = 0; x < size; ++x) {
                unsigned char rgb[3];
                lb_pixel(im, y, x, rgb);
                const size_t q = (size_t)y * size + x;
                o[q] = rgb[0]; o[plane + q] = rgb[1]; o[2 * plane + q] = rgb[2];
            }
    };
    int nt = threads > 0 ? threads : 1;
    nt = nt < size ? nt : size;
    if (nt <= 1) {
        rows(0, size);
        return YH_OK;
    }
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; ++t) pool.emplace_back(rows, size * t / nt, size * (t + 1) / nt);
    for (auto& th : pool) th.join();
    return YH_OK;
}

extern "C" int yh_resize_linear_host(const void* src, int height, int width, int stride, int new_h, int new_w,
                                     void* dst) {
    if (!src || !dst || height <= 0 || width <= 0 || new_h <= 0 || new_w <= 0) return YH_EINVAL;
    LbImage im{};
    im.src = static_cast<const unsigned char*>(src);
    im.h = height; im.w = width; im.nh = new_h; im.nw = new_w;
    im.stride = stride > 0 ? stride : 3 * width;
    if (im.stride < 3 * width) return YH_EINVAL;
    unsigned char* o = static_cast<unsigned char*>(dst);
    for (int y = 0; y < new_h; ++y)
        for (int x = 0; x < new_w; ++x) lb_resized(im, y, x, o + ((size_t)y * new_w + x) * 3);
    return YH_OK;
}
