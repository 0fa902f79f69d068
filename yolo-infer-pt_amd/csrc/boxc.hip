// Fused box branch of the detect head (16-bit handles, 64 box channels), all three levels in
// one launch: per level (nets/nn.py:240-247, 255-270)
//   box.l.0  Conv 3x3 C0 -> 64, SiLU        X (HBM) -> M (LDS)
//   box.l.1  Conv 3x3 64 -> 64, SiLU        M -> registers (rows permuted: the accumulators ARE
//                                           box.l.2's B fragments, c3k.hip's conv2 -> conv3 trick)
//   box.l.2  Conv2d 1x1 64 -> 64 (+ bias)   -> DFL softmax / expectation (nets/nn.py:222-225),
//            make_anchors (utils/util.py:85-96) and dist2bbox * stride (nn.py:264-268) -> rows
//            0..3 of the caller's y
// One workgroup (8 waves) per TH x TW output tile of one image of one level. The input tile
// with its 2-pixel halo arrives by LDS-DMA in passes of 64 channels (X); box.l.0 runs over the
// tile + a 1-pixel halo (M, zero outside the image = box.l.1's padding), one 32-pixel unit per
// wave with both 32-cout tiles (one B read feeds two MFMAs), and its output overwrites X once
// every wave is done with X; box.l.1 runs over the tile, one unit per wave. Every weight
// fragment streams through a ring of 18 KB LDS buffers (one 16-channel K block of both cout
// tiles x 9 taps per item), several items ahead. The box.l.0 / box.l.1 intermediates never reach
// HBM (at v11_n b32 640^2: 136 MB of writes and reads less than the seven per-layer launches).
//
// Bit-identical to box.l.0 / box.l.1 as conv_mx-family launches + box_dfl (common.h): the same
// canonical K order (for 16-channel block: for tap: one v_mfma_f32_32x32x16 step, fp32; for the
// K-split shapes of conv_mx.h's mx_kchunks the 64-channel chunk partials added in chunk order),
// + bias, SiLU, one rounding per layer output, box_dfl's decode arithmetic on the rounded logits.
#include "common.h"
#include "dtypes.h"

#include <algorithm>

namespace yh {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((ext_vector_type(2))) float bx_f32x2;

constexpr int BX_NW = 8;                  // waves per workgroup
constexpr int BX_THREADS = 64 * BX_NW;
constexpr int BX_ITEM = 18 * 1024;        // ring item: both 32-cout tiles x 9 taps of one K block
constexpr int BX_PPW = 3;                 // 1-KB DMA pieces per wave and item (8 x 3 >= 18)
#ifndef BX_NB_DEF
#define BX_NB_DEF 2
#endif
constexpr int BX_NB = BX_NB_DEF;          // ring buffers (2 / 3 / 5 measured alike: 142-157 us)

template <typename T> struct BMfma;
template <> struct BMfma<__bf16> {
    static __device__ __forceinline__ f32x16 step(const uint4& a, const uint4& b, const f32x16& c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                       0, 0);
    }
};
template <> struct BMfma<_Float16> {
    static __device__ __forceinline__ f32x16 step(const uint4& a, const uint4& b, const f32x16& c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                      0);
    }
};
template <typename T> struct BPk2;
template <> struct BPk2<__bf16> { typedef __attribute__((ext_vector_type(2))) __bf16 v2; };
template <> struct BPk2<_Float16> { typedef __attribute__((ext_vector_type(2))) _Float16 v2; };
// conv_mx's epilogue rounding (mx_epi's pack2)
template <typename T>
__device__ __forceinline__ unsigned bx_pack2(float a, float b) {
    return __builtin_bit_cast(unsigned, __builtin_convertvector(bx_f32x2{a, b}, typename BPk2<T>::v2));
}

__device__ __forceinline__ void bx_glds(const void* src, unsigned lds_addr) {
#if defined(__HIP_DEVICE_COMPILE__)
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds_addr) : "memory");
#else
    (void)src; (void)lds_addr;
#endif
}
__device__ __forceinline__ void bx_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// wait until at most k ring items (BX_PPW = 3 DMA instructions each) of this wave are in flight
__device__ __forceinline__ void bx_wait_items(int k) {
    switch (k) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
    }
}
// byte offset of 16-B chunk c of pixel p in a 64-channel (8-chunk) image, chunks swizzled by
// the pixel so a ds_read_b128 lane group of consecutive pixels spreads over the banks
__device__ __forceinline__ int bx_off(int p, int c) { return p * 128 + ((c ^ ((p >> 1) & 7)) << 4); }

// the decode's 16-bit exp and division (head.hip hx_exp / hx_div, misc.hip ex<T> / dv<T>)
__device__ __forceinline__ float bx_exp(float x) { return __expf(x); }
__device__ __forceinline__ float bx_div(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }

}  // namespace

// parameter image of one level (bytes): conv0 items [NCB0][tile 2][tap 9][lane 64][16 B], conv1
// items [4][2][9][64][16 B] (rows permuted for the B-fragment hand-off), the 1x1 [tile 2][kb 4]
// [64][16 B] (box_dfl's row permutation), then the fp32 biases b0[64], b1[64], b2[64]
__host__ __device__ inline int bx_prm_off_b(int C0) { return (C0 / 16 + 4) * BX_ITEM + 8 * 1024; }
int bx_prm_bytes(int C0) { return bx_prm_off_b(C0) + 3 * 64 * 4; }

// LDS of one workgroup for a TH x TW tile: the X / M region, the ring, a 1 KB dummy piece and
// the biases (768 B in a 1 KB DMA piece)
__host__ __device__ inline int bx_lds_bytes(int TH, int TW) {
    const int x = ((TH + 4) * (TW + 4) * 128 + 1023) & ~1023;
    return x + BX_NB * BX_ITEM + 2 * 1024;
}

namespace {

// 9 taps of one 16-channel K block (kb within the region's 64 channels) for both 32-cout tiles:
// B fragments from the LDS region `src` (pixel p of tap t = pb + (t / 3) rs + t % 3), A from
// the ring item wb; fragments read BX_PF taps ahead of their MFMAs (order pinned)
#ifndef BX_PF
#define BX_PF 2
#endif
template <typename T>
__device__ __forceinline__ void bx_taps(f32x16 (&d)[2], const char* src, int pb, int rs, int kb, const char* wb,
                                        int lane) {
    constexpr int PF = BX_PF, RING = BX_PF + 1;
    const int h = lane >> 5;
    uint4 fa[RING][2], fb[RING];
    auto ld = [&](int t, int buf) {
        const int p = pb + (t / 3) * rs + t % 3;
        fb[buf] = *reinterpret_cast<const uint4*>(src + p * 128 + (((2 * kb + h) ^ ((p >> 1) & 7)) << 4));
#pragma unroll
        for (int a = 0; a < 2; ++a) fa[buf][a] = *reinterpret_cast<const uint4*>(wb + ((a * 9 + t) * 64 + lane) * 16);
    };
#pragma unroll
    for (int t = 0; t < PF; ++t) ld(t, t);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
        if (t + PF < 9) ld(t + PF, (t + PF) % RING);
#pragma unroll
        for (int a = 0; a < 2; ++a) d[a] = BMfma<T>::step(fa[t % RING][a], fb[t % RING], d[a]);
    }
    __builtin_amdgcn_sched_group_barrier(0x100, 3 * PF, 0);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        if (t + PF < 9) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
    }
}

// KS: box.l.0 is a K-split shape (mx_kchunks = C0 / 64: the 64-channel chunk partials added in
// chunk order)
template <typename T, int NCB0, bool KS>
__device__ __forceinline__ void bx_body(const BoxChainArgs& A, int li, char* sm) {
    const BoxChainLevel& V = A.lv[li];
    constexpr int NITEMS = NCB0 + 5;                 // conv0 blocks, conv1's 4 blocks, the 1x1
    typedef __attribute__((address_space(3))) char* lds_c;
    const unsigned lds0 = (unsigned)(size_t)(lds_c)sm;
    const int lane = threadIdx.x & 63, l32 = lane & 31, h = lane >> 5;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // XCD-aware tile order within the level: neighbouring tiles (overlapping halos) on one L2
    const int wl = xcd_remap((int)blockIdx.x - V.wg0, A.B * V.tiles);
    const int n = wl / V.tiles, tix = wl - n * V.tiles;
    const int ty = tix / V.ntw, tx = tix - ty * V.ntw;
    const int TH = V.TH, TW = V.TW, H = V.H, W = V.W;
    const int h0 = ty * TH, w0 = tx * TW;
    const int XW = TW + 4, XH = TH + 4, MW = TW + 2, MH = TH + 2;
    const int NX = XH * XW, NM = MH * MW, NT = TH * TW;
    const int xbytes = (NX * 128 + 1023) & ~1023;
    char* XM = sm;                                   // X (64-channel pass), later M
    const int ring_off = xbytes;
    const int dummy_off = ring_off + BX_NB * BX_ITEM;
    const float* BI = reinterpret_cast<const float*>(sm + dummy_off + 1024);
    const char* prm = reinterpret_cast<const char*>(V.prm);
    const T* x = reinterpret_cast<const T*>(V.x);

    // ring item i -> buffer i % BX_NB: piece k (0..2) of wave wv is 1 KB piece 8 k + wv of the
    // item; pieces past the item's end go to the dummy KB (every wave issues BX_PPW per item)
    auto issue = [&](int i) {
        if (i >= NITEMS) return;
        const int np = i < NCB0 + 4 ? 18 : 8;
        const unsigned dst = lds0 + (unsigned)(ring_off + (i % BX_NB) * BX_ITEM);
        const char* src = prm + (size_t)i * BX_ITEM;
#pragma unroll
        for (int k = 0; k < BX_PPW; ++k) {
            const int pc = BX_NW * k + wv;
            if (pc < np) bx_glds(src + pc * 1024 + lane * 16, dst + (unsigned)(pc * 1024));
            else bx_glds(prm + lane * 16, lds0 + (unsigned)dummy_off);
        }
    };
    // X pass q (channels 64 q .. 64 q + 63) by LDS-DMA: pixel-chunk e = (pixel, chunk), zero
    // outside the image (box.l.0's padding)
    auto load_x = [&](int q) {
        for (int e0 = wv * 64; e0 < NX * 8; e0 += BX_THREADS) {
            const int e = e0 + lane;
            const int p = e >> 3, c = e & 7;
            const int r = p / XW, cc = p - r * XW;
            const int gy = h0 - 2 + r, gx = w0 - 2 + cc;
            const bool ok = e < NX * 8 && (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W;
            // the LDS address of chunk c of pixel p, swizzled (the DMA writes lane-linearly: this
            // lane's 16 B land at e0 * 16 + lane * 16, so the lane fetches the source chunk whose
            // swizzled slot that is)
            const int cs = c ^ ((p >> 1) & 7);
            const void* src = ok ? (const void*)(x + (((long long)n * H + gy) * W + gx) * V.ldx + 64 * q + 8 * cs)
                                 : A.zero;
            bx_glds(src, lds0 + (unsigned)(e0 * 16));
        }
    };

    // ---- prologue: X pass 0, the biases (48 lanes of one DMA; the rest copy zeros into the
    //      piece's tail), the first ring item
    load_x(0);
    if (wv == 0)
        bx_glds(lane < 48 ? (const void*)(prm + bx_prm_off_b(NCB0 * 16) + lane * 16) : A.zero, lds0 + (unsigned)(dummy_off + 1024));
    for (int i = 0; i < BX_NB - 1; ++i) issue(i);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bx_barrier();
    // ---- units: wave wv owns M pixels [32 wv, 32 wv + 32) (box.l.0) and tile pixels
    //      [32 wv, ...) (box.l.1 / the 1x1); lanes past the region compute clamped pixels
    const bool own0 = wv * 32 < NM, own1 = wv * 32 < NT;   // wave-uniform
    const int q0 = min(wv * 32 + l32, NM - 1);
    const int my = q0 / MW, mx = q0 - my * MW;
    const int q1 = min(wv * 32 + l32, NT - 1);
    const int oy = q1 / TW, ox = q1 - oy * TW;
    const int pb0 = my * XW + mx, pb1 = oy * MW + ox;   // tap (0, 0) pixel in X / M
    f32x16 acc[2], part[KS ? 2 : 1];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[a][e] = 0.f;
    uint4 bq[4];   // box.l.1's output = the 1x1's B fragments (K blocks 0..3)

#pragma unroll 1
    for (int i = 0; i < NITEMS; ++i) {
        // this wave's pieces of item i landed (items i + 1 .. i + NB - 2 may stay in flight), then
        // everyone's; step i - 1 is done everywhere
        bx_wait_items(min(i + BX_NB - 1, NITEMS) - (i + 1));
        bx_barrier();
        issue(i + BX_NB - 1);
        const char* wb = sm + ring_off + (i % BX_NB) * BX_ITEM;
        if (i < NCB0) {
            // ---- box.l.0, K block cb = i over X pass cb / 4
            const int cb = i;
            if (cb % 4 == 0 && cb > 0) {
                // a new 64-channel pass: every wave is past the previous one (the barrier above)
                load_x(cb / 4);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                bx_barrier();
            }
            if (own0) {
                const int kb = cb & 3;   // 16-channel block within the pass
                if constexpr (!KS) {
                    bx_taps<T>(acc, XM, pb0, XW, kb, wb, lane);
                } else {
                    if (kb == 0) {
#pragma unroll
                        for (int a = 0; a < 2; ++a)
#pragma unroll
                            for (int e = 0; e < 16; ++e) part[a][e] = 0.f;
                    }
                    bx_taps<T>(part, XM, pb0, XW, kb, wb, lane);
                    if (kb == 3) {   // the 64-channel chunk's partial, added in chunk order
#pragma unroll
                        for (int a = 0; a < 2; ++a) {
                            if (cb == 3) acc[a] = part[a];
                            else
#pragma unroll
                                for (int e = 0; e < 16; ++e) acc[a][e] += part[a][e];
                        }
                    }
                }
            }
            continue;
        }
        if (i == NCB0) {
            // ---- box.l.0's epilogue: every wave is done with X (the barrier above); bias, SiLU,
            //      one rounding, zeros outside the image -> M (over X), then box.l.1 may read it
            if (own0 && wv * 32 + l32 < NM) {
                const int gy = h0 - 1 + my, gx = w0 - 1 + mx;
                const bool in = (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W;
#pragma unroll
                for (int a = 0; a < 2; ++a) {
                    unsigned w8[8];
#pragma unroll
                    for (int e = 0; e < 16; e += 2) {
                        const int co = 32 * a + 16 * h + e;
                        w8[e >> 1] = in ? bx_pack2<T>(silu<T>(acc[a][e] + BI[co]), silu<T>(acc[a][e + 1] + BI[co + 1])) : 0u;
                    }
                    *reinterpret_cast<uint4*>(XM + bx_off(q0, 4 * a + 2 * h)) = make_uint4(w8[0], w8[1], w8[2], w8[3]);
                    *reinterpret_cast<uint4*>(XM + bx_off(q0, 4 * a + 2 * h + 1)) = make_uint4(w8[4], w8[5], w8[6], w8[7]);
                }
            }
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[a][e] = 0.f;
            bx_barrier();
        }
        if (i < NCB0 + 4) {
            // ---- box.l.1, K block kb over M
            const int kb = i - NCB0;
            if (own1) {
                bx_taps<T>(acc, XM, pb1, MW, kb, wb, lane);
                if (kb == 3) {
                    // bias, SiLU, one rounding; register 8 jj + e of tile a is channel 32 a + 16 jj
                    // + 8 h + e (the permuted rows): the 1x1's B fragment of K block 2 a + jj
                    const float* b1 = BI + 64;
#pragma unroll
                    for (int a = 0; a < 2; ++a)
#pragma unroll
                        for (int jj = 0; jj < 2; ++jj) {
                            const float* bj = b1 + 32 * a + 16 * jj + 8 * h;
                            unsigned w4[4];
#pragma unroll
                            for (int e = 0; e < 8; e += 2)
                                w4[e >> 1] = bx_pack2<T>(silu<T>(acc[a][8 * jj + e] + bj[e]), silu<T>(acc[a][8 * jj + e + 1] + bj[e + 1]));
                            bq[2 * a + jj] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
                        }
                }
            }
            continue;
        }
        // ---- box.l.2 (1x1, 64 -> 64, + bias) + DFL + anchors + dist2bbox -> y rows 0..3
        if (!own1) continue;
        float dist[2];
        const float* b2 = BI + 128;
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            f32x16 c;
#pragma unroll
            for (int e = 0; e < 16; ++e) c[e] = 0.f;
#pragma unroll
            for (int kb = 0; kb < 4; ++kb)
                c = BMfma<T>::step(*reinterpret_cast<const uint4*>(wb + ((a * 4 + kb) * 64 + lane) * 16), bq[kb], c);
            // register i: cout 32 h + 16 a + i = bin i of side 2 h + a; the conv's rounding first
            float v[16];
#pragma unroll
            for (int e = 0; e < 16; ++e) v[e] = tof(fromf<T>(c[e] + b2[32 * h + 16 * a + e]));
            float mxv = v[0];
#pragma unroll
            for (int e = 1; e < 16; ++e) mxv = fmaxf(mxv, v[e]);
            float sum = 0.f;
#pragma unroll
            for (int e = 0; e < 16; ++e) { v[e] = bx_exp(v[e] - mxv); sum += v[e]; }
            float d = 0.f;
#pragma unroll
            for (int e = 0; e < 16; ++e) d = fmaf((float)e, bx_div(v[e], sum), d);
            dist[a] = d;
        }
        const float o0 = xor32_swap(dist[0]), o1 = xor32_swap(dist[1]);
        const float dl = h ? o0 : dist[0], dt = h ? o1 : dist[1];
        const float dr = h ? dist[0] : o0, db = h ? dist[1] : o1;
        const int gy = h0 + oy, gx = w0 + ox;
        if (wv * 32 + l32 < NT && gy < H && gx < W) {
            const float ax = (float)gx + 0.5f, ay = (float)gy + 0.5f, st = V.stride;
            const float x1 = ax - dl, y1 = ay - dt;
            const float x2 = ax + dr, y2 = ay + db;
            const float r0 = h ? (x2 - x1) * st : (x1 + x2) / 2.0f * st;
            const float r1 = h ? (y2 - y1) * st : (y1 + y2) / 2.0f * st;
            const gptr<T> col = io_global<T>(A.io[1]) + ((long long)n * (4 + A.nc) + 2 * h) * A.A + V.aoff + gy * W + gx;
            col[0] = fromf<T>(r0);
            col[A.A] = fromf<T>(r1);
        }
    }
}

template <typename T>
__global__ __launch_bounds__(BX_THREADS, 2) void box_chain(const BoxChainArgs A) {
    extern __shared__ __attribute__((aligned(1024))) char bsm[];
    int li = 0;
    if (A.nlv > 1 && (int)blockIdx.x >= A.lv[1].wg0) li = 1;
    if (A.nlv > 2 && (int)blockIdx.x >= A.lv[2].wg0) li = 2;
    const bool ks = A.lv[li].nkc > 1;
    switch (A.lv[li].C0) {
        case 64: bx_body<T, 4, false>(A, li, bsm); break;
        case 128: if (ks) bx_body<T, 8, true>(A, li, bsm); else bx_body<T, 8, false>(A, li, bsm); break;
        case 256: if (ks) bx_body<T, 16, true>(A, li, bsm); else bx_body<T, 16, false>(A, li, bsm); break;
        case 512: bx_body<T, 32, false>(A, li, bsm); break;
    }
}

}  // namespace

// output tile of a level: the largest candidate with <= 8 units of 32 pixels in both convs
// (tile + 1-pixel halo, and the tile), the least padding waste first, within the 160 KB of LDS
bool bx_tile(int H, int W, int& TH, int& TW) {
    static const int cand[][2] = {{12, 16}, {8, 20}, {8, 16}, {5, 20}, {10, 10}, {8, 8}, {4, 16}, {4, 8}, {4, 4}, {2, 4}};
    double best = 1e30;
    bool found = false;
    for (auto& c : cand) {
        const int th = std::min(c[0], H), tw = std::min(c[1], W);
        if ((th + 2) * (tw + 2) > 256 || th * tw > 256 || bx_lds_bytes(th, tw) > 160 * 1024) continue;
        // cost per output: padded tiles' box.l.0 units (halo) + box.l.1 units
        const int ntw = (W + tw - 1) / tw, nth = (H + th - 1) / th;
        const double units = (double)ntw * nth * (((th + 2) * (tw + 2) + 31) / 32 * 2.0 + (th * tw + 31) / 32);
        const double cost = units / ((double)H * W);
        if (cost < best - 1e-9) {
            best = cost;
            TH = th;
            TW = tw;
            found = true;
        }
    }
    return found;
}

bool bx_ok(int C0) { return C0 == 64 || C0 == 128 || C0 == 256 || C0 == 512; }

template <typename T>
static int launch_box_chain_t(const BoxChainArgs& a, hipStream_t s) {
    int grid = 0, lds = 0;
    for (int l = 0; l < a.nlv; ++l) {
        const BoxChainLevel& v = a.lv[l];
        if (!bx_ok(v.C0) || v.wg0 != grid || v.ldx % 8 || (v.nkc != 1 && v.C0 / 64 != v.nkc)) return (int)hipErrorInvalidValue;
        if ((v.TH + 2) * (v.TW + 2) > 256 || v.TH * v.TW > 256) return (int)hipErrorInvalidValue;
        grid += a.B * v.tiles;
        lds = std::max(lds, bx_lds_bytes(v.TH, v.TW));
    }
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&box_chain<T>), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        attr = true;
    }
    hipLaunchKernelGGL((box_chain<T>), dim3((unsigned)grid), dim3(BX_THREADS), lds, s, a);
    return (int)hipGetLastError();
}

int launch_box_chain(int dtype, const BoxChainArgs& a, hipStream_t s) {
    switch (dtype) {
        case F16: return launch_box_chain_t<_Float16>(a, s);
        case BF16: return launch_box_chain_t<__bf16>(a, s);
    }
    return (int)hipErrorInvalidValue;
}

}  // namespace yh
