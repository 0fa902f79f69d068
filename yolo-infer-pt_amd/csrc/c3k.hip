// Fused C3k block (nets/nn.py:52-63, CSPModule(c, c) with two Residual(c/2, e=1.0)) for
// the 16-bit handles, hidden width h = c / 2 = 32 or 64 (the HH template parameter), on maps
// whose bands keep their intermediates in LDS (v11_n at 640 x 640: net.p4.1.res_m.0 at 40x40
// with h = 32, net.p5.1.res_m.0 / fpn.h6.res_m.0 at 20x20 with h = 64).
//
// One workgroup (16 waves) per band of RB output rows of one image (the launcher cuts each
// image into `bands` bands so that a batch fills the chip, and so that every band's region
// fits). The chain of four 3x3 convs needs a 4-row halo: a workgroup keeps the rows
// [r0 - 4, r1 + 4) of its band (clipped to the image) in LDS and each phase computes the
// rows its successors read (B: halo 3, C: 2, D: 1, E and F: the band itself); pixels outside a
// phase's rows are neither computed nor written. A 32-pixel tile per wave in every phase
// (phase A also runs the region's bottom rows past the 16 waves' 512 pixels, conv1 only):
//   A   C1 = conv1(x)            1x1 c -> h, + SiLU                   x from HBM -> LDS C1
//   B   T  = r0.conv1(C1)        3x3 h -> h, + SiLU                   LDS -> LDS
//   C   C1 = r0.conv2(T) + C1    3x3 h -> h, + SiLU, + residual       in place (nn.py:49)
//   D   T  = r1.conv1(C1)
//   E   C1 = r1.conv2(T) + C1
//   F   y  = conv3([C1 | c2])    1x1 2h -> c, + SiLU             c2 = conv2(x), from phase A
// The 3x3 convs' weights (one 18-step image per 32-cout tile and pair of 16-channel blocks)
// and then conv3's stream through a ring of 18 KB LDS buffers by LDS-DMA, several items
// ahead of the one being multiplied (one copy per workgroup, read by every wave). conv2
// never reaches LDS: its A rows are permuted (bits 2 and 3 swapped) so that a lane's
// accumulator registers 8 jj .. 8 jj + 7 ARE conv3's B fragment of K block h / 16 + 2 t + jj.
//
// Bit-identical to the per-layer conv_mx launches (conv_mx.h): every conv walks its K as
// for 16-channel block: for tap: one v_mfma_f32_32x32x16 step, + bias, SiLU, one rounding
// (pack2, as mx_epi); the residual is added to the rounded value in fp32 and rounded again.
#include "common.h"
#include "dtypes.h"

#include <algorithm>
#include <cstdlib>

namespace yh {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((ext_vector_type(2))) float ck_f32x2;

constexpr int CK_NW = 16;                // waves per workgroup
constexpr int CK_THREADS = 64 * CK_NW;
constexpr int CK_MINRB = 4;              // rows per band at least (the 4-row halo recomputation)

template <typename T> struct KMfma;
template <> struct KMfma<__bf16> {
    static __device__ __forceinline__ f32x16 step(const uint4& a, const uint4& b, const f32x16& c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                       0, 0);
    }
};
template <> struct KMfma<_Float16> {
    static __device__ __forceinline__ f32x16 step(const uint4& a, const uint4& b, const f32x16& c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                      0);
    }
};
template <typename T> struct KPk2;
template <> struct KPk2<__bf16> { typedef __attribute__((ext_vector_type(2))) __bf16 v2; };
template <> struct KPk2<_Float16> { typedef __attribute__((ext_vector_type(2))) _Float16 v2; };
// the rounding of conv_mx's epilogue (mx_epi's pack2)
template <typename T>
__device__ __forceinline__ unsigned ck_pack2(float a, float b) {
    return __builtin_bit_cast(unsigned, __builtin_convertvector(ck_f32x2{a, b}, typename KPk2<T>::v2));
}
template <typename T>
__device__ __forceinline__ float ck_lo(unsigned u) { return (float)__builtin_bit_cast(T, (unsigned short)(u & 0xffffu)); }
template <typename T>
__device__ __forceinline__ float ck_hi(unsigned u) { return (float)__builtin_bit_cast(T, (unsigned short)(u >> 16)); }

__device__ __forceinline__ void ck_glds(const void* src, unsigned lds_addr) {
#if defined(__HIP_DEVICE_COMPILE__)
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds_addr) : "memory");
#else
    (void)src; (void)lds_addr;
#endif
}
__device__ __forceinline__ void ck_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// swizzled 16-B chunk c of pixel p (C1 / T, HH channels = HH / 8 chunks per pixel):
// consecutive pixels spread over the bank slots
template <int HH>
__device__ __forceinline__ int ck_off(int p, int c) { return p * (2 * HH) + ((c ^ ((p >> 1) & (HH / 8 - 1))) << 4); }

// 16 consecutive couts of one pixel (lane half h of a 32-cout tile, fragment rows as
// c3k2.hip / conv_mx): bias, SiLU, one rounding -> 8 packed words
template <typename T>
__device__ __forceinline__ void ck_act(const f32x16& acc, const float* b, unsigned (&w)[8]) {
    // 16 biases as four 16-B reads (b is 64-B aligned: 16 h floats past a 32-float boundary)
    f32x4 bv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[i] = reinterpret_cast<const f32x4*>(b)[i];
#pragma unroll
    for (int e = 0; e < 16; e += 2)
        w[e >> 1] = ck_pack2<T>(silu<T>(acc[e] + bv[e >> 2][e & 3]), silu<T>(acc[e + 1] + bv[e >> 2][(e + 1) & 3]));
}

// 1x1 conv step chain of one 32-cout tile: NK K blocks, A fragments from LDS at w (read
// CK_PF1 steps ahead of their MFMA, the order pinned through scheduling), B in registers
#ifndef CK_PF1
#define CK_PF1 4
#endif
template <typename T, int NK>
__device__ __forceinline__ f32x16 ck_1x1(const char* w, int lane, const uint4 (&bv)[NK]) {
    constexpr int PF = CK_PF1 < NK ? CK_PF1 : NK;
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    uint4 fa[PF + 1];
#pragma unroll
    for (int st = 0; st < PF; ++st) fa[st] = *reinterpret_cast<const uint4*>(w + (st * 64 + lane) * 16);
#pragma unroll
    for (int st = 0; st < NK; ++st) {
        if (st + PF < NK) fa[(st + PF) % (PF + 1)] = *reinterpret_cast<const uint4*>(w + ((st + PF) * 64 + lane) * 16);
        acc = KMfma<T>::step(fa[st % (PF + 1)], bv[st], acc);
    }
    __builtin_amdgcn_sched_group_barrier(0x100, PF, 0);
#pragma unroll
    for (int st = 0; st < NK; ++st) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (st + PF < NK) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    return acc;
}

}  // namespace

// pixels of the largest band region: RB = ceil(H / bands) rows + 4 halo rows on each side
__host__ __device__ inline int ck_region_px(int H, int W, int bands) {
    const int rb = (H + bands - 1) / bands;
    return (rb + 8 < H ? rb + 8 : H) * W;
}

// parameter image (bytes) of a block with HH hidden channels (c = 2 HH): fragments
// [tile][step][64 lanes][16 B], then fp32 biases
struct CkLayout {
    int w1, w2, wr, w3, b1, b2, br, b3, total;
};
template <int HH>
__host__ __device__ constexpr CkLayout ck_layout() {
    constexpr int NT3 = HH / 32, NK1 = HH / 8, NK3 = 9 * (HH / 16), NTO = HH / 16;
    CkLayout L{};
    L.w1 = 0;                                // conv1: NT3 tiles x NK1 K blocks (c -> h)
    L.w2 = L.w1 + NT3 * NK1 * 1024;          // conv2: the same (rows permuted for conv3's B fragments)
    L.wr = L.w2 + NT3 * NK1 * 1024;          // 4 Residual convs: [conv][tile][NK3 steps]
    L.w3 = L.wr + 4 * NT3 * NK3 * 1024;      // conv3: NTO tiles x NK1 K blocks (2h -> c)
    L.b1 = L.w3 + NTO * NK1 * 1024;
    L.b2 = L.b1 + HH * 4;
    L.br = L.b2 + HH * 4;                    // [conv][HH]
    L.b3 = L.br + 4 * HH * 4;
    L.total = L.b3 + 2 * HH * 4;
    return L;
}

// micro benchmark builds (tools/micro, -DYH_ABLATION): s_memrealtime stamps of wave 0 per
// workgroup (0 entry, 1 prologue waited, 2 phase A done, 3 + i ring item i's barrier passed,
// 3 + NITEMS exit); nothing in the shipped library
constexpr int CK_NSTAMP = 24;
#ifdef YH_ABLATION
#define CK_STAMP(k)                                                                                       \
    do {                                                                                                  \
        if (A.trace && threadIdx.x == 0) A.trace[blockIdx.x * CK_NSTAMP + (k)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define CK_STAMP(k) do { } while (0)
#endif

namespace {

constexpr int CK_WBH = 18 * 1024;   // one weight buffer: 18 steps (two 16-channel blocks x 9 taps)
constexpr int CK_IW = 9;            // waves that issue a ring item (2 x 1 KB each, uniform)
constexpr int CK_MAXNB = 6;         // ring buffers at most
#ifndef CK_PF
#define CK_PF 3                     // 3x3 steps whose LDS reads are in flight ahead of the MFMA
#endif

// wait until at most k ring items (2 k LDS-DMA instructions) of this wave are in flight
__device__ __forceinline__ void ck_wait_items(int k) {
    switch (k) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    }
}

// LDS layout of a workgroup (bytes): C1 [rpx][hh], T [max(rpx hh, conv1 + conv2 weights)],
// nb ring buffers of 18 KB, the zero block (128 B), the biases (32 hh B)
__host__ __device__ inline int ck_tt_bytes(int hh, int rpx) {
    const int w12 = 2 * (hh / 32) * (hh / 8) * 1024;
    return rpx * 2 * hh > w12 ? rpx * 2 * hh : w12;
}

// SPLIT (h = 64, regions whose phases B..F fit 8 pixel tiles): waves w and w + 8 take the same
// pixel tile and the two 32-cout tiles of each 3x3 conv (a step multiplies two ring items, one
// per wave group; conv2's output waits in LDS for phase F): every wave has a tile in every
// phase instead of half of them, and the number of steps halves. Same per-tile arithmetic.
template <typename T, int HH, bool SPLIT>
__global__ __launch_bounds__(CK_THREADS, 1) void c3k_fused(const C3kArgs A) {
    constexpr CkLayout L = ck_layout<HH>();
    constexpr int PX = 2 * HH;                       // LDS bytes per pixel of C1 / T
    constexpr int CPX = HH / 8;                      // 16-B chunks per pixel
    constexpr int NT3 = HH / 32;                     // 32-cout tiles of conv1 / conv2 / the 3x3 convs
    constexpr int NCB = HH / 16;                     // 16-channel blocks of h
    constexpr int HALVES = NCB / 2;                  // ring items per 3x3 tile
    constexpr int NK1 = HH / 8;                      // K blocks of conv1 / conv2 / conv3 (c = 2h inputs)
    constexpr int NTO = HH / 16;                     // 32-cout tiles of conv3
    constexpr int NHS = 4 * NT3 * HALVES;            // 3x3 sub-phases (one ring item each)
    constexpr int W12 = NT3 * NK1 * 1024;            // conv1's (and conv2's) weight bytes
    constexpr int W3 = NTO * NK1 * 1024;             // conv3's weight bytes
    constexpr int TPG = 16 / NK1;                    // conv3 tiles per ring item (16 KB of it)
    constexpr int NITEMS = NHS + (NTO + TPG - 1) / TPG;
    constexpr int NS = SPLIT ? 2 : 1;                // ring items per step (one per wave group)
    constexpr int NSTEP = (NITEMS + NS - 1) / NS;
    static_assert(!SPLIT || (NT3 == 2 && NHS % 2 == 0 && NITEMS - NHS == 2), "two wave groups");
    extern __shared__ __attribute__((aligned(1024))) char sm[];
    typedef __attribute__((address_space(3))) char* lds_c;
    const unsigned lds0 = (unsigned)(size_t)(lds_c)sm;
    // band rows [r0, r1) of image n; LDS region rows [ra0, ra1) (the band + its 4-row halo)
    // XCD-aware: the bands of one image (whose halo rows overlap) on one XCD, i.e. one L2
    const int lb = xcd_remap(blockIdx.x, gridDim.x);
    const int n = lb / A.bands, band = lb - n * A.bands;
    const int RB = (A.H + A.bands - 1) / A.bands;
    const int r0 = band * RB, r1 = min(A.H, r0 + RB);
    const int ra0 = max(0, r0 - 4), ra1 = min(A.H, r1 + 4);
    const int NRP = (ra1 - ra0) * A.W;               // region pixels
    const int RPX = ck_region_px(A.H, A.W, A.bands);   // LDS pixels per region image (the largest band's)
    const int NB = A.nbuf;                           // ring buffers (2 .. CK_MAXNB)
    char* C1 = sm;                                   // [RPX][HH] (swizzled chunks)
    char* TT = sm + RPX * PX;                        // [RPX][HH]; conv1 / conv2's weights before B
    char* C2 = TT + ck_tt_bytes(HH, RPX);            // SPLIT: [RB W][HH], conv2(x) of the band's pixels
    const int wb_off = (int)(C2 - sm) + (SPLIT ? RB * A.W * PX : 0);
    char* WB = sm + wb_off;                          // the ring
    char* ZR = WB + NB * CK_WBH;                     // 128 zero bytes (out-of-image taps)
    const float* BI = reinterpret_cast<const float*>(ZR + 128);   // every bias (32 HH bytes)
    const int lane = threadIdx.x & 63, l32 = lane & 31, h = lane >> 5;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const char* prm = reinterpret_cast<const char*>(A.prm);
    CK_STAMP(0);
    if (r0 >= A.H) return;   // workgroup-uniform (no band rows: nothing issued yet)
    // LDS-DMA of `kb` 1-KB pieces from the parameter image at `src` to LDS offset `dst`
    auto dma = [&](int src, int dst, int kb) {
        for (int i = wv; i < kb; i += CK_NW) ck_glds(prm + src + i * 1024 + lane * 16, lds0 + (unsigned)(dst + i * 1024));
    };
    // ring item i -> buffer i % NB: the 3x3 sub-phases' 18-step weight images, then conv3's
    // weights in 16 KB items; waves 0..8 issue two 1-KB pieces each (pieces past an item's
    // end repeat its first piece into the buffer's unused tail), so every issuing wave has
    // the same count in flight per item
    auto issue = [&](int i) {
        if (i >= NITEMS || wv >= CK_IW) return;   // wave-uniform
        int src = L.wr + i * CK_WBH, np = 18;
        if (i >= NHS) {
            src = L.w3 + (i - NHS) * 16 * 1024;
            np = min(16, (W3 - (i - NHS) * 16 * 1024) / 1024);
        } else if (SPLIT) {   // item order (conv, half, tile): a step's two items are one conv's two tiles
            const int cv = i / (NT3 * HALVES), rem = i - cv * NT3 * HALVES, half = rem / NT3, t = rem - half * NT3;
            src = L.wr + ((cv * NT3 + t) * HALVES + half) * CK_WBH;
        }
        const unsigned dst = lds0 + (unsigned)(wb_off + (i % NB) * CK_WBH);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int pc = 2 * wv + k;
            ck_glds(prm + src + (pc < np ? pc : 0) * 1024 + lane * 16, dst + (unsigned)(pc * 1024));
        }
    };

    // prologue: conv1's and conv2's weights into T (free until the first Residual conv writes
    // it), the biases; the x fragments of the wave's tile; the first NB - 1 ring items
    dma(L.w1, (int)(TT - sm), 2 * W12 / 1024);       // w1, w2 are adjacent in the image
    dma(L.b1, (int)((const char*)BI - sm), (L.total - L.b1) / 1024);
    if (threadIdx.x < 8) *reinterpret_cast<uint4*>(ZR + threadIdx.x * 16) = make_uint4(0, 0, 0, 0);
    // the wave's pixel tile: 32 consecutive region pixels (clamped; only p < NRP is written).
    // Phases B..F only reach the first 16 tiles (the launcher's bands guarantee it); region
    // pixels past them (bottom halo rows of wide bands) get C1 from extra phase-A tiles.
    // phase A: tile wv (conv1 of all 16 tiles); phases B..F: tile bt = wv (SPLIT: wv % 8) and,
    // with SPLIT, the cout tile / ring item tg = wv / 8
    const int pa = wv * 32 + l32;
    const bool owna = wv * 32 < NRP, pva = pa < NRP;
    const int bt = SPLIT ? (wv & 7) : wv, tg = SPLIT ? (wv >> 3) : 0;
    const int p = bt * 32 + l32;
    const bool own = bt * 32 < NRP;                  // wave-uniform: the wave has a tile
    const bool pv = p < NRP;
    const int pc = pv ? p : NRP - 1;
    const int py = ra0 + pc / A.W, px = pc - (py - ra0) * A.W;   // image row / column
    const int bofs = (r0 - ra0) * A.W, nbp = (r1 - r0) * A.W;   // band pixels in the region
    // rows of the wave's tile (wave-uniform): a phase runs the tile iff it meets the phase's rows
    const int ty0 = ra0 + (bt * 32) / A.W, ty1 = ra0 + (min(bt * 32 + 31, NRP - 1)) / A.W;
    auto live = [&](int lo, int hi) { return own && ty1 >= lo && ty0 < hi; };
    auto xrow = [&](int q) {
        const int qy = ra0 + q / A.W, qx = q - (qy - ra0) * A.W;
        return reinterpret_cast<const T*>(A.x) + (((long long)n * A.H + qy) * A.W + qx) * A.ldx + 8 * h;
    };
    uint4 xb[NK1];
    {
        const T* xp = xrow(pva ? pa : NRP - 1);
#pragma unroll
        for (int kb = 0; kb < NK1; ++kb) xb[kb] = *reinterpret_cast<const uint4*>(xp + 16 * kb);
    }
    for (int i = 0; i < NB - NS; ++i) issue(i);
    if (wv < CK_IW) ck_wait_items(min(NB - NS, NITEMS));   // all but the ring items
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ck_barrier();
    CK_STAMP(1);

    // ---- A: C1 = SiLU(conv1(x)) -> LDS; conv2(x) -> registers (its rows permuted: registers
    //      8 jj .. + 7 of tile t are channels 32 t + 16 jj + 8 h .. + 7 = conv3's B fragment of
    //      K block NCB + 2 t + jj), held until phase F. B fragments from HBM, A from LDS.
    uint4 bf[NK1];
    f32x16 acc;
    auto conv1_tile = [&](int q, bool qv) {
        const char* w1 = TT;
#pragma unroll
        for (int t = 0; t < NT3; ++t) {
            const f32x16 a1 = ck_1x1<T, NK1>(w1 + t * NK1 * 1024, lane, xb);
            unsigned w[8];
            ck_act<T>(a1, BI + 32 * t + 16 * h, w);
            if (qv) {
                *reinterpret_cast<uint4*>(C1 + ck_off<HH>(q, 4 * t + 2 * h)) = make_uint4(w[0], w[1], w[2], w[3]);
                *reinterpret_cast<uint4*>(C1 + ck_off<HH>(q, 4 * t + 2 * h + 1)) = make_uint4(w[4], w[5], w[6], w[7]);
            }
        }
    };
    if (owna) {
        // SPLIT: only tiles that meet the band, conv2's output to C2 (wave-uniform)
        if (!SPLIT || (wv * 32 + 31 >= bofs && wv * 32 < bofs + nbp)) {
            const char* w2 = TT + W12;
            const float* b2 = BI + (L.b2 - L.b1) / 4;
            const int bp = pa - bofs;
            const bool bv = pva && bp >= 0 && bp < nbp;
#pragma unroll
            for (int t = 0; t < NT3; ++t) {
                acc = ck_1x1<T, NK1>(w2 + t * NK1 * 1024, lane, xb);
#pragma unroll
                for (int jj = 0; jj < 2; ++jj) {
                    const float* bj = b2 + 32 * t + 16 * jj + 8 * h;
                    unsigned w[4];
#pragma unroll
                    for (int e = 0; e < 8; e += 2)
                        w[e >> 1] = ck_pack2<T>(silu<T>(acc[8 * jj + e] + bj[e]), silu<T>(acc[8 * jj + e + 1] + bj[e + 1]));
                    if (SPLIT) {
                        if (bv) *reinterpret_cast<uint4*>(C2 + ck_off<HH>(bp, 4 * t + 2 * jj + h)) = make_uint4(w[0], w[1], w[2], w[3]);
                    } else {
                        bf[NCB + 2 * t + jj] = make_uint4(w[0], w[1], w[2], w[3]);
                    }
                }
            }
        }
        conv1_tile(pa, pva);
    }
    for (int q0 = wv * 32 + 32 * CK_NW; q0 < NRP; q0 += 32 * CK_NW) {   // wave-uniform
        const int q = q0 + l32;
        const bool qv = q < NRP;
        const T* xq = xrow(qv ? q : NRP - 1);
#pragma unroll
        for (int kb = 0; kb < NK1; ++kb) xb[kb] = *reinterpret_cast<const uint4*>(xq + 16 * kb);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (ring items too: rare, harmless)
        conv1_tile(q, qv);
    }

    // 3x3 taps of the wave's pixel: pixel byte offset within C1 / T with the chunk swizzle in
    // its low bits (-PX: outside the image, read from the zero block)
    int tq[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
        const int yy = py + t / 3 - 1, xx = px + t % 3 - 1;
        // outside the image: the zero block; outside the region (only taps of pixels whose
        // outputs no later phase reads): the zero block too
        const bool in = yy >= ra0 && yy < ra1 && (unsigned)xx < (unsigned)A.W;
        const int q = (yy - ra0) * A.W + xx;
        tq[t] = in ? (q * PX) | ((q >> 1) & (CPX - 1)) : -PX;
    }
    const int zr_off = (int)(ZR - sm);
    CK_STAMP(2);
    const float* b3 = BI + (L.b3 - L.b1) / 4;
    T* y = reinterpret_cast<T*>(A.y) + (((long long)n * A.H + py) * A.W + px) * A.ldy;
    const bool fl = live(r0, r1);

    // ---- B..E: the Residual convs, one 32-cout tile per NCB / 2 ring items (18 weight steps
    //      each); F: conv3 over [C1 | conv2] -> y, TPG tiles per ring item. Item i is in
    //      buffer i % NB; items i + 1 .. i + NB - 2 are in flight while it is multiplied, and
    //      item i + NB - 1 is issued into the buffer item i - 1 used.
#pragma unroll 1
    for (int j = 0; j < NSTEP; ++j) {
        const int i0 = j * NS;
        // this wave's pieces of the step's items landed (items issued so far: min(i0 + NB - NS,
        // NITEMS); the ones after the step's may stay in flight)
        if (wv < CK_IW) ck_wait_items(min(i0 + NB - NS, NITEMS) - min(i0 + NS, NITEMS));
        ck_barrier();   // ... and everyone's; step j - 1's buffers and the previous phase are done
        CK_STAMP(3 + j);
#pragma unroll
        for (int k = 0; k < NS; ++k) issue(i0 + NB - NS + k);
        const int i = i0 + tg;                       // this wave's item
        const char* wb = WB + (i % NB) * CK_WBH;
        if (i0 >= NHS) {
            // ---- F
            if (!fl || i >= NITEMS) continue;
            if (SPLIT) {
                const int bpc = min(max(pc - bofs, 0), nbp - 1);
#pragma unroll
                for (int kb = 0; kb < NCB; ++kb) {
                    bf[kb] = *reinterpret_cast<const uint4*>(C1 + ck_off<HH>(pc, 2 * kb + h));
                    bf[NCB + kb] = *reinterpret_cast<const uint4*>(C2 + ck_off<HH>(bpc, 2 * kb + h));
                }
            } else if (i == NHS) {
#pragma unroll
                for (int kb = 0; kb < NCB; ++kb) bf[kb] = *reinterpret_cast<const uint4*>(C1 + ck_off<HH>(pc, 2 * kb + h));
            }
            const int g = i - NHS;
#pragma unroll
            for (int tt = 0; tt < TPG; ++tt) {
                const int t = g * TPG + tt;
                if (t >= NTO) break;
                const char* w3 = wb + tt * NK1 * 1024;
                acc = ck_1x1<T, NK1>(w3, lane, bf);
                unsigned w[8];
                ck_act<T>(acc, b3 + 32 * t + 16 * h, w);
                if (pv && py >= r0 && py < r1) {
                    uint4* d = reinterpret_cast<uint4*>(y + 32 * t + 16 * h);
                    d[0] = make_uint4(w[0], w[1], w[2], w[3]);
                    d[1] = make_uint4(w[4], w[5], w[6], w[7]);
                }
            }
            continue;
        }
        int cv, t, half;
        if (SPLIT) {
            cv = i0 / (NT3 * HALVES);
            half = (i0 - cv * NT3 * HALVES) / NT3;
            t = tg;
        } else {
            cv = i / (NT3 * HALVES);
            t = (i / HALVES) % NT3;
            half = i % HALVES;
        }
        char* src = (cv & 1) ? TT : C1;
        char* dst = (cv & 1) ? C1 : TT;
        // rows this conv must produce: the band + (3 - cv) halo rows (what conv cv + 1 reads)
        const int lo = max(0, r0 - (3 - cv)), hi = min(A.H, r1 + (3 - cv));
        if (!live(lo, hi)) continue;
        const int src_off = (int)(src - sm);
        int tb[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) tb[k] = tq[k] >= 0 ? src_off + (tq[k] & ~(PX - 1)) : zr_off;
        if (half == 0) {
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[e] = 0.f;
        }
        // the item's 18 steps (16-channel blocks 2 half, 2 half + 1; 9 taps each), software
        // pipelined: step s + CK_PF's A / B fragments are read while step s multiplies
        uint4 fa[CK_PF + 1], fb[CK_PF + 1];
        auto ld = [&](int st) {
            const int j = st / 9, k = st - 9 * j, cb = 2 * half + j;
            fa[st % (CK_PF + 1)] = *reinterpret_cast<const uint4*>(wb + ((j * 9 + k) * 64 + lane) * 16);
            fb[st % (CK_PF + 1)] = *reinterpret_cast<const uint4*>(sm + tb[k] + (((2 * cb + h) ^ (tq[k] & (CPX - 1))) << 4));
        };
#pragma unroll
        for (int st = 0; st < CK_PF; ++st) ld(st);
#pragma unroll
        for (int st = 0; st < 18; ++st) {
            if (st + CK_PF < 18) ld(st + CK_PF);
            acc = KMfma<T>::step(fa[st % (CK_PF + 1)], fb[st % (CK_PF + 1)], acc);
        }
        // keep that order through scheduling (it would otherwise sink the reads to one step ahead)
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * CK_PF, 0);
#pragma unroll
        for (int st = 0; st < 18; ++st) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            if (st + CK_PF < 18) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        }
        if (half != HALVES - 1) continue;
        unsigned w[8];
        ck_act<T>(acc, BI + (L.br - L.b1) / 4 + HH * cv + 32 * t + 16 * h, w);
        if (pv && py >= lo && py < hi) {
            const int o0 = ck_off<HH>(p, 4 * t + 2 * h), o1 = ck_off<HH>(p, 4 * t + 2 * h + 1);
            if (cv & 1) {   // conv2 of a Residual: + its input (C1), rounded again (nn.py:49)
                const uint4 q0 = *reinterpret_cast<const uint4*>(C1 + o0);
                const uint4 q1 = *reinterpret_cast<const uint4*>(C1 + o1);
                const unsigned rv[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
                for (int q = 0; q < 8; ++q) w[q] = ck_pack2<T>(ck_lo<T>(w[q]) + ck_lo<T>(rv[q]), ck_hi<T>(w[q]) + ck_hi<T>(rv[q]));
            }
            *reinterpret_cast<uint4*>(dst + o0) = make_uint4(w[0], w[1], w[2], w[3]);
            *reinterpret_cast<uint4*>(dst + o1) = make_uint4(w[4], w[5], w[6], w[7]);
        }
    }
    CK_STAMP(3 + NSTEP);
}

// LDS bytes of a workgroup with region images of rpx pixels and nb ring buffers
static long long ck_lds_px(int hh, long long rpx, int nb, long long bpx = 0) {
    return rpx * 2 * hh + ck_tt_bytes(hh, (int)rpx) + bpx * 2 * hh + (long long)nb * CK_WBH + 128 + 32 * hh;
}

// pixels from a band region's first row to the last row phases B..F use (the band + 3 halo
// rows below, 4 above): they must lie in the 16 waves' tiles
static int ck_live_px(int H, int W, int bands) {
    const int rb = (H + bands - 1) / bands;
    return std::min(rb + 7, H) * W;
}

// bands per image: start from `r` and add bands until the phases' pixels fit 16 waves'
// tiles, the region two passes of them, and the LDS two ring buffers (at most one row per band)
static int ck_fit_bands(int hh, int H, int W, int r) {
    auto fits = [&](int b) {
        const int rpx = ck_region_px(H, W, b);
        return ck_live_px(H, W, b) <= 32 * CK_NW && rpx <= 2 * 32 * CK_NW && ck_lds_px(hh, rpx, 2) <= 160 * 1024;
    };
    r = std::max(1, std::min(r, H));
    while (r < H && !fits(r)) ++r;
    return r;
}

template <typename T, int HH>
int launch_c3k_t(const C3kArgs& a0, hipStream_t s) {
    C3kArgs a = a0;
    a.bands = c3k_bands(a.B, a.H, a.W, HH);
    const int rpx = ck_region_px(a.H, a.W, a.bands), bpx = (a.H + a.bands - 1) / a.bands * a.W;
    // h = 64 runs only in SPLIT mode (phases B..F within 8 tiles, the ring keeping >= 4 buffers
    // beside conv2's band: c3k_lds / c3k_bands admit no other h = 64 shape); as many ring buffers
    // as the LDS holds (YH_C3K_NB: fewer)
    const bool split = HH == 64 && ck_live_px(a.H, a.W, a.bands) <= 32 * 8 && ck_lds_px(HH, rpx, 4, bpx) <= 160 * 1024;
    if (HH == 64 && !split) return (int)hipErrorInvalidValue;
    const long long bp = split ? bpx : 0;
    a.nbuf = 2;
    while (a.nbuf < CK_MAXNB && ck_lds_px(HH, rpx, a.nbuf + 1, bp) <= 160 * 1024) ++a.nbuf;
    if (const char* e = getenv("YH_C3K_NB")) a.nbuf = std::max(split ? 4 : 2, std::min(a.nbuf, atoi(e)));
    const long long lds = ck_lds_px(HH, rpx, a.nbuf, bp);
    if (c3k_lds(a.H, a.W, HH) == 0 || ck_live_px(a.H, a.W, a.bands) > 32 * CK_NW || rpx > 2 * 32 * CK_NW ||
        lds > 160 * 1024 || a.B < 1 || a.ldx % 8 || a.ldy % 8)
        return (int)hipErrorInvalidValue;
    auto k = &c3k_fused<T, HH, HH == 64>;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    hipLaunchKernelGGL(k, dim3((unsigned)(a.B * a.bands)), dim3(CK_THREADS), (int)lds, s, a);
    return (int)hipGetLastError();
}

}  // namespace

int c3k_prm_bytes(int hh) {
    return hh == 32 ? ck_layout<32>().total : hh == 64 ? ck_layout<64>().total : 0;
}

void c3k_offsets(int hh, int (&off)[9]) {
    const CkLayout L = hh == 32 ? ck_layout<32>() : ck_layout<64>();
    const int v[9] = {L.w1, L.w2, L.wr, L.w3, L.b1, L.b2, L.br, L.b3, L.total};
    for (int i = 0; i < 9; ++i) off[i] = v[i];
}

// h = 64 runs fused only with bands that allow the SPLIT mode: its one-group form measured
// slower than the seven launches at 40 x 40 (v11_s b64: 138 vs 129 us; bench on / off equal)
static bool ck_split_fits(int H, int W, int r) {
    return ck_live_px(H, W, r) <= 32 * 8 &&
           ck_lds_px(64, ck_region_px(H, W, r), 4, (long long)((H + r - 1) / r) * W) <= 160 * 1024;
}
static int ck_split_bands(int H, int W, int r) {   // the first band count >= r that fits, else 0
    for (r = std::max(1, r); r <= H; ++r)
        if (ck_split_fits(H, W, r)) return r;
    return 0;
}

int c3k_lds(int H, int W, int hh) {
    if (H < 1 || W < 1 || (hh != 32 && hh != 64)) return 0;
    if (hh == 64) {
        const int r = ck_split_bands(H, W, 1);
        if (r == 0 || (r > 1 && (H + r - 1) / r < CK_MINRB)) return 0;
        return (int)ck_lds_px(64, ck_region_px(H, W, r), 4, (long long)((H + r - 1) / r) * W);
    }
    // the fewest bands that fit; bands of fewer than CK_MINRB rows recompute too much halo
    const int r = ck_fit_bands(hh, H, W, 1);
    const int rpx = ck_region_px(H, W, r);
    if (ck_live_px(H, W, r) > 32 * CK_NW || rpx > 2 * 32 * CK_NW || (r > 1 && (H + r - 1) / r < CK_MINRB)) return 0;
    const long long b = ck_lds_px(hh, rpx, 2);
    return b <= 160 * 1024 ? (int)b : 0;
}

int c3k_region_px(int H, int W, int bands) { return ck_region_px(H, W, bands); }

int c3k_bands(int B, int H, int W, int hh) {
    // enough workgroups for the chip (>= 128) with bands of >= CK_MINRB rows, then as many
    // more as the regions need to fit; YH_C3K_BANDS overrides the first choice
    int r = std::max(1, std::min((128 + B - 1) / B, H / CK_MINRB));
    if (const char* e = getenv("YH_C3K_BANDS")) r = std::max(1, std::min(atoi(e), H));
    if (hh == 64)
        if (const int rs = ck_split_bands(H, W, r)) return rs;
    return ck_fit_bands(hh, H, W, r);
}

int launch_c3k(int dtype, const C3kArgs& a, hipStream_t s) {
    if (a.hh == 32) {
        switch (dtype) {
            case F16: return launch_c3k_t<_Float16, 32>(a, s);
            case BF16: return launch_c3k_t<__bf16, 32>(a, s);
        }
    } else if (a.hh == 64) {
        switch (dtype) {
            case F16: return launch_c3k_t<_Float16, 64>(a, s);
            case BF16: return launch_c3k_t<__bf16, 64>(a, s);
        }
    }
    return (int)hipErrorInvalidValue;
}

}  // namespace yh
