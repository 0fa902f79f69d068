// Fused C3k block (nets/nn.py:52-63, CSPModule(c, c) with two Residual(c/2, e=1.0)) for
// the 16-bit handles, on maps small enough to keep a whole image's intermediates in LDS
// (v11_n: net.p5.1.res_m.0 and fpn.h6.res_m.0 at 20x20, c = 128, h = c / 2 = 64).
//
// One workgroup (16 waves) per band of RB output rows of one image (the launcher cuts each
// image into `bands` bands so that a batch fills the chip: one workgroup per image used 32 of
// 256 CUs at batch 32). The chain of four 3x3 convs needs a 4-row halo: a workgroup keeps the
// rows [r0 - 4, r1 + 4) of its band (clipped to the image) in LDS and each phase computes the
// rows its successors read (B: halo 3, C: 2, D: 1, E and F: the band itself); pixels outside a
// phase's rows are neither computed nor written. A 32-pixel tile per wave in every phase:
//   A   C1 = conv1(x)            1x1 c -> h, + SiLU                   x from HBM -> LDS C1
//   B   T  = r0.conv1(C1)        3x3 h -> h, + SiLU                   LDS -> LDS
//   C   C1 = r0.conv2(T) + C1    3x3 h -> h, + SiLU, + residual       in place (nn.py:49)
//   D   T  = r1.conv1(C1)
//   E   C1 = r1.conv2(T) + C1
//   F   y  = conv3([C1 | c2])    1x1 2h -> c, + SiLU             c2 = conv2(x), from phase A
// Each 3x3 conv runs as two sub-phases, one per 32-cout tile; the tile's 36-step weight
// image comes by LDS-DMA in two 18 KB halves that ping-pong between two buffers, the next
// half in flight while the current one is multiplied (one copy per workgroup, read by every
// wave, instead of one per wave). conv2
// never reaches LDS: its A rows are permuted (bits 2 and 3 swapped) so that a lane's
// accumulator registers 8 jj .. 8 jj + 7 ARE conv3's B fragment of K block 4 + 2 t + jj.
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
constexpr int CK_H = 64;                 // hidden channels (h); c = 2h
constexpr int CK_PX = 128;               // LDS bytes per pixel of C1 / T (64 channels)

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

// swizzled 16-B chunk c of pixel p (C1 / T): 16 consecutive pixels hit 16 bank slots
__device__ __forceinline__ int ck_off(int p, int c) { return p * CK_PX + ((c ^ ((p >> 1) & 7)) << 4); }

// 16 consecutive couts of one pixel (lane half h of a 32-cout tile, fragment rows as
// c3k2.hip / conv_mx): bias, SiLU, one rounding -> 8 packed words
template <typename T>
__device__ __forceinline__ void ck_act(const f32x16& acc, const float* b, unsigned (&w)[8]) {
#pragma unroll
    for (int e = 0; e < 16; e += 2) w[e >> 1] = ck_pack2<T>(silu<T>(acc[e] + b[e]), silu<T>(acc[e + 1] + b[e + 1]));
}

}  // namespace

// pixels of the largest band region: RB = ceil(H / bands) rows + 4 halo rows on each side
__host__ __device__ inline int ck_region_px(int H, int W, int bands) {
    const int rb = (H + bands - 1) / bands;
    return (rb + 8 < H ? rb + 8 : H) * W;
}

// parameter image (bytes): fragments [tile][step][64 lanes][16 B], then fp32 biases
struct CkLayout {
    int w1, w2, wr, w3, b1, b2, br, b3, total;
};
__host__ __device__ constexpr CkLayout ck_layout() {
    CkLayout L{};
    L.w1 = 0;                              // conv1: 2 tiles x 8 K blocks
    L.w2 = L.w1 + 2 * 8 * 1024;            // conv2: 2 x 8 (rows permuted for conv3's B fragments)
    L.wr = L.w2 + 2 * 8 * 1024;            // 4 Residual convs: [conv][tile][36 steps]
    L.w3 = L.wr + 4 * 2 * 36 * 1024;       // conv3: 4 tiles x 8 K blocks
    L.b1 = L.w3 + 4 * 8 * 1024;
    L.b2 = L.b1 + 64 * 4;
    L.br = L.b2 + 64 * 4;                  // [conv][64]
    L.b3 = L.br + 4 * 64 * 4;
    L.total = L.b3 + 128 * 4;
    return L;
}

namespace {

template <typename T>
__global__ __launch_bounds__(CK_THREADS, 1) void c3k_fused(const C3kArgs A) {
    constexpr CkLayout L = ck_layout();
    constexpr int WBH = 18 * 1024;                   // one weight half (18 of a tile's 36 steps)
    extern __shared__ __attribute__((aligned(1024))) char sm[];
    typedef __attribute__((address_space(3))) char* lds_c;
    const unsigned lds0 = (unsigned)(size_t)(lds_c)sm;
    const int HW = A.H * A.W;
    // band rows [r0, r1) of image n; LDS region rows [ra0, ra1) (the band + its 4-row halo)
    const int n = blockIdx.x / A.bands, band = blockIdx.x - n * A.bands;
    const int RB = (A.H + A.bands - 1) / A.bands;
    const int r0 = band * RB, r1 = min(A.H, r0 + RB);
    const int ra0 = max(0, r0 - 4), ra1 = min(A.H, r1 + 4);
    const int NRP = (ra1 - ra0) * A.W;               // region pixels
    const int RPX = ck_region_px(A.H, A.W, A.bands);   // LDS pixels per region image (the largest band's)
    char* C1 = sm;                                   // [RPX][64] (swizzled chunks)
    char* TT = sm + RPX * CK_PX;                     // [RPX][64]
    const int wb_off = 2 * RPX * CK_PX;              // two weight halves
    char* WB = sm + wb_off;
    char* ZR = WB + 2 * WBH;                         // 128 zero bytes (out-of-image taps)
    const float* BI = reinterpret_cast<const float*>(ZR + 128);   // every bias (2 KB)
    const int lane = threadIdx.x & 63, l32 = lane & 31, h = lane >> 5;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const char* prm = reinterpret_cast<const char*>(A.prm);
    if (r0 >= A.H) return;   // workgroup-uniform (no band rows: nothing issued yet)
    // LDS-DMA of `kb` 1-KB pieces from the parameter image at `src` to LDS offset `dst`
    auto dma = [&](int src, int dst, int kb) {
        for (int i = wv; i < kb; i += CK_NW) ck_glds(prm + src + i * 1024 + lane * 16, lds0 + (unsigned)(dst + i * 1024));
    };

    // prologue: conv1's weights into the second weight buffer, conv2's into T (free until the
    // first Residual conv writes it) and the first 3x3 half into the first buffer; a region too
    // small for conv2's 16 KB takes them in the first buffer, the 3x3 half then follows phase A
    const bool w2_in_t = RPX * CK_PX >= 16 * 1024;   // uniform
    dma(L.w1, wb_off + WBH, 16);
    dma(L.w2, w2_in_t ? (int)(TT - sm) : wb_off, 16);
    if (w2_in_t) dma(L.wr, wb_off, 18);
    dma(L.b1, (int)((const char*)BI - sm), (L.total - L.b1) / 1024);
    if (threadIdx.x < 8) *reinterpret_cast<uint4*>(ZR + threadIdx.x * 16) = make_uint4(0, 0, 0, 0);
    // the wave's pixel tile: 32 consecutive region pixels (clamped; only p < NRP is written)
    const int p = wv * 32 + l32;
    const bool own = wv * 32 < NRP;                  // wave-uniform: the wave has a tile
    const bool pv = p < NRP;
    const int pc = pv ? p : NRP - 1;
    const int py = ra0 + pc / A.W, px = pc - (py - ra0) * A.W;   // image row / column
    // rows of the wave's tile (wave-uniform): a phase runs the tile iff it meets the phase's rows
    const int ty0 = ra0 + (wv * 32) / A.W, ty1 = ra0 + (min(wv * 32 + 31, NRP - 1)) / A.W;
    auto live = [&](int lo, int hi) { return own && ty1 >= lo && ty0 < hi; };
    const T* xp = reinterpret_cast<const T*>(A.x) + (((long long)n * A.H + py) * A.W + px) * A.ldx + 8 * h;
    uint4 xb[8];
#pragma unroll
    for (int kb = 0; kb < 8; ++kb) xb[kb] = *reinterpret_cast<const uint4*>(xp + 16 * kb);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ck_barrier();

    // ---- A: C1 = SiLU(conv1(x)) -> LDS; conv2(x) -> registers (its rows permuted: registers
    //      8 jj .. + 7 of tile t are channels 32 t + 16 jj + 8 h .. + 7 = conv3's B fragment of
    //      K block 4 + 2 t + jj), held until phase F. B fragments from HBM, A from LDS.
    uint4 bf[8];
    f32x16 acc;
    if (own) {
        const char* w2 = w2_in_t ? TT : WB;
        const float* b2 = BI + (L.b2 - L.b1) / 4;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
            for (int kb = 0; kb < 8; ++kb)
                acc = KMfma<T>::step(*reinterpret_cast<const uint4*>(w2 + ((t * 8 + kb) * 64 + lane) * 16), xb[kb], acc);
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) {
                const float* bj = b2 + 32 * t + 16 * jj + 8 * h;
                unsigned w[4];
#pragma unroll
                for (int e = 0; e < 8; e += 2)
                    w[e >> 1] = ck_pack2<T>(silu<T>(acc[8 * jj + e] + bj[e]), silu<T>(acc[8 * jj + e + 1] + bj[e + 1]));
                bf[4 + 2 * t + jj] = make_uint4(w[0], w[1], w[2], w[3]);
            }
        }
        const char* w1 = WB + WBH;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            f32x16 acc;
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
            for (int kb = 0; kb < 8; ++kb)
                acc = KMfma<T>::step(*reinterpret_cast<const uint4*>(w1 + ((t * 8 + kb) * 64 + lane) * 16), xb[kb], acc);
            unsigned w[8];
            ck_act<T>(acc, BI + 32 * t + 16 * h, w);
            if (pv) {
                *reinterpret_cast<uint4*>(C1 + ck_off(p, 4 * t + 2 * h)) = make_uint4(w[0], w[1], w[2], w[3]);
                *reinterpret_cast<uint4*>(C1 + ck_off(p, 4 * t + 2 * h + 1)) = make_uint4(w[4], w[5], w[6], w[7]);
            }
        }
    }
    if (!w2_in_t) {
        ck_barrier();   // conv2's weights read: the first 3x3 half may land in the first buffer
        dma(L.wr, wb_off, 18);
    }

    // 3x3 taps of the wave's pixel: pixel byte offset within C1 / T with the chunk swizzle in
    // its low bits (-128: outside the image, read from the zero block)
    int tq[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
        const int yy = py + t / 3 - 1, xx = px + t % 3 - 1;
        // outside the image: the zero block; outside the region (only taps of pixels whose
        // outputs no later phase reads): the zero block too
        const bool in = yy >= ra0 && yy < ra1 && (unsigned)xx < (unsigned)A.W;
        const int q = (yy - ra0) * A.W + xx;
        tq[t] = in ? (q * CK_PX) | ((q >> 1) & 7) : -CK_PX;
    }
    const int zr_off = (int)(ZR - sm);

    // ---- B..E: the Residual convs, one 32-cout tile per sub-phase. A tile's 36 weight steps
    //      arrive as two 18 KB halves that ping-pong between two LDS buffers: the next half
    //      (of this tile or the next one; after the last one, conv3's first two tiles) is
    //      DMA'd while the current half is multiplied.
#pragma unroll 1
    for (int hs = 0; hs < 16; ++hs) {
        const int cv = hs >> 2, t = (hs >> 1) & 1, half = hs & 1;
        char* src = (cv & 1) ? TT : C1;
        char* dst = (cv & 1) ? C1 : TT;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMAs of half-step hs
        ck_barrier();   // ... and everyone's; the other buffer and the previous phase are done
        if (hs + 1 < 16) dma(L.wr + (hs + 1) * WBH, wb_off + ((hs + 1) & 1) * WBH, 18);
        else dma(L.w3, wb_off, 16);
        // rows this conv must produce: the band + (3 - cv) halo rows (what conv cv + 1 reads)
        const int lo = max(0, r0 - (3 - cv)), hi = min(A.H, r1 + (3 - cv));
        if (!live(lo, hi)) continue;
        const int src_off = (int)(src - sm);
        int tb[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) tb[k] = tq[k] >= 0 ? src_off + (tq[k] & ~(CK_PX - 1)) : zr_off;
        if (half == 0) {
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[e] = 0.f;
        }
        const char* wb = WB + half * WBH;
#pragma unroll 1
        for (int cb = 2 * half; cb < 2 * half + 2; ++cb)
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                const uint4 a = *reinterpret_cast<const uint4*>(wb + (((cb & 1) * 9 + k) * 64 + lane) * 16);
                const uint4 b = *reinterpret_cast<const uint4*>(sm + tb[k] + (((2 * cb + h) ^ (tq[k] & 7)) << 4));
                acc = KMfma<T>::step(a, b, acc);
                if (k % 3 == 2) asm volatile("" ::: "memory");   // 3 taps' reads in flight (VGPR budget)
            }
        if (half == 0) continue;
        unsigned w[8];
        ck_act<T>(acc, BI + (L.br - L.b1) / 4 + 64 * cv + 32 * t + 16 * h, w);
        if (pv && py >= lo && py < hi) {
            const int o0 = ck_off(p, 4 * t + 2 * h), o1 = ck_off(p, 4 * t + 2 * h + 1);
            if (cv & 1) {   // conv2 of a Residual: + its input (C1), rounded again (nn.py:49)
                const uint4 r0 = *reinterpret_cast<const uint4*>(C1 + o0);
                const uint4 r1 = *reinterpret_cast<const uint4*>(C1 + o1);
                const unsigned rv[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
#pragma unroll
                for (int q = 0; q < 8; ++q) w[q] = ck_pack2<T>(ck_lo<T>(w[q]) + ck_lo<T>(rv[q]), ck_hi<T>(w[q]) + ck_hi<T>(rv[q]));
            }
            *reinterpret_cast<uint4*>(dst + o0) = make_uint4(w[0], w[1], w[2], w[3]);
            *reinterpret_cast<uint4*>(dst + o1) = make_uint4(w[4], w[5], w[6], w[7]);
        }
    }
    // ---- F: conv3 over [C1 | conv2] -> y; its tiles 0-1 from the first buffer (landed during
    //      the last half-step), tiles 2-3 from the second (DMA'd now, while 0-1 multiply)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ck_barrier();
    dma(L.w3 + 16 * 1024, wb_off + WBH, 16);
    const float* b3 = BI + (L.b3 - L.b1) / 4;
    T* y = reinterpret_cast<T*>(A.y) + (((long long)n * A.H + py) * A.W + px) * A.ldy;
    const bool fl = live(r0, r1);
    if (fl) {
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) bf[kb] = *reinterpret_cast<const uint4*>(C1 + ck_off(pc, 2 * kb + h));
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        if (t == 2) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            ck_barrier();
        }
        if (!fl) continue;
        const char* w3 = WB + (t >> 1) * WBH + (t & 1) * 8 * 1024;
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
        for (int kb = 0; kb < 8; ++kb)
            acc = KMfma<T>::step(*reinterpret_cast<const uint4*>(w3 + (kb * 64 + lane) * 16), bf[kb], acc);
        unsigned w[8];
        ck_act<T>(acc, b3 + 32 * t + 16 * h, w);
        if (pv && py >= r0 && py < r1) {
            uint4* d = reinterpret_cast<uint4*>(y + 32 * t + 16 * h);
            d[0] = make_uint4(w[0], w[1], w[2], w[3]);
            d[1] = make_uint4(w[4], w[5], w[6], w[7]);
        }
    }
}

// LDS bytes for region images of rpx pixels: C1 + T, two 18 KB weight halves (also conv1 /
// conv2 / conv3's 32 KB), the zero block, the biases
static long long ck_lds_px(long long rpx) {
    return 2 * rpx * CK_PX + 36 * 1024 + 128 + (ck_layout().total - ck_layout().b1);
}

template <typename T>
int launch_c3k_t(const C3kArgs& a0, hipStream_t s) {
    C3kArgs a = a0;
    a.bands = c3k_bands(a.B, a.H, a.W);
    const long long lds = ck_lds_px(ck_region_px(a.H, a.W, a.bands));
    if (c3k_lds(a.H, a.W) == 0 || lds > 160 * 1024 || a.B < 1 || a.ldx % 8 || a.ldy % 8)
        return (int)hipErrorInvalidValue;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&c3k_fused<T>), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        attr = true;
    }
    hipLaunchKernelGGL((c3k_fused<T>), dim3((unsigned)(a.B * a.bands)), dim3(CK_THREADS), (int)lds, s, a);
    return (int)hipGetLastError();
}

}  // namespace

int c3k_prm_bytes() { return ck_layout().total; }

void c3k_offsets(int (&off)[9]) {
    const CkLayout L = ck_layout();
    const int v[9] = {L.w1, L.w2, L.wr, L.w3, L.b1, L.b2, L.br, L.b3, L.total};
    for (int i = 0; i < 9; ++i) off[i] = v[i];
}

int c3k_lds(int H, int W) {
    const long long hw = (long long)H * W;
    if (H < 1 || W < 1 || hw > 32 * CK_NW) return 0;
    const long long b = ck_lds_px(hw);
    return b <= 160 * 1024 ? (int)b : 0;
}

int c3k_region_px(int H, int W, int bands) { return ck_region_px(H, W, bands); }

int c3k_bands(int B, int H, int W) {
    // enough workgroups for the chip (>= 128) with bands of >= 4 rows; YH_C3K_BANDS overrides
    int r = std::max(1, std::min((128 + B - 1) / B, H / 4));
    if (const char* e = getenv("YH_C3K_BANDS")) r = std::max(1, std::min(atoi(e), H));
    while (r > 1 && ck_region_px(H, W, r) > 32 * CK_NW) --r;   // never: a band region <= the image
    (void)W;
    return r;
}

int launch_c3k(int dtype, const C3kArgs& a, hipStream_t s) {
    switch (dtype) {
        case F16: return launch_c3k_t<_Float16>(a, s);
        case BF16: return launch_c3k_t<__bf16>(a, s);
    }
    return (int)hipErrorInvalidValue;
}

}  // namespace yh
