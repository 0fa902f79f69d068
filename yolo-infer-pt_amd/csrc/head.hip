// Fused detect-head branches (16-bit handles).
//
//   head_cls   the cls branch of every level (nets/nn.py:244-252: DWConv 3x3 -> Conv 1x1
//              -> DWConv 3x3 -> Conv 1x1 -> Conv2d 1x1) in one launch. A workgroup owns a
//              TH x TW output tile of one image of one level; the input tile with a 2-pixel
//              halo, the first depthwise output and first pointwise output with a 1-pixel
//              halo, the second depthwise and pointwise outputs all stay in LDS; only the
//              level input is read from HBM and only the nc class logits are written
//              (direct mode: their sigmoid scores, straight into the caller's y).
//   box_dfl    the box branch's last 1x1 conv with DFL + anchors + dist2bbox in its
//              epilogue (rows 0..3 of y); with head_cls's direct mode it replaces the decode.
//
// Bit-identical to the unfused launches: the depthwise convs run dwconv3x3_c4's per-channel
// FMA chain (taps row-major, fp32, + bias, SiLU, one rounding), the pointwise convs run
// conv_mx's K order (16-channel blocks ascending, one v_mfma_f32_32x32x16 step each, fp32
// accumulator, + bias, activation, one rounding). The first pointwise output is zeroed
// outside the image: it is the second depthwise conv's zero padding.
#include "common.h"
#include "dtypes.h"

namespace yh {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <typename T> struct HMfma;
template <> struct HMfma<__bf16> {
    static __device__ __forceinline__ f32x16 step(const uint4& a, const uint4& b, const f32x16& c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                       0, 0);
    }
};
template <> struct HMfma<_Float16> {
    static __device__ __forceinline__ f32x16 step(const uint4& a, const uint4& b, const f32x16& c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                      0);
    }
};

constexpr int NWV = HEAD_CLS_THREADS / 64;
constexpr bool HC_UNITS = NWV >= 8;

// the decode's 16-bit exp and division (misc.hip ex<T> / dv<T>): same instructions, same bits
__device__ __forceinline__ float hx_exp(float x) { return __expf(x); }
__device__ __forceinline__ float hx_div(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }

// LDS-DMA: the wave's 64 lanes each copy 16 B from their own global address into LDS at
// lds_addr + 16 * lane (M0 holds the wave-uniform base; restored after the copy)
__device__ __forceinline__ void hc_glds(const void* src, unsigned lds_addr) {
#if defined(__HIP_DEVICE_COMPILE__)
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds_addr) : "memory");
#else
    (void)src; (void)lds_addr;
#endif
}

// Workgroup barrier for LDS hand-offs only: __syncthreads() also waits for every global
// load in flight (vmcnt(0)), which would drain the weight loads issued ahead of a phase.
__device__ __forceinline__ void hc_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
#ifdef YH_HC_TRACE
// experiments only (-DYH_HC_TRACE builds; the shipped library has none of this): per-workgroup
// phase stamps, read back by yh_debug_hc_trace. Slots: 0 / 8 s_memrealtime at entry / exit,
// 1 s_memtime at entry, 2..7 s_memtime after the input landed, dw1, pw1, dw2, pw2, pw3, 9 HW_ID
// | XCC_ID << 32 | level << 40.
constexpr int HC_TR = 10, HC_TR_WG = 8192;
__device__ unsigned long long hc_trace_buf[HC_TR_WG * HC_TR];
#define HC_STAMP(k, rt)                                                                                      \
    do {                                                                                                     \
        hc_barrier();                                                                                        \
        if (threadIdx.x == 0 && blockIdx.x < HC_TR_WG)                                                       \
            hc_trace_buf[(size_t)blockIdx.x * HC_TR + (k)] =                                                 \
                (rt) ? __builtin_amdgcn_s_memrealtime() : __builtin_amdgcn_s_memtime();                     \
    } while (0)
#else
#define HC_STAMP(k, rt) \
    do {                \
    } while (0)
#endif
constexpr int HC_CK = 64;    // input channels staged per pass (the first depthwise conv's chunk)
#ifndef YH_HC_RB
#define YH_HC_RB 4
#endif
constexpr int HC_RB = YH_HC_RB;   // output rows per depthwise item (register sliding window)

// LDS of one tile: region 1 = the input chunk (XH x XW x min(C0, HC_CK)), later the first /
// second pointwise outputs; region 2 = the first / second depthwise outputs
struct HcLayout {
    int SX, SD, SM, r1, x2, prm, total;   // prm: byte offset of the fp32 parameters (see hc_params)
};
__host__ __device__ inline HcLayout hc_layout(int TH, int TW, int C0, int c3) {
    HcLayout L;
    const int ck = C0 < HC_CK ? C0 : HC_CK;
    L.SX = ck + 8; L.SD = C0 + 8; L.SM = c3 + 8;
    const int MP = (TH + 2) * (TW + 2), NO = TH * TW;
    const int x = ((TH + 4) * (TW + 4) * L.SX * 2 + 1023) & ~1023;   // whole LDS-DMA instructions
    const int p1 = MP * L.SM * 2, p2 = NO * L.SM * 2;
    const int d1 = MP * L.SD * 2, d2 = NO * L.SM * 2;
    int a = x > p1 ? x : p1;
    a = a > p2 ? a : p2;
    L.r1 = (a + 15) & ~15;
    L.prm = L.r1 + (((d1 > d2 ? d1 : d2) + 15) & ~15);
    // levels with several 64-channel chunks: a second input buffer (chunk k + 1 lands during
    // chunk k's depthwise conv)
    L.x2 = 0;
    if (C0 > HC_CK) {
        L.x2 = L.prm;
        L.prm += x;
    }
    // dw1 weights [9][C0] + bias, dw2 weights [9][c3] + bias, pw1 / pw2 / pw3 bias (HC_NA * 32 each)
    L.total = L.prm + (((10 * C0 + 10 * c3 + 3 * 96) * 4 + 1023) & ~1023);
    return L;
}

// Depthwise 3x3 + bias + SiLU over channels [c_lo, c_lo + C) of region `src` (row width SW
// pixels, stride ss, channel offset 0 = c_lo) into `dst` (DH x DW pixels, stride ds, channel
// offset c_lo). An item is (4-channel group, column, block of HC_RB rows): its (HC_RB + 2) x 3
// input pixels are read once and every output row has its own FMA chain (taps row-major).
// floor(n / d) as (n * m) >> s with m = floor(2^s / d) + 1: exact for 0 <= n < 2^s / d (and
// n * m < 2^32), which the tile index ranges here satisfy (tiles of at most 24 x 36 pixels)
struct HcDiv {
    unsigned m;
    int s;
};
__device__ __forceinline__ HcDiv hc_div(int d, int s) { return HcDiv{(1u << s) / (unsigned)d + 1u, s}; }
__device__ __forceinline__ int hc_q(int n, HcDiv f) { return (int)(((unsigned)n * f.m) >> f.s); }

template <typename T>
__device__ __forceinline__ void hc_dw(const T* src, int SW, int ss, T* dst, int DH, int DW, int ds, int c_lo, int C,
                                      const float* w, int wld, const float* b) {
    const int nrb = (DH + HC_RB - 1) / HC_RB, per_g = DW * nrb, ng = C >> 2;
    const HcDiv dw = hc_div(DW, 16);
    const int rs = SW * ss;                                      // one source row (elements)
    // the first item's weights are loaded before the barrier that opens the phase
    float4 wt[9], bb;
    int wg = -1;
    auto load_w = [&](int g) {
        const int c0 = c_lo + g * 4;
#pragma unroll
        for (int k = 0; k < 9; ++k) wt[k] = *reinterpret_cast<const float4*>(w + k * wld + c0);
        bb = *reinterpret_cast<const float4*>(b + c0);
        wg = g;
    };
    hc_barrier();   // src (and the parameters in LDS) complete
    // channel group fastest: the lanes of a wave read consecutive 8-B groups of one or two pixels
    // (with the column fastest, lanes 16 apart hit one bank at the 144-B pixel stride: 37 % of
    // head_cls's LDS cycles were bank conflicts, profiles/r06_sq_all_ops_c2.txt)
    const HcDiv dn = hc_div(ng, 24);
    if ((int)threadIdx.x < ng * per_g) load_w((int)threadIdx.x - hc_q(threadIdx.x, dn) * ng);
    for (int q = threadIdx.x; q < ng * per_g; q += HEAD_CLS_THREADS) {
        const int p = hc_q(q, dn), g = q - p * ng;
        const int rb = hc_q(p, dw), c = p - rb * DW;
        const int r0 = rb * HC_RB, c0 = c_lo + g * 4;
        if (g != wg) load_w(g);
        // rows past the source's last (DH + 1) read that row (outputs discarded below)
        const T* sp = src + (r0 * SW + c) * ss + g * 4;
        const int lim = DH + 1 - r0, lim_off = lim * rs;
        uint2 xv[HC_RB + 2][3];
#pragma unroll
        for (int r = 0; r < HC_RB + 2; ++r) {
            const int ro = r <= lim ? r * rs : lim_off;
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) xv[r][kw] = *reinterpret_cast<const uint2*>(sp + ro + kw * ss);
        }
        // the input pixels as fp32 pairs once (each feeds up to three output rows)
        f32x2 xf[HC_RB + 2][3][2];
#pragma unroll
        for (int r = 0; r < HC_RB + 2; ++r)
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
                const T* xe = reinterpret_cast<const T*>(&xv[r][kw]);
                xf[r][kw][0] = f32x2{tof(xe[0]), tof(xe[1])};
                xf[r][kw][1] = f32x2{tof(xe[2]), tof(xe[3])};
            }
#pragma unroll
        for (int o = 0; o < HC_RB; ++o) {
            if (r0 + o >= DH) break;
            // two channels per packed FMA (v_pk_fma_f32): each lane of it the same fused
            // multiply-add, in the same tap order, as one fmaf per channel
            f32x2 acc01 = f32x2{0.f, 0.f}, acc23 = f32x2{0.f, 0.f};
#pragma unroll
            for (int kh = 0; kh < 3; ++kh)
#pragma unroll
                for (int kw = 0; kw < 3; ++kw) {
                    const float4 wk = wt[kh * 3 + kw];
                    acc01 = __builtin_elementwise_fma(f32x2{wk.x, wk.y}, xf[o + kh][kw][0], acc01);
                    acc23 = __builtin_elementwise_fma(f32x2{wk.z, wk.w}, xf[o + kh][kw][1], acc23);
                }
            T o4[4];
            o4[0] = fromf<T>(silu<T>(acc01.x + bb.x));
            o4[1] = fromf<T>(silu<T>(acc01.y + bb.y));
            o4[2] = fromf<T>(silu<T>(acc23.x + bb.z));
            o4[3] = fromf<T>(silu<T>(acc23.y + bb.w));
            *reinterpret_cast<uint2*>(dst + ((r0 + o) * DW + c) * ds + c0) = *reinterpret_cast<const uint2*>(o4);
        }
    }
}

// Pointwise conv phase: A = weights [rows][wld] (dtype, global; rows >= na * 32 zero-padded)
// times the NPX pixels of LDS `src` (stride ss, 16 NK channels). The A fragments of the first
// NAP 32-cout tiles are loaded ahead of the phase (hc_pw_pre, one phase earlier: their
// latency hides behind the previous phase); tiles past NAP are loaded in the loop, one tile
// ahead. Each wave takes 32-pixel B tiles round-robin (B fragments read once per B tile).
// K order: 16-channel blocks ascending. store(px, co, 4 rounded values) for couts co < M.
constexpr int HC_NA = 3;   // 32-cout tiles per pointwise conv (cout <= 96)
template <int NK, int NAP>
struct HcA {
    uint4 f[NAP][NK];
};
template <typename T, int NK, int NAP>
__device__ __forceinline__ void hc_pw_pre(const T* w, int wld, int M, HcA<NK, NAP>& A) {
    const int lane = threadIdx.x & 63, l32 = lane & 31, h = lane >> 5;
    const int na = (M + 31) >> 5;
#pragma unroll
    for (int a = 0; a < NAP; ++a) {
        const T* wrow = w + (long long)(min(a, na - 1) * 32 + l32) * wld + 8 * h;
#pragma unroll
        for (int kb = 0; kb < NK; ++kb) A.f[a][kb] = *reinterpret_cast<const uint4*>(wrow + kb * 16);
    }
}
template <typename T, int NK, int NAP, typename Store>
__device__ __forceinline__ void hc_pw_run(const T* src, int ss, int NPX, const T* w, int wld, const float* bias, int M,
                                          bool silu_act, const HcA<NK, NAP>& A, Store store) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int l32 = lane & 31, h = lane >> 5;
    const int na = (M + 31) >> 5, nb = (NPX + 31) >> 5;
    hc_barrier();   // src complete
    for (int bi = wv; bi < nb; bi += NWV) {
        const int px = bi * 32 + l32;
        const int pxc = px < NPX ? px : NPX - 1;
        uint4 bf[NK];
#pragma unroll
        for (int kb = 0; kb < NK; ++kb) bf[kb] = *reinterpret_cast<const uint4*>(src + pxc * ss + 8 * h + kb * 16);
        uint4 lf[2][NK];   // tiles past NAP: double-buffered loads
        auto load_a = [&](int a, uint4 (&dst)[NK]) {
            const T* wrow = w + (long long)(a * 32 + l32) * wld + 8 * h;
#pragma unroll
            for (int kb = 0; kb < NK; ++kb) dst[kb] = *reinterpret_cast<const uint4*>(wrow + kb * 16);
        };
        if (NAP < na) load_a(NAP, lf[NAP & 1]);
#pragma unroll
        for (int a = 0; a < HC_NA; ++a) {
            if (a >= na) break;
            if (a >= NAP && a + 1 < na) load_a(a + 1, lf[(a + 1) & 1]);
            f32x16 acc;
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[e] = 0.f;
            if (a < NAP) {
#pragma unroll
                for (int kb = 0; kb < NK; ++kb) acc = HMfma<T>::step(A.f[a < NAP ? a : 0][kb], bf[kb], acc);
            } else {
#pragma unroll
                for (int kb = 0; kb < NK; ++kb) acc = HMfma<T>::step(lf[a & 1][kb], bf[kb], acc);
            }
            if (px < NPX) {
                // register i of lane (l32, h): cout a*32 + (i & 3) + 8 (i >> 2) + 4 h, pixel px
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int co = a * 32 + 8 * q + 4 * h;
                    if (co >= M) continue;
                    const float4 bb = *reinterpret_cast<const float4*>(bias + co);
                    float v[4] = {acc[4 * q] + bb.x, acc[4 * q + 1] + bb.y, acc[4 * q + 2] + bb.z,
                                  acc[4 * q + 3] + bb.w};
                    T o4[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) o4[e] = fromf<T>(silu_act ? silu<T>(v[e]) : v[e]);
                    store(px, co, *reinterpret_cast<const uint2*>(o4));
                }
            }
        }
    }
}

template <int NK>
struct HcA<NK, 0> {};

// Pointwise phase over (32-pixel B tile, 32-cout A tile) work units, round-robin over the
// waves: the wide-K pw1 (NK > 8: the 256-channel 20x20 level) and, with 8-wave workgroups,
// every pointwise phase (no fragments held across phases). K runs in pieces of up to 8
// blocks; with two pieces the next one's A (global) and B (LDS) fragments load while the
// current one's MFMAs run. One fp32 chain per unit over the 16-channel blocks in ascending
// order: the same K order, the same bits as hc_pw_run and the per-layer 1x1 conv.
template <typename T, int NK, typename Store>
__device__ __forceinline__ void hc_pw_units(const T* src, int ss, int NPX, const T* w, int wld, const float* bias, int M,
                                            bool silu_act, Store store) {
    constexpr int KP = NK <= 8 ? NK : 8, NH = NK / KP;
    static_assert(NK % KP == 0, "whole K pieces");
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int l32 = lane & 31, h = lane >> 5;
    const int na = (M + 31) >> 5, nb = (NPX + 31) >> 5;
    // each wave takes a contiguous range of the units in A-tile-major order, so a wave with one
    // K piece (NH == 1) loads an A tile's fragments once for all its B tiles; the first unit's
    // A fragments are issued before the barrier (they do not depend on the previous phase)
    const int nu = na * nb;
    const int u0 = (wv * nu) / NWV, u1 = ((wv + 1) * nu) / NWV;
    const HcDiv dnb = hc_div(nb, 16);
    uint4 af[NH > 1 ? 2 : 1][KP], bf[NH > 1 ? 2 : 1][KP];
    auto load_a = [&](int a, int hh, int buf) {
        const T* wrow = w + (long long)(a * 32 + l32) * wld + 8 * h + hh * KP * 16;
#pragma unroll
        for (int kb = 0; kb < KP; ++kb) af[buf][kb] = *reinterpret_cast<const uint4*>(wrow + kb * 16);
    };
    auto load_b = [&](const T* brow, int hh, int buf) {
#pragma unroll
        for (int kb = 0; kb < KP; ++kb) bf[buf][kb] = *reinterpret_cast<const uint4*>(brow + (hh * KP + kb) * 16);
    };
    int a_cur = u0 < u1 ? hc_q(u0, dnb) : 0;
    if (u0 < u1) load_a(a_cur, 0, 0);
    hc_barrier();   // src complete
    for (int u = u0; u < u1; ++u) {
        const int a = hc_q(u, dnb), bi = u - a * nb;
        const int px = bi * 32 + l32;
        const int pxc = px < NPX ? px : NPX - 1;
        const T* brow = src + pxc * ss + 8 * h;
        if (NH > 1 ? u > u0 : a != a_cur) load_a(a, 0, 0);
        a_cur = a;
        load_b(brow, 0, 0);
        f32x16 acc;
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
        for (int hh = 0; hh < NH; ++hh) {
            if (hh + 1 < NH) {
                load_a(a, hh + 1, (hh + 1) & 1);
                load_b(brow, hh + 1, (hh + 1) & 1);
            }
#pragma unroll
            for (int kb = 0; kb < KP; ++kb) acc = HMfma<T>::step(af[hh & 1][kb], bf[hh & 1][kb], acc);
        }
        if (px < NPX) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int co = a * 32 + 8 * q + 4 * h;
                if (co >= M) continue;
                const float4 bb = *reinterpret_cast<const float4*>(bias + co);
                float v[4] = {acc[4 * q] + bb.x, acc[4 * q + 1] + bb.y, acc[4 * q + 2] + bb.z, acc[4 * q + 3] + bb.w};
                T o4[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) o4[e] = fromf<T>(silu_act ? silu<T>(v[e]) : v[e]);
                store(px, co, *reinterpret_cast<const uint2*>(o4));
            }
        }
    }
}

// One workgroup = one output tile of level li. NK1 = C0 / 16 and NK2 = c3 / 16 (K blocks of
// the first and the later pointwise convs); NAP1 = pw1 A tiles loaded ahead (all three when
// the registers allow).
template <typename T, int NK1, int NAP1, int NK2>
__device__ __forceinline__ void hc_body(const HeadClsArgs& A, int li, char* hsm) {
    const HeadClsLevel& V = A.lv[li];
    // XCD-aware within the level: neighbouring tiles (overlapping halos) on one XCD / L2
    const int wl = xcd_remap((int)blockIdx.x - V.wg0, A.B * V.tiles);
    const int n = wl / V.tiles, tix = wl - n * V.tiles;
    const int ty = tix / V.ntw, tx = tix - ty * V.ntw;
    const int TH = V.TH, TW = V.TW, H = V.H, W = V.W;
    const int h0 = ty * TH, w0 = tx * TW;
    const int XH = TH + 4, XW = TW + 4, MH = TH + 2, MW = TW + 2;
    const int C0 = V.C0, c3 = A.c3;
    const HcLayout L = hc_layout(TH, TW, C0, c3);
    T* R1 = reinterpret_cast<T*>(hsm);
    T* R2 = reinterpret_cast<T*>(hsm + L.r1);
    // depthwise weights and every bias in LDS (read in the phases' inner loops / epilogues)
    float* PW1 = reinterpret_cast<float*>(hsm + L.prm);
    float* PB1 = PW1 + 9 * C0;
    float* PW2 = PB1 + C0;
    float* PB2 = PW2 + 9 * c3;
    float* QB1 = PB2 + c3;
    float* QB2 = QB1 + 96;
    float* QB3 = QB2 + 96;
    // the parameters are contiguous fp32 arrays (ld == channels): one flat list of 16-B
    // chunks, loaded into registers before the input tile's loads, stored after them
    // parameters by LDS-DMA (no registers held): segment starts in 16-B chunks
    const int e0 = 9 * C0 / 4, e1 = e0 + C0 / 4, e2 = e1 + 9 * c3 / 4, e3 = e2 + c3 / 4;
    const int e4 = e3 + 24, e5 = e4 + 24, e6 = e5 + 24;
    typedef __attribute__((address_space(3))) char* lds_c;
    const unsigned lds0 = (unsigned)(size_t)(lds_c)hsm;
    {
        const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
        for (int i0 = wv * 64; i0 < e6; i0 += HEAD_CLS_THREADS) {
            const int q = i0 + lane;
            const float* src = q < e0 ? V.dw1w + 4 * q
                             : q < e1 ? V.dw1b + 4 * (q - e0)
                             : q < e2 ? V.dw2w + 4 * (q - e1)
                             : q < e3 ? V.dw2b + 4 * (q - e2)
                             : q < e4 ? V.pw1b + 4 * (q - e3)
                             : q < e5 ? V.pw2b + 4 * (q - e4)
                             : q < e6 ? V.pw3b + 4 * (q - e5) : reinterpret_cast<const float*>(A.zero);
            hc_glds(src, lds0 + (unsigned)L.prm + (unsigned)i0 * 16);
        }
    }
#ifdef YH_HC_TRACE
    if (threadIdx.x == 0 && blockIdx.x < HC_TR_WG) {
        const unsigned long long hw = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
        const unsigned long long xcc = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);
        hc_trace_buf[(size_t)blockIdx.x * HC_TR + 9] = hw | (xcc << 32) | ((unsigned long long)li << 40);
        hc_trace_buf[(size_t)blockIdx.x * HC_TR + 0] = __builtin_amdgcn_s_memrealtime();
        hc_trace_buf[(size_t)blockIdx.x * HC_TR + 1] = __builtin_amdgcn_s_memtime();
    }
#endif
    const T* x = reinterpret_cast<const T*>(V.x);
    // 8-wave workgroups run every pointwise phase as (B tile, A tile) units with no
    // fragments held across phases (HC_UNITS); 4-wave ones preload them a phase ahead
    constexpr int P1 = HC_UNITS ? 0 : NAP1;
    HcA<NK1, P1> A1;   // pw1's weights, in flight while the input tile loads
    if constexpr (P1 > 0) hc_pw_pre<T, NK1, P1>(reinterpret_cast<const T*>(V.pw1w), V.pw1ld, c3, A1);

    // 1-2. per 64-channel chunk: input tile with a 2-pixel halo (zeros outside the image =
    //      dw1's zero padding) -> R1 / X2 (alternating), then dw1 of the chunk over the MH x MW
    //      mid region -> R2; the next chunk's DMA is issued once this one has landed, before its
    //      depthwise conv
    const int ck = C0 < HC_CK ? C0 : HC_CK;
    // the padded tile (SX = ck + 8: cpp data chunks + 1 pad chunk per pixel) by LDS-DMA
    constexpr int cpp = (NK1 * 16 < HC_CK ? NK1 * 16 : HC_CK) >> 3, cpx = cpp + 1;
    const int xtotal = XH * XW * cpx;
    auto issue_x = [&](int cl, unsigned base) {
        const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
        const HcDiv dxw = hc_div(XW, 16);
        for (int i0 = wv * 64; i0 < xtotal; i0 += HEAD_CLS_THREADS) {
            const int q = i0 + lane;
            const int px = q / cpx, c = q - px * cpx;
            const int r = hc_q(px, dxw), cc = px - r * XW;
            const int gh = h0 - 2 + r, gw = w0 - 2 + cc;
            const bool ok = q < xtotal && c < cpp && (unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W;
            const void* src = ok ? (const void*)(x + (((long long)n * H + gh) * W + gw) * V.ldx + cl + c * 8) : A.zero;
            hc_glds(src, lds0 + base + (unsigned)i0 * 16);
        }
    };
    issue_x(0, 0);
    for (int cl = 0, k = 0; cl < C0; cl += ck, ++k) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMAs (and earlier loads) landed
        if (cl == 0) HC_STAMP(2, false);
        const unsigned cur = (k & 1) ? (unsigned)L.x2 : 0u;
        // the other buffer's last reader (chunk k - 1's depthwise conv) ended at the barrier below
        if (cl + ck < C0) issue_x(cl + ck, (k & 1) ? 0u : (unsigned)L.x2);
        hc_dw<T>(reinterpret_cast<const T*>(hsm + cur), XW, L.SX, R2, MH, MW, L.SD, cl, ck, PW1, C0, PB1);
        if (cl + ck < C0) hc_barrier();   // chunk k's buffer is re-filled with chunk k + 2
    }
    HC_STAMP(3, false);
    // 3. pw1: D1 (R2) -> P1 (R1), zero outside the image (dw2's zero padding)
    const HcDiv dmw = hc_div(MW, 16), dtw = hc_div(TW, 16);
    auto p1_store = [&](int px, int co, uint2 v) {
        const int r = hc_q(px, dmw), cc = px - r * MW;
        const int gh = h0 - 1 + r, gw = w0 - 1 + cc;
        if (!((unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W)) v = make_uint2(0, 0);
        *reinterpret_cast<uint2*>(R1 + px * L.SM + co) = v;
    };
    if constexpr (P1 > 0)
        hc_pw_run<T, NK1, P1>(R2, L.SD, MH * MW, reinterpret_cast<const T*>(V.pw1w), V.pw1ld, QB1, c3, true, A1,
                              p1_store);
    else
        hc_pw_units<T, NK1>(R2, L.SD, MH * MW, reinterpret_cast<const T*>(V.pw1w), V.pw1ld, QB1, c3, true, p1_store);
    constexpr int P2 = HC_UNITS ? 0 : HC_NA;
    HcA<NK2, P2> A2;   // pw2's weights, in flight during dw2
    if constexpr (P2 > 0) hc_pw_pre<T, NK2, P2>(reinterpret_cast<const T*>(V.pw2w), V.pw2ld, c3, A2);
    HC_STAMP(4, false);
    // 4. dw2 (opens with the barrier after pw1): P1 (R1) -> D2 (R2) over the TH x TW tile
    hc_dw<T>(R1, MW, L.SM, R2, TH, TW, L.SM, 0, c3, PW2, c3, PB2);
    HC_STAMP(5, false);
    // 5. pw2: D2 (R2) -> P2 (R1)
    auto p2_store = [&](int px, int co, uint2 v) { *reinterpret_cast<uint2*>(R1 + px * L.SM + co) = v; };
    if constexpr (P2 > 0)
        hc_pw_run<T, NK2, P2>(R2, L.SM, TH * TW, reinterpret_cast<const T*>(V.pw2w), V.pw2ld, QB2, c3, true, A2,
                              p2_store);
    else
        hc_pw_units<T, NK2>(R2, L.SM, TH * TW, reinterpret_cast<const T*>(V.pw2w), V.pw2ld, QB2, c3, true, p2_store);
    HC_STAMP(6, false);
    HcA<NK2, P2> A3;   // pw3's weights: issued once pw2's are dead
    if constexpr (P2 > 0) hc_pw_pre<T, NK2, P2>(reinterpret_cast<const T*>(V.pw3w), V.pw3ld, A.nc, A3);
    // 6. pw3: P2 (R1) -> class logits in the head tensor, or (direct mode) their sigmoid in
    //    the caller's y, one row per class (the decode's class part: logit rounded first)
    T* y = reinterpret_cast<T*>(V.y);
    const gptr<T> yio = A.io ? io_global<T>(A.io[1]) : nullptr;   // loaded once (see io_global)
    auto pw3 = [&](auto store) {
        if constexpr (P2 > 0)
            hc_pw_run<T, NK2, P2>(R1, L.SM, TH * TW, reinterpret_cast<const T*>(V.pw3w), V.pw3ld, QB3, A.nc, false, A3,
                                  store);
        else
            hc_pw_units<T, NK2>(R1, L.SM, TH * TW, reinterpret_cast<const T*>(V.pw3w), V.pw3ld, QB3, A.nc, false, store);
    };
    if (A.io)
        pw3([&](int px, int co, uint2 v) {
            const int r = hc_q(px, dtw), cc = px - r * TW;
            const int gh = h0 + r, gw = w0 + cc;
            if ((unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W) {
                const gptr<T> col = yio + ((long long)n * (4 + A.nc) + 4 + co) * A.A + V.aoff + gh * W + gw;
                const T* o = reinterpret_cast<const T*>(&v);
#pragma unroll
                for (int e = 0; e < 4; ++e) col[(long long)e * A.A] = fromf<T>(hx_div(1.0f, 1.0f + hx_exp(-tof(o[e]))));
            }
        });
    else
        pw3([&](int px, int co, uint2 v) {
            const int r = hc_q(px, dtw), cc = px - r * TW;
            const int gh = h0 + r, gw = w0 + cc;
            if ((unsigned)gh < (unsigned)H && (unsigned)gw < (unsigned)W)
                *reinterpret_cast<uint2*>(y + (((long long)n * H + gh) * W + gw) * V.ldy + co) = v;
        });
    HC_STAMP(7, false);
    HC_STAMP(8, true);
}

#if YH_HEAD_CLS_THREADS >= 512
#define HC_BOUNDS __launch_bounds__(HEAD_CLS_THREADS) __attribute__((amdgpu_waves_per_eu(4, 4)))
#else
#define HC_BOUNDS __launch_bounds__(HEAD_CLS_THREADS, 3)
#endif
template <typename T>
__global__ HC_BOUNDS void head_cls(const HeadClsArgs A) {
    extern __shared__ __attribute__((aligned(16))) char hsm[];
    int li = 0;
    if (A.nlv > 1 && (int)blockIdx.x >= A.lv[1].wg0) li = 1;
    if (A.nlv > 2 && (int)blockIdx.x >= A.lv[2].wg0) li = 2;
    const int nk1 = A.lv[li].C0 >> 4, nk2 = A.c3 >> 4;
    if (nk1 == 4 && nk2 == 5) hc_body<T, 4, HC_NA, 5>(A, li, hsm);
    else if (nk1 == 8 && nk2 == 5) hc_body<T, 8, 1, 5>(A, li, hsm);
    else if (nk1 == 4 && nk2 == 4) hc_body<T, 4, HC_NA, 4>(A, li, hsm);
    else if (nk1 == 8 && nk2 == 4) hc_body<T, 8, 1, 4>(A, li, hsm);
    else if (nk1 == 16 && nk2 == 5) hc_body<T, 16, 0, 5>(A, li, hsm);
    else if (nk1 == 16 && nk2 == 4) hc_body<T, 16, 0, 4>(A, li, hsm);
}

// Box tail: each wave takes BOX_DFL_TPW consecutive 32-pixel tiles of a level's flattened
// (image, row, column) pixels. The 64-cout 1x1 conv runs as two 32x32 MFMA tiles whose rows
// are permuted so that lane half h holds couts 32h .. 32h+31, i.e. the 16 bins of sides 2h and
// 2h+1 of its pixel: the DFL softmax / expectation is lane-local, one swap across the halves
// completes the four distances, and half h writes rows 2h, 2h+1 (32 consecutive anchors per
// row and store instruction).
template <typename T, int NK, int TPW>
__device__ __forceinline__ void bd_body(const BoxDflArgs& A, int li) {
    const BoxDflLevel& V = A.lv[li];
    const int lane = threadIdx.x & 63, l32 = lane & 31, h = lane >> 5, wv = threadIdx.x >> 6;
    const int HW = V.H * V.W;
    const long long M = (long long)A.B * HW;
    const long long tile0 = ((long long)(blockIdx.x - V.wg0) * 4 + wv) * TPW;
    if (tile0 * 32 >= M) return;
    const T* w = reinterpret_cast<const T*>(V.w);
    uint4 af[2][NK];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        const int co = 32 * ((l32 >> 2) & 1) + 16 * a + (l32 & 3) + 4 * (l32 >> 3);
#pragma unroll
        for (int kb = 0; kb < NK; ++kb)
            af[a][kb] = *reinterpret_cast<const uint4*>(w + (long long)co * V.wld + 8 * h + kb * 16);
    }
    const T* x = reinterpret_cast<const T*>(V.x);
    auto load_b = [&](long long t, uint4 (&bf)[NK]) {
        long long m = t * 32 + l32;
        m = m < M ? m : M - 1;
#pragma unroll
        for (int kb = 0; kb < NK; ++kb) bf[kb] = *reinterpret_cast<const uint4*>(x + m * V.ldx + 8 * h + kb * 16);
    };
    float bs[2][16];   // bias of the lane's 32 couts
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int i = 0; i < 16; i += 4) {
            const float4 q = *reinterpret_cast<const float4*>(V.b + 32 * h + 16 * a + i);
            bs[a][i] = q.x; bs[a][i + 1] = q.y; bs[a][i + 2] = q.z; bs[a][i + 3] = q.w;
        }
    uint4 bf[TPW][NK];   // every tile's loads in flight at once (HBM latency)
#pragma unroll
    for (int t = 0; t < TPW; ++t) load_b(tile0 + t, bf[t]);
    const gptr<T> yb = io_global<T>(A.io[1]);
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
        const long long tt = tile0 + t;
        if (tt * 32 >= M) break;
        float dist[2];
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            f32x16 acc;
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
            for (int kb = 0; kb < NK; ++kb) acc = HMfma<T>::step(af[a][kb], bf[t][kb], acc);
            // register i: cout 32h + 16a + i = bin i of side 2h + a; the conv's rounding first
            float v[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] = tof(fromf<T>(acc[i] + bs[a][i]));
            float mx = v[0];
#pragma unroll
            for (int i = 1; i < 16; ++i) mx = fmaxf(mx, v[i]);
            float sum = 0.f;
#pragma unroll
            for (int i = 0; i < 16; ++i) { v[i] = hx_exp(v[i] - mx); sum += v[i]; }
            float d = 0.f;
#pragma unroll
            for (int i = 0; i < 16; ++i) d = fmaf((float)i, hx_div(v[i], sum), d);
            dist[a] = d;
        }
        const float o0 = xor32_swap(dist[0]), o1 = xor32_swap(dist[1]);
        const float dl = h ? o0 : dist[0], dt = h ? o1 : dist[1];
        const float dr = h ? dist[0] : o0, db = h ? dist[1] : o1;
        const long long m = tt * 32 + l32;
        if (m < M) {
            const int n = (int)(m / HW), loc = (int)(m - (long long)n * HW);
            const int gy = loc / V.W, gx = loc - gy * V.W;
            const float ax = (float)gx + 0.5f, ay = (float)gy + 0.5f, st = V.stride;
            const float x1 = ax - dl, y1 = ay - dt;
            const float x2 = ax + dr, y2 = ay + db;
            const float r0 = h ? (x2 - x1) * st : (x1 + x2) / 2.0f * st;
            const float r1 = h ? (y2 - y1) * st : (y1 + y2) / 2.0f * st;
            const gptr<T> col = yb + ((long long)n * (4 + A.nc) + 2 * h) * A.A + V.aoff + loc;
            col[0] = fromf<T>(r0);
            col[A.A] = fromf<T>(r1);
        }
    }
}

template <typename T, int TPW>
__global__ __launch_bounds__(256) void box_dfl(const BoxDflArgs A) {
    int li = 0;
    if (A.nlv > 1 && (int)blockIdx.x >= A.lv[1].wg0) li = 1;
    if (A.nlv > 2 && (int)blockIdx.x >= A.lv[2].wg0) li = 2;
    if (A.nk == 4) bd_body<T, 4, TPW>(A, li);
    else if (A.nk == 6) bd_body<T, 6, TPW>(A, li);
}

}  // namespace

template <typename T>
static int launch_box_dfl_t(const BoxDflArgs& a, hipStream_t s) {
    if (!(a.nk == 4 || a.nk == 6)) return (int)hipErrorInvalidValue;
    int grid = 0;
    for (int l = 0; l < a.nlv; ++l) {
        const BoxDflLevel& v = a.lv[l];
        if (v.wg0 != grid || v.ldx % 8 || v.wld % 8) return (int)hipErrorInvalidValue;
        const long long tiles = ((long long)a.B * v.H * v.W + 31) / 32;
        grid += (int)((tiles + 4 * a.tpw - 1) / (4 * a.tpw));
    }
    switch (a.tpw) {
        case 1: hipLaunchKernelGGL((box_dfl<T, 1>), dim3((unsigned)grid), dim3(256), 0, s, a); break;
        case 2: hipLaunchKernelGGL((box_dfl<T, 2>), dim3((unsigned)grid), dim3(256), 0, s, a); break;
        case 4: hipLaunchKernelGGL((box_dfl<T, 4>), dim3((unsigned)grid), dim3(256), 0, s, a); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

int launch_box_dfl(int dtype, const BoxDflArgs& a, hipStream_t s) {
    switch (dtype) {
        case F16: return launch_box_dfl_t<_Float16>(a, s);
        case BF16: return launch_box_dfl_t<__bf16>(a, s);
    }
    return (int)hipErrorInvalidValue;
}

// every hc_div / hc_q quotient of a TH x TW tile is exact (n < 2^s / d for each divisor d and
// numerator range n the kernel uses), so a larger tile added to head_cls_tile cannot silently
// index the wrong rows
static bool hc_div_exact(int TH, int TW, int C0, int c3, int nc) {
    const long long XH = TH + 4, XW = TW + 4, MH = TH + 2, MW = TW + 2;
    if (XH * XW * XW >= (1 << 16) || MH * MW * MW >= (1 << 16) || (long long)TH * TW * TW >= (1 << 16)) return false;
    const int ng1 = (C0 < HC_CK ? C0 : HC_CK) / 4, ng2 = c3 / 4;
    for (int k = 0; k < 2; ++k) {   // the two depthwise phases: MH x MW (dw1) and TH x TW (dw2)
        const long long DH = k ? TH : MH, DW = k ? TW : MW, ng = k ? ng2 : ng1;
        const long long per_g = DW * ((DH + HC_RB - 1) / HC_RB);
        // item q < ng * per_g: q / ng (2^24 scale, n * m < 2^32), then (q / ng) / DW (2^16 scale)
        if (DW * per_g >= (1 << 16) || ng * ng * per_g >= (1 << 24) ||
            per_g * (1ll << 24) + ng * per_g >= (1ll << 32))
            return false;
    }
    const long long na = (std::max(c3, nc) + 31) / 32, nb = (MH * MW + 31) / 32;
    return na * nb * nb < (1 << 16);   // hc_pw_units: unit index / nb
}

int head_cls_lds(int TH, int TW, int C0, int c3, int nc) {
    if (C0 % 64 && C0 > 64) return 0;            // whole 64-channel chunks
    if (!hc_div_exact(TH, TW, C0, c3, nc)) return 0;
    // instantiated: C0 64 / 128 / 256, c3 64 / 80, at most three 32-cout tiles per pointwise conv
    if (!(C0 == 64 || C0 == 128 || C0 == 256) || !(c3 == 64 || c3 == 80) || nc > 32 * HC_NA) return 0;
    // parameter chunks: 10 (C0 + c3) / 4 + 72 <= 4 per thread
    if ((10 * (C0 + c3)) / 4 + 72 > 4 * HEAD_CLS_THREADS) return 0;
    const HcLayout L = hc_layout(TH, TW, C0, c3);
    return L.total <= HEAD_CLS_LDS && L.total <= 160 * 1024 ? L.total : 0;
}

template <typename T>
static int launch_head_cls_t(const HeadClsArgs& a, hipStream_t s) {
    int grid = 0, lds = 0;
    for (int l = 0; l < a.nlv; ++l) {
        const HeadClsLevel& v = a.lv[l];
        const int b = head_cls_lds(v.TH, v.TW, v.C0, a.c3, a.nc);
        if (b == 0 || v.wg0 != grid) return (int)hipErrorInvalidValue;
        grid += a.B * v.tiles;
        lds = lds > b ? lds : b;
    }
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&head_cls<T>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    hipLaunchKernelGGL((head_cls<T>), dim3((unsigned)grid), dim3(HEAD_CLS_THREADS), lds, s, a);
    return (int)hipGetLastError();
}

#ifdef YH_HC_TRACE
extern "C" int yh_debug_hc_trace(unsigned long long* dst, int n) {
    if (n > HC_TR_WG * HC_TR) n = HC_TR_WG * HC_TR;
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(hc_trace_buf), (size_t)n * 8, 0, hipMemcpyDeviceToHost);
}
#endif

int launch_head_cls(int dtype, const HeadClsArgs& a, hipStream_t s) {
    switch (dtype) {
        case F16: return launch_head_cls_t<_Float16>(a, s);
        case BF16: return launch_head_cls_t<__bf16>(a, s);
    }
    return (int)hipErrorInvalidValue;
}

}  // namespace yh
