// Convolution kernels for gfx950 (CDNA4):
//   conv_gemm   dense 1x1 / 3x3 (any stride) as an MFMA implicit GEMM over NHWC,
//               fused bias + SiLU/identity + residual add, writes into channel
//               slices of concat buffers (zero-copy torch.cat, nets/nn.py:78-80,
//               62-63, 94, 148, 205-208) and reads up-sampled concat inputs
//               directly (DarkFPN, nets/nn.py:195,205-206).
//   conv_first  the 3-channel stem conv (nets/nn.py:161) reading the caller's
//               NCHW tensor, VALU.
//   dwconv3x3   depthwise 3x3 (Head cls branch nn.py:248,250), VALU.
//
// Reference semantics: Conv.fuse_forward (nets/nn.py:38-39) = act(conv'(x)) with
// the BN folded into conv' (fuse_conv, nets/nn.py:8-25); Residual (nn.py:48-49)
// = x + act(conv'(...)) -> residual added after the activation.
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "dtypes.h"

namespace yh {

namespace {

constexpr int BK = 32;        // reduction depth per stage (one 16x16x32 MFMA)
constexpr int LDK = BK + 8;   // padded LDS row (elements) to spread banks
constexpr int NT_ = 256;      // threads per block (4 waves)

template <typename T, int BM, int BN>
struct ConvSmem {
    static constexpr int A_ELEMS = 2 * BM * LDK;
    static constexpr int B_ELEMS = 2 * BN * LDK;
    static constexpr int MAIN = (A_ELEMS + B_ELEMS) * (int)sizeof(T);
    static constexpr int EPI = BM * (BN + 8) * (int)sizeof(T);
    static constexpr int REGION = MAIN > EPI ? MAIN : EPI;  // epilogue reuses the staging area
};

template <typename T, int BM, int BN>
__global__ __launch_bounds__(NT_) void conv_gemm(const ConvArgs p) {
    static_assert(BM % 64 == 0 && BN % 16 == 0, "tile");
    constexpr int MT = BM / 64;             // 16-pixel MFMA tiles per wave
    constexpr int NTL = BN / 16;            // 16-cout MFMA tiles
    constexpr int CA = (BM * (BK / 8)) / NT_;  // A chunks per thread
    constexpr int NV = sizeof(T) / 2;
    using SM = ConvSmem<T, BM, BN>;

    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* As = reinterpret_cast<T*>(smem);
    T* Bs = As + SM::A_ELEMS;
    int* ktab = reinterpret_cast<int*>(smem + SM::REGION);

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int lid = xcd_remap(blockIdx.x, p.gm * p.gn);
    const int mt = lid / p.gn, nt = lid - mt * p.gn;
    const int m0 = mt * BM, n0 = nt * BN;

    for (int i = tid; i < p.Kp / 8; i += NT_) ktab[i] = p.ktab[i];

    // Per-thread A rows: row = (tid >> 2) + 64*i, k-chunk = tid & 3 (fixed).
    const int kc = tid & 3;
    int rn[CA], rhb[CA], rwb[CA];
    const int HoWo = p.Ho * p.Wo;
#pragma unroll
    for (int i = 0; i < CA; ++i) {
        const int m = m0 + (tid >> 2) + 64 * i;
        if (m < p.M) {
            const int n = m / HoWo, r = m - n * HoWo;
            const int ho = r / p.Wo, wo = r - ho * p.Wo;
            rn[i] = n;
            rhb[i] = ho * p.stride - p.pad;
            rwb[i] = wo * p.stride - p.pad;
        } else {
            rn[i] = -1; rhb[i] = 0; rwb[i] = 0;
        }
    }
    const T* in0 = reinterpret_cast<const T*>(p.in0);
    const T* in1 = reinterpret_cast<const T*>(p.in1);
    const T* wg = reinterpret_cast<const T*>(p.w);
    const long long bs0 = (long long)p.h0 * p.w0 * p.ldc0;
    const long long bs1 = (long long)p.h1 * p.w1 * p.ldc1;

    Chunk<T> ra[CA];
    Chunk<T> rb;
    const int bchunks = BN * (BK / 8);
    const bool bload = tid < bchunks || bchunks > NT_;  // BN <= 128 -> bchunks <= 512
    constexpr int CB = (BN * (BK / 8) + NT_ - 1) / NT_;
    Chunk<T> rbv[CB];

    __syncthreads();  // ktab visible

    auto load_tile = [&](int kt) {
        const int e = ktab[kt * (BK / 8) + kc];
        const int kh = e >> 24, kw = (e >> 16) & 0xff, ci = e & 0xffff;
#pragma unroll
        for (int i = 0; i < CA; ++i) {
            const int hi = rhb[i] + kh, wi = rwb[i] + kw;
            const bool ok = (ci != 0xffff) && rn[i] >= 0 && hi >= 0 && hi < p.Hi && wi >= 0 && wi < p.Wi;
            if (ok) {
                const T* src;
                if (ci < p.c0) {
                    src = in0 + rn[i] * bs0 + ((long long)(hi >> p.up0) * p.w0 + (wi >> p.up0)) * p.ldc0 + ci;
                } else {
                    src = in1 + rn[i] * bs1 + ((long long)(hi >> p.up1) * p.w1 + (wi >> p.up1)) * p.ldc1 + (ci - p.c0);
                }
                ra[i] = ld_chunk(src);
            } else {
                ra[i] = zero_chunk<T>();
            }
        }
#pragma unroll
        for (int j = 0; j < CB; ++j) {
            const int c = tid + j * NT_;
            if (c < bchunks) {
                const int co = c >> 2, kk = c & 3;
                rbv[j] = ld_chunk(wg + (long long)(n0 + co) * p.Kp + kt * BK + kk * 8);
            }
        }
    };
    auto store_tile = [&](int buf) {
        T* a = As + buf * BM * LDK;
#pragma unroll
        for (int i = 0; i < CA; ++i) st_chunk(a + ((tid >> 2) + 64 * i) * LDK + kc * 8, ra[i]);
        T* b = Bs + buf * BN * LDK;
#pragma unroll
        for (int j = 0; j < CB; ++j) {
            const int c = tid + j * NT_;
            if (c < bchunks) st_chunk(b + (c >> 2) * LDK + (c & 3) * 8, rbv[j]);
        }
    };
    (void)rb; (void)bload;

    typename Mma<T>::acc_t acc[NTL][MT];
#pragma unroll
    for (int i = 0; i < NTL; ++i)
#pragma unroll
        for (int j = 0; j < MT; ++j) acc[i][j] = typename Mma<T>::acc_t{0, 0, 0, 0};

    const int nkt = p.Kp / BK;
    load_tile(0);
    store_tile(0);
    __syncthreads();

    const int fr = lane & 15, fk = (lane >> 4) * 8;  // fragment row/col and k offset
    for (int kt = 0; kt < nkt; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nkt) load_tile(kt + 1);
        const T* a = As + cur * BM * LDK;
        const T* b = Bs + cur * BN * LDK;
        uint4 bw[NTL][NV];
#pragma unroll
        for (int i = 0; i < NTL; ++i) {
            const uint4* q = reinterpret_cast<const uint4*>(b + (i * 16 + fr) * LDK + fk);
#pragma unroll
            for (int v = 0; v < NV; ++v) bw[i][v] = q[v];
        }
#pragma unroll
        for (int j = 0; j < MT; ++j) {
            uint4 xa[NV];
            const uint4* q = reinterpret_cast<const uint4*>(a + (wave * (BM / 4) + j * 16 + fr) * LDK + fk);
#pragma unroll
            for (int v = 0; v < NV; ++v) xa[v] = q[v];
#pragma unroll
            for (int i = 0; i < NTL; ++i) Mma<T>::step(acc[i][j], bw[i], xa);
        }
        if (kt + 1 < nkt) store_tile(cur ^ 1);
        __syncthreads();
    }

    // Epilogue: bias + activation in f32, stage the tile as T in LDS, then
    // coalesced 8-channel stores (+ residual) to the NHWC output view.
    constexpr int LDE = BN + 8;
    T* Cs = reinterpret_cast<T*>(smem);
#pragma unroll
    for (int i = 0; i < NTL; ++i) {
        int co[4];
        float bv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            co[r] = i * 16 + Mma<T>::row(lane >> 4, r);
            bv[r] = p.bias[n0 + co[r]];
        }
#pragma unroll
        for (int j = 0; j < MT; ++j) {
            const int px = wave * (BM / 4) + j * 16 + fr;
            T* dst = Cs + px * LDE;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float v = Mma<T>::finish(acc[i][j][r], bv[r]);
                if (p.act == ACT_SILU) v = silu<T>(v);
                dst[co[r]] = fromf<T>(v);
            }
        }
    }
    __syncthreads();
    const T* res = reinterpret_cast<const T*>(p.res);
    T* out = reinterpret_cast<T*>(p.out);
    constexpr int CPP = BN / 8;  // chunks per pixel row of the tile
    for (int c = tid; c < BM * CPP; c += NT_) {
        const int px = c / CPP, cc = c - px * CPP;
        const int m = m0 + px, co = n0 + cc * 8;
        if (m >= p.M || co >= p.Cout) continue;
        Chunk<T> v = ld_chunk(Cs + px * LDE + cc * 8);
        if (res) {
            float f[8], g[8];
            chunk_to_f(v, f);
            chunk_to_f(ld_chunk(res + (long long)m * p.ldr + co), g);
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] += g[e];
            v = f_to_chunk<T>(f);
        }
        st_chunk(out + (long long)m * p.ldo + co, v);
    }
}



template <typename T, int BM, int BN>
int launch_conv_t(const ConvArgs& a, hipStream_t s) {
    using SM = ConvSmem<T, BM, BN>;
    const int lds = SM::REGION + (a.Kp / 8) * 4;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_gemm<T, BM, BN>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    hipLaunchKernelGGL((conv_gemm<T, BM, BN>), dim3(a.gm * a.gn), dim3(NT_), lds, s, a);
    return (int)hipGetLastError();
}

template <typename T>
int launch_conv_bm(int BM, int BN, const ConvArgs& a, hipStream_t s) {
#define YH_BN(bm)                                                        \
    switch (BN) {                                                        \
        case 16: return launch_conv_t<T, bm, 16>(a, s);                  \
        case 32: return launch_conv_t<T, bm, 32>(a, s);                  \
        case 64: return launch_conv_t<T, bm, 64>(a, s);                  \
        case 128: return launch_conv_t<T, bm, 128>(a, s);                \
        default: return (int)hipErrorInvalidValue;                       \
    }
    switch (BM) {
        case 64: YH_BN(64)
        case 128: YH_BN(128)
        case 256: YH_BN(256)
        default: return (int)hipErrorInvalidValue;
    }
#undef YH_BN
}

// Stem: Conv(3 -> Cout, k3, s2, p1) + act (nets/nn.py:161) straight from the
// caller's NCHW tensor. A block = STEM_TW consecutive output pixels of one output
// row: the 3 channels x 3 input rows x (2*STEM_TW+1) columns it needs are
// contiguous row segments in NCHW, staged into LDS with aligned 16-B loads
// (one HBM read of the input, ~1.5x with the row overlap of neighbouring
// output rows served from L2). One thread = one output pixel x all couts;
// weights ([27][Cout], packed on the host) are wave-uniform scalar loads.
constexpr int STEM_TW = 128;
constexpr int STEM_SEG = 2 * STEM_TW + 16;  // staged columns per row segment (aligned window)

// Input element U -> the value the stem sees. U == T: the caller's tensor as is.
// U == uint8_t: the reference's preprocessing (main.py:265-267, `samples.half()
// / 255.`) fused into the load, computed the way torch's device kernel does a
// division by a CPU scalar: u (exact in T) times the fp32 reciprocal 1/255,
// rounded to T.
template <typename U, typename T>
__device__ __forceinline__ float stem_in(U v) {
    if constexpr (sizeof(U) == 1) return fromf_round<T>((float)v * (1.0f / 255.0f));
    else return tof(v);
}
template <typename U, typename T>
__device__ __forceinline__ void stem_in8(const U* p, float (&f)[8]) {
    if constexpr (sizeof(U) == 1) {
        const uint2 v = *reinterpret_cast<const uint2*>(p);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = stem_in<uint8_t, T>((uint8_t)(((e < 4 ? v.x : v.y) >> (8 * (e & 3))) & 255u));
    } else {
        chunk_to_f(ld_chunk(p), f);
    }
}

// Stage the block's input window (3 channels x 3 rows x STEM_SEG columns) into the
// float LDS patch. W is a multiple of 8 and the window is 8-aligned, so each
// 8-element chunk is wholly inside the image or wholly padding: every load is
// issued before any is used (clamped address + select, no branch), one round trip.
constexpr int STEM_CPS = STEM_SEG / 8;
constexpr int STEM_NCH = (9 * STEM_CPS + STEM_TW - 1) / STEM_TW;
template <typename T, typename U>
__device__ __forceinline__ void stem_stage(const U* x, const FirstConvArgs& p, int n, int ho, int col0,
                                           float (*patch)[STEM_SEG]) {
    const long long plane = (long long)p.H * p.W;
    using Raw = typename std::conditional<sizeof(U) == 1, uint2, Chunk<U>>::type;   // 8 elements
    Raw raw[STEM_NCH];
    bool ok[STEM_NCH];
    int dst[STEM_NCH];
#pragma unroll
    for (int u = 0; u < STEM_NCH; ++u) {
        const int c = min((int)threadIdx.x + u * STEM_TW, 9 * STEM_CPS - 1);   // past the end: redo the last
        const int seg = c / STEM_CPS, ch = c - seg * STEM_CPS;
        const int ci = seg / 3, kh = seg - ci * 3;
        const int hi = 2 * ho - 1 + kh;
        const int col = col0 + ch * 8;
        ok[u] = hi >= 0 && hi < p.H && col >= 0 && col + 8 <= p.W;
        const int hc = min(max(hi, 0), p.H - 1), cc = min(max(col, 0), p.W - 8);
        raw[u] = *reinterpret_cast<const Raw*>(x + ((long long)n * 3 + ci) * plane + (long long)hc * p.W + cc);
        dst[u] = c;
    }
#pragma unroll
    for (int u = 0; u < STEM_NCH; ++u) {
        float f[8];
        if constexpr (sizeof(U) == 1) {
#pragma unroll
            for (int e = 0; e < 8; ++e)
                f[e] = stem_in<uint8_t, T>((uint8_t)((((const uint2&)raw[u]).x >> (8 * (e & 3)) & 255u) * (e < 4) +
                                                     (((const uint2&)raw[u]).y >> (8 * (e & 3)) & 255u) * (e >= 4)));
        } else {
            chunk_to_f(raw[u], f);
        }
        const int seg = dst[u] / STEM_CPS, ch = dst[u] - seg * STEM_CPS;
#pragma unroll
        for (int e = 0; e < 8; ++e) patch[seg][ch * 8 + e] = ok[u] ? f[e] : 0.f;
    }
}

template <typename T, typename U, int NC8>
__global__ __launch_bounds__(STEM_TW) void conv_first(const FirstConvArgs p) {
    __shared__ float patch[9][STEM_SEG];
    const int wo0 = blockIdx.x * STEM_TW, ho = blockIdx.y, n = blockIdx.z;
    const U* x = reinterpret_cast<const U*>(p.io[0]);
    const int col0 = 2 * wo0 - 8;  // 16-B aligned window start (8 elements before the first tap)
    stem_stage<T, U>(x, p, n, ho, col0, patch);
    __syncthreads();
    const int wo = wo0 + threadIdx.x;
    const bool live = wo < p.Wo;  // no early exit: keep the weight loads wave-uniform (scalar)
    float xv[27];
    const int lc = 2 * threadIdx.x - 1 + 8;  // local column of tap kw=0
#pragma unroll
    for (int seg = 0; seg < 9; ++seg)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) xv[seg * 3 + kw] = patch[seg][lc + kw];
    const long long m = ((long long)n * p.Ho + ho) * p.Wo + wo;
    T* out = reinterpret_cast<T*>(p.out) + m * p.ldo;
    const float* __restrict__ wgt = p.w;
    const float* __restrict__ bia = p.bias;
    constexpr int COUT = NC8 * 8;
#pragma unroll
    for (int c0 = 0; c0 < COUT; c0 += 8) {
        float acc[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = bia[c0 + e];
#pragma unroll
        for (int k = 0; k < 27; ++k) {
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[e] = fmaf(wgt[k * COUT + c0 + e], xv[k], acc[e]);
        }
        float f[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = p.act == ACT_SILU ? silu<T>(acc[e]) : acc[e];
        if (live) st_chunk(out + c0, f_to_chunk<T>(f));
    }
}

// 16-bit stem on MFMA: K = 27 taps padded to 32 = one v_mfma_f32_16x16x32 per
// 16 pixels x 16 couts. A = weights (built once per wave from the fp32 [27][Cout]
// pack), B = the im2col column of 16 pixels gathered from the LDS patch.
template <typename T, typename U, int NT>
__global__ __launch_bounds__(STEM_TW) void conv_first_mfma(const FirstConvArgs p) {
    __shared__ float patch[9][STEM_SEG];
    const int wo0 = blockIdx.x * STEM_TW, ho = blockIdx.y, n = blockIdx.z;
    const U* x = reinterpret_cast<const U*>(p.io[0]);
    const int col0 = 2 * wo0 - 8;
    stem_stage<T, U>(x, p, n, ho, col0, patch);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int fr = lane & 15, g = lane >> 4;
    // A fragments: weights[cout = 16i + fr][k = 8g + j]
    uint4 wf[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        float f[8];
        const int co = 16 * i + fr;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = 8 * g + j;
            f[j] = (k < 27 && co < p.Cout) ? p.w[k * p.Cout + co] : 0.f;
        }
        wf[i] = f_to_chunk<T>(f).v[0];
    }
    float bv[NT][4];
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int co = 16 * i + 4 * g + r;
            bv[i][r] = co < p.Cout ? p.bias[co] : 0.f;
        }
    __syncthreads();
#pragma unroll
    for (int pg = 0; pg < STEM_TW / 2 / 16; ++pg) {   // 4 groups of 16 pixels per wave
        const int px = wave * (STEM_TW / 2) + pg * 16 + fr;
        const int lc = 2 * px - 1 + 8;
        float f[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = 8 * g + j;
            const int seg = k / 3, kw = k - seg * 3;
            f[j] = k < 27 ? patch[seg][lc + kw] : 0.f;
        }
        const uint4 xf = f_to_chunk<T>(f).v[0];
        const int wo = wo0 + px;
        const long long m = ((long long)n * p.Ho + ho) * p.Wo + wo;
        T* out = reinterpret_cast<T*>(p.out) + m * p.ldo;
#pragma unroll
        for (int i = 0; i < NT; ++i) {
            f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
            Mma<T>::step(acc, &wf[i], &xf);
            const int co = 16 * i + 4 * g;
            if (wo < p.Wo && co < p.Cout) {
                unsigned u[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float v = acc[r] + bv[i][r];
                    if (p.act == ACT_SILU) v = silu<T>(v);
                    u[r] = (unsigned short)__builtin_bit_cast(short, fromf<T>(v));
                }
                *reinterpret_cast<uint2*>(out + co) = make_uint2(u[0] | (u[1] << 16), u[2] | (u[3] << 16));
            }
        }
    }
}

// 16-bit stem, 2-D tiles: a workgroup = STEM2_TR output rows x STEM2_TW pixels.
// The 2*TR+1 input rows of each channel are staged once as T (the values the
// MFMA consumes), so neighbouring output rows share their overlap row in LDS
// (input read ~(2TR+1)/(2TR) times instead of 1.5x) and every thread keeps
// STEM2_NCH 16-B loads in flight. Same k order (ci, kh, kw) and epilogue as
// conv_first_mfma -> identical outputs.
constexpr int STEM2_TW = 160, STEM2_NT = 256;
// pixel groups per wave unrolled (all 10: every group's LDS gathers and MFMA in flight
// together; 2 -> 10 measured 59.3 -> 55.9 us for the v11_n b32 stem)
#ifndef STEM2_UNROLL
#define STEM2_UNROLL 10
#endif
constexpr int STEM2_SEG = 2 * STEM2_TW + 16;         // staged columns per row segment
constexpr int STEM2_CPS = STEM2_SEG / 8;             // 8-element chunks per segment
template <typename T, typename U, int NT, int STEM2_TR>
__global__ __launch_bounds__(STEM2_NT) void conv_first_tile(const FirstConvArgs p) {
    constexpr int STEM2_ROWS = 3 * (2 * STEM2_TR + 1);   // (channel, input row) segments
    constexpr int STEM2_NCH = (STEM2_ROWS * STEM2_CPS + STEM2_NT - 1) / STEM2_NT;
    static_assert(sizeof(T) == 2, "16-bit path");
    __shared__ __attribute__((aligned(16))) T patch[STEM2_ROWS][STEM2_SEG];
    const int wo0 = blockIdx.x * STEM2_TW, ho0 = blockIdx.y * STEM2_TR, n = blockIdx.z;
    const U* x = reinterpret_cast<const U*>(p.io[0]);
    const int col0 = 2 * wo0 - 8;
    const long long plane = (long long)p.H * p.W;
    {   // stage: all loads first (clamped address + select), then the LDS stores
        using Raw = typename std::conditional<sizeof(U) == 1, uint2, uint4>::type;   // 8 elements
        Raw raw[STEM2_NCH];
        bool ok[STEM2_NCH];
        int dst[STEM2_NCH];
#pragma unroll
        for (int u = 0; u < STEM2_NCH; ++u) {
            const int c = min((int)threadIdx.x + u * STEM2_NT, STEM2_ROWS * STEM2_CPS - 1);
            const int seg = c / STEM2_CPS, ch = c - seg * STEM2_CPS;
            const int ci = seg / (2 * STEM2_TR + 1), rr = seg - ci * (2 * STEM2_TR + 1);
            const int hi = 2 * ho0 - 1 + rr;
            const int col = col0 + ch * 8;
            ok[u] = hi >= 0 && hi < p.H && col >= 0 && col + 8 <= p.W;
            const int hc = min(max(hi, 0), p.H - 1), cc = min(max(col, 0), p.W - 8);
            raw[u] = *reinterpret_cast<const Raw*>(x + ((long long)n * 3 + ci) * plane + (long long)hc * p.W + cc);
            dst[u] = c;
        }
#pragma unroll
        for (int u = 0; u < STEM2_NCH; ++u) {
            const int seg = dst[u] / STEM2_CPS, ch = dst[u] - seg * STEM2_CPS;
            uint4 v;
            if constexpr (sizeof(U) == 1) {
                float f[8];
#pragma unroll
                for (int e = 0; e < 8; ++e)
                    f[e] = stem_in<uint8_t, T>((uint8_t)(((e < 4 ? raw[u].x : raw[u].y) >> (8 * (e & 3))) & 255u));
                v = f_to_chunk<T>(f).v[0];
            } else {
                v = raw[u];
            }
            *reinterpret_cast<uint4*>(&patch[seg][ch * 8]) = ok[u] ? v : make_uint4(0, 0, 0, 0);
        }
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int fr = lane & 15, g = lane >> 4;
    uint4 wf[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        float f[8];
        const int co = 16 * i + fr;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = 8 * g + j;
            f[j] = (k < 27 && co < p.Cout) ? p.w[k * p.Cout + co] : 0.f;
        }
        wf[i] = f_to_chunk<T>(f).v[0];
    }
    float bv[NT][4];
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int co = 16 * i + 4 * g + r;
            bv[i][r] = co < p.Cout ? p.bias[co] : 0.f;
        }
    // this lane's 8 k values as (segment row offset, column offset) in the patch
    int koff[8];
    bool kok[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int k = 8 * g + j;
        const int ci = k / 9, kh = (k - ci * 9) / 3, kw = k - ci * 9 - kh * 3;
        kok[j] = k < 27;
        koff[j] = kok[j] ? (ci * (2 * STEM2_TR + 1) + kh) * STEM2_SEG + kw : 0;
    }
    __syncthreads();
    const T* pbase = &patch[0][0];
    constexpr int GPR = STEM2_TW / 16;                 // 16-pixel groups per output row
    constexpr int NG = STEM2_TR * GPR / (STEM2_NT / 64);
#pragma unroll STEM2_UNROLL
    for (int it = 0; it < NG; ++it) {
        const int gi = wave + it * (STEM2_NT / 64);
        const int tr = gi / GPR, px = (gi - tr * GPR) * 16 + fr;
        const int ho = ho0 + tr, wo = wo0 + px;
        const int b0 = 2 * tr * STEM2_SEG + 2 * px - 1 + 8;
        T xv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) xv[j] = kok[j] ? pbase[b0 + koff[j]] : fromf<T>(0.f);
        const uint4 xf = *reinterpret_cast<const uint4*>(xv);
        const long long m = ((long long)n * p.Ho + ho) * p.Wo + wo;
        T* out = reinterpret_cast<T*>(p.out) + m * p.ldo;
        const bool live = wo < p.Wo && ho < p.Ho;
#pragma unroll
        for (int i = 0; i < NT; ++i) {
            f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
            Mma<T>::step(acc, &wf[i], &xf);
            const int co = 16 * i + 4 * g;
            if (live && co < p.Cout) {
                unsigned u[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float v = acc[r] + bv[i][r];
                    if (p.act == ACT_SILU) v = silu<T>(v);
                    u[r] = (unsigned short)__builtin_bit_cast(short, fromf<T>(v));
                }
                *reinterpret_cast<uint2*>(out + co) = make_uint2(u[0] | (u[1] << 16), u[2] | (u[3] << 16));
            }
        }
    }
}

template <typename T, typename U>
int launch_first_tu(const FirstConvArgs& a, int B, hipStream_t s) {
    const dim3 grid((a.Wo + STEM_TW - 1) / STEM_TW, a.Ho, B);
    if constexpr (sizeof(T) == 2) {
        static const bool tile = [] { const char* e = getenv("YH_STEM"); return !e || atoi(e) != 1; }();
        if (tile) {
            static const int tr = [] { const char* e = getenv("YH_STEM_TR"); return e ? atoi(e) : 4; }();
            const dim3 g2((a.Wo + STEM2_TW - 1) / STEM2_TW, (a.Ho + tr - 1) / tr, B);
#define YH_ST(R)                                                                                              \
            switch ((a.Cout + 15) / 16) {                                                                     \
                case 1: hipLaunchKernelGGL((conv_first_tile<T, U, 1, R>), g2, dim3(STEM2_NT), 0, s, a); break; \
                case 2: hipLaunchKernelGGL((conv_first_tile<T, U, 2, R>), g2, dim3(STEM2_NT), 0, s, a); break; \
                case 4: hipLaunchKernelGGL((conv_first_tile<T, U, 4, R>), g2, dim3(STEM2_NT), 0, s, a); break; \
                case 6: hipLaunchKernelGGL((conv_first_tile<T, U, 6, R>), g2, dim3(STEM2_NT), 0, s, a); break; \
                default: return (int)hipErrorInvalidValue;                                                    \
            }
            if (tr == 2) { YH_ST(2) } else if (tr == 8) { YH_ST(8) } else { YH_ST(4) }
#undef YH_ST
            return (int)hipGetLastError();
        }
        switch ((a.Cout + 15) / 16) {
            case 1: hipLaunchKernelGGL((conv_first_mfma<T, U, 1>), grid, dim3(STEM_TW), 0, s, a); break;
            case 2: hipLaunchKernelGGL((conv_first_mfma<T, U, 2>), grid, dim3(STEM_TW), 0, s, a); break;
            case 4: hipLaunchKernelGGL((conv_first_mfma<T, U, 4>), grid, dim3(STEM_TW), 0, s, a); break;
            case 6: hipLaunchKernelGGL((conv_first_mfma<T, U, 6>), grid, dim3(STEM_TW), 0, s, a); break;
            default: return (int)hipErrorInvalidValue;
        }
        return (int)hipGetLastError();
    }
    switch (a.Cout) {
        case 16: hipLaunchKernelGGL((conv_first<T, U, 2>), grid, dim3(STEM_TW), 0, s, a); break;
        case 24: hipLaunchKernelGGL((conv_first<T, U, 3>), grid, dim3(STEM_TW), 0, s, a); break;
        case 32: hipLaunchKernelGGL((conv_first<T, U, 4>), grid, dim3(STEM_TW), 0, s, a); break;
        case 64: hipLaunchKernelGGL((conv_first<T, U, 8>), grid, dim3(STEM_TW), 0, s, a); break;
        case 96: hipLaunchKernelGGL((conv_first<T, U, 12>), grid, dim3(STEM_TW), 0, s, a); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

template <typename T>
int launch_first_t(const FirstConvArgs& a, int B, hipStream_t s) {
    return a.in_u8 ? launch_first_tu<T, uint8_t>(a, B, s) : launch_first_tu<T, T>(a, B, s);
}

// ---------------------------------------------------------------------------
// Stem + net.p2.0 in one launch (nets/nn.py:160-163: Conv(3, w1, 3, 2) -> Conv(w1, w2,
// 3, 2), both SiLU): the stem's output, 2x the p2.0 output in each direction plus a
// 1-pixel halo, lives only in LDS, so its HBM write and re-read (105 MB each at v11_n
// b32 640^2) disappear.
// A workgroup (4 waves) owns S2_TH x S2_TW p2.0 outputs of one image:
//   1. the 3 x (4 S2_TH + 3) x (4 S2_TW + 3) input window -> LDS (8-aligned chunks,
//      wholly inside the image or zero, exactly as conv_first_tile stages it);
//   2. the (2 S2_TH + 1) x (2 S2_TW + 1) stem pixels: conv_first_tile's arithmetic (k =
//      ci*9 + kh*3 + kw on v_mfma_f32_16x16x32, bias, SiLU, one rounding), stored NHWC
//      in LDS; pixels outside the stem map are p2.0's zero padding and stored as 0;
//   3. p2.0 on v_mfma_f32_32x32x16 in conv_mx's canonical K order (for 16-channel block:
//      for tap: one step), bias, SiLU, one rounding (mx_epi) -> HBM.
// Output is bit-identical to conv_first_tile followed by conv_mx.
constexpr int S2_TH = 4, S2_TW = 32, S2_NT = 256;
constexpr int S2_SR = 2 * S2_TH + 1, S2_SC = 2 * S2_TW + 1;   // stem region (rows, cols)
constexpr int S2_IR = 2 * S2_SR + 1;                          // input rows per channel
constexpr int S2_ICH = (4 * S2_TW + 32) / 8;                  // 8-element chunks per input row
constexpr int S2_ISEG = 8 * S2_ICH;                           // staged columns (from 4 wo0 - 32: 64-B aligned)
constexpr int S2_NPX = S2_SR * S2_SC;                         // stem pixels per tile
typedef __attribute__((ext_vector_type(16))) float f32x16_s;

template <typename T>
__device__ __forceinline__ f32x16_s s2_mfma(const uint4& a, const uint4& b, const f32x16_s& c) {
    if constexpr (std::is_same<T, __bf16>::value)
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                       0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                      0);
}
template <typename T>
__device__ __forceinline__ unsigned s2_pack2(float a, float b) {
    typedef __attribute__((ext_vector_type(2))) float f2;
    typedef __attribute__((ext_vector_type(2))) T t2;
    return __builtin_bit_cast(unsigned, __builtin_convertvector(f2{a, b}, t2));
}

template <typename T, typename U, int C1, int C2>
__global__ __launch_bounds__(S2_NT) void stem_fused(const Stem2Args p) {
    static_assert(sizeof(T) == 2, "16-bit path");
    constexpr int PS = 2 * C1 + 1;   // 16-B chunks per stored stem pixel (+1: 2-way banks on stride-2 reads)
    constexpr int KS = 9 * C1;       // p2.0 K steps
    constexpr int RPW = C2;          // output rows per wave (S2_TH rows x C2 cout tiles over 4 waves)
    static_assert(S2_TH * C2 == 4 * RPW, "4 waves");
    // + one zero row: the padded K values (k >= 27) read it instead of branching
    __shared__ __attribute__((aligned(16))) T patch[3 * S2_IR + 1][S2_ISEG];
    __shared__ uint4 sout[S2_NPX * PS];
    // (dispatch order kept: an XCD-aware order cut the input re-reads, 1.40x -> 1.00x of the
    // algorithmic bytes, but ran 75 -> 82 us)
    const int tx = blockIdx.x % p.ntw, ty = blockIdx.x / p.ntw, n = blockIdx.y;
    const int ho0 = ty * S2_TH, wo0 = tx * S2_TW;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h = lane >> 5, l32 = lane & 31;

    // p2.0 weight fragments of this wave's cout tile: issued first, consumed last
    const int a2 = wave % C2;
    uint4 af[KS];
    {
        const uint4* w2 = reinterpret_cast<const uint4*>(p.prm) + (size_t)a2 * KS * 64 + lane;
#pragma unroll
        for (int s = 0; s < KS; ++s) af[s] = w2[s * 64];
    }

    // 1. input window: rows 4 ho0 - 3 .., columns 4 wo0 - 32 .. (64-B aligned rows for 16-bit
    //    input: whole 64-B sectors, no partial-sector fetches at the row ends)
    const U* x = reinterpret_cast<const U*>(p.io[0]);
    const int ir0 = 4 * ho0 - 3, ca = 4 * wo0 - 32;
    const long long plane = (long long)p.H * p.W;
    {
        constexpr int TOT = 3 * S2_IR * S2_ICH;
        constexpr int NCH = (TOT + S2_NT - 1) / S2_NT;
        using Raw = typename std::conditional<sizeof(U) == 1, uint2, uint4>::type;
        Raw raw[NCH];
        bool ok[NCH];
#pragma unroll
        for (int u = 0; u < NCH; ++u) {
            const int c = min(tid + u * S2_NT, TOT - 1);
            const int seg = c / S2_ICH, ch = c - seg * S2_ICH;
            const int ci = seg / S2_IR, rr = seg - ci * S2_IR;
            const int hi = ir0 + rr, col = ca + 8 * ch;
            ok[u] = hi >= 0 && hi < p.H && col >= 0 && col + 8 <= p.W;
            const int hc = min(max(hi, 0), p.H - 1), cc = min(max(col, 0), p.W - 8);
            raw[u] = *reinterpret_cast<const Raw*>(x + ((long long)n * 3 + ci) * plane + (long long)hc * p.W + cc);
        }
#pragma unroll
        for (int u = 0; u < NCH; ++u) {
            const int c = tid + u * S2_NT;
            if (c >= TOT) continue;
            const int seg = c / S2_ICH, ch = c - seg * S2_ICH;
            uint4 v;
            if constexpr (sizeof(U) == 1) {
                float f[8];
#pragma unroll
                for (int e = 0; e < 8; ++e)
                    f[e] = stem_in<uint8_t, T>((uint8_t)(((e < 4 ? raw[u].x : raw[u].y) >> (8 * (e & 3))) & 255u));
                v = f_to_chunk<T>(f).v[0];
            } else {
                v = raw[u];
            }
            *reinterpret_cast<uint4*>(&patch[seg][ch * 8]) = ok[u] ? v : make_uint4(0, 0, 0, 0);
        }
    }
    if (tid < S2_ISEG / 8) *reinterpret_cast<uint4*>(&patch[3 * S2_IR][tid * 8]) = make_uint4(0, 0, 0, 0);
    // stem weights / biases (conv_first_tile's fragments)
    const int fr = lane & 15, g = lane >> 4;
    uint4 wf[C1];
    float bv[C1][4];
#pragma unroll
    for (int i = 0; i < C1; ++i) {
        float f[8];
        const int co = 16 * i + fr;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = 8 * g + j;
            f[j] = k < 27 ? p.w1[k * p.c1p + co] : 0.f;
        }
        wf[i] = f_to_chunk<T>(f).v[0];
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[i][r] = p.b1[16 * i + 4 * g + r];
    }
    int koff[8];
    bool kok[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int k = 8 * g + j;
        const int ci = k / 9, kh = (k - ci * 9) / 3, kw = k - ci * 9 - kh * 3;
        kok[j] = k < 27;
        koff[j] = kok[j] ? (ci * S2_IR + kh) * S2_ISEG + kw : 0;
    }
    __syncthreads();

    // 2. stem pixels of the region: stem row 2 ho0 - 1 + sr, col 2 wo0 - 1 + sc; every group of
    //    the wave unrolled (the LDS gathers of later groups overlap earlier groups' epilogues)
    {
        const T* pbase = &patch[0][0];
        constexpr int NG = (S2_NPX + 15) / 16, NIT = (NG + S2_NT / 64 - 1) / (S2_NT / 64);
        constexpr int ZIDX = 3 * S2_IR * S2_ISEG;   // the zero row
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            const int gi = wave + it * (S2_NT / 64);
            if (gi >= NG) break;
            const int q = min(gi * 16 + fr, S2_NPX - 1);
            const int sr = q / S2_SC, sc = q - sr * S2_SC;
            const int b0 = 2 * sr * S2_ISEG + 2 * sc + 29;
            T xv[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) xv[j] = pbase[kok[j] ? b0 + koff[j] : ZIDX];
            const uint4 xf = *reinterpret_cast<const uint4*>(xv);
            const int gs = 2 * ho0 - 1 + sr, gc = 2 * wo0 - 1 + sc;
            const bool live = gs >= 0 && gs < p.Hs && gc >= 0 && gc < p.Ws;
#pragma unroll
            for (int i = 0; i < C1; ++i) {
                f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
                Mma<T>::step(acc, &wf[i], &xf);
                unsigned u[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float v = acc[r] + bv[i][r];
                    v = silu<T>(v);
                    u[r] = live ? (unsigned short)__builtin_bit_cast(short, fromf<T>(v)) : 0u;
                }
                if (gi * 16 + fr < S2_NPX)
                    *reinterpret_cast<uint2*>(reinterpret_cast<char*>(sout) + q * PS * 16 + (16 * i + 4 * g) * 2) =
                        make_uint2(u[0] | (u[1] << 16), u[2] | (u[3] << 16));
            }
        }
    }
    __syncthreads();

    // 3. p2.0: wave -> cout tile a2, output rows r = wave / C2 + k * (4 / C2), 32 px each
    {
        const float* bias2 = reinterpret_cast<const float*>(reinterpret_cast<const char*>(p.prm) + p.prm_bias);
        const int co = 32 * a2 + 16 * h;
        float b2[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) b2[i] = bias2[co + i];
        T* out = reinterpret_cast<T*>(p.out);
#pragma unroll
        for (int k = 0; k < RPW; ++k) {
            const int r = wave / C2 + k * (4 / C2);
            f32x16_s acc;
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const int cb = s / 9, tap = s - 9 * cb, kh = tap / 3, kw = tap - 3 * kh;
                const int q = (2 * r + kh) * S2_SC + 2 * l32 + kw;
                acc = s2_mfma<T>(af[s], sout[q * PS + 2 * cb + h], acc);
            }
            // the row's 32 pixels x 32 couts through the wave's 2 KB of the (dead) input window:
            // 4 lanes per pixel store 64 contiguous bytes (one pixel per lane would write 2 x 16 B
            // of each of 32 pixels per instruction; conv_mx.hip co_stage)
            unsigned w[8];
#pragma unroll
            for (int e = 0; e < 16; e += 2) w[e >> 1] = s2_pack2<T>(silu<T>(acc[e] + b2[e]), silu<T>(acc[e + 1] + b2[e + 1]));
            char* E = reinterpret_cast<char*>(&patch[0][0]) + wave * 2048;
            const int sw = (l32 >> 1) & 3;
            *reinterpret_cast<uint4*>(E + (l32 * 4 + ((2 * h) ^ sw)) * 16) = make_uint4(w[0], w[1], w[2], w[3]);
            *reinterpret_cast<uint4*>(E + (l32 * 4 + ((2 * h + 1) ^ sw)) * 16) = make_uint4(w[4], w[5], w[6], w[7]);
            const int ho = ho0 + r;
#pragma unroll
            for (int k2 = 0; k2 < 2; ++k2) {
                const int pp = k2 * 16 + (lane >> 2), qq = lane & 3;
                const uint4 v = *reinterpret_cast<const uint4*>(E + (pp * 4 + (qq ^ ((pp >> 1) & 3))) * 16);
                const int wo = wo0 + pp;
                if (ho < p.Ho && wo < p.Wo)
                    *reinterpret_cast<uint4*>(out + (((long long)n * p.Ho + ho) * p.Wo + wo) * p.ldo + 32 * a2 + 8 * qq) = v;
            }
        }
    }
}

template <typename T, typename U>
int launch_stem2_tu(const Stem2Args& a, hipStream_t s) {
    const dim3 grid((unsigned)(a.ntw * a.nth), (unsigned)a.B);
    if (a.c1 == 16 && a.c2 == 32) hipLaunchKernelGGL((stem_fused<T, U, 1, 1>), grid, dim3(S2_NT), 0, s, a);
    else if (a.c1 == 32 && a.c2 == 64) hipLaunchKernelGGL((stem_fused<T, U, 2, 2>), grid, dim3(S2_NT), 0, s, a);
    else return (int)hipErrorInvalidValue;
    return (int)hipGetLastError();
}

// Depthwise 3x3, stride 1, pad 1 (nn.py:248,250). One thread = 8 channels x DW_ROWS
// vertically adjacent output pixels: the DW_ROWS + 2 input rows it needs are
// loaded once (no per-tap re-read of the shared rows), all loads are issued before
// any FMA (branch-free: out-of-image taps read an in-image address and are
// multiplied by 0, which adds exactly +-0 to a finite sum, so the result equals
// the skip-the-tap form bit for bit), tap order kh-major as before.
constexpr int DW_ROWS = 4;
template <typename T>
__global__ __launch_bounds__(256) void dwconv3x3(const DwArgs p) {
    const int cpp = p.C / 8;
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= p.W * cpp) return;
    const int w = t / cpp, cc = t - w * cpp;
    const int h0 = blockIdx.y * DW_ROWS, n = blockIdx.z;
    const int c0 = cc * 8;
    const T* in = reinterpret_cast<const T*>(p.in) + (long long)n * p.H * p.W * p.ldi + c0;
    float wt[9][8];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const float4 a = *reinterpret_cast<const float4*>(p.w + k * p.C + c0);
        const float4 b = *reinterpret_cast<const float4*>(p.w + k * p.C + c0 + 4);
        wt[k][0] = a.x; wt[k][1] = a.y; wt[k][2] = a.z; wt[k][3] = a.w;
        wt[k][4] = b.x; wt[k][5] = b.y; wt[k][6] = b.z; wt[k][7] = b.w;
    }
    Chunk<T> x[DW_ROWS + 2][3];
    float msk[DW_ROWS + 2][3];
#pragma unroll
    for (int r = 0; r < DW_ROWS + 2; ++r) {
        const int hi = h0 - 1 + r;
        const bool hok = (unsigned)hi < (unsigned)p.H;
        const int hc = min(max(hi, 0), p.H - 1);
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
            const int wi = w - 1 + kw;
            const bool ok = hok && (unsigned)wi < (unsigned)p.W;
            const int wc = min(max(wi, 0), p.W - 1);
            x[r][kw] = ld_chunk(in + ((long long)hc * p.W + wc) * p.ldi);
            msk[r][kw] = ok ? 1.f : 0.f;
        }
    }
    float bias[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) bias[e] = p.bias[c0 + e];
#pragma unroll
    for (int o = 0; o < DW_ROWS; ++o) {
        const int h = h0 + o;
        if (h >= p.H) break;
        float acc[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
                float f[8];
                chunk_to_f(x[o + kh][kw], f);
                const float mk = msk[o + kh][kw];
#pragma unroll
                for (int e = 0; e < 8; ++e) acc[e] = fmaf(wt[kh * 3 + kw][e], f[e] * mk, acc[e]);
            }
        float v8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            float v = acc[e] + bias[e];
            if (p.act == ACT_SILU) v = silu<T>(v);
            v8[e] = v;
        }
        const long long m = ((long long)n * p.H + h) * p.W + w;
        st_chunk(reinterpret_cast<T*>(p.out) + m * p.ldo + c0, f_to_chunk<T>(v8));
    }
}

// 16-bit types: the same per-channel arithmetic with 4 channels per thread (8-byte
// loads and stores). 8 channels hold 72 fp32 weights + 18 input chunks per thread
// (220 VGPRs, 2 waves/SIMD); 4 channels halve both. Bit-identical to dwconv3x3.
template <typename T>
__global__ __launch_bounds__(256) void dwconv3x3_c4(const DwArgs p) {
    static_assert(sizeof(T) == 2, "16-bit path");
    const int cpq = p.C / 4;
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= p.W * cpq) return;
    const int w = t / cpq, cq = t - w * cpq;
    const int h0 = blockIdx.y * DW_ROWS, n = blockIdx.z;
    const int c0 = cq * 4;
    const T* in = reinterpret_cast<const T*>(p.in) + (long long)n * p.H * p.W * p.ldi + c0;
    float wt[9][4];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const float4 a = *reinterpret_cast<const float4*>(p.w + k * p.C + c0);
        wt[k][0] = a.x; wt[k][1] = a.y; wt[k][2] = a.z; wt[k][3] = a.w;
    }
    uint2 x[DW_ROWS + 2][3];
    float msk[DW_ROWS + 2][3];
#pragma unroll
    for (int r = 0; r < DW_ROWS + 2; ++r) {
        const int hi = h0 - 1 + r;
        const bool hok = (unsigned)hi < (unsigned)p.H;
        const int hc = min(max(hi, 0), p.H - 1);
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
            const int wi = w - 1 + kw;
            const bool ok = hok && (unsigned)wi < (unsigned)p.W;
            const int wc = min(max(wi, 0), p.W - 1);
            x[r][kw] = *reinterpret_cast<const uint2*>(in + ((long long)hc * p.W + wc) * p.ldi);
            msk[r][kw] = ok ? 1.f : 0.f;
        }
    }
    float bias[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) bias[e] = p.bias[c0 + e];
#pragma unroll
    for (int o = 0; o < DW_ROWS; ++o) {
        const int h = h0 + o;
        if (h >= p.H) break;
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
                const T* xe = reinterpret_cast<const T*>(&x[o + kh][kw]);
                const float mk = msk[o + kh][kw];
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[e] = fmaf(wt[kh * 3 + kw][e], tof(xe[e]) * mk, acc[e]);
            }
        T o4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float v = acc[e] + bias[e];
            if (p.act == ACT_SILU) v = silu<T>(v);
            o4[e] = fromf<T>(v);
        }
        const long long m = ((long long)n * p.H + h) * p.W + w;
        *reinterpret_cast<uint2*>(reinterpret_cast<T*>(p.out) + m * p.ldo + c0) = *reinterpret_cast<const uint2*>(o4);
    }
}

template <typename T>
int launch_dw_t(const DwArgs& a, hipStream_t s) {
    const int B = a.M / (a.H * a.W);
    if constexpr (sizeof(T) == 2) {   // r01: 91 -> 87 us per v11_n b32 forward
        const dim3 g((unsigned)((a.W * (a.C / 4) + 255) / 256), (unsigned)((a.H + DW_ROWS - 1) / DW_ROWS), (unsigned)B);
        hipLaunchKernelGGL((dwconv3x3_c4<T>), g, dim3(256), 0, s, a);
        return (int)hipGetLastError();
    }
    const dim3 g((unsigned)((a.W * (a.C / 8) + 255) / 256), (unsigned)((a.H + DW_ROWS - 1) / DW_ROWS), (unsigned)B);
    hipLaunchKernelGGL((dwconv3x3<T>), g, dim3(256), 0, s, a);
    return (int)hipGetLastError();
}

}  // namespace

int conv_lds_bytes(int dtype, int BM, int BN, int Kp) {
    const int es = dtype_size(dtype);
    const int main_b = (2 * BM * LDK + 2 * BN * LDK) * es;
    const int epi = BM * (BN + 8) * es;
    return (main_b > epi ? main_b : epi) + (Kp / 8) * 4;
}

// Dense convs of the fp32 handle (the exact-parity mode): conv_gemm on the exact
// f32 MFMA. The 16-bit handles run the conv_mx family (conv_mx.hip).
bool conv_kernel_ok(int dtype, int kern, const ConvArgs& a) {
    (void)a;
    return dtype == F32 && kern == CONV_GEMM;
}

int launch_conv(int dtype, int kern, int BM, int BN, const ConvArgs& a, hipStream_t s) {
    if (!conv_kernel_ok(dtype, kern, a)) return (int)hipErrorInvalidValue;
    return launch_conv_bm<float>(BM, BN, a, s);
}

int launch_first_conv(int dtype, const FirstConvArgs& a, int B, hipStream_t s) {
    switch (dtype) {
        case F32: return launch_first_t<float>(a, B, s);
        case F16: return launch_first_t<_Float16>(a, B, s);
        case BF16: return launch_first_t<__bf16>(a, B, s);
    }
    return (int)hipErrorInvalidValue;
}

bool stem2_ok(int c1, int c2) { return (c1 == 16 && c2 == 32) || (c1 == 32 && c2 == 64); }
void stem2_tiles(int Ho, int Wo, int& ntw, int& nth) {
    ntw = (Wo + S2_TW - 1) / S2_TW;
    nth = (Ho + S2_TH - 1) / S2_TH;
}

int launch_stem2(int dtype, const Stem2Args& a, hipStream_t s) {
    if (!stem2_ok(a.c1, a.c2) || a.W % 8 || a.ldo % 8) return (int)hipErrorInvalidValue;
    switch (dtype) {
        case F16: return a.in_u8 ? launch_stem2_tu<_Float16, uint8_t>(a, s) : launch_stem2_tu<_Float16, _Float16>(a, s);
        case BF16: return a.in_u8 ? launch_stem2_tu<__bf16, uint8_t>(a, s) : launch_stem2_tu<__bf16, __bf16>(a, s);
    }
    return (int)hipErrorInvalidValue;
}

int launch_dwconv(int dtype, const DwArgs& a, hipStream_t s) {
    switch (dtype) {
        case F32: return launch_dw_t<float>(a, s);
        case F16: return launch_dw_t<_Float16>(a, s);
        case BF16: return launch_dw_t<__bf16>(a, s);
    }
    return (int)hipErrorInvalidValue;
}

}  // namespace yh
