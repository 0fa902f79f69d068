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

    f32x4 acc[NTL][MT];
#pragma unroll
    for (int i = 0; i < NTL; ++i)
#pragma unroll
        for (int j = 0; j < MT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

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
        const int co = i * 16 + (lane >> 4) * 4;
        float bv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = p.bias[n0 + co + r];
#pragma unroll
        for (int j = 0; j < MT; ++j) {
            const int px = wave * (BM / 4) + j * 16 + fr;
            T* dst = Cs + px * LDE + co;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float v = acc[i][j][r] + bv[r];
                if (p.act == ACT_SILU) v = silu<T>(v);
                dst[r] = fromf<T>(v);
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

template <typename T, int CPT>
__global__ __launch_bounds__(256) void conv_first(const FirstConvArgs p) {
    // Stem: Conv(3 -> Cout, k3, s2, p1) + act (nets/nn.py:161). One thread = one
    // output pixel x CPT couts; the 27 taps are gathered once into registers and
    // the weights ([27][Cout], packed on the host) are wave-uniform scalar loads.
    const float* ws = p.w;
    const float* bs = p.bias;
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    const int co0 = blockIdx.y * CPT;
    if (m >= p.M) return;
    const int HoWo = p.Ho * p.Wo;
    const int n = m / HoWo, r = m - n * HoWo;
    const int ho = r / p.Wo, wo = r - ho * p.Wo;
    const T* x = reinterpret_cast<const T*>(p.io[0]);
    const long long plane = (long long)p.H * p.W;
    const T* xn = x + (long long)n * 3 * plane;
    float xv[27];
#pragma unroll
    for (int ci = 0; ci < 3; ++ci)
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
            const int hi = ho * 2 - 1 + kh;
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
                const int wi = wo * 2 - 1 + kw;
                float v = 0.f;
                if (hi >= 0 && hi < p.H && wi >= 0 && wi < p.W) v = tof(xn[ci * plane + (long long)hi * p.W + wi]);
                xv[ci * 9 + kh * 3 + kw] = v;
            }
        }
    T* out = reinterpret_cast<T*>(p.out) + (long long)m * p.ldo + co0;
#pragma unroll
    for (int c0 = 0; c0 < CPT; c0 += 8) {
        float acc[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll
        for (int k = 0; k < 27; ++k) {
            const float* wk = ws + k * p.Cout + co0 + c0;
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[e] = fmaf(wk[e], xv[k], acc[e]);
        }
        float f[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            float v = acc[e] + bs[co0 + c0 + e];
            if (p.act == ACT_SILU) v = silu<T>(v);
            f[e] = v;
        }
        st_chunk(out + c0, f_to_chunk<T>(f));
    }
}

template <typename T>
int launch_first_t(const FirstConvArgs& a, int B, hipStream_t s) {
    (void)B;
    const dim3 blk(256);
    if (a.Cout % 16 == 0) {
        hipLaunchKernelGGL((conv_first<T, 16>), dim3((a.M + 255) / 256, a.Cout / 16), blk, 0, s, a);
    } else {
        hipLaunchKernelGGL((conv_first<T, 8>), dim3((a.M + 255) / 256, a.Cout / 8), blk, 0, s, a);
    }
    return (int)hipGetLastError();
}

template <typename T>
__global__ __launch_bounds__(256) void dwconv3x3(const DwArgs p) {
    // One thread = one pixel x 8 channels. Stride 1, pad 1 (nn.py:248,250).
    const int cpp = p.C / 8;
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)p.M * cpp) return;
    const int m = (int)(idx / cpp), cc = (int)(idx - (long long)m * cpp);
    const int HW = p.H * p.W;
    const int n = m / HW, r = m - n * HW;
    const int h = r / p.W, w = r - h * p.W;
    const int c0 = cc * 8;
    const T* in = reinterpret_cast<const T*>(p.in) + (long long)n * HW * p.ldi + c0;
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
        const int hi = h - 1 + kh;
        if (hi < 0 || hi >= p.H) continue;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
            const int wi = w - 1 + kw;
            if (wi < 0 || wi >= p.W) continue;
            float f[8];
            chunk_to_f(ld_chunk(in + ((long long)hi * p.W + wi) * p.ldi), f);
            const float* wt = p.w + (kh * 3 + kw) * p.C + c0;
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[e] = fmaf(wt[e], f[e], acc[e]);
        }
    }
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        float v = acc[e] + p.bias[c0 + e];
        if (p.act == ACT_SILU) v = silu<T>(v);
        o[e] = v;
    }
    st_chunk(reinterpret_cast<T*>(p.out) + (long long)m * p.ldo + c0, f_to_chunk<T>(o));
}

template <typename T>
int launch_dw_t(const DwArgs& a, hipStream_t s) {
    const long long n = (long long)a.M * (a.C / 8);
    hipLaunchKernelGGL((dwconv3x3<T>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
    return (int)hipGetLastError();
}

}  // namespace

int conv_lds_bytes(int dtype, int BM, int BN, int Kp) {
    const int es = dtype_size(dtype);
    const int main_b = (2 * BM * LDK + 2 * BN * LDK) * es;
    const int epi = BM * (BN + 8) * es;
    return (main_b > epi ? main_b : epi) + (Kp / 8) * 4;
}

int launch_conv(int dtype, int BM, int BN, const ConvArgs& a, hipStream_t s) {
    switch (dtype) {
        case F32: return launch_conv_bm<float>(BM, BN, a, s);
        case F16: return launch_conv_bm<_Float16>(BM, BN, a, s);
        case BF16: return launch_conv_bm<__bf16>(BM, BN, a, s);
    }
    return (int)hipErrorInvalidValue;
}

int launch_first_conv(int dtype, const FirstConvArgs& a, int B, hipStream_t s) {
    switch (dtype) {
        case F32: return launch_first_t<float>(a, B, s);
        case F16: return launch_first_t<_Float16>(a, B, s);
        case BF16: return launch_first_t<__bf16>(a, B, s);
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
