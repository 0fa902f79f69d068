// Non-GEMM kernels of the forward:
//   maxpool5    SPPF's three chained 5x5/s1/p2 max-pools (nets/nn.py:83-94)
//   psa_attention  C2PSA attention (nets/nn.py:111-123) with the positional
//               depthwise conv pe(v) fused into its epilogue
//   head_decode DFL + anchors + dist2bbox + sigmoid (nets/nn.py:255-270,
//               222-225; utils/util.py:85-96) into the caller's (B, 4+nc, A)
//   set_io      publishes the caller's x / y pointers for graph replay
#include "common.h"
#include "dtypes.h"

#include <algorithm>
#include <cstdlib>

namespace yh {

namespace {

template <typename T> __device__ __forceinline__ float ex(float x) { return __expf(x); }
template <> __device__ __forceinline__ float ex<float>(float x) { return expf(x); }
// a / b: correctly rounded on the f32 (parity) path, hardware reciprocal on the
// 16-bit paths, whose outputs are rounded to 8 / 11 mantissa bits anyway (same
// policy as silu, dtypes.h)
template <typename T> __device__ __forceinline__ float dv(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }
template <> __device__ __forceinline__ float dv<float>(float a, float b) { return a / b; }

template <typename T>
__global__ __launch_bounds__(256) void maxpool5(const T* src, T* dst, int ldc, int C, int H, int W, int M) {
    // One thread = one pixel x 8 channels; -inf padding == skip out-of-range taps.
    const int cpp = C / 8;
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)M * cpp) return;
    const int m = (int)(idx / cpp), cc = (int)(idx - (long long)m * cpp);
    const int HW = H * W;
    const int n = m / HW, r = m - n * HW;
    const int h = r / W, w = r - h * W;
    const T* base = src + (long long)n * HW * ldc + cc * 8;
    float mx[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) mx[e] = -INFINITY;
    for (int dh = -2; dh <= 2; ++dh) {
        const int hi = h + dh;
        if (hi < 0 || hi >= H) continue;
        for (int dw = -2; dw <= 2; ++dw) {
            const int wi = w + dw;
            if (wi < 0 || wi >= W) continue;
            float f[8];
            chunk_to_f(ld_chunk(base + ((long long)hi * W + wi) * ldc), f);
#pragma unroll
            for (int e = 0; e < 8; ++e) mx[e] = fmaxf(mx[e], f[e]);
        }
    }
    st_chunk(dst + (long long)m * ldc + cc * 8, f_to_chunk<T>(mx));
}

// All three pools in one launch: a workgroup owns CPW consecutive 8-channel chunks of one
// image (CPW * 16 contiguous bytes of every pixel per load and store), staged in LDS once;
// y1 = mp(x), y2 = mp(y1), y3 = mp(y2), each as a 1 x 5 row max into a scratch plane and a
// 5 x 1 column max of that (10 LDS reads per output instead of 25), stored to its concat
// slice. Max is exact and associative, so this is bit-identical to three maxpool5 launches
// (which it replaces whenever three planes fit in LDS).
// running max of 8 channels from -inf (fmaxf: NaN taps are skipped, as in maxpool5)
template <typename T>
__device__ __forceinline__ void sppf_acc(float (&mx)[8], uint4 v) {
    Chunk<T> c;
    c.v[0] = v;
    float f[8];
    chunk_to_f(c, f);
#pragma unroll
    for (int e = 0; e < 8; ++e) mx[e] = fmaxf(mx[e], f[e]);
}
constexpr int SP_LB = 4;
template <typename T>
__global__ __launch_bounds__(256) void sppf_fused(const PoolArgs a, int cpw, int xcd) {
    extern __shared__ __attribute__((aligned(16))) uint4 pln[];
    const int cpp = a.C / 8, ng = cpp / cpw;
    // xcd: an image's chunk workgroups on one XCD (consecutive logical ids), so the four 16-B
    // chunks of a 64-B segment are fetched into one L2 instead of four
    const int L = xcd ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int n = L / ng, cc = (L - n * ng) * cpw;
    const int HW = a.H * a.W, NI = HW * cpw;
    T* img = reinterpret_cast<T*>(a.buf) + (long long)n * HW * a.ldc + cc * 8;
    uint4* p0 = pln;         // pool input / output planes (ping-pong)
    uint4* p1 = pln + NI;
    uint4* rm = pln + 2 * NI;   // row maxima
    // item i = (pixel i / cpw, chunk i % cpw): consecutive threads, consecutive 16 B of a pixel;
    // SP_LB loads in flight per thread before their LDS stores
    for (int i0 = threadIdx.x; i0 < NI; i0 += SP_LB * 256) {
        uint4 v[SP_LB];
#pragma unroll
        for (int u = 0; u < SP_LB; ++u) {
            const int i = min(i0 + u * 256, NI - 1), px = i / cpw, c = i - px * cpw;
            v[u] = *reinterpret_cast<const uint4*>(img + (long long)px * a.ldc + 8 * c);
        }
#pragma unroll
        for (int u = 0; u < SP_LB; ++u)
            if (i0 + u * 256 < NI) p0[i0 + u * 256] = v[u];
    }
    __syncthreads();
    // window taps clamped into the map instead of skipped: a repeated tap leaves a max unchanged,
    // so every item reads a fixed five
    for (int it = 0; it < 3; ++it) {
        const uint4* src = (it & 1) ? p1 : p0;
        uint4* dst = (it & 1) ? p0 : p1;
#pragma unroll 2
        for (int i = threadIdx.x; i < NI; i += 256) {
            const int px = i / cpw, c = i - px * cpw;
            const int h = px / a.W, w = px - h * a.W;
            float mx[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) mx[e] = -INFINITY;
#pragma unroll
            for (int d = -2; d <= 2; ++d) sppf_acc<T>(mx, src[(h * a.W + min(max(w + d, 0), a.W - 1)) * cpw + c]);
            rm[i] = f_to_chunk<T>(mx).v[0];
        }
        __syncthreads();
#pragma unroll 2
        for (int i = threadIdx.x; i < NI; i += 256) {
            const int px = i / cpw, c = i - px * cpw;
            const int h = px / a.W, w = px - h * a.W;
            float mx[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) mx[e] = -INFINITY;
#pragma unroll
            for (int d = -2; d <= 2; ++d) sppf_acc<T>(mx, rm[(min(max(h + d, 0), a.H - 1) * a.W + w) * cpw + c]);
            const uint4 m = f_to_chunk<T>(mx).v[0];
            dst[i] = m;
            *reinterpret_cast<uint4*>(img + (long long)px * a.ldc + (it + 1) * a.C + 8 * c) = m;
        }
        __syncthreads();
    }
}

template <typename T>
int launch_sppf_t(const PoolArgs& a, hipStream_t s) {
    T* b = reinterpret_cast<T*>(a.buf);
    const int M = a.B * a.H * a.W;
    if constexpr (sizeof(T) == 2) {
        // YH_SPPF_FUSED=0 (read per launch): the three maxpool5 launches (the tests compare both)
        const char* ef = getenv("YH_SPPF_FUSED");
        if (3 * a.H * a.W * 16 <= 160 * 1024 && a.C % 8 == 0 && !(ef && atoi(ef) == 0)) {
            static bool attr_set = false;
            if (!attr_set) {
                (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&sppf_fused<T>),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
                attr_set = true;
            }
            // chunks per workgroup: 1 while that gives at most 3 workgroups per CU (v11_n b32: 21.2
            // against 22.8 us for 2; v11_x b16 1280: 81.9 against 90.4), else 2 (v11_s b64: 39.4
            // against 57.7 us for 1; 4 / 8 ran 47 / 86 us at v11_n in round 4); YH_SPPF_CPW
            // overrides. Halved until it divides the channels and the three planes fit the LDS.
            static int ncu = 0;
            if (!ncu) {
                int dev = 0;
                (void)hipGetDevice(&dev);
                if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
                    ncu = 256;
            }
            const char* e = getenv("YH_SPPF_CPW");
            int cpw = e ? std::max(1, atoi(e)) : (a.B * (a.C / 8) <= 3 * ncu ? 1 : 2);
            while (cpw > 1 && ((a.C / 8) % cpw || 3 * a.H * a.W * cpw * 16 > 160 * 1024))
                cpw >>= 1;
            // an image's chunk workgroups on one XCD (YH_SPPF_XCD=0: hardware order). r06, v11_n b32:
            // 20.4 -> 16.3 us, PMC traffic 2.34x -> 0.67x algorithmic; v11_x b16 1280: 83 -> 56 us
            const char* ex = getenv("YH_SPPF_XCD");
            const int xcd = ex ? atoi(ex) : 1;
            hipLaunchKernelGGL((sppf_fused<T>), dim3((unsigned)(a.B * (a.C / 8 / cpw))), dim3(256),
                               3 * a.H * a.W * cpw * (int)sizeof(uint4), s, a, cpw, xcd);
            return (int)hipGetLastError();
        }
    }
    const long long n = (long long)M * (a.C / 8);
    const dim3 g((unsigned)((n + 255) / 256));
    for (int i = 0; i < 3; ++i) {
        hipLaunchKernelGGL((maxpool5<T>), g, dim3(256), 0, s, b + i * a.C, b + (i + 1) * a.C, a.ldc, a.C, a.H, a.W, M);
    }
    return (int)hipGetLastError();
}

constexpr int ATT_Q = 64;   // queries per block (one wave, one query per lane)
constexpr int ATT_KB = 64;  // keys staged per LDS tile
constexpr int DK = 32, DH = 64;

template <typename T>
__global__ __launch_bounds__(ATT_Q) void psa_attention(const AttnArgs p) {
    __shared__ float ks[ATT_KB][DK];
    __shared__ float vs[ATT_KB][DH];
    const int qi = blockIdx.x * ATT_Q + threadIdx.x;
    const int head = blockIdx.y, n = blockIdx.z;
    const int per = 2 * DK + DH;
    const T* base = reinterpret_cast<const T*>(p.qkv) + (long long)n * p.T * p.ldq + head * per;
    const bool live = qi < p.T;

    float q[DK];
    if (live) {
#pragma unroll
        for (int c = 0; c < DK; c += 8) {
            float f[8];
            chunk_to_f(ld_chunk(base + (long long)qi * p.ldq + c), f);
#pragma unroll
            for (int e = 0; e < 8; ++e) q[c + e] = f[e];
        }
    } else {
#pragma unroll
        for (int c = 0; c < DK; ++c) q[c] = 0.f;
    }
    float acc[DH];
#pragma unroll
    for (int d = 0; d < DH; ++d) acc[d] = 0.f;
    float mrun = -INFINITY, lrun = 0.f;

    for (int kb = 0; kb < p.T; kb += ATT_KB) {
        const int nk = min(ATT_KB, p.T - kb);
        __syncthreads();
        if ((int)threadIdx.x < nk) {
            const T* row = base + (long long)(kb + threadIdx.x) * p.ldq;
#pragma unroll
            for (int c = 0; c < DK; c += 8) {
                float f[8];
                chunk_to_f(ld_chunk(row + DK + c), f);
#pragma unroll
                for (int e = 0; e < 8; ++e) ks[threadIdx.x][c + e] = f[e];
            }
#pragma unroll
            for (int c = 0; c < DH; c += 8) {
                float f[8];
                chunk_to_f(ld_chunk(row + 2 * DK + c), f);
#pragma unroll
                for (int e = 0; e < 8; ++e) vs[threadIdx.x][c + e] = f[e];
            }
        }
        __syncthreads();
        float s[ATT_KB];
        float mx = -INFINITY;
#pragma unroll
        for (int j = 0; j < ATT_KB; ++j) {
            float d = 0.f;
#pragma unroll
            for (int c = 0; c < DK; ++c) d = fmaf(q[c], ks[j][c], d);
            d = (j < nk) ? d * p.scale : -INFINITY;
            s[j] = d;
            mx = fmaxf(mx, d);
        }
        const float mnew = fmaxf(mrun, mx);
        const float corr = ex<T>(mrun - mnew);
        lrun *= corr;
#pragma unroll
        for (int d = 0; d < DH; ++d) acc[d] *= corr;
#pragma unroll
        for (int j = 0; j < ATT_KB; ++j) {
            const float pj = (j < nk) ? ex<T>(s[j] - mnew) : 0.f;
            lrun += pj;
#pragma unroll
            for (int d = 0; d < DH; ++d) acc[d] = fmaf(pj, vs[j][d], acc[d]);
        }
        mrun = mnew;
    }
    if (!live) return;

    // epilogue: normalise, add pe(v) = depthwise 3x3 over v (+ bias), store.
    const float inv = 1.0f / lrun;
    const int hq = qi / p.Ws, wq = qi - hq * p.Ws;
    const int C = p.heads * DH;
    float o[DH];
#pragma unroll
    for (int d = 0; d < DH; ++d) o[d] = acc[d] * inv + p.pe_b[head * DH + d];
    for (int kh = 0; kh < 3; ++kh) {
        const int hi = hq - 1 + kh;
        if (hi < 0 || hi >= p.Hs) continue;
        for (int kw = 0; kw < 3; ++kw) {
            const int wi = wq - 1 + kw;
            if (wi < 0 || wi >= p.Ws) continue;
            const T* v = base + (long long)(hi * p.Ws + wi) * p.ldq + 2 * DK;
            const float* wt = p.pe_w + (kh * 3 + kw) * C + head * DH;
#pragma unroll
            for (int c = 0; c < DH; c += 8) {
                float f[8];
                chunk_to_f(ld_chunk(v + c), f);
#pragma unroll
                for (int e = 0; e < 8; ++e) o[c + e] = fmaf(wt[c + e], f[e], o[c + e]);
            }
        }
    }
    T* out = reinterpret_cast<T*>(p.out) + ((long long)n * p.T + qi) * p.ldo + head * DH;
#pragma unroll
    for (int c = 0; c < DH; c += 8) {
        float f[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = o[c + e];
        st_chunk(out + c, f_to_chunk<T>(f));
    }
}

// ---------------------------------------------------------------------------
// 16-bit attention on MFMA. One wave = 16 queries of one (image, head); keys in
// blocks of 16:
//   S^T = K_blk . Q^T        one v_mfma_f32_16x16x32 (dk = 32): A = K rows, B = Q rows,
//                            both straight from the NHWC qkv buffer (16 B per lane);
//                            the accumulator holds S^T[key 4g+r][query li] (g = lane/16).
//   online softmax           per query = per lane column: in-lane max/sum over r plus two
//                            xor-shuffles (16, 32); exact exp, fp32 state.
//   O^T += V^T_blk . P^T     four v_mfma_f32_16x16x16 (dh = 64): B = P^T is exactly the
//                            softmax'd accumulator of the S^T MFMA (no data movement),
//                            A = V^T read from a per-wave LDS copy of V_blk with
//                            ds_read_b64_tr_b16 (hardware transpose).
// pe(v) (the depthwise positional conv, nets/nn.py:122) is added by pe_add below.
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;

template <typename T> struct Mma16;
template <> struct Mma16<__bf16> {
    static __device__ __forceinline__ f32x4 step(s16x4 a, s16x4 b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
    }
};
template <> struct Mma16<_Float16> {
    static __device__ __forceinline__ f32x4 step(s16x4 a, s16x4 b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(f16x4, a), __builtin_bit_cast(f16x4, b), c, 0, 0, 0);
    }
};

__device__ __forceinline__ s16x4 lds_tr16(const void* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef __attribute__((address_space(3))) s16x4* lp;
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(const_cast<void*>(p)));
#else
    (void)p;
    return s16x4{0, 0, 0, 0};
#endif
}

// Reductions over the four 16-lane rows of a wave (lanes l, l ^ 16, l ^ 32, l ^ 48) by gfx950's
// row swaps (v_permlane16_swap / v_permlane32_swap: VALU, no LDS round trip as a ds_bpermute
// shuffle has). Each step combines a lane's value with its xor-16 / xor-32 partner's, the two
// operands in a fixed order; max and + commute, so every lane gets the bits the shuffle form
// (own value op partner's) gives.
__device__ __forceinline__ float rows4_max(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
    const auto t = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(t[0]), __uint_as_float(t[1]));
#else
    return x;
#endif
}
__device__ __forceinline__ float rows4_sum(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    const auto t = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(t[0]) + __uint_as_float(t[1]);
#else
    return x;
#endif
}

// 16 bytes from p when ok, else zeros: a branch around the load. (The `ok ? *p : zero`
// form lets the compiler load through a select of p and a stack zero, a flat load - counted
// in lgkmcnt as well as vmcnt - even when p is global or LDS.)
template <typename P>
__device__ __forceinline__ uint4 ld16_if(bool ok, const P* p) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (ok) v = *reinterpret_cast<const uint4*>(p);
    return v;
}

template <typename T>
__global__ __launch_bounds__(256) void psa_attention_mfma(const AttnArgs p) {
    __shared__ __attribute__((aligned(16))) T vlds[4][16 * DH];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int q0 = (blockIdx.x * 4 + wave) * 16;
    const int head = blockIdx.y, n = blockIdx.z;
    if (q0 >= p.T) return;  // wave-uniform; the kernel has no block-level barrier
    const int g = lane >> 4, li = lane & 15;
    const T* base = reinterpret_cast<const T*>(p.qkv) + (long long)n * p.T * p.ldq + head * (2 * DK + DH);
    const uint4 z4 = make_uint4(0, 0, 0, 0);
    const int q = q0 + li;
    const uint4 qf = ld16_if(q < p.T, base + (long long)q * p.ldq + 8 * g);
    f32x4 o[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) o[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float mrun = -INFINITY, lrun = 0.f;
    T* vl = vlds[wave];
    for (int kb = 0; kb < p.T; kb += 16) {
        const int key = kb + li;
        const uint4 kf = ld16_if(key < p.T, base + (long long)key * p.ldq + DK + 8 * g);
        uint4 vv[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int c = lane + 64 * h, kr = c >> 3, ch = c & 7;
            vv[h] = ld16_if((kb + kr < p.T), base + (long long)(kb + kr) * p.ldq + 2 * DK + ch * 8);
        }
        f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
        Mma<T>::step(s, &kf, &qf);
        float sv[4], mx = -INFINITY;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            sv[r] = (kb + 4 * g + r < p.T) ? s[r] * p.scale : -INFINITY;
            mx = fmaxf(mx, sv[r]);
        }
        mx = rows4_max(mx);
        const float mnew = fmaxf(mrun, mx);
        const float corr = __expf(mrun - mnew);
        float ps = 0.f;
        s16x4 pb;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float pr = __expf(sv[r] - mnew);
            pb[r] = __builtin_bit_cast(short, fromf<T>(pr));
            ps += pr;
        }
        ps = rows4_sum(ps);
        lrun = lrun * corr + ps;
        mrun = mnew;
#pragma unroll
        for (int t = 0; t < 4; ++t) o[t] *= corr;
        // V block -> LDS [16 keys][64 d]
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int c = lane + 64 * h;
            *reinterpret_cast<uint4*>(vl + (c >> 3) * DH + (c & 7) * 8) = vv[h];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const s16x4 a = lds_tr16(vl + (4 * g + (li >> 2)) * DH + 16 * t + 4 * (li & 3));
            o[t] = Mma16<T>::step(a, pb, o[t]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
    }
    if (q >= p.T) return;
    const float inv = 1.0f / lrun;
    T* out = reinterpret_cast<T*>(p.out) + ((long long)n * p.T + q) * p.ldo + head * DH;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        unsigned u[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) u[r] = (unsigned short)__builtin_bit_cast(short, fromf<T>(o[t][r] * inv));
        *reinterpret_cast<uint2*>(out + 16 * t + 4 * g) = make_uint2(u[0] | (u[1] << 16), u[2] | (u[3] << 16));
    }
}

// The same attention with K and V staged in LDS once per workgroup (each wave read
// its (image, head)'s whole K and V from L2, 7x the algorithmic bytes). A workgroup of AT_NW
// waves owns AT_NW 16-query blocks of one (image, head); keys go through LDS in chunks of
// AT_KC (every key's K and V loaded once per workgroup, 16-B loads of whole token rows), and
// every wave runs exactly psa_attention_mfma's per-16-key-block arithmetic in the same key
// order, so the outputs are bit-identical. V rows are padded to 160 B: the 8 keys of a
// ds_read_b64_tr_b16 lane group then hit disjoint banks.
constexpr int AT_NW = 8, AT_KC = 256, AT_VS = DH + 16;   // V row stride (elements)
template <typename T>
__global__ __launch_bounds__(64 * AT_NW) void psa_attention_lds(const AttnArgs p) {
    __shared__ __attribute__((aligned(16))) T klds[AT_KC * DK];
    __shared__ __attribute__((aligned(16))) T vlds[AT_KC * AT_VS];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // 1-D grid, block id = (image, head) pair + pairs x query group: the query groups of one
    // pair are 8 x k ids apart (pair count a multiple of 8), i.e. on one XCD / L2, where their
    // K / V reads meet
    const int np = (int)gridDim.x / ((p.T + 16 * AT_NW - 1) / (16 * AT_NW));
    const int qg = blockIdx.x / np, pair = blockIdx.x - qg * np;
    const int n = pair / p.heads, head = pair - n * p.heads;
    const int q0 = (qg * AT_NW + wave) * 16;
    const int g = lane >> 4, li = lane & 15;
    const T* base = reinterpret_cast<const T*>(p.qkv) + (long long)n * p.T * p.ldq + head * (2 * DK + DH);
    const uint4 z4 = make_uint4(0, 0, 0, 0);
    const int q = q0 + li;
    const bool qwave = q0 < p.T;   // wave-uniform: waves past the last query block only load
    const uint4 qf = ld16_if((qwave && q < p.T), base + (long long)q * p.ldq + 8 * g);
    f32x4 o[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) o[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float mrun = -INFINITY, lrun = 0.f;
    for (int k0 = 0; k0 < p.T; k0 += AT_KC) {
        const int nk = min(AT_KC, p.T - k0);
        __syncthreads();   // the previous chunk is read by every wave
        // token row [k(32) | v(64)] = 12 chunks of 16 B: 4 K chunks, 8 V chunks; the rows of the
        // last 16-key block past the end are zeros (psa_attention_mfma's V of missing keys)
        const int nk16 = (nk + 15) & ~15;
        for (int i = threadIdx.x; i < nk16 * 12; i += 64 * AT_NW) {
            const int r = i / 12, c = i - r * 12;
            const uint4 v = ld16_if(r < nk, base + (long long)(k0 + r) * p.ldq + DK + 8 * c);
            if (c < 4) *reinterpret_cast<uint4*>(klds + r * DK + 8 * c) = v;
            else *reinterpret_cast<uint4*>(vlds + r * AT_VS + 8 * (c - 4)) = v;
        }
        __syncthreads();
        if (!qwave) continue;
        for (int kb = 0; kb < nk; kb += 16) {
            const int key = kb + li;
            const uint4 kf = ld16_if(key < nk, klds + key * DK + 8 * g);
            f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
            Mma<T>::step(s, &kf, &qf);
            float sv[4], mx = -INFINITY;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                sv[r] = (kb + 4 * g + r < nk) ? s[r] * p.scale : -INFINITY;
                mx = fmaxf(mx, sv[r]);
            }
            mx = rows4_max(mx);
            const float mnew = fmaxf(mrun, mx);
            const float corr = __expf(mrun - mnew);
            float ps = 0.f;
            s16x4 pb;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float pr = __expf(sv[r] - mnew);
                pb[r] = __builtin_bit_cast(short, fromf<T>(pr));
                ps += pr;
            }
            ps = rows4_sum(ps);
            lrun = lrun * corr + ps;
            mrun = mnew;
#pragma unroll
            for (int t = 0; t < 4; ++t) o[t] *= corr;
            const int kr = kb + 4 * g + (li >> 2);
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                s16x4 a = lds_tr16(vlds + kr * AT_VS + 16 * t + 4 * (li & 3));
                o[t] = Mma16<T>::step(a, pb, o[t]);
            }
        }
    }
    if (!qwave || q >= p.T) return;
    const float inv = 1.0f / lrun;
    T* out = reinterpret_cast<T*>(p.out) + ((long long)n * p.T + q) * p.ldo + head * DH;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        unsigned u[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) u[r] = (unsigned short)__builtin_bit_cast(short, fromf<T>(o[t][r] * inv));
        *reinterpret_cast<uint2*>(out + 16 * t + 4 * g) = make_uint2(u[0] | (u[1] << 16), u[2] | (u[3] << 16));
    }
}

// One workgroup per (image, head) with the head's whole K and V in LDS (maps of up to
// AF_TMAX tokens: v11 at 640 x 640 has 400): every qkv byte is read once, and pe_add's
// positional term is added in the epilogue from the V already in LDS, so the attention
// output is written once (7x, then 4.96x the algorithmic bytes with the
// chunked kernel and a separate pe_add). Each wave runs psa_attention_mfma's per-16-key-block
// arithmetic for its 16-query blocks in the same key order, rounds the output as that kernel
// stores it, then adds pe_b and the 3 x 3 taps in pe_add's order with pe_add's fmaf chain:
// the result is bit-identical to psa_attention_mfma / psa_attention_lds followed by pe_add.
constexpr int AF_NW = 16, AF_TMAX = 640, AF_LB = 8;
__host__ __device__ inline int af_lds_bytes(int T) {
    const int t16 = (T + 15) & ~15;
    return t16 * (DK + AT_VS) * 2 + 10 * DH * 4;
}
template <typename T, int NW>
__global__ __launch_bounds__(64 * NW) void psa_attention_full(const AttnArgs p, int B) {
    extern __shared__ __attribute__((aligned(16))) char afs[];
    const int t16 = (p.T + 15) & ~15;
    T* klds = reinterpret_cast<T*>(afs);
    T* vlds = klds + t16 * DK;
    float* pew = reinterpret_cast<float*>(vlds + t16 * AT_VS);   // [9][DH] of this head, then pe_b
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // block id = (image, head) pair + pairs x split: the workgroups of one pair are 8 x k ids
    // apart when the pair count is a multiple of 8, i.e. on the same XCD (one L2), so the second
    // one's K / V reads meet the first one's in L2
    const int np = p.heads * B, qs = gridDim.x / np;   // workgroups per (image, head), splitting the queries
    const int split = blockIdx.x / np, pair = blockIdx.x - split * np;
    const int n = pair / p.heads, head = pair - n * p.heads;
    const int g = lane >> 4, li = lane & 15;
    const int C = p.heads * DH;
    const T* base = reinterpret_cast<const T*>(p.qkv) + (long long)n * p.T * p.ldq + head * (2 * DK + DH);
    const uint4 z4 = make_uint4(0, 0, 0, 0);
    // every token row [k(32) | v(64)] once (zeros past the last token: the per-wave kernel's
    // missing keys), the head's positional weights and bias
    // (batches of AF_LB loads in flight per thread, then their LDS stores: a load-store pair per
    // iteration would put one memory round trip per iteration on the prologue's critical path)
    for (int i0 = threadIdx.x; i0 < t16 * 12; i0 += AF_LB * 64 * NW) {
        uint4 v[AF_LB];
#pragma unroll
        for (int u = 0; u < AF_LB; ++u) {
            const int i = i0 + u * 64 * NW, r = i / 12, c = i - r * 12;
            v[u] = ld16_if(i < t16 * 12 && r < p.T, base + (long long)r * p.ldq + DK + 8 * c);
        }
#pragma unroll
        for (int u = 0; u < AF_LB; ++u) {
            const int i = i0 + u * 64 * NW, r = i / 12, c = i - r * 12;
            if (i >= t16 * 12) break;
            if (c < 4) *reinterpret_cast<uint4*>(klds + r * DK + 8 * c) = v[u];
            else *reinterpret_cast<uint4*>(vlds + r * AT_VS + 8 * (c - 4)) = v[u];
        }
    }
    for (int i = threadIdx.x; i < 10 * DH; i += 64 * NW)
        pew[i] = i < 9 * DH ? p.pe_w[(i / DH) * C + head * DH + (i % DH)] : p.pe_b[head * DH + i - 9 * DH];
    __syncthreads();
    const int nqb = (p.T + 15) >> 4;
    for (int qb = split * NW + wave; qb < nqb; qb += qs * NW) {   // wave-uniform
        const int q = qb * 16 + li;
        const uint4 qf = ld16_if(q < p.T, base + (long long)q * p.ldq + 8 * g);
        f32x4 o[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) o[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        float mrun = -INFINITY, lrun = 0.f;
        // K rows past the last token are zeros up to t16; reads past t16 (the block after the
        // last) are clamped: their scores are never used
        const T* kp = klds + 8 * g;
        uint4 kf = *reinterpret_cast<const uint4*>(kp + min(li, t16 - 1) * DK);
        for (int kb = 0; kb < p.T; kb += 16) {
            f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
            Mma<T>::step(s, &kf, &qf);
            // the next block's K fragment and this block's V fragments: LDS reads issued ahead
            // of the softmax chain they do not depend on
            kf = *reinterpret_cast<const uint4*>(kp + min(kb + 16 + li, t16 - 1) * DK);
            const int kr = kb + 4 * g + (li >> 2);
            s16x4 va[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) va[t] = lds_tr16(vlds + kr * AT_VS + 16 * t + 4 * (li & 3));
            float sv[4], mx = -INFINITY;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                sv[r] = (kb + 4 * g + r < p.T) ? s[r] * p.scale : -INFINITY;
                mx = fmaxf(mx, sv[r]);
            }
            mx = rows4_max(mx);
            const float mnew = fmaxf(mrun, mx);
            const float corr = __expf(mrun - mnew);
            float ps = 0.f;
            s16x4 pb;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float pr = __expf(sv[r] - mnew);
                pb[r] = __builtin_bit_cast(short, fromf<T>(pr));
                ps += pr;
            }
            ps = rows4_sum(ps);
            lrun = lrun * corr + ps;
            mrun = mnew;
#pragma unroll
            for (int t = 0; t < 4; ++t) o[t] *= corr;
#pragma unroll
            for (int t = 0; t < 4; ++t) o[t] = Mma16<T>::step(va[t], pb, o[t]);
        }
        if (q >= p.T) continue;
        const float inv = 1.0f / lrun;
        const int hq = q / p.Ws, wq = q - hq * p.Ws;
        T* out = reinterpret_cast<T*>(p.out) + ((long long)n * p.T + q) * p.ldo + head * DH;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            float acc[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[r] = tof(fromf<T>(o[t][r] * inv)) + pew[9 * DH + 16 * t + 4 * g + r];
#pragma unroll
            for (int kh = 0; kh < 3; ++kh) {
                const int hi = hq - 1 + kh;
                if (hi < 0 || hi >= p.Hs) continue;
#pragma unroll
                for (int kw = 0; kw < 3; ++kw) {
                    const int wi = wq - 1 + kw;
                    if (wi < 0 || wi >= p.Ws) continue;
                    const T* vr = vlds + (hi * p.Ws + wi) * AT_VS + 16 * t + 4 * g;
                    const float* wt = pew + (kh * 3 + kw) * DH + 16 * t + 4 * g;
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc[r] = fmaf(wt[r], tof(vr[r]), acc[r]);
                }
            }
            unsigned u[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) u[r] = (unsigned short)__builtin_bit_cast(short, fromf<T>(acc[r]));
            *reinterpret_cast<uint2*>(out + 16 * t + 4 * g) = make_uint2(u[0] | (u[1] << 16), u[2] | (u[3] << 16));
        }
    }
}

// out[:, c] += pe_b[c] + sum_taps pe_w[tap][c] * v[nbr][c]   (c = head*dh + d; v lives in qkv)
template <typename T>
__global__ __launch_bounds__(256) void pe_add(const AttnArgs p, int B) {
    const int C = p.heads * DH, cpp = C / 8;
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)B * p.T * cpp) return;
    const int cc = (int)(idx % cpp);
    const long long tok = idx / cpp;
    const int n = (int)(tok / p.T), t = (int)(tok - (long long)n * p.T);
    const int h = t / p.Ws, w = t - h * p.Ws;
    const int c0 = cc * 8, head = c0 / DH, d0 = c0 - head * DH;
    const T* vbase = reinterpret_cast<const T*>(p.qkv) + (long long)n * p.T * p.ldq + head * (2 * DK + DH) + 2 * DK + d0;
    T* o = reinterpret_cast<T*>(p.out) + tok * p.ldo + c0;
    float acc[8];
    chunk_to_f(ld_chunk(o), acc);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += p.pe_b[c0 + e];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
        const int hi = h - 1 + kh;
        if (hi < 0 || hi >= p.Hs) continue;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
            const int wi = w - 1 + kw;
            if (wi < 0 || wi >= p.Ws) continue;
            float f[8];
            chunk_to_f(ld_chunk(vbase + (long long)(hi * p.Ws + wi) * p.ldq), f);
            const float* wt = p.pe_w + (kh * 3 + kw) * C + c0;
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[e] = fmaf(wt[e], f[e], acc[e]);
        }
    }
    st_chunk(o, f_to_chunk<T>(acc));
}

template <typename T>
int launch_attention_t(const AttnArgs& a, int B, hipStream_t s) {
    if (a.dk != DK || a.dh != DH) return (int)hipErrorInvalidValue;
    if constexpr (sizeof(T) == 2) {
        // YH_ATTN_LDS=0 (read per launch, so per captured graph): the per-wave kernel, which
        // the tests compare bit for bit
        // YH_ATTN_FULL=0 (read per launch): the chunked kernel + pe_add where the full one applies
        const char* ef = getenv("YH_ATTN_FULL");
        if (a.T <= AF_TMAX && a.Ws > 0 && a.Hs * a.Ws == a.T && !(ef && atoi(ef) == 0)) {
            static bool attr = false;
            if (!attr) {
                (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&psa_attention_full<T, 16>),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
                (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&psa_attention_full<T, 8>),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
                attr = true;
            }
            // Every wave runs one 16-query block's serial chain over all key blocks, so the launch
            // lasts about one chain when each wave has at most one block and every workgroup a CU
            // of its own (one fits per CU: the K / V staging takes ~86 KB of LDS). Default: 8-wave
            // workgroups, ceil(blocks / 8) per (image, head), when those fit the CUs in one round
            // (v11_n, batch 32: 256 workgroups, 20 us); else 16-wave ones, two per (image, head)
            // (27-28 us there; at one, 64 workgroups, 39 us). YH_ATTN_NW (8 / 16) and YH_ATTN_QS
            // (workgroups per (image, head)) override.
            static int ncu = 0;
            if (!ncu) {
                int dev = 0;
                (void)hipGetDevice(&dev);
                if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
                    ncu = 256;
            }
            const int nqb = (a.T + 15) >> 4, pairs = a.heads * B, q8 = (nqb + 7) / 8;
            const char* ew = getenv("YH_ATTN_NW");
            const int nw = ew ? (atoi(ew) == 8 ? 8 : AF_NW) : (pairs * q8 <= ncu ? 8 : AF_NW);
            const char* eq = getenv("YH_ATTN_QS");
            const int qs = std::max(1, std::min(eq ? atoi(eq) : (nw == 8 ? q8 : 2), (nqb + nw - 1) / nw));
            if (nw == 8)
                hipLaunchKernelGGL((psa_attention_full<T, 8>), dim3((unsigned)(a.heads * B * qs)), dim3(64 * 8),
                                   af_lds_bytes(a.T), s, a, B);
            else
                hipLaunchKernelGGL((psa_attention_full<T, AF_NW>), dim3((unsigned)(a.heads * B * qs)), dim3(64 * AF_NW),
                                   af_lds_bytes(a.T), s, a, B);
            return (int)hipGetLastError();
        }
        const char* e = getenv("YH_ATTN_LDS");
        if (e && atoi(e) == 0) {
            const dim3 g((a.T + 63) / 64, a.heads, B);
            hipLaunchKernelGGL((psa_attention_mfma<T>), g, dim3(256), 0, s, a);
        } else {
            const unsigned g = (unsigned)((a.T + 16 * AT_NW - 1) / (16 * AT_NW) * a.heads * B);
            hipLaunchKernelGGL((psa_attention_lds<T>), dim3(g), dim3(64 * AT_NW), 0, s, a);
        }
        const long long n = (long long)B * a.T * (a.heads * DH / 8);
        hipLaunchKernelGGL((pe_add<T>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a, B);
    } else {
        const dim3 g((a.T + ATT_Q - 1) / ATT_Q, a.heads, B);
        hipLaunchKernelGGL((psa_attention<T>), g, dim3(ATT_Q), 0, s, a);
    }
    return (int)hipGetLastError();
}

// One workgroup = 256 consecutive anchors of one image. Each thread decodes its
// anchor into a column of an LDS tile [4 + nc][256]; the tile then leaves as
// 16-B (fp32: 32-B) row chunks of the channel-major output instead of 4 + nc
// scalar stores per thread. Needs A % 8 == 0 (aligned row chunks); otherwise
// every value is stored directly (ROWS = false).
template <typename T, bool ROWS>
__global__ __launch_bounds__(256) void head_decode(const DecodeArgs p) {
    extern __shared__ __attribute__((aligned(16))) char dsm[];
    T* tile = reinterpret_cast<T*>(dsm);              // [(4 + nc)][256]
    const int n = blockIdx.y, a0 = p.a_lo + blockIdx.x * 256;
    const int a = a0 + threadIdx.x;
    const bool live = a < p.A;
    const gptr<T> yimg = io_global<T>(p.io[1]) + (long long)n * (4 + p.nc) * p.A;
    auto put = [&](int r, float v) {
        if constexpr (ROWS) tile[r * 256 + threadIdx.x] = fromf<T>(v);
        else if (live) yimg[(long long)r * p.A + a] = fromf<T>(v);
    };
    {
        const int aa = live ? a : p.A - 1;   // dead lanes decode a valid anchor that is never stored
        int l = 0, loc = aa;
        const int l0 = p.H[0] * p.W[0], l1 = p.H[1] * p.W[1];
        if (loc >= l0) { loc -= l0; l = 1; if (loc >= l1) { loc -= l1; l = 2; } }
        const int H = p.H[l], W = p.W[l];
        const int gy = loc / W, gx = loc - gy * W;
        const T* src = reinterpret_cast<const T*>(p.lvl[l]) + ((long long)n * H * W + loc) * p.ldc;

        // DFL: softmax over 16 bins per side, expectation with weights 0..15.
        float dist[4];
#pragma unroll
        for (int sd = 0; sd < 4; ++sd) {
            float v[16];
#pragma unroll
            for (int c = 0; c < 16; c += 8) {
                float f[8];
                chunk_to_f(ld_chunk(src + sd * 16 + c), f);
#pragma unroll
                for (int e = 0; e < 8; ++e) v[c + e] = f[e];
            }
            float mx = v[0];
#pragma unroll
            for (int i = 1; i < 16; ++i) mx = fmaxf(mx, v[i]);
            float sum = 0.f;
#pragma unroll
            for (int i = 0; i < 16; ++i) { v[i] = ex<T>(v[i] - mx); sum += v[i]; }
            float d = 0.f;
#pragma unroll
            for (int i = 0; i < 16; ++i) d = fmaf((float)i, dv<T>(v[i], sum), d);
            dist[sd] = d;
        }
        const float ax = (float)gx + 0.5f, ay = (float)gy + 0.5f, st = p.stride[l];
        const float x1 = ax - dist[0], y1 = ay - dist[1];
        const float x2 = ax + dist[2], y2 = ay + dist[3];
        if (p.box) {
            put(0, (x1 + x2) / 2.0f * st);
            put(1, (y1 + y2) / 2.0f * st);
            put(2, (x2 - x1) * st);
            put(3, (y2 - y1) * st);
        }
        // class scores: all chunks of a batch of DEC_CB loaded before any is used (a
        // load inside the runtime-bound loop would be waited for one round trip at a time)
        constexpr int DEC_CB = 10;
        const T* cls = src + 64;
        const int ncc = (p.nc + 7) / 8;
        for (int c0 = 0; c0 < ncc; c0 += DEC_CB) {
            Chunk<T> v[DEC_CB];
#pragma unroll
            for (int u = 0; u < DEC_CB; ++u) v[u] = ld_chunk(cls + 8 * min(c0 + u, ncc - 1));
#pragma unroll
            for (int u = 0; u < DEC_CB; ++u) {
                const int c = 8 * (c0 + u);
                if (c >= p.nc) break;
                float f[8];
                chunk_to_f(v[u], f);
#pragma unroll
                for (int e = 0; e < 8; ++e)
                    if (c + e < p.nc) put(4 + c + e, dv<T>(1.0f, 1.0f + ex<T>(-f[e])));
            }
        }
    }
    if constexpr (ROWS) {
        __syncthreads();
        const int r0 = p.box ? 0 : 4, rows = 4 + p.nc - r0;
        for (int c = threadIdx.x; c < rows * 32; c += 256) {
            const int r = r0 + (c >> 5), k = c & 31;
            const int a8 = a0 + 8 * k;
            if (a8 >= p.A) continue;
            const T* srow = tile + r * 256 + 8 * k;
            const gptr<T> drow = yimg + (long long)r * p.A + a8;
            if (a8 + 8 <= p.A) {
                st_chunk(drow, ld_chunk(srow));
            } else {
                for (int e = 0; a8 + e < p.A; ++e) drow[e] = srow[e];
            }
        }
    }
}

// 16-bit decode with the head tile staged through LDS. The head tensor's pixels are
// ldc channels apart (box 64 | cls nc | padding), so per-anchor 16-B chunk loads
// touch a new 128-B line per lane and every load instruction gathers 64 lines;
// here the workgroup first copies its 256 anchors' box+cls chunks (CH per anchor)
// as lane-consecutive 16-B pieces (each wave instruction reads whole lines), then
// each thread decodes its anchor from LDS into registers, and the (4 + nc) x 256
// output tile, written over the input tile, leaves as 512-B row runs.
constexpr int DEC_A = 256;
// BOX = false: class rows only (the box rows come from box_dfl), anchors [a_lo, A).
template <typename T, int NCC, bool BOX>   // NCC = nc / 8 class chunks
__global__ __launch_bounds__(256, 2) void head_decode_lds(const DecodeArgs p) {
    extern __shared__ __attribute__((aligned(16))) uint4 dsm4[];
    constexpr int CB = BOX ? 8 : 0;              // box chunks per anchor
    constexpr int CH = CB + NCC, CHP = CH + 1;   // chunks per anchor, padded LDS row
    const int n = blockIdx.y, a0 = p.a_lo + blockIdx.x * DEC_A;
    const int tid = threadIdx.x;
    const int l0 = p.H[0] * p.W[0], l1 = p.H[1] * p.W[1];
    auto src_of = [&](int a) {   // first chunk of anchor a of image n
        int l = 0, loc = a;
        if (loc >= l0) { loc -= l0; l = 1; if (loc >= l1) { loc -= l1; l = 2; } }
        return reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(p.lvl[l]) +
                                              ((long long)n * p.H[l] * p.W[l] + loc) * p.ldc);
    };
    {
        constexpr int BATCH = 6;
        const int total = DEC_A * CH;
        for (int q0 = 0; q0 < total; q0 += 256 * BATCH) {
            uint4 r[BATCH];
            int dst[BATCH];
#pragma unroll
            for (int u = 0; u < BATCH; ++u) {
                const int q = q0 + u * 256 + tid;
                const int ai = q / CH, c = q - ai * CH;
                const int a = min(a0 + ai, p.A - 1);
                dst[u] = q < total ? ai * CHP + c : -1;
                r[u] = q < total ? src_of(a)[c + 8 - CB] : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < BATCH; ++u)
                if (dst[u] >= 0) dsm4[dst[u]] = r[u];
        }
    }
    __syncthreads();
    const int a = a0 + tid;
    const int aa = min(a, p.A - 1);
    int l = 0, loc = aa;
    if (loc >= l0) { loc -= l0; l = 1; if (loc >= l1) { loc -= l1; l = 2; } }
    const int W = p.W[l];
    const int gy = loc / W, gx = loc - gy * W;
    const uint4* row = dsm4 + tid * CHP;
    float dist[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int sd = 0; sd < (BOX ? 4 : 0); ++sd) {
        float v[16];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            Chunk<T> ch;
            ch.v[0] = row[sd * 2 + c];
            float f[8];
            chunk_to_f(ch, f);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[c * 8 + e] = f[e];
        }
        float mx = v[0];
#pragma unroll
        for (int i = 1; i < 16; ++i) mx = fmaxf(mx, v[i]);
        float sum = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) { v[i] = ex<T>(v[i] - mx); sum += v[i]; }
        float d = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) d = fmaf((float)i, dv<T>(v[i], sum), d);
        dist[sd] = d;
    }
    uint4 cls[NCC];
#pragma unroll
    for (int c = 0; c < NCC; ++c) cls[c] = row[CB + c];
    __syncthreads();           // the input tile is dead: the output tile reuses it
    T* tile = reinterpret_cast<T*>(dsm4);   // [(4 + nc)][DEC_A]
    const float ax = (float)gx + 0.5f, ay = (float)gy + 0.5f, st = p.stride[l];
    const float x1 = ax - dist[0], y1 = ay - dist[1];
    const float x2 = ax + dist[2], y2 = ay + dist[3];
    if constexpr (BOX) {
        tile[0 * DEC_A + tid] = fromf<T>((x1 + x2) / 2.0f * st);
        tile[1 * DEC_A + tid] = fromf<T>((y1 + y2) / 2.0f * st);
        tile[2 * DEC_A + tid] = fromf<T>((x2 - x1) * st);
        tile[3 * DEC_A + tid] = fromf<T>((y2 - y1) * st);
    }
#pragma unroll
    for (int c = 0; c < NCC; ++c) {
        Chunk<T> ch;
        ch.v[0] = cls[c];
        float f[8];
        chunk_to_f(ch, f);
#pragma unroll
        for (int e = 0; e < 8; ++e) tile[(4 + 8 * c + e) * DEC_A + tid] = fromf<T>(dv<T>(1.0f, 1.0f + ex<T>(-f[e])));
    }
    __syncthreads();
    const gptr<T> yimg = io_global<T>(p.io[1]) + (long long)n * (4 + p.nc) * p.A;
    constexpr int R0 = BOX ? 0 : 4;
    const int rows = 4 + p.nc - R0;
    for (int c = tid; c < rows * (DEC_A / 8); c += 256) {
        const int r = R0 + c / (DEC_A / 8), k = c - (r - R0) * (DEC_A / 8);
        const int a8 = a0 + 8 * k;
        if (a8 >= p.A) continue;
        const T* srow = tile + r * DEC_A + 8 * k;
        const gptr<T> drow = yimg + (long long)r * p.A + a8;
        if (a8 + 8 <= p.A) st_chunk(drow, ld_chunk(srow));
        else for (int e = 0; a8 + e < p.A; ++e) drow[e] = srow[e];
    }
}

template <typename T>
int launch_decode_t(const DecodeArgs& a, hipStream_t s) {
    if (a.a_lo < 0 || a.a_lo >= a.A || (!a.box && sizeof(T) != 2)) return (int)hipErrorInvalidValue;
    const dim3 g((unsigned)((a.A - a.a_lo + 255) / 256), (unsigned)a.B);
    if constexpr (sizeof(T) == 2) {
        // instantiated for the 80-class heads (COCO); other class counts take head_decode
        constexpr int NCC = 10;
        if (a.nc == 8 * NCC && a.A % 8 == 0 && a.a_lo % 8 == 0 && a.ldc % 8 == 0 && a.ldc >= 64 + a.nc) {
            const int lds_in = DEC_A * ((a.box ? 8 : 0) + NCC + 1) * 16, lds_out = (4 + a.nc) * DEC_A * 2;
            const int lds = lds_in > lds_out ? lds_in : lds_out;
            auto kern = a.box ? &head_decode_lds<T, NCC, true> : &head_decode_lds<T, NCC, false>;
            static bool attr_set[2] = {false, false};
            if (!attr_set[a.box != 0]) {
                (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
                attr_set[a.box != 0] = true;
            }
            hipLaunchKernelGGL(kern, g, dim3(256), lds, s, a);
            return (int)hipGetLastError();
        }
    }
    const int lds = (4 + a.nc) * 256 * (int)sizeof(T);
    if (a.A % 8 == 0 && a.a_lo % 8 == 0 && lds <= 64 * 1024) {
        hipLaunchKernelGGL((head_decode<T, true>), g, dim3(256), lds, s, a);
    } else {
        hipLaunchKernelGGL((head_decode<T, false>), g, dim3(256), 0, s, a);
    }
    return (int)hipGetLastError();
}

__global__ void set_io(void** io, const void* x, void* y) {
    io[0] = const_cast<void*>(x);
    io[1] = y;
}

}  // namespace

int launch_sppf(int dtype, const PoolArgs& a, hipStream_t s) {
    switch (dtype) {
        case F32: return launch_sppf_t<float>(a, s);
        case F16: return launch_sppf_t<_Float16>(a, s);
        case BF16: return launch_sppf_t<__bf16>(a, s);
    }
    return (int)hipErrorInvalidValue;
}

int launch_attention(int dtype, const AttnArgs& a, int B, hipStream_t s) {
    switch (dtype) {
        case F32: return launch_attention_t<float>(a, B, s);
        case F16: return launch_attention_t<_Float16>(a, B, s);
        case BF16: return launch_attention_t<__bf16>(a, B, s);
    }
    return (int)hipErrorInvalidValue;
}

int launch_decode(int dtype, const DecodeArgs& a, hipStream_t s) {
    switch (dtype) {
        case F32: return launch_decode_t<float>(a, s);
        case F16: return launch_decode_t<_Float16>(a, s);
        case BF16: return launch_decode_t<__bf16>(a, s);
    }
    return (int)hipErrorInvalidValue;
}

int launch_set_io(void** io, const void* x, void* y, hipStream_t s) {
    hipLaunchKernelGGL(set_io, dim3(1), dim3(1), 0, s, io, x, y);
    return (int)hipGetLastError();
}

}  // namespace yh
