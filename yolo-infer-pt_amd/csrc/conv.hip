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

// ---------------------------------------------------------------------------
// conv_gemm2: the 16-bit (bf16 / fp16) implicit GEMM.
//   * activation and weight tiles go HBM -> LDS by LDS-DMA (global_load_lds,
//     16 B per lane, no VGPR staging), two 64-deep K stages in flight: the DMA
//     of stage k+1 overlaps the MFMAs of stage k;
//   * LDS rows are 128 B (64 k of one pixel / one cout); the eight 16-B slots of
//     row r are XOR-swizzled by (r & 7) through the per-lane SOURCE address, so
//     the DMA writes linearly and the 16-lane ds_read_b128 fragment reads hit 64
//     distinct banks;
//   * padding taps / channels read a 16-B zero page instead of branching.
constexpr int BK2 = 64;

// 16-byte LDS-DMA: lane i writes lds_base + 16*i (lds_base wave-uniform).
// Device-only builtin: kept out of the host pass so the kernel's host handle is emitted.
__device__ __forceinline__ void glds16(const void* src, char* lds_base) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef __attribute__((address_space(3))) void* lds_void_ptr;
    __builtin_amdgcn_global_load_lds(src, (lds_void_ptr)lds_base, 16, 0, 0);
#else
    (void)src; (void)lds_base;
#endif
}

// The same DMA hidden from hipcc's waitcnt pass (inline asm): the compiler then
// cannot insert the conservative vmcnt(0) in front of every ds_read of the ring
// (it cannot prove the reads miss the in-flight DMA slots). Ordering comes only
// from the kernel's own counted s_waitcnt vmcnt + barrier. M0 is saved/restored
// inside the statement (MI355X guide, section 5.7).
__device__ __forceinline__ void glds16_asm(const void* src, const char* lds_base) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef __attribute__((address_space(3))) const char* lds_cptr;
    const unsigned lds_addr = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_cptr)lds_base);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds_addr) : "memory");
#else
    (void)src; (void)lds_base;
#endif
}

template <int BM, int BN>
struct Smem2 {
    static constexpr int A_BYTES = BM * 128;
    static constexpr int B_BYTES = BN * 128;
    static constexpr int STAGE = A_BYTES + B_BYTES;
    static constexpr int MAIN = 2 * STAGE;
    static constexpr int EPI = BM * (BN + 8) * 2;
    static constexpr int REGION = MAIN > EPI ? MAIN : EPI;
};

template <typename T, int BM, int BN>
__global__ __launch_bounds__(NT_) void conv_gemm2(const ConvArgs p) {
    static_assert(sizeof(T) == 2, "16-bit path");
    static_assert(BM % 64 == 0 && BN % 16 == 0, "tile");
    constexpr int MT = BM / 64;
    constexpr int NTL = BN / 16;
    constexpr int AI = BM / 32;   // A wave-instructions (8 rows x 128 B) per wave per stage
    using SM = Smem2<BM, BN>;

    extern __shared__ __attribute__((aligned(16))) char smem[];
    int* ktab = reinterpret_cast<int*>(smem + SM::REGION);

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int lid = xcd_remap(blockIdx.x, p.gm * p.gn);
    const int mt = lid / p.gn, nt = lid - mt * p.gn;
    const int m0 = mt * BM, n0 = nt * BN;
    for (int i = tid; i < p.Kp / 8; i += NT_) ktab[i] = p.ktab[i];

    const int lrow = lane >> 3;                 // row within a DMA instruction
    const int cidx = (lane & 7) ^ lrow;         // logical 16-B chunk this lane fetches
    const int HoWo = p.Ho * p.Wo;
    int rn[AI], rhb[AI], rwb[AI];
#pragma unroll
    for (int i = 0; i < AI; ++i) {
        const int m = m0 + (wave + 4 * i) * 8 + lrow;
        if (m < p.M) {
            const int n = m / HoWo, r = m - n * HoWo;
            const int ho = r / p.Wo, wo = r - ho * p.Wo;
            rn[i] = n; rhb[i] = ho * p.stride - p.pad; rwb[i] = wo * p.stride - p.pad;
        } else {
            rn[i] = -1; rhb[i] = 0; rwb[i] = 0;
        }
    }
    const T* in0 = reinterpret_cast<const T*>(p.in0);
    const T* in1 = reinterpret_cast<const T*>(p.in1);
    const T* wg = reinterpret_cast<const T*>(p.w);
    const long long bs0 = (long long)p.h0 * p.w0 * p.ldc0;
    const long long bs1 = (long long)p.h1 * p.w1 * p.ldc1;
    __syncthreads();  // ktab

    auto issue = [&](int kt, int buf) {
        char* a = smem + buf * SM::STAGE;
        char* b = a + SM::A_BYTES;
        const int e = ktab[kt * 8 + cidx];
        const int kh = e >> 24, kw = (e >> 16) & 0xff, ci = e & 0xffff;
#pragma unroll
        for (int i = 0; i < AI; ++i) {
            const int hi = rhb[i] + kh, wi = rwb[i] + kw;
            const void* src = p.zero;
            if (ci != 0xffff && rn[i] >= 0 && hi >= 0 && hi < p.Hi && wi >= 0 && wi < p.Wi) {
                if (ci < p.c0)
                    src = in0 + rn[i] * bs0 + ((long long)(hi >> p.up0) * p.w0 + (wi >> p.up0)) * p.ldc0 + ci;
                else
                    src = in1 + rn[i] * bs1 + ((long long)(hi >> p.up1) * p.w1 + (wi >> p.up1)) * p.ldc1 + (ci - p.c0);
            }
            glds16(src, a + (wave + 4 * i) * 1024);
        }
        for (int ii = wave; ii < BN / 8; ii += 4) {
            const T* src = wg + (long long)(n0 + ii * 8 + lrow) * p.Kp + kt * BK2 + cidx * 8;
            glds16(src, b + ii * 1024);
        }
    };

    f32x4 acc[NTL][MT];
#pragma unroll
    for (int i = 0; i < NTL; ++i)
#pragma unroll
        for (int j = 0; j < MT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nkt = p.Kp / BK2;
    const int fr = lane & 15, fq = lane >> 4;
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < nkt; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nkt) issue(kt + 1, cur ^ 1);
        const char* a = smem + cur * SM::STAGE;
        const char* b = a + SM::A_BYTES;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int chunk = kk * 4 + fq;
            uint4 wf[NTL];
#pragma unroll
            for (int i = 0; i < NTL; ++i) {
                const int row = i * 16 + fr;
                wf[i] = *reinterpret_cast<const uint4*>(b + row * 128 + ((chunk ^ (row & 7)) << 4));
            }
#pragma unroll
            for (int j = 0; j < MT; ++j) {
                const int row = wave * (BM / 4) + j * 16 + fr;
                const uint4 xa = *reinterpret_cast<const uint4*>(a + row * 128 + ((chunk ^ (row & 7)) << 4));
#pragma unroll
                for (int i = 0; i < NTL; ++i) Mma<T>::step(acc[i][j], &wf[i], &xa);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    constexpr int LDE = BN + 8;
    T* Cs = reinterpret_cast<T*>(smem);
#pragma unroll
    for (int i = 0; i < NTL; ++i) {
        const int co = i * 16 + fq * 4;
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
    constexpr int CPP = BN / 8;
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

// ---------------------------------------------------------------------------
// conv_stream: persistent, software-pipelined version of conv_gemm2 for the
// 16-bit types. Each workgroup walks a contiguous run of (M-tile, N-tile) pairs
// of its XCD and streams their 64-deep K stages through an NS-slot LDS ring by
// LDS-DMA, keeping NS-1 stages in flight across tile boundaries (the epilogue
// of one tile overlaps the DMA of the next tiles). Every wave issues exactly
// LPS DMA instructions per stage (short B tiles and non-final stages pad with
// zero-page DMAs into a scratch KiB), so one counted `s_waitcnt vmcnt` retires a
// stage; barriers are raw s_barrier so nothing drains the DMA queue. The
// residual (nets/nn.py:49,135-136) is fetched by inline-asm loads issued one
// stage ahead of its use and waited with a counted vmcnt.
template <int BM, int BN, int NS, bool RES>
struct SmemS {
    static constexpr int A_BYTES = BM * 128;
    static constexpr int B_BYTES = BN * 128;
    static constexpr int STAGE = A_BYTES + B_BYTES;
    static constexpr int RING = NS * STAGE;
    static constexpr int DUMMY = RING;                  // 1 KiB sink for padding DMAs
    static constexpr int EPI = DUMMY + 1024;            // [BM][BN+8] output tile
    static constexpr int EPI_BYTES = BM * (BN + 8) * 2;
    static constexpr int TAIL = EPI + EPI_BYTES;        // ktab, bias follow
};

__device__ __forceinline__ void vm_wait(int n) {
    // counted wait; n is wave-uniform and small
    switch (n) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
        case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
        case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
        case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
        case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
        case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
        case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
        case 15: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
        case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
        case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
        case 20: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
        case 24: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
        case 30: asm volatile("s_waitcnt vmcnt(30)" ::: "memory"); break;
        case 32: asm volatile("s_waitcnt vmcnt(32)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}

__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}

template <typename T, int BM, int BN, int NS, bool RES>
__global__ __launch_bounds__(NT_) void conv_stream(const ConvArgs p) {
    static_assert(sizeof(T) == 2, "16-bit path");
    constexpr int MT = BM / 64;
    constexpr int NTL = BN / 16;
    constexpr int AI = BM / 32;                        // A DMA instructions per wave per stage
    constexpr int BI = BN / 32 > 0 ? BN / 32 : 1;      // B DMA instructions per wave per stage
    constexpr int CPP = BN / 8;                        // 16-B chunks per output pixel row
    constexpr int RPW = (BM * CPP) / NT_ > 0 ? (BM * CPP) / NT_ : 1;  // residual chunks per thread
    constexpr int LPS = AI + BI;
    using SM = SmemS<BM, BN, NS, RES>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int* ktab = reinterpret_cast<int*>(smem + SM::TAIL);
    float* bias_s = reinterpret_cast<float*>(smem + SM::TAIL + p.Kp / 8 * 4);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int ntiles = p.gm * p.gn;
    // contiguous tile range per XCD (blocks b and b+8 share an XCD), round-robin inside it
    const int nblk = gridDim.x, xcd = blockIdx.x & 7, q = blockIdx.x >> 3, per_xcd = nblk >> 3;
    const int t_lo = (int)(((long long)ntiles * xcd) / 8), t_hi = (int)(((long long)ntiles * (xcd + 1)) / 8);
    const int my_tiles = t_hi - t_lo > q ? (t_hi - t_lo - q + per_xcd - 1) / per_xcd : 0;
    const int nkt = p.Kp / BK2;
    const int total = my_tiles * nkt;

    for (int i = tid; i < p.Kp / 8; i += NT_) ktab[i] = p.ktab[i];
    for (int i = tid; i < p.gn * BN; i += NT_) bias_s[i] = p.bias[i];
    __syncthreads();   // no DMA in flight yet: the plain barrier is free here
    if (total == 0) return;

    const int lrow = lane >> 3, cidx = (lane & 7) ^ lrow;
    const int HoWo = p.Ho * p.Wo;
    const T* in0 = reinterpret_cast<const T*>(p.in0);
    const T* in1 = reinterpret_cast<const T*>(p.in1);
    const T* wg = reinterpret_cast<const T*>(p.w);
    const long long bs0 = (long long)p.h0 * p.w0 * p.ldc0;
    const long long bs1 = (long long)p.h1 * p.w1 * p.ldc1;

    // issue-side state
    int iss = 0, iss_tile = -1, iss_m0 = 0, iss_n0 = 0;
    int rn[AI], rhb[AI], rwb[AI];
    auto tile_of = [&](int j, int& m0, int& n0) {
        const int t = t_lo + q + j * per_xcd;
        const int mt = t / p.gn, nt = t - mt * p.gn;
        m0 = mt * BM; n0 = nt * BN;
    };
    auto issue = [&]() {
        char* slot = smem + (iss % NS) * SM::STAGE;
        if (iss < total) {
            const int j = iss / nkt, kt = iss - j * nkt;
            if (j != iss_tile) {
                iss_tile = j;
                tile_of(j, iss_m0, iss_n0);
#pragma unroll
                for (int i = 0; i < AI; ++i) {
                    const int m = iss_m0 + (wave + 4 * i) * 8 + lrow;
                    if (m < p.M) {
                        const int n = m / HoWo, r = m - n * HoWo;
                        const int ho = r / p.Wo, wo = r - ho * p.Wo;
                        rn[i] = n; rhb[i] = ho * p.stride - p.pad; rwb[i] = wo * p.stride - p.pad;
                    } else {
                        rn[i] = -1; rhb[i] = 0; rwb[i] = 0;
                    }
                }
            }
            const int e = ktab[kt * 8 + cidx];
            const int kh = e >> 24, kw = (e >> 16) & 0xff, ci = e & 0xffff;
#pragma unroll
            for (int i = 0; i < AI; ++i) {
                const int hi = rhb[i] + kh, wi = rwb[i] + kw;
                const void* src = p.zero;
                if (ci != 0xffff && rn[i] >= 0 && hi >= 0 && hi < p.Hi && wi >= 0 && wi < p.Wi) {
                    if (ci < p.c0)
                        src = in0 + rn[i] * bs0 + ((long long)(hi >> p.up0) * p.w0 + (wi >> p.up0)) * p.ldc0 + ci;
                    else
                        src = in1 + rn[i] * bs1 + ((long long)(hi >> p.up1) * p.w1 + (wi >> p.up1)) * p.ldc1 + (ci - p.c0);
                }
                glds16_asm(src, slot + (wave + 4 * i) * 1024);
            }
#pragma unroll
            for (int i = 0; i < BI; ++i) {
                const int ii = wave + 4 * i;
                if (ii < BN / 8) {
                    const T* src = wg + (long long)(iss_n0 + ii * 8 + lrow) * p.Kp + kt * BK2 + cidx * 8;
                    glds16_asm(src, slot + SM::A_BYTES + ii * 1024);
                } else {
                    glds16_asm(p.zero, smem + SM::DUMMY);
                }
            }
        } else {
            // pipeline tail: keep the per-stage count uniform with zero-page DMAs
#pragma unroll
            for (int i = 0; i < LPS; ++i) glds16_asm(p.zero, smem + SM::DUMMY);
        }
        ++iss;
    };

    f32x4 acc[NTL][MT];
#pragma unroll
    for (int i = 0; i < NTL; ++i)
#pragma unroll
        for (int j = 0; j < MT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int sidx = 0; sidx < NS - 1; ++sidx) issue();

    const int fr = lane & 15, fq = lane >> 4;
    const T* res = reinterpret_cast<const T*>(p.res);
    T* out = reinterpret_cast<T*>(p.out);
    T* Cs = reinterpret_cast<T*>(smem + SM::EPI);
    constexpr int LDE = BN + 8;
    for (int g = 0; g < total; ++g) {
        vm_wait(LPS * (NS - 2));   // this wave's DMAs of stage g have landed
        lds_barrier();             // ... and everyone's; everyone is done with stage g-1
        const int j = g / nkt, kt = g - j * nkt;
        const bool last = kt == nkt - 1;
        int m0, n0;
        tile_of(j, m0, n0);
        static_assert(!RES || RPW <= 4, "residual chunks per thread");
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        u32x4 rv0 = {0u, 0u, 0u, 0u}, rv1 = rv0, rv2 = rv0, rv3 = rv0;
        if constexpr (RES) {
            if (last) {  // residual of this tile, issued before the next stage's DMA
                auto rsrc = [&](int r) {
                    const int c = tid + r * NT_;
                    const int px = c / CPP, cc = c - px * CPP;
                    const int m = min(m0 + px, p.M - 1), co = min(n0 + cc * 8, p.Cout - 8);
                    return res + (long long)m * p.ldr + co;
                };
                asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(rv0) : "v"(rsrc(0)) : "memory");
                if constexpr (RPW > 1) asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(rv1) : "v"(rsrc(1)) : "memory");
                if constexpr (RPW > 2) asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(rv2) : "v"(rsrc(2)) : "memory");
                if constexpr (RPW > 3) asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(rv3) : "v"(rsrc(3)) : "memory");
            }
        }
        issue();   // stage g + NS - 1 into the slot stage g-1 used
        const char* a = smem + (g % NS) * SM::STAGE;
        const char* b = a + SM::A_BYTES;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int chunk = kk * 4 + fq;
            uint4 wf[NTL];
#pragma unroll
            for (int i = 0; i < NTL; ++i) {
                const int row = i * 16 + fr;
                wf[i] = *reinterpret_cast<const uint4*>(b + row * 128 + ((chunk ^ (row & 7)) << 4));
            }
#pragma unroll
            for (int jj = 0; jj < MT; ++jj) {
                const int row = wave * (BM / 4) + jj * 16 + fr;
                const uint4 xa = *reinterpret_cast<const uint4*>(a + row * 128 + ((chunk ^ (row & 7)) << 4));
#pragma unroll
                for (int i = 0; i < NTL; ++i) Mma<T>::step(acc[i][jj], &wf[i], &xa);
            }
        }
        if (last) {
#pragma unroll
            for (int i = 0; i < NTL; ++i) {
                const int co = i * 16 + fq * 4;
#pragma unroll
                for (int jj = 0; jj < MT; ++jj) {
                    const int px = wave * (BM / 4) + jj * 16 + fr;
                    T* dst = Cs + px * LDE + co;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        float v = acc[i][jj][r] + bias_s[n0 + co + r];
                        if (p.act == ACT_SILU) v = silu<T>(v);
                        dst[r] = fromf<T>(v);
                    }
                    acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
                }
            }
            lds_barrier();
            if constexpr (RES) {
                // the residual loads are older than the LPS DMAs just issued: vmcnt(LPS)
                static_assert(LPS >= 3 && LPS <= 12, "residual wait count");
#define YH_RWAIT(N) asm volatile("s_waitcnt vmcnt(" #N ")" : "+v"(rv0), "+v"(rv1), "+v"(rv2), "+v"(rv3) :: "memory")
                if constexpr (LPS == 3) YH_RWAIT(3);
                else if constexpr (LPS == 4) YH_RWAIT(4);
                else if constexpr (LPS == 5) YH_RWAIT(5);
                else if constexpr (LPS == 6) YH_RWAIT(6);
                else if constexpr (LPS == 8) YH_RWAIT(8);
                else if constexpr (LPS == 9) YH_RWAIT(9);
                else if constexpr (LPS == 10) YH_RWAIT(10);
                else YH_RWAIT(12);
#undef YH_RWAIT
            }
#pragma unroll
            for (int r = 0; r < RPW; ++r) {
                const int c = tid + r * NT_;
                if (c >= BM * CPP) break;
                const int px = c / CPP, cc = c - px * CPP;
                const int m = m0 + px, co = n0 + cc * 8;
                Chunk<T> v = ld_chunk(Cs + px * LDE + cc * 8);
                if constexpr (RES) {
                    float f[8], gg[8];
                    Chunk<T> rc;
                    rc.v[0] = __builtin_bit_cast(uint4, r == 0 ? rv0 : r == 1 ? rv1 : r == 2 ? rv2 : rv3);
                    chunk_to_f(v, f);
                    chunk_to_f(rc, gg);
#pragma unroll
                    for (int e = 0; e < 8; ++e) f[e] += gg[e];
                    v = f_to_chunk<T>(f);
                }
                if (m < p.M && co < p.Cout) st_chunk(out + (long long)m * p.ldo + co, v);
            }
        }
    }
    vm_wait(0);
}

template <typename T, int BM, int BN, int NS>
int launch_stream_t(const ConvArgs& a, hipStream_t s, int blocks_per_cu) {
    constexpr bool RES_OK = (BM * (BN / 8)) / NT_ <= 4;
    const int lds_res = SmemS<BM, BN, NS, true>::TAIL + a.Kp / 8 * 4 + a.gn * BN * 4;
    static bool attr[2] = {false, false};
    const bool res = a.res != nullptr;
    if (res && !RES_OK) return (int)hipErrorInvalidValue;
    const int ntiles = a.gm * a.gn;
    int grid = 256 * blocks_per_cu;
    if (grid > ntiles) grid = ((ntiles + 7) / 8) * 8;
    if constexpr (RES_OK) {
        if (res) {
            if (!attr[1]) {
                (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_stream<T, BM, BN, NS, true>),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
                attr[1] = true;
            }
            hipLaunchKernelGGL((conv_stream<T, BM, BN, NS, true>), dim3(grid), dim3(NT_), lds_res, s, a);
            return (int)hipGetLastError();
        }
    }
    if (!attr[0]) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_stream<T, BM, BN, NS, false>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr[0] = true;
    }
    hipLaunchKernelGGL((conv_stream<T, BM, BN, NS, false>), dim3(grid), dim3(NT_), lds_res, s, a);
    return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// conv_direct: barrier-free implicit GEMM for the 16-bit types.
//
// A workgroup (8 waves) keeps one Cout slice of the packed weights resident in
// LDS for its whole life and its waves stream pixel tiles independently: each
// wave owns 16*MT output pixels x all BN couts of the slice, loads its pixel
// operand (16 B of 8 channels per lane = one MFMA B-fragment) straight from
// global memory into VGPRs D k-steps ahead of use, reads the weight fragments
// from LDS and runs 16x16x32 MFMAs. There is no LDS staging of activations and
// no barrier after the one-time weight fill, so latency is hidden by the
// per-wave prefetch depth and by occupancy (4 waves/SIMD), not by block-wide
// pipelining. The 3x3 halo re-reads (9 taps of each input pixel) are served by
// L1/L2; HBM sees the input roughly once per Cout slice.
//
// Weight rows are permuted on the LDS fill so that the MFMA accumulator layout
// (lane = pixel, 4 consecutive rows per lane quarter) lands 4*NTL *contiguous*
// output channels in every lane: MFMA row (i, 4q + r) <- cout q*4*NTL + 4i + r.
// The epilogue then stores straight from registers in 16-B chunks (bias, SiLU,
// residual add in fp32), no LDS transpose.
constexpr int DIRECT_WAVES = 8;
constexpr int DIRECT_NT = DIRECT_WAVES * 64;
constexpr int DIRECT_LDS_CAP = 80 * 1024;   // weight slice + ktab per block: 2 blocks per CU

// KM: 0 = 1x1 stride 1 (two segments, nearest-up allowed); 1 = general kxk over
// the k-table (one plain segment); 2 = 3x3 with Cin % 32 == 0, walked tap-major so
// the tap's pixel address is computed once per tap, not once per 32-channel step.
template <typename T, int NTL, int MT, int KM, int D>
__global__ __launch_bounds__(DIRECT_NT, 2) void conv_direct(const ConvArgs p) {
    constexpr bool K3 = KM != 0;
    static_assert(sizeof(T) == 2, "16-bit path");
    constexpr int BN = NTL * 16;   // D = k-steps in flight per wave
    constexpr int RUN = 4 * NTL;  // contiguous couts per lane
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int ldw = p.Kp * 2 + 16;                       // padded LDS row: conflict-free b128 reads
    int* ktab = reinterpret_cast<int*>(smem + BN * ldw);
    const int S = p.gn, PT = p.gm;
    const int slice = blockIdx.x % S, bs = blockIdx.x / S, nbs = gridDim.x / S;
    const int n0 = slice * BN;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int kc8 = p.Kp / 8;
    {
        const T* wg = reinterpret_cast<const T*>(p.w);
        constexpr int FB = 8;   // loads in flight per thread during the fill
        for (int c0 = tid; c0 < BN * kc8; c0 += DIRECT_NT * FB) {
            // straight-line: out-of-range slots redo the last chunk (same value, same place)
            uint4 v[FB];
            int dst[FB];
#pragma unroll
            for (int u = 0; u < FB; ++u) {
                const int c = min(c0 + u * DIRECT_NT, BN * kc8 - 1);
                const int R = c / kc8, kc = c - R * kc8;
                const int i = R >> 4, q = (R >> 2) & 3, r = R & 3;
                const int co = n0 + q * RUN + 4 * i + r;
                v[u] = *reinterpret_cast<const uint4*>(wg + (long long)co * p.Kp + kc * 8);
                dst[u] = R * ldw + kc * 16;
            }
#pragma unroll
            for (int u = 0; u < FB; ++u) *reinterpret_cast<uint4*>(smem + dst[u]) = v[u];
        }
        if constexpr (KM == 1)
            for (int c = tid; c < kc8 + 8 * D; c += DIRECT_NT) ktab[c] = c < kc8 ? p.ktab[c] : 0xffff;
    }
    __syncthreads();

    const int t_lo = (int)((long long)PT * bs / nbs), t_hi = (int)((long long)PT * (bs + 1) / nbs);
    const int p16 = lane & 15, q = lane >> 4;
    const int nks = (p.K + 31) / 32;
    const int nkp = (nks + D - 1) / D * D;
    const int kmax = p.Kp / 32 - 1;
    const int HoWo = p.Ho * p.Wo;
    const T* in0 = reinterpret_cast<const T*>(p.in0);
    const T* in1 = reinterpret_cast<const T*>(p.in1);
    const T* zero = reinterpret_cast<const T*>(p.zero);
    const long long bs0 = (long long)p.h0 * p.w0 * p.ldc0;
    const long long bs1 = (long long)p.h1 * p.w1 * p.ldc1;
    const int co = n0 + q * RUN;   // this lane's first output channel
    const char* wrow = smem + p16 * ldw + q * 16;

    for (int t = t_lo + wave; t < t_hi; t += DIRECT_WAVES) {
        const int m0 = t * 16 * MT;
        // per-pixel loader state
        int rn[MT], rhb[MT], rwb[MT];
        const T* pb0[MT];
        const T* pb1[MT];
#pragma unroll
        for (int j = 0; j < MT; ++j) {
            const int m = m0 + j * 16 + p16;
            const int mm = m < p.M ? m : p.M - 1;
            const int n = mm / HoWo, rr = mm - n * HoWo;
            const int ho = rr / p.Wo, wo = rr - ho * p.Wo;
            rn[j] = m < p.M ? n : -1;
            rhb[j] = m < p.M ? ho * p.stride - p.pad : -(1 << 20);   // out-of-range rows read the zero page
            rwb[j] = wo * p.stride - p.pad;
            if constexpr (K3) {
                pb0[j] = in0 + n * bs0;
                pb1[j] = nullptr;
            } else {
                pb0[j] = in0 + n * bs0 + ((long long)(ho >> p.up0) * p.w0 + (wo >> p.up0)) * p.ldc0;
                pb1[j] = in1 + n * bs1 + ((long long)(ho >> p.up1) * p.w1 + (wo >> p.up1)) * p.ldc1 - p.c0;
            }
        }
        // tap-major walk (KM == 2): wave-uniform (tap, 32-channel block) counters
        int l_tap = 0, l_cb = 0;
        const int ncb = p.Cin >> 5;
        const T* tp[MT];
        bool tv[MT];
        auto set_tap = [&]() {
            const int kh = l_tap / 3, kw = l_tap - kh * 3;
#pragma unroll
            for (int j = 0; j < MT; ++j) {
                const int hi = rhb[j] + kh, wi = rwb[j] + kw;
                tv[j] = (l_tap < 9) & ((unsigned)hi < (unsigned)p.Hi) & ((unsigned)wi < (unsigned)p.Wi);
                tp[j] = pb0[j] + ((long long)hi * p.w0 + wi) * p.ldc0 + q * 8;
            }
        };
        if constexpr (KM == 2) set_tap();
        // Branch-free address selection (v_cndmask): a divergent branch here makes
        // hipcc drain the loads in flight at the join.
        auto load = [&](int ks, uint4 (&dst)[MT]) {
            if constexpr (KM == 2) {
#pragma unroll
                for (int j = 0; j < MT; ++j)
                    dst[j] = *reinterpret_cast<const uint4*>(tv[j] ? tp[j] + l_cb * 32 : zero);
                if (++l_cb == ncb) {   // uniform: next tap
                    l_cb = 0;
                    ++l_tap;
                    set_tap();
                }
            } else if constexpr (KM == 1) {
                const int e = ktab[ks * 4 + q];   // padded with 0xffff past K
                const int kh = e >> 24, kw = (e >> 16) & 0xff, ci = e & 0xffff;
#pragma unroll
                for (int j = 0; j < MT; ++j) {
                    const int hi = rhb[j] + kh, wi = rwb[j] + kw;
                    const bool ok = (ci != 0xffff) & ((unsigned)hi < (unsigned)p.Hi) & ((unsigned)wi < (unsigned)p.Wi);
                    const T* src = pb0[j] + ((long long)hi * p.w0 + wi) * p.ldc0 + ci;
                    dst[j] = *reinterpret_cast<const uint4*>(ok ? src : zero);
                }
            } else {
                const int ci = ks * 32 + q * 8;
                const bool in_k = ci < p.Cin, seg0 = ci < p.c0;
#pragma unroll
                for (int j = 0; j < MT; ++j) {
                    const T* src = (seg0 ? pb0[j] : pb1[j]) + ci;
                    dst[j] = *reinterpret_cast<const uint4*>((in_k && rn[j] >= 0) ? src : zero);
                }
            }
        };

        f32x4 acc[NTL][MT];
#pragma unroll
        for (int i = 0; i < NTL; ++i)
#pragma unroll
            for (int j = 0; j < MT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        uint4 buf[D][MT];
#pragma unroll
        for (int d = 0; d < D; ++d) load(d, buf[d]);
        // The step count is padded to a multiple of D so the unrolled body has no
        // branches (a skipped step would make hipcc drain the loads to avoid
        // overwriting registers with loads still in flight). Padded steps read
        // the zero page against a clamped (finite) weight row: they add 0.
        for (int ks = 0; ks < nkp; ks += D) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const int kwr = min(ks + d, kmax);
                uint4 wf[NTL];
#pragma unroll
                for (int i = 0; i < NTL; ++i)
                    wf[i] = *reinterpret_cast<const uint4*>(wrow + i * 16 * ldw + kwr * 64);
#pragma unroll
                for (int j = 0; j < MT; ++j)
#pragma unroll
                    for (int i = 0; i < NTL; ++i) Mma<T>::step(acc[i][j], &wf[i], &buf[d][j]);
                load(ks + d + D, buf[d]);
            }
        }

        // epilogue: lane holds couts [co, co + RUN) of pixels m0 + j*16 + p16
        if (co < p.Cout) {
            float bv[RUN];
#pragma unroll
            for (int e = 0; e < RUN; ++e) bv[e] = p.bias[co + e];
            const T* res = reinterpret_cast<const T*>(p.res);
            T* out = reinterpret_cast<T*>(p.out);
#pragma unroll
            for (int j = 0; j < MT; ++j) {
                const int m = m0 + j * 16 + p16;
                if (m >= p.M) continue;
                float v[RUN];
#pragma unroll
                for (int e = 0; e < RUN; ++e) {
                    float x = acc[e >> 2][j][e & 3] + bv[e];
                    if (p.act == ACT_SILU) x = silu<T>(x);
                    v[e] = x;
                }
                if constexpr (RUN % 8 == 0) {
#pragma unroll
                    for (int c8 = 0; c8 < RUN / 8; ++c8) {
                        if (co + c8 * 8 >= p.Cout) break;
                        float f[8];
#pragma unroll
                        for (int e = 0; e < 8; ++e) f[e] = fromf_round<T>(v[c8 * 8 + e]);
                        if (res) {
                            float g[8];
                            chunk_to_f(ld_chunk(res + (long long)m * p.ldr + co + c8 * 8), g);
#pragma unroll
                            for (int e = 0; e < 8; ++e) f[e] += g[e];
                        }
                        st_chunk(out + (long long)m * p.ldo + co + c8 * 8, f_to_chunk<T>(f));
                    }
                } else {
                    // RUN = 4 or 20 (NTL 1 / 5): 8-byte stores, 8-byte aligned (co = n0 + q * RUN)
#pragma unroll
                    for (int c4 = 0; c4 < RUN / 4; ++c4) {
                        if (co + c4 * 4 >= p.Cout) break;
                        T o[4];
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            float x = fromf_round<T>(v[c4 * 4 + e]);
                            if (res) x += tof(res[(long long)m * p.ldr + co + c4 * 4 + e]);
                            o[e] = fromf<T>(x);
                        }
                        *reinterpret_cast<uint2*>(out + (long long)m * p.ldo + co + c4 * 4) =
                            *reinterpret_cast<const uint2*>(o);
                    }
                }
            }
        }
    }
}

template <typename T, int NTL, int MT, int KM, int D>
int launch_direct_t(const ConvArgs& a, int lds, int S, hipStream_t s) {
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_direct<T, NTL, MT, KM, D>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    ConvArgs b = a;
    b.gn = S;
    b.gm = (a.M + 16 * MT - 1) / (16 * MT);
    // 2 blocks per CU, but never fewer than one pixel tile per wave
    int nbs = (512 + S - 1) / S;
    const int need = (b.gm + DIRECT_WAVES - 1) / DIRECT_WAVES;
    if (nbs > need) nbs = need;
    if (nbs < 1) nbs = 1;
    hipLaunchKernelGGL((conv_direct<T, NTL, MT, KM, D>), dim3(nbs * S), dim3(DIRECT_NT), lds, s, b);
    return (int)hipGetLastError();
}

// conv_direct plan: Cout slice width (16 * ntl) and LDS bytes; false when the
// layer does not fit the kernel (3x3 over a concat / upsampled input, or a
// weight slice beyond the LDS budget even at 16 couts).
bool direct_plan(const ConvArgs& a, int* ntl_out, int* lds_out) {
    const bool k1 = a.KH == 1 && a.KW == 1 && a.stride == 1 && a.pad == 0;
    if (!k1 && (a.c1 != 0 || a.up0 != 0)) return false;
    // 80 couts (the v11_n class branch, c3 = 80) as one 5-tile slice: two 64-wide slices
    // would read the input twice and spend 3/8 of their MFMAs on padding
    int ntl = a.Cout <= 16 ? 1 : a.Cout <= 32 ? 2 : a.Cout == 80 ? 5 : 4;
    auto lds_of = [&](int n) { return n * 16 * (a.Kp * 2 + 16) + (a.Kp / 8 + 32) * 4; };
    if (ntl == 5 && lds_of(5) > DIRECT_LDS_CAP) ntl = 4;
    while (ntl > 1 && lds_of(ntl) > DIRECT_LDS_CAP) ntl >>= 1;
    if (lds_of(ntl) > DIRECT_LDS_CAP) return false;
    if (ntl_out) *ntl_out = ntl;
    if (lds_out) *lds_out = lds_of(ntl);
    return true;
}

template <typename T>
int launch_direct(const ConvArgs& a, hipStream_t s) {
    int ntl = 0, lds = 0;
    if (!direct_plan(a, &ntl, &lds)) return (int)hipErrorInvalidValue;
    const bool k1 = a.KH == 1 && a.KW == 1 && a.stride == 1 && a.pad == 0;
    const int S = (a.Cout + ntl * 16 - 1) / (ntl * 16);
    const bool short_k = (a.K + 31) / 32 <= 2;
    const bool tap_major = a.KH == 3 && a.KW == 3 && a.Cin % 32 == 0;
#define YH_DIR(n)                                                                          \
    if (k1) return short_k ? launch_direct_t<T, n, 2, 0, 2>(a, lds, S, s)                  \
                           : launch_direct_t<T, n, 2, 0, 4>(a, lds, S, s);                 \
    if (tap_major) return launch_direct_t<T, n, 2, 2, 4>(a, lds, S, s);                    \
    return short_k ? launch_direct_t<T, n, 2, 1, 2>(a, lds, S, s)                          \
                   : launch_direct_t<T, n, 2, 1, 4>(a, lds, S, s);
    switch (ntl) {
        case 1: YH_DIR(1)
        case 2: YH_DIR(2)
        case 5:   // 1x1: 2 k-steps in flight keeps 4 waves/SIMD (D = 4 needs 132 VGPRs)
            if (k1) return launch_direct_t<T, 5, 2, 0, 2>(a, lds, S, s);
            YH_DIR(5)
        default: YH_DIR(4)
    }
#undef YH_DIR
}

// ---------------------------------------------------------------------------
// conv_tiny: 3x3 stride-1 convs with few input channels (Cin = 8 / 16 / 32, e.g.
// the 160x160 and 80x80 C3k2 bottlenecks 16->8->16 and 32->16->32). A
// workgroup owns TH full output rows of one image and one cout slice: the weight
// slice and the input rows (+1 halo row / column, zero border) are staged in LDS
// once with all loads in flight. The k-table is the same for every pixel, so each
// lane turns its k-steps into LDS offsets once (padding steps point at a zero
// chunk); a job's fragment reads are then independent ds_read_b128s from one base.
// K order and epilogue are conv_direct's -> bit-identical outputs.
struct TinyPlan {
    int TH, PC, pst, nrb, ntl, slices, B, lds, zoff;
};
constexpr int TINY_NT = 256;
constexpr int TINY_BUDGET = 64 * 1024;   // two or more workgroups per CU
constexpr int TINY_KS = 10;              // k-steps: Kp <= 320 (Cin <= 32)

template <typename T, int NTL>
__global__ __launch_bounds__(TINY_NT) void conv_tiny(const ConvArgs p, const TinyPlan g) {
    static_assert(sizeof(T) == 2, "16-bit path");
    constexpr int BN = NTL * 16, RUN = 4 * NTL, MT = 2;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int ldw = p.Kp * 2 + 16;
    const int kc8 = p.Kp / 8;
    char* wl = smem;                     // BN rows x ldw
    char* pl = smem + BN * ldw;          // patch, then a 16-B zero chunk at g.zoff
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int p16 = lane & 15, q = lane >> 4;
    const int bid = blockIdx.x;
    const int slice = bid % g.slices, rem = bid / g.slices;
    const int n = rem / g.nrb, rb = rem - n * g.nrb;
    const int ho0 = rb * g.TH, th = min(g.TH, p.Ho - ho0);
    const int n0 = slice * BN;
    const int cpp = p.c0 / 8;   // 16-B chunks per input pixel
    {   // weights (rows permuted as conv_direct) and input rows: loads first, then stores
        const T* wg = reinterpret_cast<const T*>(p.w);
        constexpr int FB = 8;
        const int wtot = BN * kc8;
        for (int c0 = tid; c0 < wtot; c0 += TINY_NT * FB) {
            uint4 v[FB];
            int dst[FB];
#pragma unroll
            for (int u = 0; u < FB; ++u) {
                const int c = min(c0 + u * TINY_NT, wtot - 1);
                const int R = c / kc8, kc = c - R * kc8;
                const int i = R >> 4, qq = (R >> 2) & 3, r = R & 3;
                const int co = n0 + qq * RUN + 4 * i + r;
                v[u] = *reinterpret_cast<const uint4*>(wg + (long long)co * p.Kp + kc * 8);
                dst[u] = R * ldw + kc * 16;
            }
#pragma unroll
            for (int u = 0; u < FB; ++u) *reinterpret_cast<uint4*>(wl + dst[u]) = v[u];
        }
        const T* in0 = reinterpret_cast<const T*>(p.in0) + (long long)n * p.h0 * p.w0 * p.ldc0;
        const int hi0 = ho0 - 1;
        const int ptot = (th + 2) * g.PC * cpp;
        for (int c0 = tid; c0 < ptot; c0 += TINY_NT * FB) {
            uint4 v[FB];
            int dst[FB];
            bool ok[FB];
#pragma unroll
            for (int u = 0; u < FB; ++u) {
                const int cc = min(c0 + u * TINY_NT, ptot - 1);
                const int px = cc / cpp, ch = cc - px * cpp;
                const int pr = px / g.PC, pc = px - pr * g.PC;
                const int hi = hi0 + pr, wi = pc - 1;
                ok[u] = (unsigned)hi < (unsigned)p.Hi && (unsigned)wi < (unsigned)p.Wi;
                const int hc = min(max(hi, 0), p.Hi - 1), wc = min(max(wi, 0), p.Wi - 1);
                v[u] = *reinterpret_cast<const uint4*>(in0 + ((long long)hc * p.w0 + wc) * p.ldc0 + ch * 8);
                dst[u] = px * g.pst + ch * 16;
            }
#pragma unroll
            for (int u = 0; u < FB; ++u)
                *reinterpret_cast<uint4*>(pl + dst[u]) = ok[u] ? v[u] : make_uint4(0, 0, 0, 0);
        }
        if (tid == 0) *reinterpret_cast<uint4*>(pl + g.zoff) = make_uint4(0, 0, 0, 0);
    }
    // this lane's k-steps as patch offsets relative to the pixel's (r, c) tap-(0,0) base;
    // padding steps read the zero chunk (an absolute offset: base is subtracted back)
    const int nks = (p.K + 31) / 32;
    int toff[TINY_KS];
    bool tpad[TINY_KS];
#pragma unroll
    for (int k = 0; k < TINY_KS; ++k) {
        const int e = k < nks ? p.ktab[k * 4 + q] : 0xffff;
        const int kh = e >> 24, kw = (e >> 16) & 0xff, ci = e & 0xffff;
        tpad[k] = ci == 0xffff;
        toff[k] = tpad[k] ? 0 : (kh * g.PC + kw) * g.pst + ci * 2;
    }
    __syncthreads();
    const int npx = th * p.Wo;
    const int njob = (npx + 16 * MT - 1) / (16 * MT);
    const int co = n0 + q * RUN;
    const char* wrow = wl + p16 * ldw + q * 16;
    float bv[RUN];
#pragma unroll
    for (int e = 0; e < RUN; ++e) bv[e] = co + e < p.Cout ? p.bias[co + e] : 0.f;
    const T* res = reinterpret_cast<const T*>(p.res);
    T* out = reinterpret_cast<T*>(p.out);
    for (int job = wave; job < njob; job += TINY_NT / 64) {
        int mg[MT];
        const char* base[MT];
#pragma unroll
        for (int j = 0; j < MT; ++j) {
            const int idx = (job * MT + j) * 16 + p16;
            const bool v = idx < npx;
            const int r = v ? idx / p.Wo : 0, c = v ? idx - r * p.Wo : 0;
            base[j] = pl + (r * g.PC + c) * g.pst;
            mg[j] = v ? (n * p.Ho + ho0 + r) * p.Wo + c : -1;
        }
        f32x4 acc[NTL][MT];
#pragma unroll
        for (int i = 0; i < NTL; ++i)
#pragma unroll
            for (int j = 0; j < MT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        uint4 xa[TINY_KS][MT];
#pragma unroll
        for (int k = 0; k < TINY_KS; ++k)
#pragma unroll
            for (int j = 0; j < MT; ++j)
                xa[k][j] = *reinterpret_cast<const uint4*>(tpad[k] ? pl + g.zoff : base[j] + toff[k]);
        // all TINY_KS steps, branch-free: steps past K read the zero chunk against a
        // clamped (finite) weight step and add exactly 0
        const int kmax = p.Kp / 32 - 1;
#pragma unroll
        for (int k = 0; k < TINY_KS; ++k) {
            uint4 wf[NTL];
#pragma unroll
            for (int i = 0; i < NTL; ++i)
                wf[i] = *reinterpret_cast<const uint4*>(wrow + i * 16 * ldw + min(k, kmax) * 64);
#pragma unroll
            for (int j = 0; j < MT; ++j)
#pragma unroll
                for (int i = 0; i < NTL; ++i) Mma<T>::step(acc[i][j], &wf[i], &xa[k][j]);
        }
        if (co >= p.Cout) continue;
#pragma unroll
        for (int j = 0; j < MT; ++j) {
            const int m = mg[j];
            if (m < 0) continue;
            float vv[RUN];
#pragma unroll
            for (int e = 0; e < RUN; ++e) {
                float x = acc[e >> 2][j][e & 3] + bv[e];
                if (p.act == ACT_SILU) x = silu<T>(x);
                vv[e] = x;
            }
            if constexpr (RUN >= 8) {
#pragma unroll
                for (int c8 = 0; c8 < RUN / 8; ++c8) {
                    if (co + c8 * 8 >= p.Cout) break;
                    float f[8];
#pragma unroll
                    for (int e = 0; e < 8; ++e) f[e] = fromf_round<T>(vv[c8 * 8 + e]);
                    if (res) {
                        float gg[8];
                        chunk_to_f(ld_chunk(res + (long long)m * p.ldr + co + c8 * 8), gg);
#pragma unroll
                        for (int e = 0; e < 8; ++e) f[e] += gg[e];
                    }
                    st_chunk(out + (long long)m * p.ldo + co + c8 * 8, f_to_chunk<T>(f));
                }
            } else {
                T o[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float x = fromf_round<T>(vv[e]);
                    if (res) x += tof(res[(long long)m * p.ldr + co + e]);
                    o[e] = fromf<T>(x);
                }
                *reinterpret_cast<uint2*>(out + (long long)m * p.ldo + co) = *reinterpret_cast<const uint2*>(o);
            }
        }
    }
}

bool tiny_plan(const ConvArgs& a, TinyPlan* out) {
    if (!(a.KH == 3 && a.KW == 3 && a.pad == 1 && a.stride == 1)) return false;
    if (a.c1 != 0 || a.up0 != 0 || a.c0 % 8 != 0 || a.c0 > 32 || a.Cin != a.c0) return false;
    if (a.Hi != a.h0 || a.Wi != a.w0 || a.Hi != a.Ho || a.Wi != a.Wo) return false;
    if ((a.K + 31) / 32 > TINY_KS) return false;
    TinyPlan g{};
    g.ntl = a.Cout <= 16 ? 1 : a.Cout <= 32 ? 2 : 4;
    g.PC = a.Wi + 2;
    g.pst = a.c0 * 2 + 16;
    const int wbytes = 16 * g.ntl * (a.Kp * 2 + 16);
    int th = 0;
    for (int t = 1; t <= a.Ho; ++t) {
        if (wbytes + (t + 2) * g.PC * g.pst + 16 > TINY_BUDGET) break;
        th = t;
    }
    if (th == 0) return false;
    g.nrb = (a.Ho + th - 1) / th;
    g.TH = (a.Ho + g.nrb - 1) / g.nrb;
    g.slices = (a.Cout + 16 * g.ntl - 1) / (16 * g.ntl);
    g.B = a.M / (a.Ho * a.Wo);
    g.zoff = (g.TH + 2) * g.PC * g.pst;
    g.lds = wbytes + g.zoff + 16;
    if (out) *out = g;
    return true;
}

template <typename T>
int launch_tiny(const ConvArgs& a, hipStream_t s) {
    TinyPlan g{};
    if (!tiny_plan(a, &g)) return (int)hipErrorInvalidValue;
    const dim3 grid((unsigned)(g.B * g.nrb * g.slices));
    switch (g.ntl) {
        case 1: hipLaunchKernelGGL((conv_tiny<T, 1>), grid, dim3(TINY_NT), g.lds, s, a, g); break;
        case 2: hipLaunchKernelGGL((conv_tiny<T, 2>), grid, dim3(TINY_NT), g.lds, s, a, g); break;
        default: hipLaunchKernelGGL((conv_tiny<T, 4>), grid, dim3(TINY_NT), g.lds, s, a, g); break;
    }
    return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// conv_gemm2k: conv_gemm2 (BM 64) with the K walk split over the workgroup's
// waves, for layers whose few tiles leave CUs idle and whose long K loop is a
// chain of LDS-DMA round trips (e.g. head.box.2.0: 200 tiles, 36 stages).
// Wave w = g*KS + z walks K stages z, z+KS, ... for rows g*16*KS .. +16*KS of
// the tile; the KS stages of one iteration are in flight together. Partial sums
// meet in LDS and are added in the fixed order z = 0, 1, .., KS-1 - so the
// result is deterministic, but rounds differently from the single-chain kernels:
// the engine selects this kernel by a shape rule (ConvArgs::ks), never by timing.
template <int BN, int KS>
struct Smem2K {
    static constexpr int STAGE = 64 * 128 + BN * 128;
    static constexpr int MAIN = 2 * KS * STAGE;
    static constexpr int RED = 4 * (BN / 16) * KS * 64 * 16;   // every wave's accumulators
    static constexpr int EPI = 64 * (BN + 8) * 2;
    static constexpr int R1 = MAIN > RED ? MAIN : RED;
    static constexpr int REGION = R1 > EPI ? R1 : EPI;
};

template <typename T, int BN, int KS>
__global__ __launch_bounds__(NT_) void conv_gemm2k(const ConvArgs p) {
    static_assert(sizeof(T) == 2, "16-bit path");
    constexpr int BM = 64;
    constexpr int NTL = BN / 16;
    constexpr int AI = BM / 32;
    constexpr int MT = KS;          // 16-row MFMA tiles per wave (rows = 16 * KS)
    using SM = Smem2K<BN, KS>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int* ktab = reinterpret_cast<int*>(smem + SM::REGION);

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int z = wave % KS, g = wave / KS;
    const int lid = xcd_remap(blockIdx.x, p.gm * p.gn);
    const int mt = lid / p.gn, nt = lid - mt * p.gn;
    const int m0 = mt * BM, n0 = nt * BN;
    for (int i = tid; i < p.Kp / 8; i += NT_) ktab[i] = p.ktab[i];

    const int lrow = lane >> 3;
    const int cidx = (lane & 7) ^ lrow;
    const int HoWo = p.Ho * p.Wo;
    int rn[AI], rhb[AI], rwb[AI];
#pragma unroll
    for (int i = 0; i < AI; ++i) {
        const int m = m0 + (wave + 4 * i) * 8 + lrow;
        if (m < p.M) {
            const int n = m / HoWo, r = m - n * HoWo;
            const int ho = r / p.Wo, wo = r - ho * p.Wo;
            rn[i] = n; rhb[i] = ho * p.stride - p.pad; rwb[i] = wo * p.stride - p.pad;
        } else {
            rn[i] = -1; rhb[i] = 0; rwb[i] = 0;
        }
    }
    const T* in0 = reinterpret_cast<const T*>(p.in0);
    const T* in1 = reinterpret_cast<const T*>(p.in1);
    const T* wg = reinterpret_cast<const T*>(p.w);
    const long long bs0 = (long long)p.h0 * p.w0 * p.ldc0;
    const long long bs1 = (long long)p.h1 * p.w1 * p.ldc1;
    __syncthreads();  // ktab

    auto issue = [&](int kt, char* a) {
        char* b = a + BM * 128;
        const int e = ktab[kt * 8 + cidx];
        const int kh = e >> 24, kw = (e >> 16) & 0xff, ci = e & 0xffff;
#pragma unroll
        for (int i = 0; i < AI; ++i) {
            const int hi = rhb[i] + kh, wi = rwb[i] + kw;
            const void* src = p.zero;
            if (ci != 0xffff && rn[i] >= 0 && hi >= 0 && hi < p.Hi && wi >= 0 && wi < p.Wi) {
                if (ci < p.c0)
                    src = in0 + rn[i] * bs0 + ((long long)(hi >> p.up0) * p.w0 + (wi >> p.up0)) * p.ldc0 + ci;
                else
                    src = in1 + rn[i] * bs1 + ((long long)(hi >> p.up1) * p.w1 + (wi >> p.up1)) * p.ldc1 + (ci - p.c0);
            }
            glds16(src, a + (wave + 4 * i) * 1024);
        }
        for (int ii = wave; ii < BN / 8; ii += 4) {
            const T* src = wg + (long long)(n0 + ii * 8 + lrow) * p.Kp + kt * BK2 + cidx * 8;
            glds16(src, b + ii * 1024);
        }
    };
    const int nkt = p.Kp / BK2;
    auto issue_iter = [&](int it, int buf) {
        for (int zz = 0; zz < KS; ++zz) {
            const int kt = it * KS + zz;
            if (kt < nkt) issue(kt, smem + buf * KS * SM::STAGE + zz * SM::STAGE);
        }
    };

    f32x4 acc[NTL][MT];
#pragma unroll
    for (int i = 0; i < NTL; ++i)
#pragma unroll
        for (int j = 0; j < MT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nit = (nkt + KS - 1) / KS;
    const int fr = lane & 15, fq = lane >> 4;
    issue_iter(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int it = 0; it < nit; ++it) {
        const int cur = it & 1;
        if (it + 1 < nit) issue_iter(it + 1, cur ^ 1);
        if (it * KS + z < nkt) {   // wave-uniform
            const char* a = smem + cur * KS * SM::STAGE + z * SM::STAGE;
            const char* b = a + BM * 128;
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                const int chunk = kk * 4 + fq;
                uint4 wf[NTL];
#pragma unroll
                for (int i = 0; i < NTL; ++i) {
                    const int row = i * 16 + fr;
                    wf[i] = *reinterpret_cast<const uint4*>(b + row * 128 + ((chunk ^ (row & 7)) << 4));
                }
#pragma unroll
                for (int j = 0; j < MT; ++j) {
                    const int row = g * (16 * KS) + j * 16 + fr;
                    const uint4 xa = *reinterpret_cast<const uint4*>(a + row * 128 + ((chunk ^ (row & 7)) << 4));
#pragma unroll
                    for (int i = 0; i < NTL; ++i) Mma<T>::step(acc[i][j], &wf[i], &xa);
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    // partials -> LDS, then wave w sums rows w*16 .. w*16+15 over z in order
    f32x4* red = reinterpret_cast<f32x4*>(smem);
#pragma unroll
    for (int i = 0; i < NTL; ++i)
#pragma unroll
        for (int j = 0; j < MT; ++j) red[((wave * NTL + i) * MT + j) * 64 + lane] = acc[i][j];
    __syncthreads();
    f32x4 sum[NTL];
    {
        const int gw = wave / KS, jw = wave % KS;   // (group, tile) holding rows wave*16..
#pragma unroll
        for (int i = 0; i < NTL; ++i) {
            sum[i] = red[(((gw * KS + 0) * NTL + i) * MT + jw) * 64 + lane];
            for (int zz = 1; zz < KS; ++zz) sum[i] += red[(((gw * KS + zz) * NTL + i) * MT + jw) * 64 + lane];
        }
    }
    __syncthreads();   // the epilogue's staging reuses the reduction area

    constexpr int LDE = BN + 8;
    T* Cs = reinterpret_cast<T*>(smem);
#pragma unroll
    for (int i = 0; i < NTL; ++i) {
        const int co = i * 16 + fq * 4;
        float bv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = p.bias[n0 + co + r];
        const int px = wave * 16 + fr;
        T* dst = Cs + px * LDE + co;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float v = sum[i][r] + bv[r];
            if (p.act == ACT_SILU) v = silu<T>(v);
            dst[r] = fromf<T>(v);
        }
    }
    __syncthreads();
    const T* res = reinterpret_cast<const T*>(p.res);
    T* out = reinterpret_cast<T*>(p.out);
    constexpr int CPP = BN / 8;
    for (int c = tid; c < BM * CPP; c += NT_) {
        const int px = c / CPP, cc = c - px * CPP;
        const int m = m0 + px, co = n0 + cc * 8;
        if (m >= p.M || co >= p.Cout) continue;
        Chunk<T> v = ld_chunk(Cs + px * LDE + cc * 8);
        if (res) {
            float f[8], gg[8];
            chunk_to_f(v, f);
            chunk_to_f(ld_chunk(res + (long long)m * p.ldr + co), gg);
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] += gg[e];
            v = f_to_chunk<T>(f);
        }
        st_chunk(out + (long long)m * p.ldo + co, v);
    }
}

template <typename T, int BN, int KS>
int launch_conv2k_t(const ConvArgs& a, hipStream_t s) {
    using SM = Smem2K<BN, KS>;
    const int lds = SM::REGION + (a.Kp / 8) * 4;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_gemm2k<T, BN, KS>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    ConvArgs b = a;
    b.gm = (a.M + 63) / 64;
    b.gn = (a.Cout + BN - 1) / BN;
    hipLaunchKernelGGL((conv_gemm2k<T, BN, KS>), dim3(b.gm * b.gn), dim3(NT_), lds, s, b);
    return (int)hipGetLastError();
}

template <typename T>
int launch_conv2k(const ConvArgs& a, int BN, hipStream_t s) {
    if (a.ks == 4) {
        switch (BN) {
            case 16: return launch_conv2k_t<T, 16, 4>(a, s);
            case 32: return launch_conv2k_t<T, 32, 4>(a, s);
            case 64: return launch_conv2k_t<T, 64, 4>(a, s);
        }
    } else if (a.ks == 2) {
        switch (BN) {
            case 16: return launch_conv2k_t<T, 16, 2>(a, s);
            case 32: return launch_conv2k_t<T, 32, 2>(a, s);
            case 64: return launch_conv2k_t<T, 64, 2>(a, s);
            case 128: return launch_conv2k_t<T, 128, 2>(a, s);
        }
    }
    return (int)hipErrorInvalidValue;
}

template <typename T, int BM, int BN>
int launch_conv2_t(const ConvArgs& a, hipStream_t s) {
    using SM = Smem2<BM, BN>;
    const int lds = SM::REGION + (a.Kp / 8) * 4;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_gemm2<T, BM, BN>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    hipLaunchKernelGGL((conv_gemm2<T, BM, BN>), dim3(a.gm * a.gn), dim3(NT_), lds, s, a);
    return (int)hipGetLastError();
}

template <typename T>
int launch_conv2_bm(int BM, int BN, const ConvArgs& a, hipStream_t s) {
#define YH_BN2(bm)                                                       \
    switch (BN) {                                                        \
        case 16: return launch_conv2_t<T, bm, 16>(a, s);                 \
        case 32: return launch_conv2_t<T, bm, 32>(a, s);                 \
        case 64: return launch_conv2_t<T, bm, 64>(a, s);                 \
        case 128: return launch_conv2_t<T, bm, 128>(a, s);               \
        default: return (int)hipErrorInvalidValue;                       \
    }
    switch (BM) {
        case 64: YH_BN2(64)
        case 128: YH_BN2(128)
        case 256: YH_BN2(256)
        default: return (int)hipErrorInvalidValue;
    }
#undef YH_BN2
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
#pragma unroll 2
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

template <typename T, int BM, int NS>
int launch_stream_bn(int BN, const ConvArgs& a, hipStream_t s, int bpc) {
    switch (BN) {
        case 16: return launch_stream_t<T, BM, 16, NS>(a, s, bpc);
        case 32: return launch_stream_t<T, BM, 32, NS>(a, s, bpc);
        case 64: return launch_stream_t<T, BM, 64, NS>(a, s, bpc);
        case 128: return launch_stream_t<T, BM, 128, (NS > 4 ? 4 : NS)>(a, s, bpc);
    }
    return (int)hipErrorInvalidValue;
}

// BM 64. NS = 2 (the ring depth that wins on large layers: more blocks per CU)
// or a deep ring (NS = 4 / 8: NS-1 stages in flight, for the small 20x20 /
// 40x40 layers whose few tiles leave CUs idle and whose K loop is latency-bound).
// Blocks per CU from the LDS footprint.
template <typename T>
int launch_stream(int BN, int NS, const ConvArgs& a, hipStream_t s) {
    const int ns = (BN == 128 && NS > 4) ? 4 : NS;
    const int lds = ns * (64 + BN) * 128 + 1024 + 64 * (BN + 8) * 2 + a.Kp / 2 + a.gn * BN * 4;
    if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
    int bpc = (160 * 1024) / lds;
    bpc = bpc < 1 ? 1 : bpc > 8 ? 8 : bpc;
    switch (NS) {
        case 2: return launch_stream_bn<T, 64, 2>(BN, a, s, bpc);
        case 4: return launch_stream_bn<T, 64, 4>(BN, a, s, bpc);
        case 8: return launch_stream_bn<T, 64, 8>(BN, a, s, bpc);
    }
    return (int)hipErrorInvalidValue;
}

bool conv_kernel_ok(int dtype, int kern, const ConvArgs& a) {
    if (a.Kp % BK2 != 0) return false;
    if (dtype == F32) return kern == CONV_GEMM;
    if (kern == CONV_DIRECT) return direct_plan(a, nullptr, nullptr);
    if (kern == CONV_TINY) return tiny_plan(a, nullptr);
    if (kern == CONV_STREAM4 || kern == CONV_STREAM8) {
        // deep rings only pay off while the tiles leave CUs idle; LDS must fit
        const int BN = a.Cout <= 16 ? 16 : a.Cout <= 32 ? 32 : a.Cout <= 64 ? 64 : 128;
        const int ns = kern == CONV_STREAM4 ? 4 : (BN == 128 ? 4 : 8);
        if (kern == CONV_STREAM8 && BN == 128) return false;
        if (a.res && BN > 64) return false;
        const int lds = ns * (64 + BN) * 128 + 1024 + 64 * (BN + 8) * 2 + a.Kp / 2 + ((a.Cout + BN - 1) / BN) * BN * 4;
        return lds <= 160 * 1024 && a.Kp / BK2 >= 2;
    }
    return kern >= CONV_GEMM && kern <= CONV_STREAM;
}

int launch_conv(int dtype, int kern, int BM, int BN, const ConvArgs& a, hipStream_t s) {
    if (dtype != F32 && a.ks > 1)   // shape-ruled K split (deterministic, see conv_gemm2k)
        return dtype == F16 ? launch_conv2k<_Float16>(a, BN, s) : launch_conv2k<__bf16>(a, BN, s);
    if (!conv_kernel_ok(dtype, kern, a)) return (int)hipErrorInvalidValue;
    if (dtype == F32) return launch_conv_bm<float>(BM, BN, a, s);
    const bool h = dtype == F16;
    switch (kern) {
        case CONV_GEMM:
            return h ? launch_conv2_bm<_Float16>(BM, BN, a, s) : launch_conv2_bm<__bf16>(BM, BN, a, s);
        case CONV_GEMM64:
        case CONV_GEMM128: {
            ConvArgs b = a;
            const int bm = kern == CONV_GEMM64 ? 64 : 128;
            b.gm = (a.M + bm - 1) / bm;
            return h ? launch_conv2_bm<_Float16>(bm, BN, b, s) : launch_conv2_bm<__bf16>(bm, BN, b, s);
        }
        case CONV_STREAM:
        case CONV_STREAM4:
        case CONV_STREAM8: {
            ConvArgs b = a;
            if (a.res && BN > 64) BN = 64;  // residual epilogue keeps <= 4 chunks per thread
            b.gm = (a.M + 63) / 64;
            b.gn = (a.Cout + BN - 1) / BN;
            const int ns = kern == CONV_STREAM ? 2 : kern == CONV_STREAM4 ? 4 : 8;
            return h ? launch_stream<_Float16>(BN, ns, b, s) : launch_stream<__bf16>(BN, ns, b, s);
        }
        case CONV_DIRECT:
            return h ? launch_direct<_Float16>(a, s) : launch_direct<__bf16>(a, s);
        case CONV_TINY:
            return h ? launch_tiny<_Float16>(a, s) : launch_tiny<__bf16>(a, s);
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
