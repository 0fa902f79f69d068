// Pointwise chains (16-bit handles): runs of consecutive 1x1 convs (nets/nn.py:28-39 Conv with
// k = 1, the Residual add of nn.py:49, channel-slice concats) on one map, as one launch.
// v11_n's 20x20 tail has three: the C3k2 conv2 -> SPPF conv1 pair (nn.py:66-94), SPPF conv2 ->
// C2PSA conv1 -> qkv (nn.py:83-148) and the PSABlock after the attention core, proj (+x) ->
// ffn 1x1 -> ffn 1x1 (+x) -> C2PSA conv2 over [a | b] (nn.py:97-148).
//
// A workgroup owns P consecutive pixels of the flattened (image, row, column) map - a 1x1 conv
// needs no halo - and runs the stages in order with a barrier between them:
//   prologue  every global input and residual of the chain (views no earlier stage writes) ->
//             LDS by LDS-DMA, padded by one 16-B chunk per pixel;
//   stage     (32-cout A tile, 32-pixel B tiles) units over the waves; A fragments come from the
//             conv's 16-bit weights in fragment order (one contiguous KB per load; L2, warmed by
//             the prologue), 8 K blocks per piece with the next piece in flight; B fragments from LDS; epilogue: bias, activation,
//             one rounding, the residual (LDS) added in fp32 and rounded again; every output goes to its
//             global view (all tensors stay materialised as in the per-layer forward) and, when a
//             later stage reads it, to an LDS region of its own.
// Bit-identical to the per-layer conv_mx launches: each stage walks K as one 32x32x16 MFMA step
// per 16-channel block in ascending order (conv_mx.h), from a zero fp32 accumulator.
#include "common.h"
#include "dtypes.h"

namespace yh {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <typename T> struct PMfma;
template <> struct PMfma<__bf16> {
    static __device__ __forceinline__ f32x16 step(const uint4& a, const uint4& b, const f32x16& c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                       0, 0);
    }
};
template <> struct PMfma<_Float16> {
    static __device__ __forceinline__ f32x16 step(const uint4& a, const uint4& b, const f32x16& c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                      0);
    }
};

constexpr int PNW = PWC_THREADS / 64;

__device__ __forceinline__ void pc_glds(const void* src, unsigned lds_addr) {
#if defined(__HIP_DEVICE_COMPILE__)
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds_addr) : "memory");
#else
    (void)src; (void)lds_addr;
#endif
}
__device__ __forceinline__ void pc_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

typedef __attribute__((address_space(3))) const uint4* pc_lp4;
typedef __attribute__((address_space(3))) const uint2* pc_lp2;
typedef __attribute__((address_space(3))) uint2* pc_sp2;
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ uint4 pc_rd(unsigned addr) { return *reinterpret_cast<pc_lp4>((size_t)addr); }
__device__ __forceinline__ uint2 pc_rd2(unsigned addr) { return *reinterpret_cast<pc_lp2>((size_t)addr); }
__device__ __forceinline__ void pc_wr2(unsigned addr, uint2 v) { *reinterpret_cast<pc_sp2>((size_t)addr) = v; }
#else
__device__ __forceinline__ uint4 pc_rd(unsigned) { return uint4{}; }
__device__ __forceinline__ uint2 pc_rd2(unsigned) { return uint2{}; }
__device__ __forceinline__ void pc_wr2(unsigned, uint2) {}
#endif

#ifdef YH_PWC_TRACE
// experiments only (-DYH_PWC_TRACE builds): per-workgroup s_memtime after the prologue and after
// each stage (slots 1..), s_memrealtime at entry / exit (slots 0 / 15); the last launch wins
__device__ unsigned long long pwc_trace_buf[1024 * 32];
#define PWC_STAMP(k, rt)                                                                           \
    do {                                                                                           \
        if (threadIdx.x == 0 && blockIdx.x < 1024)                                                 \
            pwc_trace_buf[blockIdx.x * 32 + (k)] =                                                 \
                (rt) ? __builtin_amdgcn_s_memrealtime() : __builtin_amdgcn_s_memtime();            \
    } while (0)
#else
#define PWC_STAMP(k, rt) \
    do {                 \
    } while (0)
#endif

template <typename T>
__global__ __launch_bounds__(PWC_THREADS) void pw_chain(const PwChainArgs A) {
    PWC_STAMP(0, true);
    PWC_STAMP(30, false);
#ifndef YH_PWC_NOTOUCH
    touch_kernargs<sizeof(PwChainArgs)>();
#endif
    extern __shared__ __attribute__((aligned(16))) char sm[];
    typedef __attribute__((address_space(3))) char* lds_c;
    const unsigned lds0 = (unsigned)(size_t)(lds_c)sm;
    const int lane = threadIdx.x & 63, l32 = lane & 31, h = lane >> 5;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long long m0 = (long long)blockIdx.x * A.P;
    const int np = (int)(A.M - m0 < A.P ? A.M - m0 : A.P);

    const int nb = (np + 31) >> 5;   // B tiles holding pixels of the map (1 or 2)
    // a unit = one A tile and both B tiles (A fragments loaded once), or one B tile when that
    // gives more units than waves
    auto nsplit_of = [&](int s) { return ((A.st[s].N >> 5) >= PNW || nb < 2) ? 1 : 2; };
    auto nu_of = [&](int s) { return (A.st[s].N >> 5) * nsplit_of(s); };
    // A fragments of one step (stage s, unit u, piece pc: 8 K blocks of the unit's 32 couts)
    // (fragment-ordered weights: each of the 8 loads is one contiguous KB of the wave)
    auto load_a = [&](int s, int u, int pc, uint4 (&f)[8]) {
        const PwcStage& S = A.st[s];
        const int a = nsplit_of(s) == 1 ? u : (u >> 1);
        const char* wb = reinterpret_cast<const char*>(S.w) + (((long long)a * (S.wld >> 4) + pc * 8) * 64 + lane) * 16;
#pragma unroll
        for (int i = 0; i < 8; ++i) f[i] = *reinterpret_cast<const uint4*>(wb + i * 1024);
    };
    // the wave's steps in order - stages, its units, their pieces - with the next step's A
    // fragments in flight during the current one, across unit and stage boundaries (a stage's
    // first weights load before the barrier that opens it)
    // (ps, pu, ppc): the step two ahead of the current one, whose A fragments are requested now
    int ps = 0, pu = wv, ppc = 0;
    while (ps < A.nst && pu >= nu_of(ps)) {
        ++ps;
        pu = wv;
    }
    auto advance = [&]() {
        if (ps >= A.nst) return;
        if (++ppc < (A.st[ps].K >> 7)) return;
        ppc = 0;
        pu += PNW;
        if (pu < nu_of(ps)) return;
        do {
            ++ps;
            pu = wv;
        } while (ps < A.nst && pu >= nu_of(ps));
    };
    // a two-step ring of A fragments: step k's in ring[k & 1], step k + 1's in flight
    uint4 ring[2][8];
    if (ps < A.nst) load_a(ps, pu, ppc, ring[0]);   // in flight with the prologue's DMAs
    advance();   // (step 1's fragments are requested after the prologue's barrier: the prologue
                 // then waits for 64 KB less per workgroup, the CU's L2 intake being its bound)
    int kstep = 0;
    PWC_STAMP(24, false);

    // prologue: the chain's global inputs -> LDS (pixel p, chunk c at (p * (nchunk + 1) + c) * 16;
    // the pad chunk and pixels past the map read zeros)
#if defined(YH_PWC_TRACE) && defined(YH_PWC_NOIN)
    if (A.nload < 0)
#endif
    for (int g = 0; g < A.nload; ++g) {
        const PwcLoad& L = A.ld[g];
        const int cpx = L.nchunk + 1, total = A.P * cpx;
        for (int i0 = wv * 64; i0 < total; i0 += PWC_THREADS) {
            const int q = i0 + lane;
            const int px = q / cpx, c = q - px * cpx;
            const bool ok = q < total && c < L.nchunk && px < np;
            const void* src = ok ? (const void*)(reinterpret_cast<const char*>(L.g) + ((m0 + px) * L.ldg + c * 8) * 2)
                                 : A.zero;
            pc_glds(src, lds0 + (unsigned)L.lds + (unsigned)i0 * 16);
        }
    }
    PWC_STAMP(25, false);
    // L2 warm-up: the workgroups of one XCD (round-robin dispatch: blockIdx % 8) together touch
    // every stage's weights once, 1 KB per DMA into a scratch KB, so the stages' A-fragment loads
    // hit L2 instead of each paying an HBM / MALL round trip (sink < 0: no warm-up)
    if (A.sink >= 0) {
        const int G = (int)((gridDim.x + 7) >> 3), gi = (int)(blockIdx.x >> 3);
        const unsigned sink = lds0 + (unsigned)A.sink;
        int q0 = 0;
        for (int s = 0; s < A.nst; ++s) {
            const int nq = (A.st[s].N * A.st[s].wld * 2) >> 10;   // whole KB (rows are 128-B multiples)
            const char* w = reinterpret_cast<const char*>(A.st[s].w);
            for (int q = (gi + G - q0 % G) % G + wv * G; q < nq; q += PNW * G) pc_glds(w + ((size_t)q << 10) + lane * 16, sink);
            q0 += nq;
        }
    }
    PWC_STAMP(26, false);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    PWC_STAMP(27, false);
    pc_barrier();
    PWC_STAMP(1, false);
    if (ps < A.nst) load_a(ps, pu, ppc, ring[1]);

    for (int s = 0; s < A.nst; ++s) {
        const PwcStage& S = A.st[s];
        const int nsplit = nsplit_of(s), nu = nu_of(s), npc = S.K >> 7;
        const bool silu_act = S.act == ACT_SILU;
        // the stage's epilogue fields in registers once (not re-read from the kernel arguments)
        const int res_lds = S.res_lds, res_ldl = S.res_ldl, out_lds = S.out_lds, out_ldl = S.out_ldl, ldo = S.ldo;
        void* const out = S.out;
        for (int u = wv; u < nu; u += PNW) {
            const int a = nsplit == 1 ? u : (u >> 1);
            const int j0 = nsplit == 1 ? 0 : (u & 1);
            const bool two = nsplit == 1 && nb == 2;
            f32x16 acc0, acc1;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                acc0[e] = 0.f;
                acc1[e] = 0.f;
            }
            // the unit's biases, loaded before the next step's A fragments are issued (vmcnt is in
            // order: a wait for a later load would also wait for that prefetch)
            float4 bq[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) bq[q] = *reinterpret_cast<const float4*>(S.bias + a * 32 + 8 * q + 4 * h);
            if (u == wv) PWC_STAMP(2 + 5 * s, false);
            for (int pc = 0; pc < npc; ++pc) {
                uint4 f[8];
                advance();
                if (kstep & 1) {
#pragma unroll
                    for (int i = 0; i < 8; ++i) f[i] = ring[1][i];
                    if (ps < A.nst) load_a(ps, pu, ppc, ring[1]);
                } else {
#pragma unroll
                    for (int i = 0; i < 8; ++i) f[i] = ring[0][i];
                    if (ps < A.nst) load_a(ps, pu, ppc, ring[0]);
                }
                ++kstep;
                // the piece's run; its B fragments (8 K blocks of one or two B tiles) read from LDS
                // together, then the MFMA steps in block order
                int r = 0, base = 0;
                while (base + (S.run[r].nkb >> 3) <= pc) {
                    base += S.run[r].nkb >> 3;
                    ++r;
                }
                const int rl = S.run[r].lds, rld = S.run[r].ld;
                const unsigned b0 = lds0 + (unsigned)rl + (unsigned)(((j0 * 32 + l32) * rld + (pc - base) * 128 + 8 * h) * 2);
                if (two) {
                    const unsigned b1 = b0 + (unsigned)(32 * rld * 2);
                    uint4 x0[8], x1[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        x0[i] = pc_rd(b0 + i * 32);
                        x1[i] = pc_rd(b1 + i * 32);
                    }
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        acc0 = PMfma<T>::step(f[i], x0[i], acc0);
                        acc1 = PMfma<T>::step(f[i], x1[i], acc1);
                    }
                } else {
                    uint4 x0[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) x0[i] = pc_rd(b0 + i * 32);
#pragma unroll
                    for (int i = 0; i < 8; ++i) acc0 = PMfma<T>::step(f[i], x0[i], acc0);
                }
            }
            // register i of lane (l32, h): cout a * 32 + (i & 3) + 8 (i >> 2) + 4 h, pixel j * 32 + l32
            auto epi = [&](int j, const f32x16& acc) {
                const int px = j * 32 + l32;
                if (px >= np) return;
                const long long m = m0 + px;
                uint2 rr[4];
                if (res_lds >= 0) {
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        rr[q] = pc_rd2(lds0 + (unsigned)res_lds + (unsigned)((px * res_ldl + a * 32 + 8 * q + 4 * h) * 2));
                }
                T* orow = reinterpret_cast<T*>(out) + m * ldo;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int co = a * 32 + 8 * q + 4 * h;
                    const float4 bb = bq[q];
                    const float v[4] = {acc[4 * q] + bb.x, acc[4 * q + 1] + bb.y, acc[4 * q + 2] + bb.z,
                                        acc[4 * q + 3] + bb.w};
                    T o[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) o[e] = fromf<T>(silu_act ? silu<T>(v[e]) : v[e]);
                    if (res_lds >= 0) {
                        const T* rv = reinterpret_cast<const T*>(&rr[q]);
#pragma unroll
                        for (int e = 0; e < 4; ++e) o[e] = fromf<T>(tof(o[e]) + tof(rv[e]));
                    }
                    const uint2 ov = *reinterpret_cast<const uint2*>(o);
                    *reinterpret_cast<uint2*>(orow + co) = ov;
                    if (out_lds >= 0) pc_wr2(lds0 + (unsigned)out_lds + (unsigned)((px * out_ldl + co) * 2), ov);
                }
            };
            if (u == wv) {
                asm volatile("s_nop 0" ::: "memory");
                PWC_STAMP(2 + 5 * s + 1, false);
            }
            epi(j0, acc0);
            if (two) epi(1, acc1);
            if (u == wv) PWC_STAMP(2 + 5 * s + 2, false);
        }
        PWC_STAMP(2 + 5 * s + 3, false);   // wave 0's units done
        pc_barrier();   // this stage's LDS outputs are complete for the next stage
        PWC_STAMP(2 + 5 * s + 4, false);
    }
    PWC_STAMP(31, true);
}

template <typename T>
int launch_pw_chain_t(const PwChainArgs& a, int lds, hipStream_t s) {
    if (!(a.P == 32 || a.P == 64) || a.nst < 1 || a.nst > PWC_MAX_STAGES || a.nload > PWC_MAX_LOADS || a.M <= 0 ||
        lds > 160 * 1024)
        return (int)hipErrorInvalidValue;
    for (int k = 0; k < a.nst; ++k) {
        const PwcStage& st = a.st[k];
        int nkb = 0;
        for (int r = 0; r < st.nrun; ++r) {
            if (st.run[r].nkb % 8) return (int)hipErrorInvalidValue;
            nkb += st.run[r].nkb;
        }
        if (st.nrun < 1 || st.nrun > PWC_MAX_RUNS || nkb * 16 != st.K || st.N % 32 || st.wld < st.K ||
            st.ldo % 4)
            return (int)hipErrorInvalidValue;
    }
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&pw_chain<T>), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        attr = true;
    }
    const long long grid = (a.M + a.P - 1) / a.P;
    hipLaunchKernelGGL((pw_chain<T>), dim3((unsigned)grid), dim3(PWC_THREADS), lds, s, a);
    return (int)hipGetLastError();
}

}  // namespace

#ifdef YH_PWC_TRACE
extern "C" int yh_debug_pwc_trace(unsigned long long* dst, int n) {
    if (n > 1024 * 32) n = 1024 * 32;
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(pwc_trace_buf), (size_t)n * 8, 0, hipMemcpyDeviceToHost);
}
#endif

int launch_pw_chain(int dtype, const PwChainArgs& a, int lds, hipStream_t s) {
    switch (dtype) {
        case F16: return launch_pw_chain_t<_Float16>(a, lds, s);
        case BF16: return launch_pw_chain_t<__bf16>(a, lds, s);
    }
    return (int)hipErrorInvalidValue;
}

}  // namespace yh
