// Level program for gfx950: one persistent launch runs a run of consecutive ops
// whose outputs live on the 40x40 / 20x20 pyramid levels (C3k2 / C3k / SPPF /
// C2PSA / FPN / detect-head layers of nets/nn.py:139-270 at strides 16 and 32).
//
// Why: at batch 32 these layers are 12800..51200-pixel GEMMs. As one kernel per
// layer they are bound by launch latency, by too few workgroups to fill 256 CUs
// and by serial K loops (10-45 us each for 1-15 GFLOP); here every op is a
// short phase of one launch.
//
// Execution model:
//   * the grid is NC clusters x G workgroups; cluster c owns images c, c+NC, ...;
//     its G members share one XCD (blocks b and b+8 are dealt to one XCD) so the
//     hand-offs stay in that XCD's L2;
//   * every op splits the image's output pixels into G contiguous ranges of
//     16-pixel tiles (attention: the (head, 16-query) tiles over all G*4 waves),
//     then the cluster meets at a barrier;
//   * activations produced inside the launch move only through sc1 buffer stores
//     and sc1 buffer loads (L1 bypass), signalled by an agent-scope atomic
//     arrival counter polled with sc1 loads (MI355X_MICROARCH.md, inter-workgroup
//     visibility, table row 1). The engine lays tensors out so that no region is
//     rewritten after another workgroup has read it within the launch;
//   * activations are addressed as 32-bit byte offsets from the workspace base
//     through one buffer resource; an out-of-range offset reads zeros, which is
//     how padding taps and padded K steps are fed.
//
// Arithmetic is the same as the per-layer kernels, operation for operation:
// dense convs accumulate K in 32-deep v_mfma_f32_16x16x32 steps in increasing k
// with the weights as the A operand (conv.hip), depthwise / pool / attention /
// positional-conv epilogues follow dwconv3x3, maxpool5, psa_attention_mfma and
// pe_add. The fused forward is bit-identical to the unfused one (tested).
#include "common.h"
#include "dtypes.h"

namespace yh {

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v2i __attribute__((ext_vector_type(2)));
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;

constexpr int LP_T = 512;          // threads per workgroup (8 waves: 2 per SIMD)
constexpr int LP_W = LP_T / 64;
constexpr int LP_MT = 4;          // pixel tiles per wave block (register blocking)
constexpr int LP_D = 4;            // k steps in flight per wave
// Buffer range: offsets are unsigned and range-checked against num_records =
// 0x7fffffff by their START address, so "no data" is 2^31 (>= num_records):
// loads return 0, stores are dropped. Real offsets stay below 2^31 - 4096.
constexpr int OFF_NONE = (int)0x80000000u;
constexpr int KTAB_MAX = 2048;     // staged k-table entries (Kp/8 + padding)
constexpr int ADK = 32, ADH = 64;  // PSA head dims (nets/nn.py:104-106)
constexpr int SC1 = 16;            // cache-policy bit of the buffer intrinsics: sc1

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ uint4 ld16(__amdgpu_buffer_rsrc_t r, int off) {
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, SC1));
}
__device__ __forceinline__ uint2 ld8(__amdgpu_buffer_rsrc_t r, int off) {
    return __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, SC1));
}
// Activation stores. sc1 stores write through and drop the line from the XCD's
// L2, so a reader on any XCD fetches the new bytes; when every member of the
// cluster runs on one XCD (checked at launch, g_plain) plain stores keep the line
// in that shared L2, where the members' sc1 (L1-bypassing) loads find it.
__device__ __forceinline__ void st16(__amdgpu_buffer_rsrc_t r, int off, uint4 v, bool plain) {
    if (plain) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v), r, off, 0, 0);
    else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v), r, off, 0, SC1);
}
__device__ __forceinline__ void st8(__amdgpu_buffer_rsrc_t r, int off, uint2 v, bool plain) {
    if (plain) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2i, v), r, off, 0, 0);
    else __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2i, v), r, off, 0, SC1);
}
// Read-only operands (weights, biases, k-tables) whose pointers come from the op
// descriptors in memory: load through global (address space 1) pointers so they
// count on vmcnt only; a generic pointer would issue flat loads, which count on
// lgkmcnt too and make every LDS wait drain all loads in flight.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ldg16(const void* p) {
    return __builtin_bit_cast(uint4, *(const __attribute__((address_space(1))) u32x4*)p);
}
__device__ __forceinline__ float ldgf(const float* p) {
    return *(const __attribute__((address_space(1))) float*)p;
}
__device__ __forceinline__ int ldgi(const int* p) {
    return *(const __attribute__((address_space(1))) int*)p;
}
__device__ __forceinline__ int boff(const void* p, const void* base) {
    return (int)((const char*)p - (const char*)base);
}
template <typename T>
__device__ __forceinline__ void u4_to_f(uint4 u, float (&f)[8]) {
    Chunk<T> c;
    c.v[0] = u;
    chunk_to_f(c, f);
}
template <typename T>
__device__ __forceinline__ uint4 f_to_u4(const float (&f)[8]) {
    return f_to_chunk<T>(f).v[0];
}

// Cluster barrier: every wave drains its stores, the workgroup syncs, lane 0
// arrives on the cluster counter (agent-scope atomic); the last arriver resets
// the counter and bumps the generation word that the others poll with sc1 loads.
// Bounded: a barrier that never completes sets *err and lets the launch finish.
__device__ __forceinline__ void cluster_barrier(unsigned* cnt, unsigned* gen, int G, int* err) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned g0 = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == (unsigned)G - 1u) {
            const unsigned was = __hip_atomic_exchange(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::"v"(was) : "memory");
            __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            unsigned spins = 0;
            while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g0) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1u << 24)) {
                    __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
        }
    }
    __syncthreads();
}

// Epilogue of one lane: couts [co, co + 4*NT) of pixel m (bias, SiLU, rounding
// to T, residual added in fp32 after the activation, sc1 stores) - conv_direct's.
// Bounds-checked read-only loads of the level program: an index outside the
// allocation (which would be an engine planning bug) reads 0 and flags *err
// (bit 2 weights, bit 3 bias) instead of faulting.
__device__ __forceinline__ void lp_flag(int* err, int bit) {
    if (err) __hip_atomic_fetch_or(err, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T, int NT>
__device__ __forceinline__ void load_bias(const ConvArgs& p, int co, float (&bv)[4 * NT], int bcount, int* err) {
#pragma unroll
    for (int e = 0; e < 4 * NT; ++e) {   // bias is padded to coutp_pad
        const bool ok = co + e < bcount && co + e >= 0;
        if (!ok) lp_flag(err, 8);
        bv[e] = ok ? ldgf(p.bias + co + e) : 0.f;
    }
}
template <typename T, int NT>
__device__ __forceinline__ void conv_store(const ConvArgs& p, __amdgpu_buffer_rsrc_t R, int outo, int reso, int m,
                                           int co, const f32x4 (&acc)[NT], const float (&bv)[4 * NT], bool plain) {
    constexpr int RUN = 4 * NT;
    float v[RUN];
#pragma unroll
    for (int e = 0; e < RUN; ++e) {
        float x = acc[e >> 2][e & 3] + bv[e];
        if (p.act == ACT_SILU) x = silu<T>(x);
        v[e] = fromf_round<T>(x);
    }
    if constexpr (RUN >= 8) {
#pragma unroll
        for (int c8 = 0; c8 < RUN / 8; ++c8) {
            if (co + c8 * 8 >= p.Cout) break;
            float f[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] = v[c8 * 8 + e];
            if (p.res) {
                float g[8];
                u4_to_f<T>(ld16(R, reso + (m * p.ldr + co + c8 * 8) * 2), g);
#pragma unroll
                for (int e = 0; e < 8; ++e) f[e] += g[e];
            }
            st16(R, outo + (m * p.ldo + co + c8 * 8) * 2, f_to_u4<T>(f), plain);
        }
    } else {
        float g[4] = {0.f, 0.f, 0.f, 0.f};
        if (p.res) {
            const uint2 r2 = ld8(R, reso + (m * p.ldr + co) * 2);
            const T* rt = reinterpret_cast<const T*>(&r2);
#pragma unroll
            for (int e = 0; e < 4; ++e) g[e] = tof(rt[e]);
        }
        T o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = fromf<T>(p.res ? v[e] + g[e] : v[e]);
        st8(R, outo + (m * p.ldo + co) * 2, *reinterpret_cast<const uint2*>(o), plain);
    }
}

// ---------------------------------------------------------------- dense conv
// Wave work unit = one 16-pixel tile x 16*NT output channels. Lane (li, q):
// pixel li of the tile, k chunk q (8 channels) of every 32-deep step. Weight
// rows are loaded permuted (MFMA row 4g'+r' of tile i <- cout g'*4NT + 4i + r')
// so each lane ends with 4*NT contiguous output channels of its pixel.
template <typename T, int NT>
__device__ __forceinline__ void conv_op(const ConvArgs& p, __amdgpu_buffer_rsrc_t R, const void* base, int n, int t0, int t1,
                        const int* kt, int wave, int lane, bool plain) {
    constexpr int RUN = 4 * NT;
    const int li = lane & 15, q = lane >> 4;
    const int P = p.Ho * p.Wo;
    const int nch = (p.Cout + 16 * NT - 1) / (16 * NT);
    const int units = (t1 - t0) * nch;
    const int in0 = boff(p.in0, base) + n * (p.h0 * p.w0 * p.ldc0 * 2);
    const int in1 = boff(p.in1, base) + n * (p.h1 * p.w1 * p.ldc1 * 2);
    const int outo = boff(p.out, base) + n * (P * p.ldo * 2);
    const int reso = p.res ? boff(p.res, base) + n * (P * p.ldr * 2) : 0;
    const int nks = (p.K + 31) >> 5;
    const int nkp = (nks + LP_D - 1) / LP_D * LP_D;
    const int kmax = p.Kp / 32 - 1;
    const T* wg = reinterpret_cast<const T*>(p.w);
    for (int u = wave; u < units; u += LP_W) {
        const int pt = t0 + u / nch, c0 = (u % nch) * 16 * NT;
        const int pix = pt * 16 + li;
        const bool pv = pix < P;
        const int ho = pix / p.Wo, wo = pix - ho * p.Wo;
        const int rh = pv ? ho * p.stride - p.pad : -(1 << 20), rw = wo * p.stride - p.pad;
        const T* wrow = wg + (long long)(c0 + (li >> 2) * RUN + (li & 3)) * p.Kp + q * 8;
        auto aoff = [&](int ks) {
            const int e = kt[ks * 4 + q];
            const int kh = e >> 24, kw = (e >> 16) & 0xff, ci = e & 0xffff;
            const int hi = rh + kh, wi = rw + kw;
            const bool ok = (ci != 0xffff) & ((unsigned)hi < (unsigned)p.Hi) & ((unsigned)wi < (unsigned)p.Wi);
            const int o = ci < p.c0 ? in0 + (((hi >> p.up0) * p.w0 + (wi >> p.up0)) * p.ldc0 + ci) * 2
                                    : in1 + (((hi >> p.up1) * p.w1 + (wi >> p.up1)) * p.ldc1 + (ci - p.c0)) * 2;
            return ok ? o : OFF_NONE;
        };
        f32x4 acc[NT];
#pragma unroll
        for (int i = 0; i < NT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        uint4 ab[LP_D], bb[LP_D][NT];
        auto load = [&](int ks, int d) {
            ab[d] = ld16(R, aoff(ks));
            const int kw_ = min(ks, kmax);
#pragma unroll
            for (int i = 0; i < NT; ++i)
                bb[d][i] = ldg16(wrow + (long long)(4 * i) * p.Kp + kw_ * 32);
        };
#pragma unroll
        for (int d = 0; d < LP_D; ++d) load(d, d);
        for (int ks = 0; ks < nkp; ks += LP_D) {
#pragma unroll
            for (int d = 0; d < LP_D; ++d) {
#pragma unroll
                for (int i = 0; i < NT; ++i) Mma<T>::step(acc[i], &bb[d][i], &ab[d]);
                load(ks + d + LP_D, d);
            }
        }
        const int co = c0 + q * RUN;
        if (!pv || co >= p.Cout) continue;
        float bv[RUN];
        load_bias<T, NT>(p, co, bv, 1 << 30, nullptr);
        conv_store<T, NT>(p, R, outo, reso, pix, co, acc, bv, plain);
    }
}

// Patch variant: the workgroup walks its output pixels in bands of op.band
// 16-pixel tiles. For each band it copies the input rows the band needs (the
// conv's halo rows included, a zero border column on each side, all input
// channels of both concat segments, nearest-upsampled segments expanded) into
// LDS with sc1 loads; every wave reads its pixel fragments from LDS (ds_read_b128;
// a 16-B pad per pixel keeps 16 consecutive pixels on distinct banks) through the
// op's k-offset table (koff: LDS byte offset of every 8-channel K chunk relative
// to the tap-(0,0) pixel, -1 = padding -> the zero fragment at LDS[0..16)).
// Weights stream through two LDS buffers in chunks of op.kcs k steps, shared by
// all 8 waves: the loads of chunk c+1 are in flight while chunk c is multiplied.
// Weight rows are stored permuted (LDS row 16i + l of a 16*NT-cout group holds
// cout (l>>2)*4NT + 4i + (l&3)), so 16 lanes read 16 consecutive rows (conflict
// free with the 16-B row pad) and each lane ends with 4*NT contiguous couts.
// A wave owns one block of <= LP_MT pixel tiles x NT cout tiles per band.
template <typename T, int NT>
__device__ __forceinline__ void conv_patch(const LevelOp& op, __amdgpu_buffer_rsrc_t R, const void* base, int n, int p0,
                                           int p1, int ch0, int ch1, const int* koff, char* lds, int wave, int lane,
                                           unsigned long long* tr, int* err, bool plain) {
    const ConvArgs& p = op.c;
    constexpr int RUN = 4 * NT;
    const int ps = op.pstride, wp = op.wp, nck = p.Cin / 8;
    const int P = p.Ho * p.Wo;
    const int in0 = boff(p.in0, base) + n * (p.h0 * p.w0 * p.ldc0 * 2);
    const int in1 = boff(p.in1, base) + n * (p.h1 * p.w1 * p.ldc1 * 2);
    const int li = lane & 15, q = lane >> 4;
    const int outo = boff(p.out, base) + n * (P * p.ldo * 2);
    const int reso = p.res ? boff(p.res, base) + n * (P * p.ldr * 2) : 0;
    const int nch = ch1 - ch0;                   // cout chunks (16*NT couts) of this workgroup
    const int wrows = nch * 16 * NT;
    const int nks = (p.K + 31) >> 5;
    const int kcs = op.kcs, wpitch = op.wpitch;
    const int nchunks = (nks + kcs - 1) / kcs;
    const int wpieces = kcs * 4;                 // 16-B pieces per weight row and chunk
    const int witems = wrows * wpieces;
    char* wbuf0 = lds + op.woff;
    char* wbuf1 = wbuf0 + wrows * wpitch;
    const char* wg = reinterpret_cast<const char*>(p.w);
    const int WN = op.wn, WM = LP_W / WN;
    const int wn = wave % WN, wm = wave / WN;
    constexpr int WREG = 8;                      // weight pieces staged per thread per chunk (<= 64 KB chunk)
    // chunk c of the weights -> registers (source rows permuted, see above)
    auto wload = [&](int c, uint4 (&r)[WREG]) {
#pragma unroll
        for (int u = 0; u < WREG; ++u) {
            const int it = threadIdx.x + u * LP_T;
            r[u] = make_uint4(0, 0, 0, 0);
            if (it < witems) {
                const int row = it / wpieces, pc = it - row * wpieces;
                const int g = row / (16 * NT), rr = row - g * 16 * NT, i = rr >> 4, l = rr & 15;
                const int cout = (ch0 + g) * 16 * NT + (l >> 2) * RUN + 4 * i + (l & 3);
                const int k = (c * kcs) * 32 + pc * 8;
                if (k < p.Kp) {
                    const long long e = (long long)cout * p.Kp + k;
                    if (e >= 0 && e + 8 <= op.wcount) r[u] = ldg16(wg + e * 2);
                    else lp_flag(err, 4);
                }
            }
        }
    };
    auto wstore = [&](char* buf, const uint4 (&r)[WREG]) {
#pragma unroll
        for (int u = 0; u < WREG; ++u) {
            const int it = threadIdx.x + u * LP_T;
            if (it < witems) {
                const int row = it / wpieces, pc = it - row * wpieces;
                *reinterpret_cast<uint4*>(buf + row * wpitch + pc * 16) = r[u];
            }
        }
    };
    if (threadIdx.x == 0) *reinterpret_cast<uint4*>(lds) = make_uint4(0, 0, 0, 0);
    for (int q0 = p0; q0 < p1; q0 += 16 * op.band) {
        const int q1 = min(p1, q0 + 16 * op.band);
        const int ho0 = q0 / p.Wo, ho1 = (q1 - 1) / p.Wo;
        const int r0 = ho0 * p.stride - p.pad;
        const int nrows = (ho1 - ho0) * p.stride + p.KH;
        uint4 wr[WREG];
        wload(0, wr);                                 // first weight chunk, overlapping the patch loads
        __syncthreads();                              // the previous band is consumed
        const int items = nrows * wp * nck;
        for (int b0 = threadIdx.x; b0 < items; b0 += 4 * LP_T) {
            uint4 v[4];
            int dst[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int it = b0 + u * LP_T;
                int o = OFF_NONE;
                dst[u] = -1;
                if (it < items) {
                    const int ch = it % nck, rc = it / nck, c = rc % wp, r = rc / wp;
                    const int hi = r0 + r, wi = c - p.pad, ci = ch * 8;
                    if ((unsigned)hi < (unsigned)p.Hi && (unsigned)wi < (unsigned)p.Wi)
                        o = ci < p.c0 ? in0 + (((hi >> p.up0) * p.w0 + (wi >> p.up0)) * p.ldc0 + ci) * 2
                                      : in1 + (((hi >> p.up1) * p.w1 + (wi >> p.up1)) * p.ldc1 + (ci - p.c0)) * 2;
                    dst[u] = 16 + (r * wp + c) * ps + ch * 16;
                }
                v[u] = ld16(R, o);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (dst[u] >= 0) *reinterpret_cast<uint4*>(lds + dst[u]) = v[u];
        }
        wstore(wbuf0, wr);
        __syncthreads();
        if (tr && q0 == p0) tr[3] = __builtin_amdgcn_s_memrealtime();
        // this wave's block: pixel tiles [mb, mb + mt) x cout chunk wn
        const int t0 = q0 / 16, t1 = (q1 + 15) / 16;
        const int per = (t1 - t0 + WM - 1) / WM;
        const int mb = t0 + wm * per, mt = max(0, min(per, t1 - mb));
        const bool active = mt > 0 && wn < nch;       // wave-uniform
        const int c0 = (ch0 + wn) * 16 * NT;
        int lbj[LP_MT];
#pragma unroll
        for (int j = 0; j < LP_MT; ++j) {
            const int pix = (mb + min(j, max(mt, 1) - 1)) * 16 + li;
            const int pc = pix < q1 ? pix : q1 - 1;
            const int ho = pc / p.Wo, wo = pc - ho * p.Wo;
            lbj[j] = 16 + (((ho - ho0) * p.stride) * wp + wo * p.stride) * ps;
        }
        float bv[RUN];
        load_bias<T, NT>(p, min(c0 + q * RUN, p.Cout - 1), bv, op.bcount, err);
        f32x4 acc[LP_MT][NT];
#pragma unroll
        for (int j = 0; j < LP_MT; ++j)
#pragma unroll
            for (int i = 0; i < NT; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int wrow0 = (wn * 16 * NT + li) * wpitch + q * 16;   // LDS row of MFMA tile 0 for this lane
        for (int c = 0; c < nchunks; ++c) {
            const bool more = c + 1 < nchunks;
            if (more) wload(c + 1, wr);
            const char* wb = (c & 1) ? wbuf1 : wbuf0;
            const int ks0 = c * kcs, ks1 = min(nks, ks0 + kcs);
            if (active) {
                for (int ks = ks0; ks < ks1; ++ks) {
                    const int ko = koff[ks * 4 + q];
                    uint4 b[NT];
#pragma unroll
                    for (int i = 0; i < NT; ++i)
                        b[i] = *reinterpret_cast<const uint4*>(wb + wrow0 + i * 16 * wpitch + (ks - ks0) * 64);
#pragma unroll
                    for (int j = 0; j < LP_MT; ++j) {
                        if (j < mt) {   // wave-uniform
                            const uint4 a = *reinterpret_cast<const uint4*>(lds + (ko < 0 ? 0 : lbj[j] + ko));
#pragma unroll
                            for (int i = 0; i < NT; ++i) Mma<T>::step(acc[j][i], &b[i], &a);
                        }
                    }
                }
            }
            if (more) wstore((c & 1) ? wbuf0 : wbuf1, wr);
            __syncthreads();
        }
        if (tr && q0 == p0) tr[4] = __builtin_amdgcn_s_memrealtime();
        if (!active) continue;
        const int co = c0 + q * RUN;
#pragma unroll
        for (int j = 0; j < LP_MT; ++j) {
            const int pix = (mb + j) * 16 + li;
            if (j < mt && pix < q1 && co < p.Cout) conv_store<T, NT>(p, R, outo, reso, pix, co, acc[j], bv, plain);
        }
    }
}

// ---------------------------------------------------------------- depthwise 3x3
// One thread item = one pixel x 8 channels of this workgroup's pixel range
// (dwconv3x3 in conv.hip, nets/nn.py:248,250). All nine taps are loaded before
// any is used (out-of-image taps read zeros: adding w*0 to the fp32 sum leaves it
// bit-identical to skipping the tap, as dwconv3x3 does).
template <typename T>
__device__ __forceinline__ void dw_op(const DwArgs& p, __amdgpu_buffer_rsrc_t R, const void* base, int n, int p0, int p1,
                                      bool plain) {
    const int cpp = p.C / 8, HW = p.H * p.W;
    const int ino = boff(p.in, base) + n * (HW * p.ldi * 2);
    const int outo = boff(p.out, base) + n * (HW * p.ldo * 2);
    const int items = (p1 - p0) * cpp;
    for (int it = threadIdx.x; it < items; it += LP_T) {
        const int px = p0 + it / cpp, c0 = (it % cpp) * 8;
        const int h = px / p.W, w = px - h * p.W;
        uint4 tap[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const int hi = h - 1 + k / 3, wi = w - 1 + k % 3;
            const bool ok = ((unsigned)hi < (unsigned)p.H) & ((unsigned)wi < (unsigned)p.W);
            tap[k] = ld16(R, ok ? ino + ((hi * p.W + wi) * p.ldi + c0) * 2 : OFF_NONE);
        }
        float acc[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            float f[8];
            u4_to_f<T>(tap[k], f);
            const float* wt = p.w + k * p.C + c0;
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[e] = fmaf(ldgf(wt + e), f[e], acc[e]);
        }
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            float v = acc[e] + ldgf(p.bias + c0 + e);
            if (p.act == ACT_SILU) v = silu<T>(v);
            o[e] = v;
        }
        st16(R, outo + (px * p.ldo + c0) * 2, f_to_u4<T>(o), plain);
    }
}

// ---------------------------------------------------------------- SPPF max-pool
// One 5x5 / stride 1 / pad 2 max-pool (-inf padding) from concat slice `step`
// into slice step+1 (maxpool5 in misc.hip, nets/nn.py:90-94). The 25 taps of a
// row of 5 are loaded together; out-of-image taps are masked out of the max.
template <typename T>
__device__ __forceinline__ void pool_op(const PoolArgs& p, int step, __amdgpu_buffer_rsrc_t R, const void* base, int n, int p0,
                                        int p1, bool plain) {
    const int cpp = p.C / 8, HW = p.H * p.W;
    const int img = boff(p.buf, base) + n * (HW * p.ldc * 2);
    const int src = img + step * p.C * 2, dst = img + (step + 1) * p.C * 2;
    const int items = (p1 - p0) * cpp;
    for (int it = threadIdx.x; it < items; it += LP_T) {
        const int px = p0 + it / cpp, c0 = (it % cpp) * 8;
        const int h = px / p.W, w = px - h * p.W;
        float mx[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) mx[e] = -INFINITY;
#pragma unroll
        for (int dh = -2; dh <= 2; ++dh) {
            const int hi = h + dh;
            uint4 row[5];
            bool ok[5];
#pragma unroll
            for (int dw = -2; dw <= 2; ++dw) {
                const int wi = w + dw;
                ok[dw + 2] = ((unsigned)hi < (unsigned)p.H) & ((unsigned)wi < (unsigned)p.W);
                row[dw + 2] = ld16(R, ok[dw + 2] ? src + ((hi * p.W + wi) * p.ldc + c0) * 2 : OFF_NONE);
            }
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                float f[8];
                u4_to_f<T>(row[k], f);
#pragma unroll
                for (int e = 0; e < 8; ++e) mx[e] = ok[k] ? fmaxf(mx[e], f[e]) : mx[e];
            }
        }
        st16(R, dst + (px * p.ldc + c0) * 2, f_to_u4<T>(mx), plain);
    }
}

// ---------------------------------------------------------------- PSA attention
template <typename T> struct Mma16L;
template <> struct Mma16L<__bf16> {
    static __device__ __forceinline__ f32x4 step(s16x4 a, s16x4 b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
    }
};
template <> struct Mma16L<_Float16> {
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

// One wave = 16 queries of one head (psa_attention_mfma in misc.hip), then the
// positional dwconv pe(v) + bias of those 16 pixels (pe_add), all in registers.
template <typename T>
__device__ __forceinline__ void attn_tile(const AttnArgs& p, __amdgpu_buffer_rsrc_t R, const void* base, int n, int head, int q0,
                          T* vl, int lane, bool plain) {
    const int g = lane >> 4, li = lane & 15;
    const int per = 2 * ADK + ADH;
    const int qkv = boff(p.qkv, base) + n * (p.T * p.ldq * 2) + head * per * 2;
    const int q = q0 + li;
    const uint4 qf = ld16(R, q < p.T ? qkv + (q * p.ldq + 8 * g) * 2 : OFF_NONE);
    f32x4 o[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) o[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float mrun = -INFINITY, lrun = 0.f;
    for (int kb = 0; kb < p.T; kb += 16) {
        const int key = kb + li;
        const uint4 kf = ld16(R, key < p.T ? qkv + (key * p.ldq + ADK + 8 * g) * 2 : OFF_NONE);
        uint4 vv[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int c = lane + 64 * h, kr = c >> 3, ch = c & 7;
            vv[h] = ld16(R, kb + kr < p.T ? qkv + ((kb + kr) * p.ldq + 2 * ADK + ch * 8) * 2 : OFF_NONE);
        }
        f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
        Mma<T>::step(s, &kf, &qf);
        float sv[4], mx = -INFINITY;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            sv[r] = (kb + 4 * g + r < p.T) ? s[r] * p.scale : -INFINITY;
            mx = fmaxf(mx, sv[r]);
        }
        mx = fmaxf(mx, __shfl_xor(mx, 16));
        mx = fmaxf(mx, __shfl_xor(mx, 32));
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
        ps += __shfl_xor(ps, 16);
        ps += __shfl_xor(ps, 32);
        lrun = lrun * corr + ps;
        mrun = mnew;
#pragma unroll
        for (int t = 0; t < 4; ++t) o[t] *= corr;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int c = lane + 64 * h;
            *reinterpret_cast<uint4*>(vl + (c >> 3) * ADH + (c & 7) * 8) = vv[h];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const s16x4 a = lds_tr16(vl + (4 * g + (li >> 2)) * ADH + 16 * t + 4 * (li & 3));
            o[t] = Mma16L<T>::step(a, pb, o[t]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
    }
    if (q >= p.T) return;
    // epilogue: O rounded to T (the stored attention output), then pe_add's
    // arithmetic: + pe_b, then the 3x3 depthwise taps over v in (kh, kw) order.
    const float inv = 1.0f / lrun;
    const int C = p.heads * ADH;
    const int hq = q / p.Ws, wq = q - hq * p.Ws;
    float acc[4][4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int c = head * ADH + 16 * t + 4 * g + r;
            acc[t][r] = fromf_round<T>(o[t][r] * inv) + ldgf(p.pe_b + c);
        }
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
        const int hi = hq - 1 + kh;
        if (hi < 0 || hi >= p.Hs) continue;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
            const int wi = wq - 1 + kw;
            if (wi < 0 || wi >= p.Ws) continue;
            const int vrow = qkv + ((hi * p.Ws + wi) * p.ldq + 2 * ADK) * 2;
            const float* wt = p.pe_w + (kh * 3 + kw) * C + head * ADH;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const uint2 v2 = ld8(R, vrow + (16 * t + 4 * g) * 2);
                const T* vt = reinterpret_cast<const T*>(&v2);
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[t][r] = fmaf(ldgf(wt + 16 * t + 4 * g + r), tof(vt[r]), acc[t][r]);
            }
        }
    }
    const int outo = boff(p.out, base) + ((n * p.T + q) * p.ldo + head * ADH) * 2;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        T ov[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) ov[r] = fromf<T>(acc[t][r]);
        st8(R, outo + (16 * t + 4 * g) * 2, *reinterpret_cast<const uint2*>(ov), plain);
    }
}

// ---------------------------------------------------------------- program
template <typename T>
__global__ __launch_bounds__(LP_T) void level_program(const LevelArgs a, const LevelOp* __restrict__ ops) {
    __shared__ int ktab[KTAB_MAX];
    __shared__ __attribute__((aligned(16))) T vlds[LP_W][16 * ADH];
    extern __shared__ __attribute__((aligned(16))) char patch_lds[];
    const int b = blockIdx.x, xcd = b & 7, slot = b >> 3;
    const int cl = (slot / a.G) * 8 + xcd, member = slot % a.G;
    unsigned* cnt = a.bar + cl * 64;
    unsigned* gen = cnt + 32;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const __amdgpu_buffer_rsrc_t R = make_rsrc(a.base);
    // Placement check: do all members of this cluster run on one XCD?
    __shared__ int s_plain;
    {
        unsigned* xcc_slot = a.bar + 32 * 64 + cl * 32;
        if (threadIdx.x == 0)
            __hip_atomic_store(xcc_slot + member, __builtin_amdgcn_s_getreg((3 << 11) | 20) & 0xfu, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        cluster_barrier(cnt, gen, a.G, a.err);
        if (threadIdx.x == 0) {
            const unsigned x0 = __hip_atomic_load(xcc_slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            int same = a.plain_ok;
            for (int m = 1; m < a.G; ++m)
                same &= __hip_atomic_load(xcc_slot + m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == x0;
            s_plain = same;
        }
        __syncthreads();
    }
    const bool plain = s_plain != 0;
    const int npass = (a.B + a.NC - 1) / a.NC;
    for (int pass = 0; pass < npass; ++pass) {
        const int n = pass * a.NC + cl;
        const bool live = n < a.B;
        for (int oi = 0; oi < a.nops; ++oi) {
            // The descriptor is copied into registers: read through the pointer, every
            // field use after a (buffer) store would be reloaded from memory.
            const LevelOp* opp = ops + oi;
            const int kind = opp->kind;
            unsigned long long* tr = (a.trace && blockIdx.x == 0 && threadIdx.x == 0 && pass == 0) ? a.trace + 8 * oi : nullptr;
            if (tr) tr[1] = __builtin_amdgcn_s_memrealtime();
            if (live && !((a.skip >> kind) & 1)) {
                if (kind == LOP_CONV) {
                    LevelOp op;
                    op.kind = kind; op.nt = opp->nt; op.patch = opp->patch; op.pstride = opp->pstride;
                    op.wp = opp->wp; op.band = opp->band; op.wn = opp->wn;
                    op.kcs = opp->kcs; op.wpitch = opp->wpitch; op.woff = opp->woff; op.pc = opp->pc;
                    op.wcount = opp->wcount; op.bcount = opp->bcount;
                    op.c = opp->c;
                    const ConvArgs& c = op.c;
                    const int kc8 = c.Kp / 8;
                    const int P = c.Ho * c.Wo, npt = (P + 15) / 16;
                    if (op.patch) {
                        for (int i = threadIdx.x; i < KTAB_MAX; i += LP_T) {
                            int ko = -1;
                            if (i < kc8) {
                                const int e = ldgi(c.ktab + i);
                                const int kh = e >> 24, kw = (e >> 16) & 0xff, ci = e & 0xffff;
                                ko = ci == 0xffff ? -1 : (kh * op.wp + kw) * op.pstride + ci * 2;
                            }
                            ktab[i] = ko;
                        }
                        // the cluster is split pm (pixel ranges) x pc (cout chunk ranges)
                        const int pc = op.pc, pm = a.G / pc, mp = member / pc, mc = member - mp * pc;
                        const int nchall = (c.Cout + 16 * op.nt - 1) / (16 * op.nt);
                        const int ch0 = mc * nchall / pc, ch1 = (mc + 1) * nchall / pc;
                        const int p0 = mp * npt / pm * 16, p1 = min(P, (mp + 1) * npt / pm * 16);
                        if (tr) tr[2] = __builtin_amdgcn_s_memrealtime();
                        if (p1 > p0 && ch1 > ch0) {
                            if (op.nt == 4) conv_patch<T, 4>(op, R, a.base, n, p0, p1, ch0, ch1, ktab, patch_lds, wave, lane, tr, a.err, plain);
                            else if (op.nt == 2) conv_patch<T, 2>(op, R, a.base, n, p0, p1, ch0, ch1, ktab, patch_lds, wave, lane, tr, a.err, plain);
                            else conv_patch<T, 1>(op, R, a.base, n, p0, p1, ch0, ch1, ktab, patch_lds, wave, lane, tr, a.err, plain);
                        }
                    } else {
                        for (int i = threadIdx.x; i < KTAB_MAX; i += LP_T) ktab[i] = i < kc8 ? ldgi(c.ktab + i) : 0xffff;
                        __syncthreads();
                        const int t0 = member * npt / a.G, t1 = (member + 1) * npt / a.G;
                        if (op.nt == 4) conv_op<T, 4>(c, R, a.base, n, t0, t1, ktab, wave, lane, plain);
                        else if (op.nt == 2) conv_op<T, 2>(c, R, a.base, n, t0, t1, ktab, wave, lane, plain);
                        else conv_op<T, 1>(c, R, a.base, n, t0, t1, ktab, wave, lane, plain);
                    }
                } else if (kind == LOP_DW) {
                    const DwArgs d = opp->d;
                    const int P = d.H * d.W, npt = (P + 15) / 16;
                    const int p0 = member * npt / a.G * 16, p1 = min(P, (member + 1) * npt / a.G * 16);
                    dw_op<T>(d, R, a.base, n, p0, p1, plain);
                } else if (kind == LOP_POOL) {
                    const PoolArgs pl = opp->pl;
                    const int step = opp->step;
                    const int P = pl.H * pl.W, npt = (P + 15) / 16;
                    const int p0 = member * npt / a.G * 16, p1 = min(P, (member + 1) * npt / a.G * 16);
                    pool_op<T>(pl, step, R, a.base, n, p0, p1, plain);
                } else {
                    const AttnArgs at = opp->at;
                    const int qt = (at.T + 15) / 16, tasks = at.heads * qt;
                    for (int tk = member * LP_W + wave; tk < tasks; tk += a.G * LP_W)
                        attn_tile<T>(at, R, a.base, n, tk / qt, (tk % qt) * 16, vlds[wave], lane, plain);
                }
            }
            if (tr) tr[5] = __builtin_amdgcn_s_memrealtime();
            // Ops that only read their own pixels of data this workgroup wrote need no
            // cluster barrier: its own stores drained + a workgroup barrier suffice.
            if (oi + 1 < a.nops && ops[oi + 1].sync) {   // uniform
                cluster_barrier(cnt, gen, a.G, a.err);
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
            }
            if (tr) tr[6] = __builtin_amdgcn_s_memrealtime();
        }
    }
}

}  // namespace

int launch_level(int dtype, const LevelArgs& a, hipStream_t s) {
    if (a.NC % 8 != 0 || a.G <= 0 || a.nops <= 0) return (int)hipErrorInvalidValue;
    const dim3 grid(a.NC * a.G);
    // dynamic LDS limit = per-workgroup opt-in maximum minus the kernel's static LDS
    static int max_dyn = -1;
    if (max_dyn < 0) {
        int dev = 0, optin = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&optin, hipDeviceAttributeSharedMemPerBlockOptin, dev) != hipSuccess)
            return (int)hipErrorInvalidValue;
        hipFuncAttributes fa16{}, fa16b{};
        if (hipFuncGetAttributes(&fa16, reinterpret_cast<const void*>(&level_program<_Float16>)) != hipSuccess ||
            hipFuncGetAttributes(&fa16b, reinterpret_cast<const void*>(&level_program<__bf16>)) != hipSuccess)
            return (int)hipErrorInvalidValue;
        const int st = (int)(fa16.sharedSizeBytes > fa16b.sharedSizeBytes ? fa16.sharedSizeBytes : fa16b.sharedSizeBytes);
        max_dyn = optin - st;
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(&level_program<_Float16>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, max_dyn) != hipSuccess ||
            hipFuncSetAttribute(reinterpret_cast<const void*>(&level_program<__bf16>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, max_dyn) != hipSuccess) {
            max_dyn = 0;
            return (int)hipErrorInvalidValue;
        }
    }
    if (a.lds_patch > max_dyn) return (int)hipErrorInvalidValue;
    switch (dtype) {
        case F16: hipLaunchKernelGGL((level_program<_Float16>), grid, dim3(LP_T), a.lds_patch, s, a, a.ops); break;
        case BF16: hipLaunchKernelGGL((level_program<__bf16>), grid, dim3(LP_T), a.lds_patch, s, a, a.ops); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

int level_ktab_max() { return KTAB_MAX - 8 * LP_D; }   // max Kp/8 of a fused conv

}  // namespace yh
