// conv_rw: the dense 3x3 conv (nets/nn.py:28-39 Conv, s 1 / 2, fused bias + SiLU, the
// Residual add of nn.py:49) with the layer's weights resident in VGPRs. Kind 2 of the
// conv_mx plan family: same canonical K order (conv_mx.h), so bit-identical to every
// other plan of a layer and freely chosen by the per-shape tuner.
//
// Why another structure (profiles/r02_conv_ablation.txt): in conv_mx /
// conv_mxr every wave streams its own patch stage by stage with one stage in flight, and
// the weights occupy most of the LDS, so patch DMA, MFMA and epilogue ran in series.
// Here the weights of a wave's 32 couts live in its VGPRs for the whole launch (Cin <= 64:
// at most 36 k-steps x 4 VGPRs), which frees the whole LDS for a ring of NS patch slots
// SHARED by the workgroup:
//   * one persistent workgroup of NW = NCG x NPG waves per CU walks a strided stream of
//     output tiles (TH x TW pixels of one image, all couts of its slice); wave (cg, pg)
//     owns cout group cg (32 couts) and MB 32-pixel B tiles of pixel group pg;
//   * a slot holds a tile's whole input patch (every input channel, full 128-B pixel lines
//     for Cin = 64), filled by LDS-DMA (global_load_lds_dwordx4) by all waves; the slots
//     of the next NS-1 tiles are in flight while a tile is multiplied;
//   * per tile: counted vmcnt (the wave's own DMA of this tile landed; later DMAs and the
//     previous tiles' stores stay in flight) -> one barrier -> issue the DMA of tile
//     it + NS - 1 into the slot the previous tile freed -> MFMAs -> epilogue;
//   * layers with a residual (RES) bring the tile's residual values into the same slot by
//     LDS-DMA, so the loop issues no VGPR-destination loads at all: hipcc then inserts no
//     vmcnt wait of its own (a wait for a register load would also drain the patch DMAs
//     issued before it, in order);
//   * the epilogue's 16-B stores are buffer instructions issued by every lane for every
//     pixel (out-of-image pixels get an offset past the buffer's range, which the
//     hardware drops), so the vmcnt arithmetic is exact.
#include "conv_mx.h"
#include "dtypes.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

#ifndef RW_PF
#define RW_PF 1   // B-fragment prefetch distance of the MFMA loop, in k-steps
#endif


namespace yh {

typedef __attribute__((ext_vector_type(16))) float rw_f32x16;
typedef __attribute__((ext_vector_type(4))) unsigned int rw_u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int rw_u32x2;
typedef __attribute__((ext_vector_type(2))) float rw_f32x2;

RwGeo rw_geo(int S, int cin, int ncg, int npg, int mb, int tw, bool res, int nkc) {
    RwGeo g;
    g.nw = ncg * nkc * npg;
    g.cpp = cin / 8;
    g.nks = cin / 16 * 9;   // the whole K walk (the packed image); a wave runs nks / nkc steps
    g.tpx = npg * mb * 32;
    g.th = g.tpx / tw;
    g.pr = S * (g.th - 1) + 3;
    g.pc = S * (tw - 1) + 3;
    g.nbi = (g.pr * g.pc * g.cpp + 64 * g.nw - 1) / (64 * g.nw);
    g.nbr = res ? (g.tpx * ncg * 4 + 64 * g.nw - 1) / (64 * g.nw) : 0;
    g.slot = (g.nbi + g.nbr) * g.nw * 1024;
    // K-split layers: every chunk's fp32 partial tile in LDS (the reduction and the epilogue
    // are shared by the chunk waves); otherwise one 32-pixel x 32-cout staging tile per wave for
    // the coalesced epilogue. + the slice's bias, + the counter mode's slot counters (2 x 8 words)
    g.red = nkc > 1 ? nkc * ncg * npg * mb * 4096 : 0;
    g.epi = (nkc > 1 ? 0 : ncg * npg * 2048) + ncg * 128 + 64;
    return g;
}

// ablation switches of the micro benchmark (tools/micro, -DYH_ABLATION); off in the shipped
// library: dbg 4 no MFMA, 8 no epilogue stores, 16 no K-chunk reduction and no epilogue; trace = per-workgroup stamps (entry, prologue done,
// first tile done, exit)
#ifdef YH_ABLATION
#define RW_DBG(bit) (p.dbg & (bit))
#define RW_TRACE (p.trace)
#else
#define RW_DBG(bit) 0
#define RW_TRACE ((unsigned long long*)nullptr)
#endif

namespace {

constexpr unsigned RW_OOB = 0x7ffffff0u;         // buffer offset past every valid byte: dropped
constexpr int RW_NUM_RECORDS = 0x7ffffff0;

__device__ __forceinline__ void rw_glds(const void* src, unsigned lds_addr) {
#if defined(__HIP_DEVICE_COMPILE__)
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds_addr) : "memory");
#else
    (void)src; (void)lds_addr;
#endif
}

template <int N>
__device__ __forceinline__ void rw_vmwait() {
    static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits");
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory");
}

__device__ __forceinline__ void rw_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}

// counter mode: wait (bounded) until the LDS word at p reaches target. Returns false if the
// bound ran out: the caller then poisons its tile with NaN, so a stalled hand-off shows up as
// wrong outputs every test catches, not as a silent race (and not as a hang or a trap)
__device__ __forceinline__ bool rw_spin(const unsigned* p, unsigned target) {
    for (int k = 0; k < (1 << 22); ++k) {
        const unsigned v = __builtin_amdgcn_readfirstlane(*reinterpret_cast<const volatile unsigned*>(p));
        if (v >= target) return true;
        __builtin_amdgcn_s_sleep(1);
    }
    return false;
}
__device__ __forceinline__ void rw_signal(unsigned* p, int lane) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's LDS reads of the slot are done
    if (lane == 0) __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// LDS column of patch column pcol (and back): stride 2 stores a row's even columns first
template <int S, int PC>
__host__ __device__ constexpr int rw_lcol(int pcol) {
    return S == 2 ? ((pcol & 1) ? (PC + 1) / 2 + (pcol >> 1) : (pcol >> 1)) : pcol;
}
template <int S, int PC>
__host__ __device__ constexpr int rw_gcol(int lcol) {
    return S == 2 ? (lcol < (PC + 1) / 2 ? 2 * lcol : 2 * (lcol - (PC + 1) / 2) + 1) : lcol;
}

__device__ __forceinline__ uint32_t rw_fdiv(uint32_t x, FastDiv d) {
    return (uint32_t)(((uint64_t)__umulhi(x, d.m) + x) >> d.s);
}

template <typename T> struct RwMfma;
template <> struct RwMfma<__bf16> {
    static __device__ __forceinline__ rw_f32x16 step(const uint4& a, const uint4& b, const rw_f32x16& c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                       0, 0);
    }
};
template <> struct RwMfma<_Float16> {
    static __device__ __forceinline__ rw_f32x16 step(const uint4& a, const uint4& b, const rw_f32x16& c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                      0);
    }
};

template <typename T> struct RwPk2;
template <> struct RwPk2<__bf16> { typedef __attribute__((ext_vector_type(2))) __bf16 v2; };
template <> struct RwPk2<_Float16> { typedef __attribute__((ext_vector_type(2))) _Float16 v2; };
template <typename T>
__device__ __forceinline__ unsigned rw_pack2(float a, float b) {
    return __builtin_bit_cast(unsigned, __builtin_convertvector(rw_f32x2{a, b}, typename RwPk2<T>::v2));
}
template <typename T>
__device__ __forceinline__ float rw_lo(unsigned u) { return (float)__builtin_bit_cast(T, (unsigned short)(u & 0xffffu)); }
template <typename T>
__device__ __forceinline__ float rw_hi(unsigned u) { return (float)__builtin_bit_cast(T, (unsigned short)(u >> 16)); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rw_rsrc(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, RW_NUM_RECORDS, 0x00020000);
}

}  // namespace

// CM (counter mode, NKC = 1): no workgroup barrier per tile. Tile it + NS - 2 is issued at
// iteration it into the slot tile it - 2 used, once every wave has signalled it done with that
// tile (LDS counter); a wave starts tile it once every wave has signalled its pieces of tile it
// landed. Waves may drift up to a tile apart: the second half of the waves starts half a tile
// late, so on each SIMD one wave's epilogue (VALU: SiLU, the staging, the stores) runs beside
// the other's MFMAs instead of after them. Same arithmetic, same bits.
template <typename T, int S, int CIN, int NCG, int NPG, int MB, int TW, int NS, bool RES, int NKC, bool CM>
__global__ __launch_bounds__(64 * NCG * NKC * NPG, (NCG * NKC * NPG >= 8 || NCG > 1 || CIN <= 32) ? 2 : 1) void conv_rw(
    const MxArgs p) {
    constexpr int NW = NCG * NKC * NPG;
    constexpr int CPP = CIN / 8;                 // 16-B chunks per input pixel
    constexpr int NKT = CIN / 16 * 9;            // k-steps of the whole walk (canonical: cb, then tap)
    constexpr int NKS = NKT / NKC;               // k-steps of a wave's K chunk
    constexpr int CBC = CIN / 16 / NKC;          // 16-channel blocks per K chunk
    constexpr int TPX = NPG * MB * 32;
    constexpr int TH = TPX / TW;
    constexpr int PR = S * (TH - 1) + 3, PC = S * (TW - 1) + 3;
    constexpr int NBI = (PR * PC * CPP + 64 * NW - 1) / (64 * NW);
    constexpr int RCH = NCG * 4;                 // residual chunks per pixel (the slice's couts)
    constexpr int RSH = NCG == 1 ? 2 : NCG == 2 ? 1 : 0;   // residual image swizzle: chunk ^ (px >> RSH)
    constexpr int NBR = RES ? (TPX * RCH + 64 * NW - 1) / (64 * NW) : 0;
    constexpr int SLOT = (NBI + NBR) * NW * 1024;
    constexpr int RED = NKC > 1 ? NKC * NCG * NPG * MB * 4096 : 0;   // K-chunk partials (rw_geo's red)
    constexpr int EST = NKC > 1 ? 0 : NCG * NPG * 2048;              // epilogue staging tiles (NKC = 1)
    static_assert(TPX % TW == 0 && (CPP & (CPP - 1)) == 0 && NS >= 2 && NKT % NKC == 0, "rw geometry");
    // VMEM ops a wave issues after its DMAs of tile it, still uncounted at the wait of
    // iteration it: the epilogues of the NS-1 earlier tiles (NKC = 1: 2 stores per B tile;
    // K-split: 4 / NKC per B tile from every chunk wave) and the DMAs of NS-2 tiles
    constexpr int SPT = NKC > 1 ? MB * (4 / NKC) : 2 * MB;
    constexpr int CNT0 = (NS - 1) * SPT + (NS - 2) * (NBI + NBR);
    static_assert(NKC == 1 || NKC == 2 || NKC == 4, "K chunks");
    static_assert(CNT0 <= 63, "vmcnt range");
    // counter mode: tiles issued D = NS - 2 ahead; at the wait for tile it's DMA, the wave has
    // issued since then the DMAs of D - 1 tiles and the stores of D epilogues
    constexpr int DPC = NS - 2;
    constexpr int CNTP = DPC * 2 * MB + (DPC - 1) * (NBI + NBR);
    static_assert(!CM || (NKC == 1 && NS >= 3 && CNTP <= 63), "counter mode geometry");

    const unsigned long long t_entry = RW_TRACE ? __builtin_amdgcn_s_memrealtime() : 0ull;
    extern __shared__ __attribute__((aligned(1024))) uint4 sm4[];
    typedef __attribute__((address_space(3))) uint4* lds_p;
    const unsigned lds0 = (unsigned)(size_t)(lds_p)sm4;
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int cg = wv % NCG, kc = (wv / NCG) % NKC, pg = wv / (NCG * NKC);
    const int h = lane >> 5, r32 = lane & 31;

    // workgroup -> (cout slice, stream of tiles); the nslices workgroups of one tile are
    // adjacent (same XCD under round-robin dispatch: the patch's second read hits L2)
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int wps = gridDim.x / p.nslices;
    const int lw = L / p.nslices, sl = L - lw * p.nslices;
    const int ntile = p.ntasks;
    const int n_it = lw < ntile ? (ntile - lw + wps - 1) / wps : 0;
    if (n_it == 0) return;   // workgroup-uniform

    const int sw_sh = p.sw_sh, sw_mr = p.sw_mr;
    auto swz = [&](int prow, int pcol) { return ((pcol >> sw_sh) + prow * sw_mr) & (CPP - 1); };

    // ---- patch fill slots of this lane (tile independent): packed prow | pcol << 8, and
    //      the byte offset of the source chunk from the tile's tap-(0,0) pixel. A stride-2 patch
    //      row is stored de-interleaved (its even columns, then its odd ones: rw_lcol), so a tap's
    //      32 B-fragment pixels are consecutive in LDS as at stride 1; otherwise every 16-lane
    //      group of a ds_read_b128 hit 8 of the 16 bank slots (2-way conflicts on every read)
    int fgeo[NBI], foff[NBI];
#pragma unroll
    for (int i = 0; i < NBI; ++i) {
        const int q = (i * NW + wv) * 64 + lane;
        const int ppix = q / CPP, cs = q & (CPP - 1);
        const int prow = ppix / PC, lcol = ppix - prow * PC;
        const int pcol = rw_gcol<S, PC>(lcol);
        const int c = cs ^ swz(prow, lcol);
        fgeo[i] = ppix < PR * PC ? (prow | (pcol << 8)) : -1;
        foff[i] = (prow * p.Wi + pcol) * p.ldc0 * 2 + c * 16;
    }
    // ---- B fragment chunk index per (tap, B tile) in a slot, and the epilogue pixel
    int bidx[9][MB], pty[MB], ptx[MB];
#pragma unroll
    for (int j = 0; j < MB; ++j) {
        const int px = (pg * MB + j) * 32 + r32;
        pty[j] = px / TW;
        ptx[j] = px % TW;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int prow = S * pty[j] + t / 3, pcol = S * ptx[j] + t % 3;
            // the wave's K chunk starts at block kc * CBC: its chunk bits are folded in here,
            // so the k-step loop XORs compile-time block offsets only
            const int lcol = rw_lcol<S, PC>(pcol);
            bidx[t][j] = ((prow * PC + lcol) * CPP + (h ^ swz(prow, lcol))) ^ (2 * kc * CBC);
        }
    }

    // ---- residual fill slots: tile pixel, chunk within the slice's couts (stored at
    //      chunk ^ (px >> RSH) of the pixel's RCH chunks: conflict-free epilogue reads)
    int rgeo[NBR > 0 ? NBR : 1];
#pragma unroll
    for (int i = 0; i < NBR; ++i) {
        const int q = (i * NW + wv) * 64 + lane;
        const int px = q / RCH, cs = q & (RCH - 1);
        rgeo[i] = px < TPX ? ((px << 4) | (cs ^ ((px >> RSH) & (RCH - 1)))) : -1;
    }

    auto tile_pos = [&](int it, int& n, int& ty0, int& tx0) {
        const int t = lw + it * wps;
        const uint32_t b = rw_fdiv((uint32_t)t, p.d_ntw);
        tx0 = (t - (int)b * p.ntw) * TW;
        const uint32_t c = rw_fdiv(b, p.d_nth);
        ty0 = ((int)b - (int)c * p.nth) * TH;
        n = (int)c;
    };
    // DMA of tile `it`'s patch into slot `slot` (zeros past the stream's end, so every
    // iteration issues the same number of DMAs)
    auto issue = [&](int it, int slot) {
        const unsigned sb = lds0 + (unsigned)(slot * SLOT) + (unsigned)wv * 1024u;
        if (it < n_it) {
            int n, ty0, tx0;
            tile_pos(it, n, ty0, tx0);
            const int gy0 = S * ty0 - 1, gx0 = S * tx0 - 1;
            const char* base = p.in0 + (((long long)n * p.Hi + gy0) * p.Wi + gx0) * p.ldc0 * 2;
#pragma unroll
            for (int i = 0; i < NBI; ++i) {
                const int g = fgeo[i];
                const int gy = gy0 + (g & 255), gx = gx0 + ((g >> 8) & 255);
                const bool ok = g >= 0 && (unsigned)gy < (unsigned)p.Hi && (unsigned)gx < (unsigned)p.Wi;
                rw_glds(ok ? (const void*)(base + foff[i]) : (const void*)p.zero, sb + (unsigned)(i * NW * 1024));
            }
            if constexpr (RES) {
                const int cbase = (sl * NCG) * 64;   // byte offset of the slice's couts
#pragma unroll
                for (int i = 0; i < NBR; ++i) {
                    const int g = rgeo[i];
                    const int px = g >> 4, c = g & 15;
                    const int oy = ty0 + px / TW, ox = tx0 + px % TW;
                    const bool ok = g >= 0 && oy < p.Ho && ox < p.Wo;
                    const char* src = p.res + (((long long)n * p.Ho + oy) * p.Wo + ox) * p.ldr * 2 + cbase + c * 16;
                    rw_glds(ok ? (const void*)src : (const void*)p.zero, sb + (unsigned)((NBI + i) * NW * 1024));
                }
            }
        } else {
#pragma unroll
            for (int i = 0; i < NBI + NBR; ++i) rw_glds(p.zero, sb + (unsigned)(i * NW * 1024));
        }
    };

    // ---- prologue: the weights and bias, and the first NS-1 tiles' patches in flight.
    //      With several pixel groups (NPG > 1) NPG waves need each cout group's image: the
    //      workgroup's images (NCG x NKT KB) come by LDS-DMA once into the (still idle) slot
    //      ring and every wave reads its fragments from there, instead of NPG reads of each
    //      image from L2 (r04 micro bench, box.0.0 shape: a 5 us setup, 75 MB of L2 reads per
    //      launch against 37 MB of patches); the first patches are issued after that.
    constexpr bool WLDS = NPG > 1 && NCG * NKT * 1024 <= NS * SLOT;
    const int co0 = (sl * NCG + cg) * 32;
    uint4 wf[NKS];
    if constexpr (WLDS) {
        // the images go to the END of the ring: the first tiles whose slots lie below them are
        // issued before the images, the others once every wave holds its fragments
        constexpr int NQ = NCG * NKT;
        constexpr int WOFF = NS * SLOT - NQ * 1024;
        constexpr int EARLY = WOFF / SLOT < NS - 1 ? WOFF / SLOT : NS - 1;
        for (int k = 0; k < EARLY; ++k) issue(k, k);
        const char* wimg = p.w + (long long)(sl * NCG) * NKT * 1024;
        // every workgroup starts at another 1 KB piece: the 256 workgroups do not all read the
        // same lines at the same moment
        const int rot = (int)(blockIdx.x % NQ);
        for (int q0 = wv; q0 < NQ; q0 += NW) {
            const int q = q0 + rot < NQ ? q0 + rot : q0 + rot - NQ;
            rw_glds(wimg + ((long long)q * 64 + lane) * 16, lds0 + (unsigned)(WOFF + q * 1024));
        }
        rw_vmwait<0>();
        rw_barrier();
        const char* wl = reinterpret_cast<const char*>(sm4) + WOFF + ((cg * NKT + kc * NKS) * 64 + lane) * 16;
#pragma unroll
        for (int s = 0; s < NKS; ++s) wf[s] = *reinterpret_cast<const uint4*>(wl + s * 1024);
        rw_barrier();   // every wave holds its fragments: the rest of the ring may be filled
        for (int k = EARLY; k < NS - 1; ++k) issue(k, k);
    } else {
        for (int k = 0; k < NS - 1; ++k) issue(k, k);
        const char* wsrc = p.w + ((long long)(sl * NCG + cg) * NKT * 64 + kc * NKS * 64 + lane) * 16;
#pragma unroll
        for (int s = 0; s < NKS; ++s) wf[s] = *reinterpret_cast<const uint4*>(wsrc + (long long)s * 1024);
    }
    // the slice's bias in LDS (read per B tile in the epilogue: 16 VGPRs free for the fragment
    // prefetch ring)
    float* bias_l = reinterpret_cast<float*>(reinterpret_cast<char*>(sm4) + NS * SLOT + RED + EST);
    if ((int)threadIdx.x < NCG * 32) bias_l[threadIdx.x] = p.bias[(sl * NCG) * 32 + threadIdx.x];
    // the compiler waits for these loads HERE (not at their first use inside the loop,
    // where its vmcnt(0) would drain the patch ring every iteration)
#pragma unroll
    for (int s = 0; s < NKS; ++s) asm volatile("" :: "v"(wf[s].x), "v"(wf[s].y), "v"(wf[s].z), "v"(wf[s].w));
    // counter mode: landed[NS] then done[NS], zeroed before the barrier below
    unsigned* cnt = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(sm4) + NS * SLOT + RED + EST + NCG * 128);
    if (CM && (int)threadIdx.x < 2 * NS) cnt[threadIdx.x] = 0u;
    rw_vmwait<0>();
    rw_barrier();
    const unsigned long long t_setup = RW_TRACE ? __builtin_amdgcn_s_memrealtime() : 0ull;
    unsigned long long t_first = 0ull;

    const __amdgpu_buffer_rsrc_t ro = rw_rsrc(p.out);
    const bool silu_act = p.act == ACT_SILU;

    rw_f32x16 acc[MB];
    // ---- epilogue (chunk-0 waves): bias, activation, one rounding (the conv output), the
    //      residual added in fp32 and rounded again (nets/nn.py:49). The wave's 32 pixels x
    //      32 couts go through its private LDS staging tile (lane (r32, h) writes its 16
    //      couts, 4 lanes per pixel read 64 contiguous bytes back: every store instruction
    //      writes 16 pixels x 64 B instead of 32 pixels x 2 x 16 B; conv_mx.hip co_stage)
    auto epilogue = [&](int it) {
        int n, ty0, tx0;
        tile_pos(it, n, ty0, tx0);
        char* E = reinterpret_cast<char*>(sm4) + NS * SLOT + RED + (pg * NCG + cg) * 2048;
        const int qr = lane & 3, pr0 = lane >> 2;
        float bv[16];
#pragma unroll
        for (int e = 0; e < 16; e += 4) {
            const float4 b4 = *reinterpret_cast<const float4*>(bias_l + cg * 32 + 16 * h + e);
            bv[e] = b4.x; bv[e + 1] = b4.y; bv[e + 2] = b4.z; bv[e + 3] = b4.w;
        }
#pragma unroll
        for (int j = 0; j < MB; ++j) {
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                unsigned w[4];
#pragma unroll
                for (int e = 0; e < 8; e += 2) {
                    float x0 = acc[j][8 * c + e] + bv[8 * c + e], x1 = acc[j][8 * c + e + 1] + bv[8 * c + e + 1];
                    if (silu_act) {
                        x0 = silu<T>(x0);
                        x1 = silu<T>(x1);
                    }
                    w[e >> 1] = rw_pack2<T>(x0, x1);
                }
                const int q = 2 * h + c;
                *reinterpret_cast<uint4*>(E + (r32 * 4 + (q ^ ((r32 >> 1) & 3))) * 16) = make_uint4(w[0], w[1], w[2], w[3]);
            }
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int pp = k * 16 + pr0;
                const uint4 v = *reinterpret_cast<const uint4*>(E + (pp * 4 + (qr ^ ((pp >> 1) & 3))) * 16);
                unsigned w[4] = {v.x, v.y, v.z, v.w};
                const int px = (pg * MB + j) * 32 + pp;
                const int oy = ty0 + px / TW, ox = tx0 + px % TW;
                const bool ok = oy < p.Ho && ox < p.Wo;
                const long long m = ((long long)n * p.Ho + oy) * p.Wo + ox;
                if constexpr (RES) {
                    const int f = (px >> RSH) & (RCH - 1);
                    const char* rb = reinterpret_cast<const char*>(sm4) + (it % NS) * SLOT + NBI * NW * 1024 + px * RCH * 16;
                    const uint4 r = *reinterpret_cast<const uint4*>(rb + ((cg * 4 + qr) ^ f) * 16);
                    const unsigned rv[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        w[q] = rw_pack2<T>(rw_lo<T>(w[q]) + rw_lo<T>(rv[q]), rw_hi<T>(w[q]) + rw_hi<T>(rv[q]));
                }
                const unsigned oo = ok ? (unsigned)(m * p.ldo * 2) + (unsigned)(co0 + 8 * qr) * 2u : RW_OOB;
                const unsigned od = RW_DBG(8) ? RW_OOB : oo;
                __builtin_amdgcn_raw_buffer_store_b128(rw_u32x4{w[0], w[1], w[2], w[3]}, ro, od, 0, 0);
            }
        }
    };
    // ---- K-split epilogue: the NKC chunk waves of a (cg, pg) tile share the reduction and the
    //      epilogue. Every chunk's fp32 partials sit in LDS ([chunk][pg][cg][j] tiles: 32 pixel
    //      rows of 8 16-B chunks of 4 couts, chunk c of pixel p at c ^ (p & 7)); wave kc takes
    //      pixels kc * 32 / NKC .. of each B tile, lane (pixel, 4-cout chunk c4) sums its four
    //      couts in chunk order (((P0 + P1) + P2) + P3: the canonical order), adds the bias,
    //      activates, rounds (+ residual, rounded again) and stores 8 B; 8 lanes write a
    //      pixel's 64 contiguous bytes.
    auto red_tile = [&](int k2, int j) {
        return reinterpret_cast<float*>(reinterpret_cast<char*>(sm4) + NS * SLOT) +
               (((k2 * NPG + pg) * NCG + cg) * MB + j) * 1024;
    };
    auto epilogue_split = [&](int it) {
        int n, ty0, tx0;
        tile_pos(it, n, ty0, tx0);
        constexpr int PPW = 32 / NKC, NR = PPW / 8;
        const int c4 = lane & 7;
        const float4 bv = *reinterpret_cast<const float4*>(bias_l + cg * 32 + 4 * c4);
#pragma unroll
        for (int j = 0; j < MB; ++j) {
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const int pp = kc * PPW + r * 8 + (lane >> 3);
                const int off = pp * 32 + (c4 ^ (pp & 7)) * 4;
                float4 v = *reinterpret_cast<const float4*>(red_tile(0, j) + off);
#pragma unroll
                for (int k2 = 1; k2 < NKC; ++k2) {
                    const float4 u = *reinterpret_cast<const float4*>(red_tile(k2, j) + off);
                    v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
                }
                float x0 = v.x + bv.x, x1 = v.y + bv.y, x2 = v.z + bv.z, x3 = v.w + bv.w;
                // selects, not a branch: one basic block the scheduler can spread between MFMAs
                x0 = silu_act ? silu<T>(x0) : x0;
                x1 = silu_act ? silu<T>(x1) : x1;
                x2 = silu_act ? silu<T>(x2) : x2;
                x3 = silu_act ? silu<T>(x3) : x3;
                unsigned w[2] = {rw_pack2<T>(x0, x1), rw_pack2<T>(x2, x3)};
                const int px = (pg * MB + j) * 32 + pp;
                const int oy = ty0 + px / TW, ox = tx0 + px % TW;
                const bool ok = oy < p.Ho && ox < p.Wo;
                const long long m = ((long long)n * p.Ho + oy) * p.Wo + ox;
                if constexpr (RES) {
                    const int f = (px >> RSH) & (RCH - 1);
                    const char* rb = reinterpret_cast<const char*>(sm4) + (it % NS) * SLOT + NBI * NW * 1024 + px * RCH * 16;
                    const uint2 rr = *reinterpret_cast<const uint2*>(rb + ((cg * 4 + (c4 >> 1)) ^ f) * 16 + (c4 & 1) * 8);
                    const unsigned rv[2] = {rr.x, rr.y};
#pragma unroll
                    for (int q = 0; q < 2; ++q)
                        w[q] = rw_pack2<T>(rw_lo<T>(w[q]) + rw_lo<T>(rv[q]), rw_hi<T>(w[q]) + rw_hi<T>(rv[q]));
                }
                const unsigned oo = ok ? (unsigned)(m * p.ldo * 2) + (unsigned)(co0 + 4 * c4) * 2u : RW_OOB;
                const unsigned od = RW_DBG(8) ? RW_OOB : oo;
                __builtin_amdgcn_raw_buffer_store_b64(rw_u32x2{w[0], w[1]}, ro, od, 0, 0);
            }
        }
    };
    // K-split layers without a residual run tile it - 1's epilogue in iteration it, beside tile
    // it's MFMAs (the partials wait in LDS; the residual would sit in a slot the ring has already
    // re-filled). Iteration 0 issues the same number of stores to the dropped offset, so the
    // vmcnt arithmetic (CNT0) holds from the first iteration on.
    constexpr bool DEFER = NKC > 1 && !RES && !CM;
    auto dummy_stores = [&]() {
        constexpr int NR = 32 / NKC / 8;
#pragma unroll
        for (int k = 0; k < MB * NR; ++k) __builtin_amdgcn_raw_buffer_store_b64(rw_u32x2{0u, 0u}, ro, RW_OOB, 0, 0);
    };
    unsigned long long t_wait = 0ull;   // diagnostic builds, dbg 64: time spent in the loop-top waits
    if constexpr (CM) {
        // the prologue issued tiles 0 .. NS - 2; tiles 0 .. DPC - 1 are the ones this loop expects
        // (issue distance DPC): the remaining one (NS - 2) is also in flight, counted like the rest
        if (wv >= NW / 2) {   // the second half of the waves starts half a tile late
#pragma unroll 1
            for (int k = 0; k < p.pc_delay; ++k) __builtin_amdgcn_s_sleep(32);
        }
    }
    bool stalled = false;   // counter mode: a hand-off wait ran out (rw_spin)
    for (int it = 0; it < n_it; ++it) {
        if constexpr (CM) {
            const int sl_it = it % NS;
            if (it >= NS - 1) {
                // tiles past the prologue's: this wave's pieces landed, then everyone's (the count
                // of slot sl_it's tiles from NS - 1 on, this one included)
                const int first = sl_it == NS - 1 ? NS - 1 : sl_it + NS;
                rw_vmwait<CNTP>();
                rw_signal(cnt + sl_it, lane);
                stalled |= !rw_spin(cnt + sl_it, (unsigned)(NW * ((it - first) / NS + 1)));
            }
            if (it >= 1) {
                // tile it + NS - 2 into the slot tile it - 2 used, once every wave is done with it
                // (tile NS - 1, issued at it = 1, takes the ring's unused last slot)
                if (it >= 2) stalled |= !rw_spin(cnt + NS + (it - 2) % NS, (unsigned)(NW * ((it - 2) / NS + 1)));
                issue(it + NS - 2, (it + NS - 2) % NS);
            }
        } else if (it > 0) {
            const unsigned long long tw0 = (RW_TRACE && RW_DBG(64)) ? __builtin_amdgcn_s_memrealtime() : 0ull;
            rw_vmwait<CNT0>();
            rw_barrier();   // tile it complete in its slot; slot (it - 1) % NS read by every wave
            if (RW_TRACE && RW_DBG(64)) t_wait += __builtin_amdgcn_s_memrealtime() - tw0;
            if (RW_TRACE && it == 1) t_first = __builtin_amdgcn_s_memrealtime();
        }
        if constexpr (!CM) issue(it + NS - 1, (it + NS - 1) % NS);
        if constexpr (DEFER) {
            if (it > 0) epilogue_split(it - 1);
            else dummy_stores();
        }

        // ---- MFMAs: one k-step = one 32x32x16 step per B tile, fragments of step s+1
        //      read while step s multiplies
        {
            const char* Bp = reinterpret_cast<const char*>(sm4) + (it % NS) * SLOT;
            auto rd = [](const char* q) { return *reinterpret_cast<const uint4*>(__builtin_assume_aligned(q, 16)); };
            // B fragments read RW_PF k-steps ahead (a ring of RW_PF + 1): one ds_read_b128 feeds
            // one 32-cycle MFMA, shorter than the read's latency
            constexpr int PF = RW_PF, RING = RW_PF + 1;
            uint4 bf[RING][MB];
            auto load = [&](int s, int buf) {
                const int cb = s / 9, t = s - (s / 9) * 9;
#pragma unroll
                for (int j = 0; j < MB; ++j) bf[buf][j] = rd(Bp + (bidx[t][j] ^ (2 * cb)) * 16);
            };
#pragma unroll
            for (int j = 0; j < MB; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
#pragma unroll
            for (int s = 0; s < PF && s < NKS; ++s) load(s, s % RING);
            __builtin_amdgcn_sched_group_barrier(0x100, MB * (PF < NKS ? PF : NKS), 0);
#pragma unroll
            for (int s = 0; s < NKS; ++s) {
                if (s + PF < NKS) load(s + PF, (s + PF) % RING);
                if (RW_DBG(4)) continue;
#pragma unroll
                for (int j = 0; j < MB; ++j) acc[j] = RwMfma<T>::step(wf[s], bf[s % RING][j], acc[j]);
                if (s + PF < NKS) __builtin_amdgcn_sched_group_barrier(0x100, MB, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, MB, 0);
            }
        }

        if constexpr (CM) {
            if (stalled) {
#pragma unroll
                for (int j = 0; j < MB; ++j)
#pragma unroll
                    for (int e = 0; e < 16; ++e) acc[j][e] = __builtin_nanf("");
            }
        }
        if (RW_DBG(16)) continue;   // ablation: no K-chunk reduction, no epilogue
        // ---- K chunks: every chunk wave's partial tile to LDS (lane (r32, h) holds couts
        //      16 h .. 16 h + 15 of pixel r32: 4 swizzled 16-B chunks), then the shared epilogue
        if constexpr (NKC > 1) {
            if constexpr (DEFER) rw_barrier();   // every wave's epilogue reads of tile it - 1 are done
#pragma unroll
            for (int j = 0; j < MB; ++j) {
                float* t = red_tile(kc, j) + r32 * 32;
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    *reinterpret_cast<float4*>(t + (((4 * h + q) ^ (r32 & 7)) * 4)) =
                        make_float4(acc[j][4 * q], acc[j][4 * q + 1], acc[j][4 * q + 2], acc[j][4 * q + 3]);
            }
            if constexpr (!DEFER) {
                rw_barrier();
                epilogue_split(it);
            }
        } else {
            epilogue(it);
        }
        if constexpr (CM) rw_signal(cnt + NS + it % NS, lane);
    }
    if constexpr (DEFER) {
        rw_barrier();   // the last tile's partials
        epilogue_split(n_it - 1);
    }
    if (RW_TRACE && threadIdx.x == 0) {
        unsigned long long* tr = RW_TRACE + blockIdx.x * 4;
        tr[0] = t_entry; tr[1] = t_setup; tr[2] = t_first ? t_first : t_setup; tr[3] = __builtin_amdgcn_s_memrealtime();
        if (RW_DBG(64)) tr[2] = t_setup + t_wait;   // "first" column = the summed loop-top waits
    }
}

// ------------------------------------------------------------------ host side
namespace {

// extra LDS cycles of the B-fragment reads of one wave over a whole tile (ds_read_b128
// lane groups, 16-B slots of a 256-B bank row), for swizzle f = ((lcol >> sh) + prow mr) & (cpp-1)
int rw_conflicts(const RwGeo& g, int S, int tw, int mb, int npg, int sh, int mr) {
    static const int grp[4][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                                   {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
                                   {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
                                   {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
    const int cpp = g.cpp, ncb = cpp / 2;
    int total = 0;
    for (int pgi = 0; pgi < npg; ++pgi)
        for (int j = 0; j < mb; ++j)
            for (int t = 0; t < 9; ++t)
                for (int cb = 0; cb < ncb; ++cb)
                    for (int q = 0; q < 4; ++q) {
                        int cnt[16] = {0};
                        long long seen[16][16];
                        for (int u = 0; u < 16; ++u) {
                            const int lane = grp[q][u], h = lane >> 5, r = lane & 31;
                            const int px = (pgi * mb + j) * 32 + r;
                            const int prow = S * (px / tw) + t / 3, pcol = S * (px % tw) + t % 3;
                            // the kernel's LDS column (rw_lcol: stride 2 de-interleaves a patch row)
                            const int lcol = S == 2 ? ((pcol & 1) ? (g.pc + 1) / 2 + (pcol >> 1) : (pcol >> 1)) : pcol;
                            const int f = ((lcol >> sh) + prow * mr) & (cpp - 1);
                            const long long a = ((long long)(prow * g.pc + lcol) * cpp + ((2 * cb + h) ^ f)) * 16;
                            const int slot = (int)((a / 16) & 15);
                            bool dup = false;
                            for (int k = 0; k < cnt[slot]; ++k) dup |= seen[slot][k] == a;
                            if (!dup) seen[slot][cnt[slot]++] = a;
                        }
                        int mx = 0;
                        for (int s = 0; s < 16; ++s) mx = std::max(mx, cnt[s]);
                        total += mx - 1;
                    }
    return total;
}

}  // namespace

MxPlan mx_plan_w(const MxShape& sh, const MxConfig& c, int num_cus) {
    MxPlan pl;
    pl.cfg = c;
    if (sh.ks != 3 || c.ks != 3 || sh.s != c.s || sh.c1 != 0 || sh.up0 != 0) return pl;
    // a wave keeps 64 input channels' weights (36 k-steps) at most: wider layers are K-split
    if (c.ncb * 16 != sh.cin || c.nkc != mx_kchunks(sh) || sh.cin / c.nkc > 64) return pl;
    if (!(sh.cin / c.nkc == 16 || sh.cin / c.nkc == 32 || sh.cin / c.nkc == 64)) return pl;
    const int ncg = c.na, npg = c.wm, bn = 32 * ncg;
    if (sh.cout % bn) return pl;
    // 32-bit buffer offsets: every byte the epilogue addresses below 2^31
    const double M = (double)sh.B * sh.Ho * sh.Wo;
    const int ldo = sh.ldo > 0 ? sh.ldo : sh.cout, ldr = sh.ldr > 0 ? sh.ldr : sh.cout;
    if (M * std::max(ldo, ldr) * 2.0 + 64 > (double)RW_NUM_RECORDS) return pl;
    const bool res = sh.ldr > 0;
    const RwGeo g = rw_geo(sh.s, sh.cin, ncg, npg, c.mb, c.tw, res, c.nkc);
    if (g.tpx % c.tw || g.th < 1 || (res && sh.s != 1)) return pl;
    pl.TW = c.tw; pl.TH = g.th;
    pl.PR = g.pr; pl.PC = g.pc;
    pl.bc_log2 = 0;
    pl.nbi = g.nbi;
    pl.ains = g.nbr;   // conv_rw: residual DMA instructions per wave and tile
    pl.nst = 1;
    pl.nslices = sh.cout / bn;
    pl.ntw = (sh.Wo + c.tw - 1) / c.tw;
    pl.nth = (sh.Ho + g.th - 1) / g.th;
    pl.ntasks = sh.B * pl.ntw * pl.nth;
    pl.bbytes = g.slot;
    pl.abytes = 0;
    pl.lds = c.nbuf * g.slot + g.red + g.epi;
    if (pl.lds > 160 * 1024 || g.nw > 16) return pl;
    pl.wstage = pl.nslices * ncg * g.nks * 1024;   // packed weight bytes
    int best = 1 << 30, bsh = 0, bmr = 0;
    for (int s2 = 0; s2 <= 4; ++s2)
        for (int mr = 0; mr < g.cpp; ++mr) {
            const int cf = rw_conflicts(g, sh.s, c.tw, c.mb, npg, s2, mr);
            if (cf < best) { best = cf; bsh = s2; bmr = mr; }
        }
    pl.sw_sh = bsh; pl.sw_mr = bmr; pl.conflicts = best;
    // every kernel keeps <= 256 VGPRs (2 waves per SIMD): 4-wave workgroups run two per CU where
    // the LDS allows, so each SIMD's two waves come from different workgroups and drift apart
    // (one's epilogue / barrier wait beside the other's MFMAs); 8-wave ones run one per CU
    const bool two = g.nw == 4 && (ncg > 1 || sh.cin <= 32);   // (the 1-cout-group Cin 64 kernel needs > 256)
    const int per_cu = std::max(1, std::min((160 * 1024) / pl.lds, two ? 2 : 1));
    // every wave loads its cout group's whole weight image: fewer, longer-lived workgroups
    // (gdiv) trade parallelism for weight traffic on small layers
    const int wps = std::max(1, std::min(pl.ntasks, per_cu * num_cus / pl.nslices) / std::max(1, c.gdiv));
    pl.grid = wps * pl.nslices;
    pl.ok = true;
    return pl;
}

void mx_candidates_w(const MxShape& sh, std::vector<MxConfig>& out) {
    if (sh.ks != 3 || sh.c1 != 0 || sh.up0 != 0 || sh.cout % 32) return;
    const int nkc = mx_kchunks(sh);
    if (!(sh.cin == 16 || sh.cin == 32 || sh.cin == 64 || nkc > 1)) return;
    // small layers (fewer tiles than 2 per CU) also get the grid halved and quartered
    const bool small = (double)sh.B * sh.Ho * sh.Wo < 2.0 * 256 * 64;
    auto add = [&](int ncg, int npg, int mb, int tw, int ns, int pc = 0) {
        MxConfig c{};
        c.kind = 2; c.ks = 3; c.s = sh.s; c.na = ncg; c.mb = mb; c.wn = ncg; c.wm = npg; c.ncb = sh.cin / 16;
        c.tw = tw; c.nbuf = ns; c.nkc = nkc; c.pc = pc;
        for (int gd : {1, 2, 4}) {
            if (gd > 1 && !small) break;
            c.gdiv = gd;
            out.push_back(c);
        }
    };
    const int ncg = sh.cout % 64 == 0 ? 2 : 1;
    // the instantiated set (launch_rw_cfg)
    if (nkc > 1) {
        if (sh.s == 1 && sh.cin == 128) {
            add(2, 2, 1, 8, 3); add(2, 1, 1, 8, 3); add(2, 1, 1, 8, 4);
            if (sh.cout % 128 == 0) add(4, 1, 1, 8, 3);
        } else if (sh.s == 1 && sh.cin == 256) {
            add(2, 1, 1, 8, 3); add(2, 1, 1, 4, 3);
        } else if (sh.s == 2 && sh.cin == 128) {
            add(2, 2, 1, 8, 2); add(2, 1, 1, 8, 3);
            if (sh.cout % 128 == 0) add(4, 1, 1, 8, 3);
        }
    } else if (sh.s == 1) {
        if (sh.cin == 64 && ncg == 2) {
            add(2, 4, 1, 16, 4); add(2, 4, 1, 8, 4); add(2, 2, 1, 8, 4); add(2, 2, 1, 4, 4); add(2, 2, 1, 8, 3);
            // counter mode (YH_RW_CM=1 only: bit-identical, measured slower, r05 micro bench box0.0:
            // 26.8-27.5 us against 25.5 us for the barrier ring)
            if (getenv("YH_RW_CM")) { add(2, 4, 1, 16, 4, 1); add(2, 4, 1, 16, 5, 1); add(2, 4, 1, 8, 4, 1); }
        } else if (sh.cin == 64 && ncg == 1) {
            add(1, 8, 1, 16, 3); add(1, 4, 1, 8, 4);
        } else if (sh.cin == 32 && ncg == 1) {
            add(1, 4, 1, 8, 4); add(1, 8, 1, 16, 4);
        } else if (sh.cin == 32 && ncg == 2) {
            add(2, 2, 1, 8, 4); add(2, 4, 1, 16, 4);
        }
    } else if (sh.cin == 64 && ncg == 2) {
        add(2, 2, 1, 8, 3); add(2, 4, 1, 16, 2);
        if (getenv("YH_RW_CM")) add(2, 2, 1, 8, 3, 1);
        // 128 couts in one workgroup: the patch is read once, not once per 64-cout slice
        if (sh.cout % 128 == 0) { add(4, 2, 1, 8, 3); add(4, 1, 1, 8, 4); }
    }
}

std::vector<uint16_t> mx_pack_w(const MxPlan& pl, const MxShape& sh, const float* wf, int cin_logical,
                                const std::vector<int>& phys2log, bool bf16, int cout_logical) {
    const int ncg = pl.cfg.na, nks = sh.cin / 16 * 9;
    std::vector<uint16_t> out((size_t)pl.wstage / 2, 0);
    for (int sl = 0; sl < pl.nslices; ++sl)
        for (int g = 0; g < ncg; ++g)
            for (int s = 0; s < nks; ++s)
                for (int lane = 0; lane < 64; ++lane) {
                    const int R = lane & 31, hh = lane >> 5;
                    // row permutation: lane half h of the accumulator holds couts 16h .. 16h+15
                    const int co = (sl * ncg + g) * 32 + 16 * ((R >> 2) & 1) + (R & 3) + 4 * (R >> 3);
                    const int cb = s / 9, tap = s % 9;
                    for (int e = 0; e < 8; ++e) {
                        const int ci = cb * 16 + hh * 8 + e;
                        if (co >= sh.cout || co >= cout_logical || ci >= (int)phys2log.size()) continue;
                        const int cl = phys2log[ci];
                        if (cl < 0) continue;
                        const float v = wf[((size_t)co * cin_logical + cl) * 9 + tap];
                        uint32_t u;
                        std::memcpy(&u, &v, 4);
                        uint16_t hv;
                        if (bf16) {
                            hv = ((u & 0x7fffffffu) > 0x7f800000u) ? (uint16_t)((u >> 16) | 0x40)
                                                                  : (uint16_t)((u + 0x7fffu + ((u >> 16) & 1)) >> 16);
                        } else {
                            _Float16 f16 = (_Float16)v;
                            std::memcpy(&hv, &f16, 2);
                        }
                        out[(((size_t)(sl * ncg + g) * nks + s) * 64 + lane) * 8 + e] = hv;
                    }
                }
    return out;
}

namespace {

template <typename T, int S, int CIN, int NCG, int NPG, int MB, int TW, int NS, bool RES, int NKC, bool CM = false>
int launch_rw_t(const MxPlan& pl, const MxArgs& a, hipStream_t s) {
    const RwGeo g = rw_geo(S, CIN, NCG, NPG, MB, TW, RES, NKC);
    if (g.nbi != pl.nbi || NS * g.slot + g.red + g.epi != pl.lds || RES != (a.res != nullptr)) return (int)hipErrorInvalidValue;
    static bool attr = false;
    auto k = &conv_rw<T, S, CIN, NCG, NPG, MB, TW, NS, RES, NKC, CM>;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        attr = true;
    }
    hipLaunchKernelGGL(k, dim3(pl.grid), dim3(64 * NCG * NKC * NPG), pl.lds, s, a);
    return (int)hipGetLastError();
}

template <typename T>
int launch_rw_cfg(const MxPlan& pl, const MxArgs& a, hipStream_t s) {
    const MxConfig& c = pl.cfg;
#define YH_RW(S_, CIN_, NCG_, NPG_, MB_, TW_, NS_, NKC_)                                                    \
    if (c.s == S_ && c.ncb * 16 == CIN_ && c.na == NCG_ && c.wm == NPG_ && c.mb == MB_ && c.tw == TW_ &&     \
        c.nbuf == NS_ && c.nkc == NKC_ && c.pc == 0) {                                                       \
        if (S_ == 1 && a.res) return launch_rw_t<T, S_, CIN_, NCG_, NPG_, MB_, TW_, NS_, (S_ == 1), NKC_>(pl, a, s); \
        return launch_rw_t<T, S_, CIN_, NCG_, NPG_, MB_, TW_, NS_, false, NKC_>(pl, a, s);                     \
    }
#define YH_RWP(S_, CIN_, NCG_, NPG_, MB_, TW_, NS_)                                                          \
    if (c.s == S_ && c.ncb * 16 == CIN_ && c.na == NCG_ && c.wm == NPG_ && c.mb == MB_ && c.tw == TW_ &&     \
        c.nbuf == NS_ && c.nkc == 1 && c.pc == 1) {                                                          \
        if (S_ == 1 && a.res) return launch_rw_t<T, S_, CIN_, NCG_, NPG_, MB_, TW_, NS_, (S_ == 1), 1, true>(pl, a, s); \
        return launch_rw_t<T, S_, CIN_, NCG_, NPG_, MB_, TW_, NS_, false, 1, true>(pl, a, s);                   \
    }
    // counter mode (pc = 1)
    YH_RWP(1, 64, 2, 4, 1, 16, 4)
    YH_RWP(1, 64, 2, 4, 1, 16, 5)
    YH_RWP(1, 64, 2, 4, 1, 8, 4)
    YH_RWP(2, 64, 2, 2, 1, 8, 3)
#undef YH_RWP
    YH_RW(1, 64, 2, 4, 1, 16, 4, 1)
    YH_RW(1, 64, 2, 4, 1, 8, 4, 1)
    YH_RW(1, 64, 2, 2, 1, 8, 4, 1)
    YH_RW(1, 64, 2, 2, 1, 4, 4, 1)
    YH_RW(1, 64, 2, 2, 1, 8, 3, 1)
    YH_RW(1, 64, 1, 8, 1, 16, 3, 1)
    YH_RW(1, 64, 1, 4, 1, 8, 4, 1)
    YH_RW(1, 32, 1, 4, 1, 8, 4, 1)
    YH_RW(1, 32, 1, 8, 1, 16, 4, 1)
    YH_RW(1, 32, 2, 2, 1, 8, 4, 1)
    YH_RW(1, 32, 2, 4, 1, 16, 4, 1)
    YH_RW(2, 64, 2, 2, 1, 8, 3, 1)
    YH_RW(2, 64, 2, 4, 1, 16, 2, 1)
    YH_RW(2, 64, 4, 2, 1, 8, 3, 1)
    YH_RW(2, 64, 4, 1, 1, 8, 4, 1)
    // K-split (mx_kchunks): 128 / 256 input channels, one 64-channel chunk per wave
    YH_RW(1, 128, 2, 2, 1, 8, 3, 2)
    YH_RW(1, 128, 2, 1, 1, 8, 3, 2)
    YH_RW(1, 128, 2, 1, 1, 8, 4, 2)
    YH_RW(1, 128, 4, 1, 1, 8, 3, 2)
    YH_RW(1, 256, 2, 1, 1, 8, 3, 4)
    YH_RW(1, 256, 2, 1, 1, 4, 3, 4)
    YH_RW(2, 128, 2, 2, 1, 8, 2, 2)
    YH_RW(2, 128, 2, 1, 1, 8, 3, 2)
    YH_RW(2, 128, 4, 1, 1, 8, 3, 2)
#undef YH_RW
    return (int)hipErrorInvalidValue;
}

}  // namespace

int launch_rw(int dtype, const MxPlan& pl, const MxArgs& a0, hipStream_t s) {
    MxArgs a = a0;
    // counter mode: how long the second half of the waves starts late (YH_RW_DELAY, read per
    // launch: s_sleep(32) rounds of 2048 cycles)
    const char* e = getenv("YH_RW_DELAY");
    a.pc_delay = e ? std::max(0, atoi(e)) : 1;
    if (dtype == BF16) return launch_rw_cfg<__bf16>(pl, a, s);
    if (dtype == F16) return launch_rw_cfg<_Float16>(pl, a, s);
    return (int)hipErrorInvalidValue;
}

}  // namespace yh
