// conv_mx: dense 1x1 / 3x3 convolution (nets/nn.py:28-39 Conv, fused bias + SiLU,
// Residual add nn.py:49, concat / upsample views nn.py:66-94, 203-209) for the
// 16-bit handles on v_mfma_f32_32x32x16_{bf16,f16}.
//
// Structure (one persistent workgroup of NW waves per task stream):
//   * a task is an output tile of one image (3x3: TH rows x TW cols; 1x1: TW
//     consecutive pixels) times one BN-wide cout slice;
//   * its K walk is cut into stages of NCB 16-channel blocks. A stage brings two
//     LDS images in by LDS-DMA (global_load_lds_dwordx4, 16 B per lane, linear
//     destination): the weight image of the stage (pre-packed in HBM exactly as
//     it lies in LDS) and the input PATCH of the task for those channels (every
//     input pixel the tile's taps touch, with a zero border, once: the 3x3 halo is
//     re-read from LDS, not from L2). Stage g+1 is in flight while stage g is
//     multiplied (two LDS buffers, counted vmcnt, raw s_barrier);
//   * every wave owns NA 32-cout x MB 32-pixel accumulator tiles; each k-step reads
//     NA + MB fragments with ds_read_b128 (weights: row stride odd in 16-B slots;
//     patch: 16-B chunks XOR-swizzled by the stored pixel so the 16 lanes of a
//     read group hit distinct bank slots) and issues NA x MB MFMAs;
//   * the weight rows are permuted at pack time so every lane's accumulators are
//     16*NA CONTIGUOUS output channels: the epilogue (bias, SiLU, rounding,
//     residual) stores 16-B chunks straight from registers.
// Reduction order: see conv_mx.h (for cb16: for tap: one MFMA step).
#include "conv_mx.h"
#include "dtypes.h"

#include <algorithm>
#include <cstring>

namespace yh {

typedef __attribute__((ext_vector_type(16))) float f32x16;

// ablation switches of the micro benchmark (tools/micro, -DYH_ABLATION); constant 0 / off
// in the shipped library
#ifdef YH_ABLATION
#define MX_DBG(bit) (p.dbg & (bit))
#define MX_TRACE (p.trace)
#else
#define MX_DBG(bit) 0
#define MX_TRACE ((unsigned long long*)nullptr)
#endif

namespace {

// 16-byte LDS-DMA hidden from hipcc's waitcnt pass (ordering: the kernel's own
// counted vmcnt + barrier). M0 is saved and restored inside the statement.
__device__ __forceinline__ void mx_glds(const void* src, unsigned lds_addr) {
#if defined(__HIP_DEVICE_COMPILE__)
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds_addr) : "memory");
#else
    (void)src; (void)lds_addr;
#endif
}

__device__ __forceinline__ void mx_vmwait(int n) {
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
        case 17: asm volatile("s_waitcnt vmcnt(17)" ::: "memory"); break;
        case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
        case 19: asm volatile("s_waitcnt vmcnt(19)" ::: "memory"); break;
        case 20: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
        case 21: asm volatile("s_waitcnt vmcnt(21)" ::: "memory"); break;
        case 22: asm volatile("s_waitcnt vmcnt(22)" ::: "memory"); break;
        case 23: asm volatile("s_waitcnt vmcnt(23)" ::: "memory"); break;
        case 24: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}

__device__ __forceinline__ void mx_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}

__device__ __forceinline__ uint32_t fdiv(uint32_t x, FastDiv d) {
    return (uint32_t)(((uint64_t)__umulhi(x, d.m) + x) >> d.s);
}

template <typename T> struct Mfma32;
template <> struct Mfma32<__bf16> {
    static __device__ __forceinline__ f32x16 step(const uint4& a, const uint4& b, const f32x16& c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                       0, 0);
    }
};
template <> struct Mfma32<_Float16> {
    static __device__ __forceinline__ f32x16 step(const uint4& a, const uint4& b, const f32x16& c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                      0);
    }
};

__device__ __forceinline__ uint4 lds_rd(unsigned addr) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef __attribute__((address_space(3))) const uint4* lp;
    return *reinterpret_cast<lp>((size_t)addr);
#else
    (void)addr;
    return uint4{};
#endif
}

}  // namespace


// Epilogue of one 32-pixel B tile of a wave: the lane holds 16*NA consecutive couts
// of its pixel in acc[a][j] (cout 16a + i <-> acc[a][i]). Adds the bias, applies
// SiLU, rounds to T once (the reference's conv output), adds the residual in fp32
// and rounds again (nets/nn.py:49, 135-136), stores 16-B chunks. Only `nc8` chunks
// (couts [8*c8, 8*c8+8) < Cout) are stored; loads are unconditional (callers clamp
// the addresses), so no load is ever left unconsumed.
typedef __attribute__((ext_vector_type(2))) float f32x2;
template <typename T> struct Pk2;
template <> struct Pk2<__bf16> {
    typedef __attribute__((ext_vector_type(2))) __bf16 v2;
};
template <> struct Pk2<_Float16> {
    typedef __attribute__((ext_vector_type(2))) _Float16 v2;
};
template <typename T>
__device__ __forceinline__ unsigned pack2(float a, float b) {
    typedef typename Pk2<T>::v2 v2;
    return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a, b}, v2));
}
template <typename T>
__device__ __forceinline__ float lo16(unsigned u) {
    const unsigned short s = (unsigned short)(u & 0xffffu);
    return (float)__builtin_bit_cast(T, s);
}
template <typename T>
__device__ __forceinline__ float hi16(unsigned u) {
    const unsigned short s = (unsigned short)(u >> 16);
    return (float)__builtin_bit_cast(T, s);
}
template <typename T, int NA, bool SILU, bool RES>
__device__ __forceinline__ void mx_epi(const f32x16 (&acc)[NA], const float* bv, T* outp, const T* resp, int nc8) {
#pragma unroll
    for (int c8 = 0; c8 < 2 * NA; ++c8) {
        unsigned w[4];
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
            const int i0 = c8 * 8 + e, i1 = i0 + 1;
            float x0 = acc[i0 >> 4][i0 & 15] + bv[i0];
            float x1 = acc[i1 >> 4][i1 & 15] + bv[i1];
            if constexpr (SILU) {
                x0 = silu<T>(x0);
                x1 = silu<T>(x1);
            }
            w[e >> 1] = pack2<T>(x0, x1);
        }
        if constexpr (RES) {
            const uint4 r = *reinterpret_cast<const uint4*>(resp + c8 * 8);
            const unsigned rr[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
            for (int q = 0; q < 4; ++q)
                w[q] = pack2<T>(lo16<T>(w[q]) + lo16<T>(rr[q]), hi16<T>(w[q]) + hi16<T>(rr[q]));
        }
        if (c8 < nc8) *reinterpret_cast<uint4*>(outp + c8 * 8) = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

// Coalesced epilogue (tools/micro/access_rate: 16-B stores with one pixel per lane, 32 B of
// each of 32 lines per wave-instruction, write 2.3 TB/s against 4.6 TB/s for whole-line
// instructions, MALL-resident, 3.6 against 5.8-6.1 TB/s to HBM). The wave's 32-pixel x BN-cout
// B tile goes through LDS: each lane writes its pixel's 16*NA couts (bias, activation, one
// rounding done), then reads back LPP = 4*NA lanes per pixel, so every store instruction writes
// 64 / LPP whole pixel rows of BN*2 bytes; the residual is read in the same shape and added after
// the rounding, as in mx_epi (bit-identical). Row slots are XOR-swizzled by the pixel: the
// ds_write_b128 groups of 8 lanes (8 pixels, one chunk) and the ds_read_b128 groups hit
// distinct banks.
template <int NA>
__device__ __forceinline__ int co_swz(int p) { return NA == 1 ? ((p >> 1) & 3) : (p & 7); }

template <typename T, int NA, bool SILU>
__device__ __forceinline__ void co_stage(const f32x16 (&acc)[NA], const float* bv, char* E, int l32, int h) {
    constexpr int LPP = 4 * NA;
#pragma unroll
    for (int c8 = 0; c8 < 2 * NA; ++c8) {
        unsigned w[4];
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
            const int i0 = c8 * 8 + e, i1 = i0 + 1;
            float x0 = acc[i0 >> 4][i0 & 15] + bv[i0];
            float x1 = acc[i1 >> 4][i1 & 15] + bv[i1];
            if constexpr (SILU) {
                x0 = silu<T>(x0);
                x1 = silu<T>(x1);
            }
            w[e >> 1] = pack2<T>(x0, x1);
        }
        const int q = 2 * NA * h + c8;
        *reinterpret_cast<uint4*>(E + (l32 * LPP + (q ^ co_swz<NA>(l32))) * 16) = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

template <typename T>
__device__ __forceinline__ uint4 co_addres(uint4 v, const T* rp) {
    const uint4 r = *reinterpret_cast<const uint4*>(rp);
    const unsigned vv[4] = {v.x, v.y, v.z, v.w}, rr[4] = {r.x, r.y, r.z, r.w};
    unsigned w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) w[q] = pack2<T>(lo16<T>(vv[q]) + lo16<T>(rr[q]), hi16<T>(vv[q]) + hi16<T>(rr[q]));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// One 32-pixel B tile through the wave's staging image E (64 * 32 * NA bytes): stage, read back
// 4*NA lanes per pixel, add the residual, store. bt = B tile index within the task, c0 = first
// cout of the wave's BN-wide block; (n, hh0, ww0) = the task's origin (KS 1: flat pixel ww0).
template <typename T, int NA, int KS>
__device__ __forceinline__ void co_tile(const f32x16 (&aj)[NA], const float* bv, bool silu_act, char* E, int lane,
                                        const MxArgs& p, int n, int hh0, int ww0, int bt, int c0, const T* res, T* out,
                                        bool no_store) {
    constexpr int LPP = 4 * NA, PPI = 64 / LPP;
    const int l32 = lane & 31, h = lane >> 5;
    if (silu_act) co_stage<T, NA, true>(aj, bv, E, l32, h);
    else co_stage<T, NA, false>(aj, bv, E, l32, h);
    const int qr = lane % LPP, pr0 = lane / LPP;
    const int cq = c0 + 8 * qr;
    const bool cq_ok = cq < p.cout;
#pragma unroll
    for (int k = 0; k < 2 * NA; ++k) {
        const int pp = k * PPI + pr0;
        const uint4 v = *reinterpret_cast<const uint4*>(E + (pp * LPP + (qr ^ co_swz<NA>(pp))) * 16);
        long long m;
        bool ok;
        if constexpr (KS == 3) {
            const int bc = 1 << p.bc_log2, btw = p.TW >> p.bc_log2;
            const int btr = bt / btw, btc = bt - btr * btw;
            const int ho = hh0 + btr * (32 >> p.bc_log2) + (pp >> p.bc_log2);
            const int wo = ww0 + btc * bc + (pp & (bc - 1));
            ok = ho < p.Ho && wo < p.Wo;
            m = ((long long)n * p.Ho + ho) * p.Wo + wo;
        } else {
            const int mm = ww0 + bt * 32 + pp;
            ok = mm < p.M;
            m = mm;
        }
        ok = ok && cq_ok;
        if (!ok) m = 0;
        const int cc = ok ? cq : 0;
        uint4 o = v;
        if (res) o = co_addres<T>(v, res + m * p.ldr + cc);
        if (ok && !no_store) *reinterpret_cast<uint4*>(out + m * p.ldo + cc) = o;
    }
}

template <typename T, int KS, int S, int NA, int MB, int WN, int WM, int NCB>
__global__ __launch_bounds__(64 * WN * WM, 2) void conv_mx(const MxArgs p) {
    constexpr int NW = WN * WM, NT = 64 * NW;
    constexpr int CPS = 2 * NCB;              // 16-B chunks per stored patch pixel per stage
    constexpr int TAPS = KS * KS;
    constexpr int RS = 2 * TAPS * NCB + 1;    // weight-row chunks (odd: conflict-free row reads)
    constexpr int BN = 32 * NA * WN;
    constexpr int AINS = (BN * RS + NT - 1) / NT;
    constexpr int ACH = AINS * NT;            // weight chunks per stage buffer
    constexpr int NSTEP = NCB * TAPS;         // MFMA k-steps per stage
    static_assert(sizeof(T) == 2, "16-bit path");
    // all LDS addressing in 16-B chunks from one aligned uint4 array: ds_read_b128
    extern __shared__ __attribute__((aligned(1024))) uint4 sm4[];
    typedef __attribute__((address_space(3))) uint4* lds_p;
    const unsigned lds0 = (unsigned)(size_t)(lds_p)sm4;

    const unsigned long long t_entry = MX_TRACE ? __builtin_amdgcn_s_memrealtime() : 0ull;
    const int nbi = p.nbi;
    const int stage_ch = ACH + nbi * NT;      // chunks per stage buffer
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wn = wv / WM, wm = wv - wn * WM;
    const int h = lane >> 5, l32 = lane & 31;

    // ---- contiguous task range per workgroup, consecutive workgroups of an XCD adjacent
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    const int t_lo = (int)((long long)p.ntasks * L / gridDim.x);
    const int t_hi = (int)((long long)p.ntasks * (L + 1) / gridDim.x);
    const int nstages = (t_hi - t_lo) * p.nst;
    if (nstages <= 0) return;

    // ---- per-lane constants
    const int a_lane = (wn * NA * 32 + l32) * RS + h;   // chunk index of the lane's weight fragment
    const bool gen1 = KS == 1 && (p.up0 | p.up1);       // 1x1 with an upsampled segment: per-task gather
    // fill slots (task independent): packed (rs | wi_rel << 10 | c << 22 | valid << 31) and the
    // byte offset of the slot's source chunk from the task's tap-(0,0) pixel (segment 0 / 1)
    int slot_geo[MX_MAXB], slot_off0[MX_MAXB], slot_off1[MX_MAXB];
#pragma unroll
    for (int i = 0; i < MX_MAXB; ++i) {
        const uint32_t q = (uint32_t)((i * NW + wv) * 64 + lane);
        const uint32_t rs = fdiv(q, p.d_pcc);
        const uint32_t rem = q - rs * (uint32_t)(p.PC * CPS);
        const uint32_t lc = rem / CPS, cpos = rem & (CPS - 1);
        const uint32_t f = ((lc >> p.sw_sh) + rs * p.sw_mr) & (CPS - 1);
        const uint32_t c = cpos ^ f;
        const bool vpos = (int)rs < p.PR && i < nbi;
        uint32_t wrel = lc;
        if constexpr (KS == 3 && S == 2) wrel = (int)lc <= p.TW ? 2 * lc : 2 * (lc - p.TW - 1) + 1;
        slot_geo[i] = vpos ? (int)(rs | (wrel << 10) | (c << 22) | (1u << 31)) : 0;
        slot_off0[i] = ((int)rs * p.Wi + (int)wrel) * p.ldc0 * 2 + (int)c * 16;
        slot_off1[i] = ((int)rs * p.Wi + (int)wrel) * p.ldc1 * 2 + (int)c * 16;
    }
    // B fragment chunk indices per (tap, B tile), buffer-relative; epilogue pixel of each tile
    int bidx[TAPS][MB];
    int pix_r[MB], pix_c[MB];
#pragma unroll
    for (int j = 0; j < MB; ++j) {
        const int bt = wm * MB + j;
        int r, cc;
        if constexpr (KS == 3) {
            const int bc = 1 << p.bc_log2;
            const int btw = p.TW >> p.bc_log2;
            const int btr = bt / btw, btc = bt - btr * btw;
            r = btr * (32 >> p.bc_log2) + (l32 >> p.bc_log2);
            cc = btc * bc + (l32 & (bc - 1));
        } else {
            r = 0;
            cc = bt * 32 + l32;
        }
        pix_r[j] = r;
        pix_c[j] = cc;
#pragma unroll
        for (int t = 0; t < TAPS; ++t) {
            const int kh = t / KS, kw = t - (t / KS) * KS;
            int rs, lc;
            if constexpr (KS == 1) {
                rs = 0; lc = cc;
            } else if constexpr (S == 1) {
                rs = r + kh; lc = cc + kw;
            } else {
                rs = 2 * r + kh;
                lc = kw == 0 ? cc : (kw == 1 ? p.TW + 1 + cc : cc + 1);
            }
            const int f = ((lc >> p.sw_sh) + rs * p.sw_mr) & (CPS - 1);
            bidx[t][j] = (rs * p.PC + lc) * CPS + (h ^ f);
        }
    }

    // ---- fill state (the task whose stages are being issued)
    const char* sptr[MX_MAXB];
    int fill_seg = -1;
    int f_n = 0, f_h0 = 0, f_w0 = 0, f_sl = 0;
    auto decompose = [&](int tk, int& n, int& hh0, int& ww0, int& sl) {
        const uint32_t a = fdiv((uint32_t)tk, p.d_nsl);
        sl = tk - (int)a * p.nslices;
        const uint32_t b = fdiv(a, p.d_ntw);
        const int tw = (int)(a - b * p.ntw);
        if constexpr (KS == 3) {
            const uint32_t c = fdiv(b, p.d_nth);
            const int th = (int)(b - c * p.nth);
            n = (int)c;
            hh0 = th * p.TH;
            ww0 = tw * p.TW;
        } else {
            n = 0; hh0 = 0;
            ww0 = tw * p.TW;   // flat pixel index of the task's first pixel
        }
    };
    // per task: 64-bit source of each slot's chunk (zero page when out of the image)
    auto setup_slots = [&](int seg) {
        const char* base = seg ? p.in1 : p.in0;
        const int ldc = seg ? p.ldc1 : p.ldc0;
        if constexpr (KS == 3) {
            // tap-(0,0) pixel of the task; a slot is inside the image iff its row / col are
            const long long b0 = (((long long)f_n * p.Hi + (S * f_h0 - 1)) * p.Wi + (S * f_w0 - 1)) * ldc * 2;
            const int rlo = 1 - S * f_h0, rhi = p.Hi + 1 - S * f_h0;
            const int clo = 1 - S * f_w0, chi = p.Wi + 1 - S * f_w0;
#pragma unroll
            for (int i = 0; i < MX_MAXB; ++i) {
                const int g = slot_geo[i];
                const int rs = g & 1023, wr = (g >> 10) & 4095;
                const bool ok = g < 0 && rs >= rlo && rs < rhi && wr >= clo && wr < chi;
                sptr[i] = ok ? base + b0 + slot_off0[i] : nullptr;
            }
        } else {
            const int up = seg ? p.up1 : p.up0;
            const int hs = seg ? p.hs1 : p.hs0, ws = seg ? p.ws1 : p.ws0;
#pragma unroll
            for (int i = 0; i < MX_MAXB; ++i) {
                const int g = slot_geo[i];
                const int lc = (g >> 10) & 4095, c = (g >> 22) & 15;
                const int m = f_w0 + lc;
                const bool ok = g < 0 && m < p.M;
                if (!gen1) {
                    sptr[i] = ok ? base + (long long)f_w0 * ldc * 2 + (seg ? slot_off1[i] : slot_off0[i]) : nullptr;
                } else {
                    const uint32_t n = fdiv((uint32_t)m, p.d_howo);
                    const uint32_t rr = (uint32_t)m - n * (uint32_t)(p.Ho * p.Wo);
                    const uint32_t ho = fdiv(rr, p.d_wo);
                    const uint32_t wo = rr - ho * (uint32_t)p.Wo;
                    const long long pix = ((long long)n * hs + (ho >> up)) * ws + (wo >> up);
                    sptr[i] = ok ? base + pix * ldc * 2 + c * 16 : nullptr;
                }
            }
        }
        fill_seg = seg;
    };
    auto issue = [&](int g, int buf) {
        const int tk = t_lo + g / p.nst, st = g - (g / p.nst) * p.nst;
        if (st == 0) {
            decompose(tk, f_n, f_h0, f_w0, f_sl);
            fill_seg = -1;
        }
        const unsigned sbase = lds0 + (unsigned)(buf * stage_ch * 16);
        // weights: contiguous stage image
        if (!MX_DBG(1)) {
            const char* wsrc = p.w + ((long long)f_sl * p.nst + st) * p.wstage + (long long)(wv * 64 + lane) * 16;
#pragma unroll
            for (int i = 0; i < AINS; ++i)
                mx_glds(wsrc + (long long)i * NT * 16, sbase + (unsigned)((i * NW + wv) * 1024));
        }
        // patch
        const int ch0 = st * NCB * 16;
        const int seg = (p.in1 != nullptr && ch0 >= p.c0) ? 1 : 0;
        if (seg != fill_seg) setup_slots(seg);
        const int coff = (seg ? ch0 - p.c0 : ch0) * 2;
        const int clim = (p.cin - ch0) >> 3;   // chunks of this stage inside Cin
        const unsigned bb = sbase + ACH * 16;
        if (!MX_DBG(2)) {
#pragma unroll
            for (int i = 0; i < MX_MAXB; ++i) {
                if (i < nbi) {
                    const int c = (slot_geo[i] >> 22) & 15;
                    const bool ok = sptr[i] != nullptr && c < clim;
                    mx_glds(ok ? (const void*)(sptr[i] + coff) : (const void*)p.zero, bb + (unsigned)((i * NW + wv) * 1024));
                }
            }
        }
    };

    f32x16 acc[NA][MB];
    const int per_stage = (MX_DBG(1) ? 0 : AINS) + (MX_DBG(2) ? 0 : nbi);
    const int co_lane = wn * NA * 32 + 16 * NA * h;   // lane's first cout within the slice

    // one stage: NSTEP k-steps, fragments of step s+1 read while step s multiplies
    auto compute = [&](const int sb) {
        const char* A = reinterpret_cast<const char*>(sm4) + (sb + a_lane) * 16;
        const char* Bp = reinterpret_cast<const char*>(sm4) + (sb + ACH) * 16;
        auto rd = [](const char* q) { return *reinterpret_cast<const uint4*>(__builtin_assume_aligned(q, 16)); };
        uint4 af[2][NA], bf[2][MB];
        auto load = [&](int s, int buf) {
            const int cbl = s / TAPS, t = s - (s / TAPS) * TAPS;
#pragma unroll
            for (int a = 0; a < NA; ++a) af[buf][a] = rd(A + (a * 32 * RS + s * 2) * 16);
#pragma unroll
            for (int j = 0; j < MB; ++j) bf[buf][j] = rd(Bp + (bidx[t][j] ^ (cbl * 2)) * 16);
        };
        load(0, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, NA + MB, 0);
#pragma unroll
        for (int s = 0; s < NSTEP; ++s) {
            if (s + 1 < NSTEP) load(s + 1, (s + 1) & 1);
#pragma unroll
            for (int a = 0; a < NA; ++a)
#pragma unroll
                for (int j = 0; j < MB; ++j) acc[a][j] = Mfma32<T>::step(af[s & 1][a], bf[s & 1][j], acc[a][j]);
            // keep the next step's fragment reads ahead of this step's MFMAs
            if (s + 1 < NSTEP) __builtin_amdgcn_sched_group_barrier(0x100, NA + MB, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, NA * MB, 0);
        }
    };

    // bias of every cout of the layer, staged once in LDS after the two stage buffers
    const int bias_ch = 2 * stage_ch;
    {
        const int nb = p.nslices * BN / 4;   // float4 chunks
        for (int i = threadIdx.x; i < nb; i += NT)
            sm4[bias_ch + i] = *reinterpret_cast<const uint4*>(p.bias + i * 4);
    }

    // Epilogue: bias, activation, rounding, residual, 16-B stores. Branch-free apart from
    // the stores (and the uniform residual switch): every load it issues is consumed on
    // every path, so no load is left in flight across the loop back-edge (hipcc would
    // otherwise wait for it in the next compute phase, draining the prefetch DMA).
    // coalesced epilogue (co_tile): after a barrier every wave has multiplied the last stage, so
    // that stage's buffer (weights + patch) is free until the next iteration issues into it,
    // which is after the barrier that closes this one
    const bool co_fits = NW * 2048 * NA <= stage_ch * 16;   // uniform
    auto epilogue = [&](int tk, int g) {
        int n, hh0, ww0, sl;
        decompose(tk, n, hh0, ww0, sl);
        const int co = sl * BN + co_lane;
        const bool co_ok = co < p.cout;
        float bv[16 * NA];
#pragma unroll
        for (int e = 0; e < 16 * NA; e += 4) {
            const uint4 b4 = sm4[bias_ch + (sl * BN + co_lane + e) / 4];
            bv[e] = __uint_as_float(b4.x); bv[e + 1] = __uint_as_float(b4.y);
            bv[e + 2] = __uint_as_float(b4.z); bv[e + 3] = __uint_as_float(b4.w);
        }
        const T* res = reinterpret_cast<const T*>(p.res);
        T* out = reinterpret_cast<T*>(p.out);
        if (co_fits) {
            mx_barrier();
            char* E = reinterpret_cast<char*>(sm4) + ((g & 1) * stage_ch) * 16 + wv * 2048 * NA;
#pragma unroll
            for (int j = 0; j < MB; ++j) {
                f32x16 aj[NA];
#pragma unroll
                for (int a = 0; a < NA; ++a) aj[a] = acc[a][j];
                co_tile<T, NA, KS>(aj, bv, p.act == ACT_SILU, E, lane, p, n, hh0, ww0, wm * MB + j, sl * BN + wn * NA * 32,
                                   res, out, false);
            }
            return;
        }
#pragma unroll
        for (int j = 0; j < MB; ++j) {
            long long m;
            bool ok;
            if constexpr (KS == 3) {
                const int ho = hh0 + pix_r[j], wo = ww0 + pix_c[j];
                ok = ho < p.Ho && wo < p.Wo;
                m = ((long long)n * p.Ho + ho) * p.Wo + wo;
            } else {
                const int mm = ww0 + pix_c[j];
                ok = mm < p.M;
                m = mm;
            }
            ok = ok && co_ok;
            if (!ok) m = 0;
            const int cc = ok ? co : 0;
            const int nc8 = ok ? min(2 * NA, (p.cout - co) >> 3) : 0;
            f32x16 aj[NA];
#pragma unroll
            for (int a = 0; a < NA; ++a) aj[a] = acc[a][j];
            T* op = out + m * p.ldo + cc;
            const T* rp = res + m * p.ldr + cc;
            if (p.act == ACT_SILU) {
                if (res) mx_epi<T, NA, true, true>(aj, bv, op, rp, nc8);
                else mx_epi<T, NA, true, false>(aj, bv, op, rp, nc8);
            } else {
                if (res) mx_epi<T, NA, false, true>(aj, bv, op, rp, nc8);
                else mx_epi<T, NA, false, false>(aj, bv, op, rp, nc8);
            }
        }
    };

    unsigned long long t_setup = MX_TRACE ? __builtin_amdgcn_s_memrealtime() : 0ull, t_first = 0;
    issue(0, 0);
    for (int g = 0; g < nstages; ++g) {
        const bool more = g + 1 < nstages;
        if (more) issue(g + 1, (g + 1) & 1);
        mx_vmwait(more ? per_stage : 0);
        mx_barrier();
        if (MX_TRACE && g == 0) t_first = __builtin_amdgcn_s_memrealtime();
        const int st = g - (g / p.nst) * p.nst;
        if (st == 0) {
#pragma unroll
            for (int a = 0; a < NA; ++a)
#pragma unroll
                for (int j = 0; j < MB; ++j)
#pragma unroll
                    for (int e = 0; e < 16; ++e) acc[a][j][e] = 0.f;
        }
        if (!(MX_DBG(4))) compute((g & 1) * stage_ch);
        if (st == p.nst - 1 && !(MX_DBG(8))) epilogue(t_lo + g / p.nst, g);
        mx_barrier();
    }
    if (MX_TRACE && threadIdx.x == 0) {
        unsigned long long* tr = MX_TRACE + blockIdx.x * 4;
        tr[0] = t_entry; tr[1] = t_setup; tr[2] = t_first; tr[3] = __builtin_amdgcn_s_memrealtime();
    }
}


// ---------------------------------------------------------------------------
// conv_mxr: the same reduction, for layers whose whole weight slice fits in LDS
// (3x3 with Cin <= 64-128, most 1x1). The workgroup (NW waves, one per CU) loads its
// BN-cout weight slice and bias ONCE; after that single barrier every wave runs its
// own pipeline with no further workgroup synchronisation: it owns a contiguous run of
// wave tiles (MB 32-pixel B tiles), brings each tile's input patch in one 16-channel
// stage group at a time by LDS-DMA into its private double buffer (stage g+1 in flight
// while g multiplies, the wave's own counted vmcnt is the only ordering needed), and
// writes the tile out from registers. The waves drift apart, so one wave's epilogue
// (VALU) overlaps its SIMD partner's MFMAs.
template <typename T, int KS, int S, int NA, int MB, int NCB, int NBI, int NW, int NBUF>
__global__ __launch_bounds__(64 * NW, 2) void conv_mxr(const MxArgs p) {
    constexpr int CPS = 2 * NCB;
    constexpr int TAPS = KS * KS;
    constexpr int BN = 32 * NA;
    constexpr int NSTEP = NCB * TAPS;
    constexpr int BUFCH = NBI * 64;             // chunks per patch buffer
    static_assert(sizeof(T) == 2, "16-bit path");
    extern __shared__ __attribute__((aligned(1024))) uint4 sm4[];
    typedef __attribute__((address_space(3))) uint4* lds_p;
    const unsigned lds0 = (unsigned)(size_t)(lds_p)sm4;

    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, l32 = lane & 31;
    // LDS: [weights: BN rows x rsw chunks, padded to wch] [bias: BN floats] [NW x 2 patch buffers]
    const int rsw = p.nst * NCB * TAPS * 2 + 1;
    const int wch = p.wstage / 16;
    const int bias_ch = wch;
    const int pbuf = bias_ch + BN / 4 + wv * NBUF * BUFCH;

    // ---- workgroup -> (cout slice, run of wave tiles); consecutive workgroups of an XCD adjacent
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    // slice fastest: the nslices workgroups that read the same patches run side by side
    // on one XCD, so all but the first read of a patch hit that XCD's L2
    const int wps = gridDim.x / p.nslices;       // workgroups per slice (grid = nslices * wps)
    const int lw = L / p.nslices, sl = L - lw * p.nslices;
    const int ntile = p.ntasks;                  // wave tiles per slice
    const int gw = lw * NW + wv, GW = wps * NW;
    const int t_lo = (int)((long long)ntile * gw / GW), t_hi = (int)((long long)ntile * (gw + 1) / GW);

    // ---- resident weights + bias
    {
        const char* wsrc = p.w + (long long)sl * p.wstage;
        if (!(MX_DBG(1024)))
            for (int q = wv * 64; q < wch; q += 64 * NW)   // wch: a multiple of 64 chunks
                mx_glds(wsrc + (long long)(q + lane) * 16, lds0 + (unsigned)q * 16);
        if (threadIdx.x < BN / 4)
            sm4[bias_ch + threadIdx.x] = *reinterpret_cast<const uint4*>(p.bias + sl * BN + threadIdx.x * 4);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    if (t_lo >= t_hi) return;

    // ---- per-lane constants (tile independent)
    int a_idx[NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) a_idx[a] = (a * 32 + l32) * rsw + h;
    int slot_geo[NBI], slot_off0[NBI], slot_off1[NBI];
#pragma unroll
    for (int i = 0; i < NBI; ++i) {
        const uint32_t q = (uint32_t)(i * 64 + lane);
        const uint32_t rs = fdiv(q, p.d_pcc);
        const uint32_t rem = q - rs * (uint32_t)(p.PC * CPS);
        const uint32_t lc = rem / CPS, cpos = rem & (CPS - 1);
        const uint32_t f = ((lc >> p.sw_sh) + rs * p.sw_mr) & (CPS - 1);
        const uint32_t c = cpos ^ f;
        const bool vpos = (int)rs < p.PR;
        uint32_t wrel = lc;
        if constexpr (KS == 3 && S == 2) wrel = (int)lc <= p.TW ? 2 * lc : 2 * (lc - p.TW - 1) + 1;
        slot_geo[i] = vpos ? (int)(rs | (wrel << 10) | (c << 22) | (1u << 31)) : 0;
        slot_off0[i] = ((int)rs * p.Wi + (int)wrel) * p.ldc0 * 2 + (int)c * 16;
        slot_off1[i] = ((int)rs * p.Wi + (int)wrel) * p.ldc1 * 2 + (int)c * 16;
    }
    int bidx[TAPS][MB];
    int pix_r[MB], pix_c[MB];
#pragma unroll
    for (int j = 0; j < MB; ++j) {
        int r, cc;
        if constexpr (KS == 3) {
            const int bc = 1 << p.bc_log2;
            const int btw = p.TW >> p.bc_log2;
            const int btr = j / btw, btc = j - btr * btw;
            r = btr * (32 >> p.bc_log2) + (l32 >> p.bc_log2);
            cc = btc * bc + (l32 & (bc - 1));
        } else {
            r = 0;
            cc = j * 32 + l32;
        }
        pix_r[j] = r;
        pix_c[j] = cc;
#pragma unroll
        for (int t = 0; t < TAPS; ++t) {
            const int kh = t / KS, kw = t - (t / KS) * KS;
            int rs, lc;
            if constexpr (KS == 1) {
                rs = 0; lc = cc;
            } else if constexpr (S == 1) {
                rs = r + kh; lc = cc + kw;
            } else {
                rs = 2 * r + kh;
                lc = kw == 0 ? cc : (kw == 1 ? p.TW + 1 + cc : cc + 1);
            }
            const int f = ((lc >> p.sw_sh) + rs * p.sw_mr) & (CPS - 1);
            bidx[t][j] = (rs * p.PC + lc) * CPS + (h ^ f);
        }
    }
    const bool gen1 = KS == 1 && (p.up0 | p.up1);

    // ---- per-tile fill state
    const char* sptr[NBI];
    int fill_seg = -1;
    int f_n = 0, f_h0 = 0, f_w0 = 0;
    auto tile_pos = [&](int tk, int& n, int& hh0, int& ww0) {
        if constexpr (KS == 3) {
            const uint32_t b = fdiv((uint32_t)tk, p.d_ntw);
            const int tw = tk - (int)b * p.ntw;
            const uint32_t c = fdiv(b, p.d_nth);
            n = (int)c;
            hh0 = ((int)b - (int)c * p.nth) * p.TH;
            ww0 = tw * p.TW;
        } else {
            n = 0; hh0 = 0;
            ww0 = tk * p.TW;
        }
    };
    auto setup_slots = [&](int seg) {
        const char* base = seg ? p.in1 : p.in0;
        const int ldc = seg ? p.ldc1 : p.ldc0;
        if constexpr (KS == 3) {
            const long long b0 = (((long long)f_n * p.Hi + (S * f_h0 - 1)) * p.Wi + (S * f_w0 - 1)) * ldc * 2;
            const int rlo = 1 - S * f_h0, rhi = p.Hi + 1 - S * f_h0;
            const int clo = 1 - S * f_w0, chi = p.Wi + 1 - S * f_w0;
#pragma unroll
            for (int i = 0; i < NBI; ++i) {
                const int g = slot_geo[i];
                const int rs = g & 1023, wr = (g >> 10) & 4095;
                const bool ok = g < 0 && rs >= rlo && rs < rhi && wr >= clo && wr < chi;
                sptr[i] = ok ? base + b0 + slot_off0[i] : nullptr;
            }
        } else {
            const int up = seg ? p.up1 : p.up0;
            const int hs = seg ? p.hs1 : p.hs0, ws = seg ? p.ws1 : p.ws0;
#pragma unroll
            for (int i = 0; i < NBI; ++i) {
                const int g = slot_geo[i];
                const int lc = (g >> 10) & 4095, c = (g >> 22) & 15;
                const int m = f_w0 + lc;
                const bool ok = g < 0 && m < p.M;
                if (!gen1) {
                    sptr[i] = ok ? base + (long long)f_w0 * ldc * 2 + (seg ? slot_off1[i] : slot_off0[i]) : nullptr;
                } else {
                    const uint32_t n = fdiv((uint32_t)m, p.d_howo);
                    const uint32_t rr = (uint32_t)m - n * (uint32_t)(p.Ho * p.Wo);
                    const uint32_t ho = fdiv(rr, p.d_wo);
                    const uint32_t wo = rr - ho * (uint32_t)p.Wo;
                    const long long pix = ((long long)n * hs + (ho >> up)) * ws + (wo >> up);
                    sptr[i] = ok ? base + pix * ldc * 2 + c * 16 : nullptr;
                }
            }
        }
        fill_seg = seg;
    };
    auto issue = [&](int g) {
        const int tk = t_lo + g / p.nst, st = g - (g / p.nst) * p.nst;
        if (st == 0) {
            tile_pos(tk, f_n, f_h0, f_w0);
            fill_seg = -1;
        }
        const int ch0 = st * NCB * 16;
        const int seg = (p.in1 != nullptr && ch0 >= p.c0) ? 1 : 0;
        if (seg != fill_seg) setup_slots(seg);
        const int coff = (seg ? ch0 - p.c0 : ch0) * 2;
        const int clim = (p.cin - ch0) >> 3;
        const unsigned bb = lds0 + (unsigned)((pbuf + (NBUF == 2 ? (g & 1) : 0) * BUFCH) * 16);
#pragma unroll
        for (int i = 0; i < NBI; ++i) {
            const int c = (slot_geo[i] >> 22) & 15;
            const bool ok = sptr[i] != nullptr && c < clim && !MX_DBG(2);
            mx_glds(ok ? (const void*)(sptr[i] + coff) : (const void*)p.zero, bb + (unsigned)(i * 1024));
        }
    };

    f32x16 acc[NA][MB];
    auto compute = [&](int g) {
        const int st = g - (g / p.nst) * p.nst;
        const char* A = reinterpret_cast<const char*>(sm4) + (st * NSTEP * 2) * 16;
        const char* Bp = reinterpret_cast<const char*>(sm4) + (pbuf + (NBUF == 2 ? (g & 1) : 0) * BUFCH) * 16;
        auto rd = [](const char* q) { return *reinterpret_cast<const uint4*>(__builtin_assume_aligned(q, 16)); };
        uint4 af[2][NA], bf[2][MB];
        auto load = [&](int s, int buf) {
            const int cbl = s / TAPS, t = s - (s / TAPS) * TAPS;
#pragma unroll
            for (int a = 0; a < NA; ++a) af[buf][a] = rd(A + (a_idx[a] + s * 2) * 16);
#pragma unroll
            for (int j = 0; j < MB; ++j) bf[buf][j] = rd(Bp + (bidx[t][j] ^ (cbl * 2)) * 16);
        };
        load(0, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, NA + MB, 0);
#pragma unroll
        for (int s = 0; s < NSTEP; ++s) {
            if (s + 1 < NSTEP) load(s + 1, (s + 1) & 1);
#pragma unroll
            for (int a = 0; a < NA; ++a)
#pragma unroll
                for (int j = 0; j < MB; ++j) acc[a][j] = Mfma32<T>::step(af[s & 1][a], bf[s & 1][j], acc[a][j]);
            if (s + 1 < NSTEP) __builtin_amdgcn_sched_group_barrier(0x100, NA + MB, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, NA * MB, 0);
        }
    };

    const int co = sl * BN + 16 * NA * h;
    const bool co_ok = co < p.cout;
    // coalesced epilogue through the patch buffer the last stage just freed (NBUF 2: the next
    // stage's DMA goes to the other buffer; the one after it is issued only after these reads)
    constexpr bool CO = NBUF == 2 && NBI * 1024 >= 2048 * NA;
    auto epilogue = [&](int tk, int g) {
        int n, hh0, ww0;
        tile_pos(tk, n, hh0, ww0);
        float bv[16 * NA];
#pragma unroll
        for (int e = 0; e < 16 * NA; e += 4) {
            const uint4 b4 = sm4[bias_ch + (16 * NA * h + e) / 4];
            bv[e] = __uint_as_float(b4.x); bv[e + 1] = __uint_as_float(b4.y);
            bv[e + 2] = __uint_as_float(b4.z); bv[e + 3] = __uint_as_float(b4.w);
        }
        const T* res = reinterpret_cast<const T*>(p.res);
        T* out = reinterpret_cast<T*>(p.out);
        if constexpr (CO) {
            char* E = reinterpret_cast<char*>(sm4) + (pbuf + (g & 1) * BUFCH) * 16;
#pragma unroll
            for (int j = 0; j < MB; ++j) {
                f32x16 aj[NA];
#pragma unroll
                for (int a = 0; a < NA; ++a) aj[a] = acc[a][j];
                co_tile<T, NA, KS>(aj, bv, p.act == ACT_SILU && !(MX_DBG(16)), E, lane, p, n, hh0, ww0, j, sl * BN, res,
                                   out, MX_DBG(8));
            }
            return;
        }
#pragma unroll
        for (int j = 0; j < MB; ++j) {
            long long m;
            bool ok;
            if constexpr (KS == 3) {
                const int ho = hh0 + pix_r[j], wo = ww0 + pix_c[j];
                ok = ho < p.Ho && wo < p.Wo;
                m = ((long long)n * p.Ho + ho) * p.Wo + wo;
            } else {
                const int mm = ww0 + pix_c[j];
                ok = mm < p.M;
                m = mm;
            }
            ok = ok && co_ok;
            if (!ok) m = 0;
            const int cc = ok ? co : 0;
            const int nc8 = ok ? min(2 * NA, (p.cout - co) >> 3) : 0;
            f32x16 aj[NA];
#pragma unroll
            for (int a = 0; a < NA; ++a) aj[a] = acc[a][j];
            T* op = out + m * p.ldo + cc;
            const T* rp = res + m * p.ldr + cc;
            if (p.act == ACT_SILU && !(MX_DBG(16))) {
                if (res) mx_epi<T, NA, true, true>(aj, bv, op, rp, nc8);
                else mx_epi<T, NA, true, false>(aj, bv, op, rp, nc8);
            } else {
                if (res) mx_epi<T, NA, false, true>(aj, bv, op, rp, nc8);
                else mx_epi<T, NA, false, false>(aj, bv, op, rp, nc8);
            }
        }
    };

    const int nstages = (t_hi - t_lo) * p.nst;
    issue(0);
    for (int g = 0; g < nstages; ++g) {
        const bool more = g + 1 < nstages;
        if (NBUF == 2 && more) {
            issue(g + 1);
            asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NBI) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const int st = g - (g / p.nst) * p.nst;
        if (st == 0) {
#pragma unroll
            for (int a = 0; a < NA; ++a)
#pragma unroll
                for (int j = 0; j < MB; ++j)
#pragma unroll
                    for (int e = 0; e < 16; ++e) acc[a][j][e] = 0.f;
        }
        if (!(MX_DBG(4))) compute(g);
        // single buffer: the next stage's DMA may only start once this stage's reads are done
        if (NBUF == 1 && more) issue(g + 1);
        if (st == p.nst - 1 && !(MX_DBG(8) && !CO)) epilogue(t_lo + g / p.nst, g);
    }
}

// ------------------------------------------------------------------ host side
namespace {

int ilog2(int v) {
    int l = 0;
    while ((1 << l) < v) ++l;
    return l;
}

// bank conflicts of the B-fragment reads: extra LDS cycles summed over the taps and
// B tiles of one task (ds_read_b128 lane groups, 16-B slots of a 256-B bank row)
int simulate_conflicts(const MxPlan& pl, int sh, int mr) {
    const MxConfig& c = pl.cfg;
    const int CPS = 2 * c.ncb;
    static const int grp[4][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                                   {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
                                   {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
                                   {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
    const int taps = c.ks * c.ks;
    const int nbt = c.wm * c.mb;
    int total = 0;
    for (int bt = 0; bt < nbt; ++bt)
        for (int t = 0; t < taps; ++t)
            for (int cbl = 0; cbl < c.ncb; ++cbl)
                for (int g = 0; g < 4; ++g) {
                    int slotcnt[16] = {0};
                    long long seen[16][16];
                    int nseen[16] = {0};
                    for (int u = 0; u < 16; ++u) {
                        const int lane = grp[g][u], h = lane >> 5, l32 = lane & 31;
                        int r, cc;
                        if (c.ks == 3) {
                            const int bc = 1 << pl.bc_log2, btw = pl.TW >> pl.bc_log2;
                            const int btr = bt / btw, btc = bt % btw;
                            r = btr * (32 >> pl.bc_log2) + (l32 >> pl.bc_log2);
                            cc = btc * bc + (l32 & (bc - 1));
                        } else {
                            r = 0;
                            cc = bt * 32 + l32;
                        }
                        const int kh = t / c.ks, kw = t % c.ks;
                        int rs, lc;
                        if (c.ks == 1) { rs = 0; lc = cc; }
                        else if (c.s == 1) { rs = r + kh; lc = cc + kw; }
                        else { rs = 2 * r + kh; lc = kw == 0 ? cc : (kw == 1 ? pl.TW + 1 + cc : cc + 1); }
                        const int f = ((lc >> sh) + rs * mr) & (CPS - 1);
                        const long long addr = ((long long)(rs * pl.PC + lc) * CPS + ((2 * cbl + h) ^ f)) * 16;
                        const int slot = (int)((addr / 16) & 15);
                        bool dup = false;
                        for (int k = 0; k < nseen[slot]; ++k) dup |= seen[slot][k] == addr;
                        if (!dup) { seen[slot][nseen[slot]++] = addr; ++slotcnt[slot]; }
                    }
                    int mx = 0;
                    for (int s = 0; s < 16; ++s) mx = std::max(mx, slotcnt[s]);
                    total += mx - 1;
                }
    return total;
}

}  // namespace

static MxPlan mx_plan_r(const MxShape& sh, const MxConfig& cfg, int num_cus);

MxPlan mx_plan(const MxShape& sh, const MxConfig& cfg, int num_cus) {
    if (cfg.kind == 2) return mx_plan_w(sh, cfg, num_cus);
    // K-split layers follow the chunked order, which only the conv_rw kernels implement
    if (mx_kchunks(sh) > 1) {
        MxPlan none;
        none.cfg = cfg;
        return none;
    }
    if (cfg.kind == 1) return mx_plan_r(sh, cfg, num_cus);
    MxPlan pl;
    pl.cfg = cfg;
    const MxConfig& c = cfg;
    if (c.ks != sh.ks || (c.ks == 1 && c.s != 1) || (c.ks == 3 && sh.s != c.s)) return pl;
    if (sh.ks == 3 && (sh.c1 != 0 || sh.up0 != 0)) return pl;
    const int NW = c.nw(), NT = 64 * NW, BN = c.bn(), CPS = 2 * c.ncb, taps = c.ks * c.ks;
    const int ncb16 = (sh.cin + 15) / 16;
    if (sh.c1 != 0 && sh.c0 % (16 * c.ncb) != 0) return pl;
    pl.nst = (ncb16 + c.ncb - 1) / c.ncb;
    pl.nslices = (sh.cout + BN - 1) / BN;
    const int tile_px = 32 * c.wm * c.mb;
    if (c.ks == 3) {
        int bc = sh.Wo % 16 == 0 ? 16 : sh.Wo % 8 == 0 ? 8 : 4;
        // widest B tile whose row count divides the task's rows; task as square-ish as possible
        int best_tw = 0, best_th = 0;
        double best_cost = 1e30;
        for (int bcc : {16, 8, 4}) {
            if (bcc > bc) continue;
            for (int tw = bcc; tw <= 256; tw += bcc) {
                if (tile_px % tw) continue;
                const int th = tile_px / tw;
                if (th % (32 / bcc)) continue;
                const int ntw = (sh.Wo + tw - 1) / tw, nth = (sh.Ho + th - 1) / th;
                const double waste = (double)ntw * tw * nth * th / ((double)sh.Wo * sh.Ho);
                const int pc = c.s == 1 ? tw + 2 : 2 * tw + 1, pr = c.s == 1 ? th + 2 : 2 * th + 1;
                const double halo = (double)pc * pr / (double)(c.s * c.s * tw * th);
                const double cost = waste * (1.0 + 0.5 * (halo - 1.0));
                if (cost < best_cost - 1e-9) { best_cost = cost; best_tw = tw; best_th = th; bc = bcc; }
            }
            if (best_tw) { bc = std::min(bc, bcc); break; }
        }
        if (!best_tw) return pl;
        pl.TW = best_tw; pl.TH = best_th; pl.bc_log2 = ilog2(bc);
        // re-derive bc from the chosen tw (largest of 16/8/4 that divides tw and whose rows divide th)
        for (int bcc : {16, 8, 4})
            if (pl.TW % bcc == 0 && pl.TH % (32 / bcc) == 0 && bcc <= (sh.Wo % 16 == 0 ? 16 : sh.Wo % 8 == 0 ? 8 : 4)) {
                pl.bc_log2 = ilog2(bcc);
                break;
            }
        pl.PC = c.s == 1 ? pl.TW + 2 : 2 * pl.TW + 1;
        pl.PR = c.s == 1 ? pl.TH + 2 : 2 * pl.TH + 1;
        pl.ntw = (sh.Wo + pl.TW - 1) / pl.TW;
        pl.nth = (sh.Ho + pl.TH - 1) / pl.TH;
        pl.ntasks = sh.B * pl.nth * pl.ntw * pl.nslices;
    } else {
        pl.TW = tile_px;
        pl.TH = 1;
        pl.bc_log2 = 5;
        pl.PC = pl.TW;
        pl.PR = 1;
        const long long M = (long long)sh.B * sh.Ho * sh.Wo;
        pl.ntw = (int)((M + pl.TW - 1) / pl.TW);
        pl.nth = 1;
        pl.ntasks = pl.ntw * pl.nslices;
    }
    const int bchunks = pl.PR * pl.PC * CPS;
    pl.nbi = (bchunks + NT - 1) / NT;
    if (pl.nbi > MX_MAXB) return pl;
    const int RS = 2 * taps * c.ncb + 1;
    pl.ains = (BN * RS + NT - 1) / NT;
    pl.abytes = pl.ains * NT * 16;
    pl.bbytes = pl.nbi * NT * 16;
    pl.lds = 2 * (pl.abytes + pl.bbytes) + pl.nslices * BN * 4;
    if (pl.lds > 160 * 1024) return pl;
    pl.wstage = pl.abytes;
    // swizzle search
    int best = 1 << 30, bsh = 0, bmr = 0;
    for (int s2 = 0; s2 <= 4; ++s2)
        for (int mr = 0; mr < CPS; ++mr) {
            const int cf = simulate_conflicts(pl, s2, mr);
            if (cf < best) { best = cf; bsh = s2; bmr = mr; }
        }
    pl.sw_sh = bsh; pl.sw_mr = bmr; pl.conflicts = best;
    const int per_cu = std::max(1, std::min(8, (160 * 1024) / pl.lds));
    const int wgs = std::max(1, std::min(per_cu, 8 / NW));   // <= 2 waves per SIMD (VGPR budget)
    pl.grid = std::min(pl.ntasks, num_cus * wgs);
    pl.ok = true;
    return pl;
}

// conv_mxr plan: per-wave tile of MB B tiles; weights of one BN slice resident.
static MxPlan mx_plan_r(const MxShape& sh, const MxConfig& cfg, int num_cus) {
    MxPlan pl;
    pl.cfg = cfg;
    const MxConfig& c = cfg;
    if (c.ks != sh.ks || (c.ks == 1 && c.s != 1) || (c.ks == 3 && sh.s != c.s)) return pl;
    if (sh.ks == 3 && (sh.c1 != 0 || sh.up0 != 0)) return pl;
    const int NW = c.wm, BN = 32 * c.na, CPS = 2 * c.ncb, taps = c.ks * c.ks;
    const int ncb16 = (sh.cin + 15) / 16;
    if (sh.c1 != 0 && sh.c0 % (16 * c.ncb) != 0) return pl;
    pl.nst = (ncb16 + c.ncb - 1) / c.ncb;
    pl.nslices = (sh.cout + BN - 1) / BN;
    const int tile_px = 32 * c.mb;
    if (c.ks == 3) {
        const int bcmax = sh.Wo % 16 == 0 ? 16 : sh.Wo % 8 == 0 ? 8 : 4;
        int best_tw = 0, best_th = 0, best_bc = 0;
        double best = 1e30;
        for (int bc : {16, 8, 4}) {
            if (bc > bcmax) continue;
            for (int tw = bc; tw <= tile_px; tw += bc) {
                if (tile_px % tw) continue;
                const int th = tile_px / tw;
                if (th % (32 / bc)) continue;
                const int ntw = (sh.Wo + tw - 1) / tw, nth = (sh.Ho + th - 1) / th;
                const double waste = (double)ntw * tw * nth * th / ((double)sh.Wo * sh.Ho);
                const int pc = c.s == 1 ? tw + 2 : 2 * tw + 1, pr = c.s == 1 ? th + 2 : 2 * th + 1;
                if ((pr * pc * CPS + 63) / 64 > c.nbi) continue;
                // bank conflicts of this shape under its best swizzle
                MxPlan t = pl;
                t.TW = tw; t.TH = th; t.bc_log2 = ilog2(bc); t.PC = pc; t.PR = pr;
                t.cfg.wm = 1;
                int cf = 1 << 30;
                for (int s2 = 0; s2 <= 4; ++s2)
                    for (int mr = 0; mr < CPS; ++mr) cf = std::min(cf, simulate_conflicts(t, s2, mr));
                const double cost = waste * pr * pc * (1.0 + 0.5 * cf / (double)(taps * c.ncb * 4 * c.mb));
                if (cost < best - 1e-9) { best = cost; best_tw = tw; best_th = th; best_bc = bc; }
            }
        }
        if (!best_tw) return pl;
        pl.TW = best_tw; pl.TH = best_th; pl.bc_log2 = ilog2(best_bc);
        pl.PC = c.s == 1 ? pl.TW + 2 : 2 * pl.TW + 1;
        pl.PR = c.s == 1 ? pl.TH + 2 : 2 * pl.TH + 1;
        pl.ntw = (sh.Wo + pl.TW - 1) / pl.TW;
        pl.nth = (sh.Ho + pl.TH - 1) / pl.TH;
        pl.ntasks = sh.B * pl.nth * pl.ntw;   // wave tiles per slice
    } else {
        pl.TW = tile_px; pl.TH = 1; pl.bc_log2 = 5; pl.PC = pl.TW; pl.PR = 1;
        const long long M = (long long)sh.B * sh.Ho * sh.Wo;
        pl.ntw = (int)((M + pl.TW - 1) / pl.TW);
        pl.nth = 1;
        pl.ntasks = pl.ntw;
        if ((pl.PC * CPS + 63) / 64 > c.nbi) return pl;
    }
    pl.nbi = c.nbi;
    const int rsw = pl.nst * c.ncb * taps * 2 + 1;
    const int wch = (BN * rsw + 63) / 64 * 64;
    pl.wstage = wch * 16;
    pl.abytes = pl.wstage;
    pl.bbytes = c.nbi * 1024;
    pl.lds = pl.wstage + BN * 4 + NW * c.nbuf * pl.bbytes;
    if (pl.lds > 160 * 1024) return pl;
    int best = 1 << 30, bsh = 0, bmr = 0;
    MxPlan sim = pl;
    sim.cfg.wm = 1;   // one wave's tile
    for (int s2 = 0; s2 <= 4; ++s2)
        for (int mr = 0; mr < CPS; ++mr) {
            const int cf = simulate_conflicts(sim, s2, mr);
            if (cf < best) { best = cf; bsh = s2; bmr = mr; }
        }
    pl.sw_sh = bsh; pl.sw_mr = bmr; pl.conflicts = best;
    const int wps = std::max(1, std::min(num_cus / std::max(1, std::min(pl.nslices, num_cus)),
                                         (pl.ntasks + NW - 1) / NW));
    pl.grid = wps * pl.nslices;
    pl.ok = true;
    return pl;
}

std::vector<MxPlan> mx_candidates(const MxShape& sh, int num_cus) {
    std::vector<MxConfig> cfgs;
    auto add = [&](int na, int mb, int wn, int wm, int ncb) {
        MxConfig c{};
        c.kind = 0; c.ks = sh.ks; c.s = sh.ks == 1 ? 1 : sh.s; c.na = na; c.mb = mb; c.wn = wn; c.wm = wm; c.ncb = ncb;
        cfgs.push_back(c);
    };
    const bool narrow = sh.cout <= 32;
    const int ncbmax = sh.ks == 1 ? 4 : 2;
    for (int ncb = 1; ncb <= ncbmax; ncb *= 2) {
        if (ncb > 1 && (sh.cin + 15) / 16 < ncb) break;
        if (narrow) { add(1, 2, 1, 4, ncb); add(1, 4, 1, 4, ncb); }
        else {
            add(2, 2, 1, 4, ncb);
            add(1, 4, 1, 4, ncb);
            if (sh.cout > 64) add(2, 2, 2, 2, ncb);
            // 256-cout slices for wide layers: the input patch is read by half as many slices
            if (sh.cout >= 512) add(2, 2, 4, 2, ncb);
        }
    }
    // resident-weight per-wave kernels (instantiated set, see launch_mxr_cfg)
    auto addr = [&](int na, int mb, int ncb, int nbi, int nbuf = 2, int nw = 8) {
        MxConfig c{};
        c.kind = 1; c.ks = sh.ks; c.s = sh.ks == 1 ? 1 : sh.s; c.na = na; c.mb = mb; c.wn = 1; c.wm = nw;
        c.ncb = ncb; c.nbi = nbi; c.nbuf = nbuf;
        cfgs.push_back(c);
    };
    // 32-pixel wave tiles (mb 1) give small layers (40x40, 20x20) 2-4x more wave tasks
    if (sh.ks == 3 && sh.s == 1) {
        if (narrow) { addr(1, 2, 1, 4); addr(1, 2, 2, 7); addr(1, 4, 1, 6); addr(1, 1, 1, 2); addr(1, 1, 2, 4); }
        else { addr(2, 2, 1, 4); addr(2, 2, 2, 7); addr(2, 1, 1, 2); addr(2, 1, 2, 4); }
    } else if (sh.ks == 3) {
        // stride 2: a 4x8 wave tile (9x17 patch) double-buffered, or an 8x8 tile (17x17)
        // single-buffered; 32-cout slices for weights too large to keep whole
        // 16-channel stages read 32 B of each input pixel per stage: on an input far beyond
        // L2 (net.p3.0: 105 MB) that costs 2x its bytes in HBM traffic (PMC), and in-situ
        // timing does not separate the two reliably, so only 32-channel stages there
        const bool big_in = (double)sh.B * sh.Hi * sh.Wi * sh.cin * 2.0 > 64e6 && sh.cin >= 64;
        if (narrow) { addr(1, 1, 1, 5); addr(1, 2, 1, 10, 1); }
        else {
            if (!big_in) { addr(2, 1, 1, 5); addr(2, 2, 1, 10, 1); addr(1, 1, 1, 5); addr(1, 2, 1, 10, 1); }
            addr(2, 1, 2, 10, 2, 4); addr(1, 1, 2, 10, 2, 4);
        }
    } else {
        if (narrow) { addr(1, 2, 1, 2); addr(1, 2, 2, 4); addr(1, 2, 4, 8); addr(1, 4, 1, 4); addr(1, 4, 2, 8);
                      addr(1, 1, 2, 2); addr(1, 1, 4, 4); }
        else { addr(2, 2, 1, 2); addr(2, 2, 2, 4); addr(2, 2, 4, 8); addr(2, 1, 2, 2); addr(2, 1, 4, 4); }
    }
    // weights in VGPRs, shared patch ring (conv_rw.hip)
    mx_candidates_w(sh, cfgs);
    std::vector<MxPlan> out;
    for (auto& c : cfgs) {
        MxPlan p = mx_plan(sh, c, num_cus);
        if (p.ok) out.push_back(p);
    }
    return out;
}

std::vector<uint16_t> mx_pack(const MxPlan& pl, const MxShape& sh, const float* wf, int cin_logical,
                              const std::vector<int>& phys2log, bool bf16, int cout_logical) {
    const MxConfig& c = pl.cfg;
    if (c.kind == 2) return mx_pack_w(pl, sh, wf, cin_logical, phys2log, bf16, cout_logical);
    if (c.kind == 1) {
        // resident: per slice one image [BN rows][rsw chunks], chunk (cb16*taps + t)*2 + hh
        const int BN = 32 * c.na, NA = c.na, taps = c.ks * c.ks, rsw = pl.nst * c.ncb * taps * 2 + 1;
        const size_t img_el = (size_t)pl.wstage / 2;
        std::vector<uint16_t> out((size_t)pl.nslices * img_el, 0);
        for (int sl = 0; sl < pl.nslices; ++sl) {
            uint16_t* img = out.data() + (size_t)sl * img_el;
            for (int row = 0; row < BN; ++row) {
                const int a = row / 32, R = row % 32;
                const int cout = sl * BN + 16 * NA * ((R >> 2) & 1) + 16 * a + (R & 3) + 4 * (R >> 3);
                if (cout >= sh.cout || cout >= cout_logical) continue;
                for (int cb = 0; cb < pl.nst * c.ncb; ++cb)
                    for (int t = 0; t < taps; ++t)
                        for (int hh = 0; hh < 2; ++hh)
                            for (int e = 0; e < 8; ++e) {
                                const int ci = cb * 16 + hh * 8 + e;
                                if (ci >= (int)phys2log.size()) continue;
                                const int cl = phys2log[ci];
                                if (cl < 0) continue;
                                const float v = wf[((size_t)cout * cin_logical + cl) * taps + t];
                                uint16_t hv;
                                {
                                    uint32_t u;
                                    std::memcpy(&u, &v, 4);
                                    if (bf16) {
                                        hv = ((u & 0x7fffffffu) > 0x7f800000u) ? (uint16_t)((u >> 16) | 0x40)
                                                                              : (uint16_t)((u + 0x7fffu + ((u >> 16) & 1)) >> 16);
                                    } else {
                                        _Float16 f16 = (_Float16)v;
                                        std::memcpy(&hv, &f16, 2);
                                    }
                                }
                                img[(size_t)(row * rsw + (cb * taps + t) * 2 + hh) * 8 + e] = hv;
                            }
            }
        }
        return out;
    }
    const int BN = c.bn(), NA = c.na, taps = c.ks * c.ks, RS = 2 * taps * c.ncb + 1;
    const size_t stage_el = (size_t)pl.wstage / 2;
    std::vector<uint16_t> out((size_t)pl.nslices * pl.nst * stage_el, 0);
    auto cvt = [&](float f) -> uint16_t {
        uint32_t u;
        std::memcpy(&u, &f, 4);
        if (bf16) {
            if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
            return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1)) >> 16);
        }
        _Float16 hv = (_Float16)f;
        uint16_t r;
        std::memcpy(&r, &hv, 2);
        return r;
    };
    for (int sl = 0; sl < pl.nslices; ++sl)
        for (int st = 0; st < pl.nst; ++st) {
            uint16_t* img = out.data() + ((size_t)sl * pl.nst + st) * stage_el;
            for (int row = 0; row < BN; ++row) {
                const int wgrp = row / (32 * NA), a = (row / 32) % NA, R = row % 32;
                const int cout = sl * BN + wgrp * NA * 32 + 16 * NA * ((R >> 2) & 1) + 16 * a + (R & 3) + 4 * (R >> 3);
                if (cout >= sh.cout || cout >= cout_logical) continue;
                for (int cbl = 0; cbl < c.ncb; ++cbl)
                    for (int t = 0; t < taps; ++t)
                        for (int hh = 0; hh < 2; ++hh)
                            for (int e = 0; e < 8; ++e) {
                                const int ci = (st * c.ncb + cbl) * 16 + hh * 8 + e;
                                if (ci >= (int)phys2log.size()) continue;
                                const int cl = phys2log[ci];
                                if (cl < 0) continue;
                                const float v = wf[((size_t)cout * cin_logical + cl) * taps + t];
                                img[(size_t)(row * RS + (cbl * taps + t) * 2 + hh) * 8 + e] = cvt(v);
                            }
            }
        }
    return out;
}

void mx_fill_args(const MxPlan& pl, const MxShape& sh, MxArgs& a) {
    a.Hi = sh.Hi; a.Wi = sh.Wi; a.Ho = sh.Ho; a.Wo = sh.Wo; a.B = sh.B;
    a.cin = sh.cin; a.c0 = sh.c0; a.up0 = sh.up0; a.up1 = sh.up1;
    a.nst = pl.nst;
    a.wstage = pl.wstage;
    a.cout = sh.cout;
    a.TH = pl.TH; a.TW = pl.TW; a.ntw = pl.ntw; a.nth = pl.nth; a.nslices = pl.nslices; a.ntasks = pl.ntasks;
    a.bc_log2 = pl.bc_log2; a.PC = pl.PC; a.PR = pl.PR; a.nbi = pl.nbi;
    a.sw_sh = pl.sw_sh; a.sw_mr = pl.sw_mr;
    const int CPS = 2 * pl.cfg.ncb;
    a.d_pcc = make_fastdiv((uint32_t)(pl.PC * CPS));
    a.d_cps = make_fastdiv((uint32_t)CPS);
    a.d_wo = make_fastdiv((uint32_t)sh.Wo);
    a.d_howo = make_fastdiv((uint32_t)(sh.Ho * sh.Wo));
    a.d_ntw = make_fastdiv((uint32_t)pl.ntw);
    a.d_nth = make_fastdiv((uint32_t)pl.nth);
    a.d_nsl = make_fastdiv((uint32_t)pl.nslices);
    a.M = sh.B * sh.Ho * sh.Wo;
}

namespace {

template <typename T, int KS, int S, int NA, int MB, int WN, int WM, int NCB>
int launch_mx_t(const MxPlan& pl, const MxArgs& a, hipStream_t s) {
    static bool attr = false;
    auto k = &conv_mx<T, KS, S, NA, MB, WN, WM, NCB>;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        attr = true;
    }
    hipLaunchKernelGGL(k, dim3(pl.grid), dim3(64 * WN * WM), pl.lds, s, a);
    return (int)hipGetLastError();
}

template <typename T, int KS, int S>
int launch_mx_cfg(const MxPlan& pl, const MxArgs& a, hipStream_t s) {
    const MxConfig& c = pl.cfg;
#define YH_MX(NA_, MB_, WN_, WM_)                                                              \
    if (c.na == NA_ && c.mb == MB_ && c.wn == WN_ && c.wm == WM_) {                                \
        if (c.ncb == 1) return launch_mx_t<T, KS, S, NA_, MB_, WN_, WM_, 1>(pl, a, s);             \
        if (c.ncb == 2) return launch_mx_t<T, KS, S, NA_, MB_, WN_, WM_, 2>(pl, a, s);             \
        if constexpr (KS == 1)                                                                     \
            if (c.ncb == 4) return launch_mx_t<T, KS, S, NA_, MB_, WN_, WM_, 4>(pl, a, s);         \
    }
    YH_MX(2, 2, 1, 4)
    YH_MX(1, 4, 1, 4)
    YH_MX(1, 2, 1, 4)
    YH_MX(2, 2, 2, 2)
    YH_MX(2, 2, 4, 2)
#undef YH_MX
    return (int)hipErrorInvalidValue;
}

template <typename T, int KS, int S, int NA, int MB, int NCB, int NBI, int NBUF, int NW>
int launch_mxr_t(const MxPlan& pl, const MxArgs& a, hipStream_t s) {
    static bool attr = false;
    auto k = &conv_mxr<T, KS, S, NA, MB, NCB, NBI, NW, NBUF>;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        attr = true;
    }
    hipLaunchKernelGGL(k, dim3(pl.grid), dim3(64 * NW), pl.lds, s, a);
    return (int)hipGetLastError();
}

template <typename T>
int launch_mxr_cfg(const MxPlan& pl, const MxArgs& a, hipStream_t s) {
    const MxConfig& c = pl.cfg;
#define YH_MXRW(KS_, S_, NA_, MB_, NCB_, NBI_, NBUF_, NW_)                                            \
    if (c.ks == KS_ && c.s == S_ && c.na == NA_ && c.mb == MB_ && c.ncb == NCB_ && c.nbi == NBI_ &&      \
        c.nbuf == NBUF_ && c.wm == NW_)                                                                 \
        return launch_mxr_t<T, KS_, S_, NA_, MB_, NCB_, NBI_, NBUF_, NW_>(pl, a, s);
#define YH_MXR(KS_, S_, NA_, MB_, NCB_, NBI_, NBUF_) YH_MXRW(KS_, S_, NA_, MB_, NCB_, NBI_, NBUF_, 8)
    // stride 2, 32-channel stages with 4 waves: each stage reads 64 of a pixel's 128 B
    YH_MXRW(3, 2, 2, 1, 2, 10, 2, 4)
    YH_MXRW(3, 2, 1, 1, 2, 10, 2, 4)
    YH_MXR(3, 1, 2, 2, 1, 4, 2)
    YH_MXR(3, 1, 2, 2, 2, 7, 2)
    YH_MXR(3, 1, 1, 2, 1, 4, 2)
    YH_MXR(3, 1, 1, 2, 2, 7, 2)
    YH_MXR(3, 1, 1, 4, 1, 6, 2)
    YH_MXR(3, 2, 2, 2, 1, 10, 1)
    YH_MXR(3, 2, 1, 2, 1, 10, 1)
    YH_MXR(3, 2, 2, 1, 1, 5, 2)
    YH_MXR(3, 2, 1, 1, 1, 5, 2)
    YH_MXR(3, 1, 2, 1, 1, 2, 2)
    YH_MXR(3, 1, 2, 1, 2, 4, 2)
    YH_MXR(3, 1, 1, 1, 1, 2, 2)
    YH_MXR(3, 1, 1, 1, 2, 4, 2)
    YH_MXR(1, 1, 2, 1, 2, 2, 2)
    YH_MXR(1, 1, 2, 1, 4, 4, 2)
    YH_MXR(1, 1, 1, 1, 2, 2, 2)
    YH_MXR(1, 1, 1, 1, 4, 4, 2)
    YH_MXR(1, 1, 2, 2, 1, 2, 2)
    YH_MXR(1, 1, 2, 2, 2, 4, 2)
    YH_MXR(1, 1, 2, 2, 4, 8, 2)
    YH_MXR(1, 1, 1, 2, 1, 2, 2)
    YH_MXR(1, 1, 1, 2, 2, 4, 2)
    YH_MXR(1, 1, 1, 2, 4, 8, 2)
    YH_MXR(1, 1, 1, 4, 1, 4, 2)
    YH_MXR(1, 1, 1, 4, 2, 8, 2)
#undef YH_MXR
#undef YH_MXRW
    return (int)hipErrorInvalidValue;
}

template <typename T>
int launch_mx_dt(const MxPlan& pl, const MxArgs& a, hipStream_t s) {
    if (pl.cfg.kind == 1) return launch_mxr_cfg<T>(pl, a, s);
    if (pl.cfg.ks == 1) return launch_mx_cfg<T, 1, 1>(pl, a, s);
    if (pl.cfg.s == 1) return launch_mx_cfg<T, 3, 1>(pl, a, s);
    return launch_mx_cfg<T, 3, 2>(pl, a, s);
}

}  // namespace

int launch_mx(int dtype, const MxPlan& pl, const MxArgs& a, hipStream_t s) {
    if (!pl.ok) return (int)hipErrorInvalidValue;
    if (pl.cfg.kind == 2) return launch_rw(dtype, pl, a, s);
    if (dtype == BF16) return launch_mx_dt<__bf16>(pl, a, s);
    if (dtype == F16) return launch_mx_dt<_Float16>(pl, a, s);
    return (int)hipErrorInvalidValue;
}

}  // namespace yh
