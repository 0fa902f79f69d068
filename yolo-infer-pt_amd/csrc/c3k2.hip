// Fused C3k2 block (nets/nn.py:66-80, n = 1, csp = False) for the 16-bit handles.
//
// One persistent workgroup (8 waves) per CU walks TH x TW output tiles of the block:
//   P0  input tile with a 2-pixel halo -> LDS (LDS-DMA, zeros outside the image)
//   P1  conv1 1x1 Cin -> 2c + SiLU on the whole halo tile -> T1 = [a | b]; pixels
//       outside the image are zeroed (they are the next conv's zero padding)
//   P2  Residual conv1 3x3 c -> c/2 + SiLU on b, 1-pixel halo -> R1 (zeroed outside)
//   P3  Residual conv2 3x3 c/2 -> c + SiLU, + b (nn.py:49) -> C2
//   P4  conv2 1x1 over cat [a | b | C2] (3c) -> cout + SiLU -> the block output in HBM
// The packed weights (MFMA fragments in lane order, one 1 KB image per 32-cout tile and
// K step) and biases are copied to LDS once per workgroup; the next tile's input DMA
// runs during P2-P4.
//
// Bit-identical to the per-layer conv_mx launches (conv_mx.h): each conv walks its K
// as  for 16-channel block: for tap: one v_mfma_f32_32x32x16 step  (channels past a
// layer's width are zero), adds the bias, applies SiLU and rounds once; the residual
// is added to the rounded value in fp32 and rounded again (mx_epi).
//
// Fragment rows are permuted like conv_mx's packed weights: lane half hh of a 32-cout
// tile a holds couts 32a + 16hh .. +15 in its 16 accumulator registers, so every
// epilogue store is two 16-B chunks.
#include "common.h"
#include "dtypes.h"

namespace yh {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <typename T> struct CMfma;
template <> struct CMfma<__bf16> {
    static __device__ __forceinline__ f32x16 step(const uint4& a, const uint4& b, const f32x16& c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                       0, 0);
    }
};
template <> struct CMfma<_Float16> {
    static __device__ __forceinline__ f32x16 step(const uint4& a, const uint4& b, const f32x16& c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                      0);
    }
};

constexpr int NWV = CSP_THREADS / 64;

__device__ __forceinline__ void cs_glds(const void* src, unsigned lds_addr) {
#if defined(__HIP_DEVICE_COMPILE__)
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds_addr) : "memory");
#else
    (void)src; (void)lds_addr;
#endif
}
__device__ __forceinline__ void cs_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ uint4 cs_rd(unsigned addr) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef __attribute__((address_space(3))) const uint4* lp;
    return *reinterpret_cast<lp>((size_t)addr);
#else
    (void)addr;
    return uint4{};
#endif
}
__device__ __forceinline__ void cs_wr(unsigned addr, uint4 v) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef __attribute__((address_space(3))) uint4* lp;
    *reinterpret_cast<lp>((size_t)addr) = v;
#else
    (void)addr; (void)v;
#endif
}
__device__ __forceinline__ float4 cs_rdf(unsigned addr) {
    const uint4 u = cs_rd(addr);
    return make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
}

// Parameter image layout (bytes), shared with the host packer through csp_prm_bytes.
struct CsLayout {
    int w1, w2, w3, w4, b1, b2, b3, b4, prm;
};
__host__ __device__ constexpr CsLayout cs_layout(int ni, int nc, int no) {
    const int nh = (nc + 1) / 2, na3 = (nc + 1) / 2;
    CsLayout L{};
    L.w1 = 0;
    L.w2 = L.w1 + nc * ni * 1024;            // conv1: nc 32-cout tiles x ni steps
    L.w3 = L.w2 + 9 * nc * 1024;             // res conv1: one tile x 9 nc steps
    L.w4 = L.w3 + na3 * 9 * nh * 1024;       // res conv2: na3 tiles x 9 nh steps
    L.b1 = L.w4 + no * 3 * nc * 1024;        // conv2: no tiles x 3 nc steps
    L.b2 = L.b1 + 32 * nc * 4;
    L.b3 = L.b2 + 32 * 4;
    L.b4 = L.b3 + 32 * na3 * 4;
    L.prm = (L.b4 + 32 * no * 4 + 1023) & ~1023;
    return L;
}
struct CsTile {
    int lx, lt, lr, lc, total;
};
__host__ __device__ inline CsTile cs_tile(int TH, int TW, int ni, int nc, int no) {
    const int nh = (nc + 1) / 2;
    const CsLayout L = cs_layout(ni, nc, no);
    const int XP = (TH + 4) * (TW + 4), MP = (TH + 2) * (TW + 2), NP = TH * TW;
    CsTile t{};
    t.lx = L.prm;
    t.lt = t.lx + (ni ? ((XP * (16 * ni + 8) * 2 + 1023) & ~1023) : 0);   // tail mode: no X region
    t.lr = t.lt + XP * (32 * nc + 8) * 2;
    t.lc = t.lr + MP * (16 * nh + 8) * 2;
    t.total = t.lc + NP * (16 * nc + 8) * 2;
    return t;
}

// 16 consecutive outputs of one pixel (couts co0 .. co0 + 15): bias, SiLU, one rounding
template <typename T>
__device__ __forceinline__ void cs_act(const f32x16& acc, unsigned bias_addr, uint4 (&o)[2]) {
    float v[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float4 b = cs_rdf(bias_addr + 16 * q);
        v[4 * q] = acc[4 * q] + b.x;
        v[4 * q + 1] = acc[4 * q + 1] + b.y;
        v[4 * q + 2] = acc[4 * q + 2] + b.z;
        v[4 * q + 3] = acc[4 * q + 3] + b.w;
    }
    T t[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) t[i] = fromf<T>(silu<T>(v[i]));
    o[0] = *reinterpret_cast<const uint4*>(&t[0]);
    o[1] = *reinterpret_cast<const uint4*>(&t[8]);
}

// One conv phase: the NA x nb work items (32-cout A tile a, 32-pixel B tile) of an
// npx-pixel region go round-robin to the waves; a wave runs two items at once (two
// independent MFMA chains) while it has two. A image a = aimg + a * NK KB (fragments in lane
// order); baddr(px, k) = LDS byte address of the lane's 8 K values of step k for region
// pixel px; epi(a, px, acc) for pixels < npx.
template <typename T, int NA, int NK, typename BAddr, typename Epi>
__device__ __forceinline__ void cs_phase(unsigned aimg, int npx, BAddr baddr, Epi epi) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, l32 = lane & 31;
    const int items = NA * ((npx + 31) >> 5);
    for (int i0 = wv; i0 < items; i0 += 2 * NWV) {
        const int i1 = i0 + NWV;
        const int a0 = i0 % NA, a1 = i1 % NA;
        const int p0 = (i0 / NA) * 32 + l32, p1 = (i1 / NA) * 32 + l32;
        const int c0 = p0 < npx ? p0 : npx - 1, c1 = p1 < npx ? p1 : npx - 1;
        const unsigned ai0 = aimg + (unsigned)(a0 * NK * 1024 + lane * 16);
        const unsigned ai1 = aimg + (unsigned)(a1 * NK * 1024 + lane * 16);
        f32x16 acc0, acc1;
#pragma unroll
        for (int e = 0; e < 16; ++e) { acc0[e] = 0.f; acc1[e] = 0.f; }
        if (i1 < items) {   // wave-uniform
#pragma unroll
            for (int k = 0; k < NK; ++k) {
                const uint4 f0 = cs_rd(ai0 + k * 1024), f1 = NA > 1 ? cs_rd(ai1 + k * 1024) : f0;
                const uint4 x0 = cs_rd(baddr(c0, k)), x1 = cs_rd(baddr(c1, k));
                acc0 = CMfma<T>::step(f0, x0, acc0);
                acc1 = CMfma<T>::step(f1, x1, acc1);
            }
            if (p0 < npx) epi(a0, p0, acc0);
            if (p1 < npx) epi(a1, p1, acc1);
        } else {
#pragma unroll
            for (int k = 0; k < NK; ++k) acc0 = CMfma<T>::step(cs_rd(ai0 + k * 1024), cs_rd(baddr(c0, k)), acc0);
            if (p0 < npx) epi(a0, p0, acc0);
        }
    }
}

template <typename T, int NI, int NC, int NO>
__global__ __launch_bounds__(CSP_THREADS) void csp_fused(const CspArgs A) {
    constexpr int NH = (NC + 1) / 2, NA3 = (NC + 1) / 2;
    constexpr int SX = 16 * NI + 8, ST = 32 * NC + 8, SR = 16 * NH + 8, SC = 16 * NC + 8;
    constexpr CsLayout L = cs_layout(NI, NC, NO);
    extern __shared__ __attribute__((aligned(16))) char sm[];
    typedef __attribute__((address_space(3))) char* lds_c;
    const unsigned lds0 = (unsigned)(size_t)(lds_c)sm;
    const int TH = A.TH, TW = A.TW, XW = TW + 4, MW = TW + 2;
    const int XP = (TH + 4) * XW, MP = (TH + 2) * MW, NP = TH * TW;
    const CsTile G = cs_tile(TH, TW, NI, NC, NO);
    const unsigned LX = lds0 + G.lx, LT = lds0 + G.lt, LR = lds0 + G.lr, LC = lds0 + G.lc;
    const int lane = threadIdx.x & 63, hh = lane >> 5;
    const int wvu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const T* x = reinterpret_cast<const T*>(A.x);
    T* y = reinterpret_cast<T*>(A.y);

    // parameters: once per workgroup
    {
        const char* prm = reinterpret_cast<const char*>(A.prm);
        for (int i0 = wvu * 64; i0 < L.prm / 16; i0 += CSP_THREADS) cs_glds(prm + (size_t)(i0 + lane) * 16, lds0 + i0 * 16);
    }
    // tail mode (NI == 0): the block input is conv1's output [a | b] (2c channels, computed
    // by its own launch) and lands straight in T1; P1 is skipped
    constexpr bool TAIL = NI == 0;
    constexpr int NCH = TAIL ? 4 * NC : 2 * NI;   // 16-B data chunks per pixel
    constexpr int CPX = NCH + 1;                  // + one padding chunk per stored pixel
    const unsigned LD = TAIL ? LT : LX;
    auto load_x = [&](int t) {
        const int n = t / A.tiles, tix = t - n * A.tiles;
        const int ty = tix / A.ntw, tx = tix - ty * A.ntw;
        const int h0 = ty * TH - 2, w0 = tx * TW - 2;
        const int total = XP * CPX;
        for (int i0 = wvu * 64; i0 < total; i0 += CSP_THREADS) {
            const int q = i0 + lane;
            const int px = q / CPX, c = q - px * CPX;
            const int r = px / XW, cc = px - r * XW;
            const int gh = h0 + r, gw = w0 + cc;
            const bool ok = q < total && c < NCH && (unsigned)gh < (unsigned)A.H && (unsigned)gw < (unsigned)A.W;
            const void* src = ok ? (const void*)(x + (((long long)n * A.H + gh) * A.W + gw) * A.ldx + c * 8) : A.zero;
            cs_glds(src, LD + i0 * 16);
        }
    };
    // XCD-aware: the workgroups of one XCD take neighbouring tiles (overlapping halos, one L2)
    const int t0 = xcd_remap(blockIdx.x, gridDim.x);
    if (t0 < A.ntiles) load_x(t0);

    for (int t = t0; t < A.ntiles; t += gridDim.x) {
        const int n = t / A.tiles, tix = t - n * A.tiles;
        const int ty = tix / A.ntw, tx = tix - ty * A.ntw;
        const int h0 = ty * TH, w0 = tx * TW;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMAs (and stores) done
        cs_barrier();

        // P1: conv1 over the halo tile, X -> T1 (zero outside the image)
        if constexpr (!TAIL) {
        cs_phase<T, NC, NI>(
                lds0 + L.w1, XP,
                [&](int px, int k) { return LX + (unsigned)(px * SX + 16 * k + 8 * hh) * 2; },
                [&](int a, int px, const f32x16& acc) {
                    uint4 o[2];
                    cs_act<T>(acc, lds0 + L.b1 + (32 * a + 16 * hh) * 4, o);
                    const int r = px / XW, cc = px - r * XW;
                    const int gh = h0 - 2 + r, gw = w0 - 2 + cc;
                    if (!((unsigned)gh < (unsigned)A.H && (unsigned)gw < (unsigned)A.W)) o[0] = o[1] = make_uint4(0, 0, 0, 0);
                    const unsigned d = LT + (unsigned)(px * ST + 32 * a + 16 * hh) * 2;
                    cs_wr(d, o[0]);
                    cs_wr(d + 16, o[1]);
                });
        cs_barrier();
        if (t + (int)gridDim.x < A.ntiles) load_x(t + gridDim.x);   // X is dead: next tile's input
        }

        // P2: Residual conv1 (3x3, b -> R1) over the 1-pixel halo region
        cs_phase<T, 1, 9 * NC>(
            lds0 + L.w2, MP,
            [&](int px, int k) {
                const int cb = k / 9, tap = k - 9 * (k / 9), kh = tap / 3, kw = tap - 3 * (tap / 3);
                const int r = px / MW, cc = px - r * MW;
                return LT + (unsigned)(((r + kh) * XW + cc + kw) * ST + 16 * NC + 16 * cb + 8 * hh) * 2;
            },
            [&](int, int px, const f32x16& acc) {
                if (16 * hh >= 16 * NH) return;
                uint4 o[2];
                cs_act<T>(acc, lds0 + L.b2 + 16 * hh * 4, o);
                const int r = px / MW, cc = px - r * MW;
                const int gh = h0 - 1 + r, gw = w0 - 1 + cc;
                if (!((unsigned)gh < (unsigned)A.H && (unsigned)gw < (unsigned)A.W)) o[0] = o[1] = make_uint4(0, 0, 0, 0);
                const unsigned d = LR + (unsigned)(px * SR + 16 * hh) * 2;
                cs_wr(d, o[0]);
                cs_wr(d + 16, o[1]);
            });
        cs_barrier();

        // P3: Residual conv2 (3x3, R1 -> C2) + b over the tile
        cs_phase<T, NA3, 9 * NH>(
                lds0 + L.w3, NP,
                [&](int px, int k) {
                    const int cb = k / 9, tap = k - 9 * (k / 9), kh = tap / 3, kw = tap - 3 * (tap / 3);
                    const int r = px / TW, cc = px - r * TW;
                    return LR + (unsigned)(((r + kh) * MW + cc + kw) * SR + 16 * cb + 8 * hh) * 2;
                },
                [&](int a, int px, const f32x16& acc) {
                    const int co = 32 * a + 16 * hh;
                    if (co >= 16 * NC) return;
                    uint4 o[2];
                    cs_act<T>(acc, lds0 + L.b3 + co * 4, o);
                    const int r = px / TW, cc = px - r * TW;
                    const unsigned rs = LT + (unsigned)(((r + 2) * XW + cc + 2) * ST + 16 * NC + co) * 2;
#pragma unroll
                    for (int hf = 0; hf < 2; ++hf) {
                        const uint4 rv = cs_rd(rs + 16 * hf);
                        const T* ov = reinterpret_cast<const T*>(&o[hf]);
                        const T* rr = reinterpret_cast<const T*>(&rv);
                        T s[8];
#pragma unroll
                        for (int e = 0; e < 8; ++e) s[e] = fromf<T>(tof(ov[e]) + tof(rr[e]));
                        o[hf] = *reinterpret_cast<const uint4*>(s);
                    }
                    const unsigned d = LC + (unsigned)(px * SC + co) * 2;
                    cs_wr(d, o[0]);
                    cs_wr(d + 16, o[1]);
                });
        cs_barrier();

        // P4: conv2 over cat [a | b | C2] -> block output
        cs_phase<T, NO, 3 * NC>(
                lds0 + L.w4, NP,
                [&](int px, int k) {
                    const int r = px / TW, cc = px - r * TW;
                    return k < 2 * NC ? LT + (unsigned)(((r + 2) * XW + cc + 2) * ST + 16 * k + 8 * hh) * 2
                                      : LC + (unsigned)(px * SC + 16 * (k - 2 * NC) + 8 * hh) * 2;
                },
                [&](int a, int px, const f32x16& acc) {
                    uint4 o[2];
                    const int co = 32 * a + 16 * hh;
                    cs_act<T>(acc, lds0 + L.b4 + co * 4, o);
                    const int r = px / TW, cc = px - r * TW;
                    const int gh = h0 + r, gw = w0 + cc;
                    if ((unsigned)gh < (unsigned)A.H && (unsigned)gw < (unsigned)A.W) {
                        uint4* d = reinterpret_cast<uint4*>(y + (((long long)n * A.H + gh) * A.W + gw) * A.ldy + co);
                        d[0] = o[0];
                        d[1] = o[1];
                    }
                });
        if constexpr (TAIL) {   // T1 is read until here: the next tile's input after a barrier
            cs_barrier();
            if (t + (int)gridDim.x < A.ntiles) load_x(t + gridDim.x);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// instantiated (ni, nc, no): v11_n p2.1 (2, 1, 2), p3.1 and v11_s p2.1 (4, 2, 4); tail mode
// (ni = 0): v11_n fpn.h2 (0, 2, 2), p3.1 (0, 2, 4)
#define YH_CSP_LIST(X) X(2, 1, 2) X(4, 2, 4) X(0, 2, 2) X(0, 2, 4)

template <typename T>
int launch_csp_t(const CspArgs& a, int grid, hipStream_t s) {
    const int lds = csp_lds(a.TH, a.TW, a.ni, a.nc, a.no);
    if (lds == 0 || grid <= 0 || a.ldx % 8 || a.ldy % 8) return (int)hipErrorInvalidValue;
#define YH_CSP_CASE(NI, NC, NO)                                                                              \
    if (a.ni == NI && a.nc == NC && a.no == NO) {                                                            \
        static bool attr = false;                                                                            \
        if (!attr) {                                                                                         \
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&csp_fused<T, NI, NC, NO>),              \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);               \
            attr = true;                                                                                     \
        }                                                                                                    \
        hipLaunchKernelGGL((csp_fused<T, NI, NC, NO>), dim3((unsigned)grid), dim3(CSP_THREADS), lds, s, a); \
        return (int)hipGetLastError();                                                                       \
    }
    YH_CSP_LIST(YH_CSP_CASE)
#undef YH_CSP_CASE
    return (int)hipErrorInvalidValue;
}

}  // namespace

int csp_prm_bytes(int ni, int nc, int no) { return cs_layout(ni, nc, no).prm; }

void csp_offsets(int ni, int nc, int no, int (&off)[9]) {
    const CsLayout L = cs_layout(ni, nc, no);
    const int v[9] = {L.w1, L.w2, L.w3, L.w4, L.b1, L.b2, L.b3, L.b4, L.prm};
    for (int i = 0; i < 9; ++i) off[i] = v[i];
}

int csp_lds(int TH, int TW, int ni, int nc, int no) {
    bool inst = false;
#define YH_CSP_HAS(NI, NC, NO) inst = inst || (ni == NI && nc == NC && no == NO);
    YH_CSP_LIST(YH_CSP_HAS)
#undef YH_CSP_HAS
    if (!inst || TH < 1 || TW < 1) return 0;
    const int b = cs_tile(TH, TW, ni, nc, no).total;
    return b <= 160 * 1024 ? b : 0;
}

int launch_csp(int dtype, const CspArgs& a, int grid, hipStream_t s) {
    switch (dtype) {
        case F16: return launch_csp_t<_Float16>(a, grid, s);
        case BF16: return launch_csp_t<__bf16>(a, grid, s);
    }
    return (int)hipErrorInvalidValue;
}

}  // namespace yh
