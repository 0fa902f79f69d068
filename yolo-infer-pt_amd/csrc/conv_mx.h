// conv_mx: the dense-conv kernel family of the 16-bit handles (bf16 / fp16) on
// v_mfma_f32_32x32x16. Host-side planning (task geometry, LDS layout, bank
// swizzle) and weight packing are shared by the engine and the micro benchmark.
//
// Reference ops: Conv (nets/nn.py:28-39) with k in {1, 3}, s in {1, 2}, plus the
// Residual add (nets/nn.py:49), the C3k2 / C3k / SPPF / C2PSA concats
// (nn.py:52-148, 203-209: channel-slice views) and DarkFPN's nearest x2 upsample
// (nn.py:195, 205-206: folded into the pixel gather).
//
// Canonical reduction order (every kernel of the family follows it, so every
// plan of a layer gives bit-identical outputs and the tuner may pick freely):
//   the input channels are cut into 16-channel blocks cb (channels past Cin are
//   zero); the K walk is  for cb: for tap (kh, kw) row-major:  one 32x32x16 MFMA
//   step accumulating W[co][cb*16 .. +16][tap] . X[cb*16 .. +16][tap-shifted pixel].
// K-split layers (mx_kchunks > 1: 3x3 convs with 128 / 256 input channels on maps of at
// most 40 x 40): the walk is cut into 64-channel chunks, each chunk's partial sum runs the
// order above from zero, and the partials are added in chunk order (((P0 + P1) + P2) + P3)
// in fp32 before the bias. Every plan of such a layer (conv_rw kinds only) follows it.
#pragma once
#include <stdint.h>
#include <vector>
#include "common.h"

namespace yh {

// q = (umulhi(x, m) + x) >> s  for every 32-bit x (Granlund-Montgomery, 64-bit add)
struct FastDiv {
    uint32_t m = 1, s = 0;
};
inline FastDiv make_fastdiv(uint32_t d) {
    FastDiv f;
    uint32_t l = 0;
    while ((1ull << l) < d) ++l;
    f.s = l;
    f.m = (uint32_t)(((((unsigned __int128)1) << 32) * ((1ull << l) - d)) / d + 1);
    return f;
}

constexpr int MX_MAXB = 8;   // B-patch DMA instructions per wave per stage (max)

struct MxArgs {
    const char* in0; const char* in1;   // segment bases (bytes): channels [0, c0) | [c0, cin)
    int ldc0, ldc1;                     // pixel strides in elements
    int c0;                             // channels of segment 0 (a multiple of 16*NCB when c1 > 0)
    int cin;                            // physical input channels; chunks >= cin/8 read zero
    int up0, up1;                       // nearest x2 upsample of a segment (1x1 only)
    int hs0, ws0, hs1, ws1;             // source spatial sizes of the segments
    int Hi, Wi, Ho, Wo, B;
    int nst;                            // K stages per task = ceil(cb blocks / NCB)
    const char* w;                      // packed stage images [slice][stage][wstage bytes]
    int wstage;                         // bytes of one stage image (padded to the DMA grain)
    const float* bias;                  // [cout padded]
    char* out; int ldo;                 // output view (channel offset applied), pixel stride (elements)
    const char* res; int ldr;           // optional residual view, added after the activation
    int cout;                           // physical couts written
    int act;
    const char* zero;                   // >= 16 zero bytes
    // tasks: KS == 3: TH x TW output tiles of one image; KS == 1: TW consecutive pixels (TH = 1)
    int TH, TW, ntw, nth, nslices, ntasks;
    int bc_log2;                        // B tile = (32 >> bc_log2) rows x (1 << bc_log2) cols (KS == 3)
    int PC, PR;                         // stored patch cols / rows
    int nbi;                            // B-patch DMA instructions per wave per stage (<= MX_MAXB)
    int sw_sh, sw_mr;                   // bank swizzle f(rs, lc) = ((lc >> sh) + rs * mr) & (CPs - 1)
    FastDiv d_pcc, d_cps;               // divide by PC*CPs (patch row), CPs
    FastDiv d_wo, d_howo;               // KS == 1: flat pixel -> (n, ho, wo)
    FastDiv d_ntw, d_nth, d_nsl;        // task id decomposition
    int M;                              // B * Ho * Wo
    int pc_delay;                       // conv_rw counter mode: s_sleep(32) rounds of the late half
#ifdef YH_ABLATION
    // tools/micro builds only (-DYH_ABLATION; the shipped library has neither field):
    int dbg;                            // 1 no weight DMA, 2 no patch DMA, 4 no MFMA, 8 no epilogue
                                        // stores; conv_mxr also 16 no SiLU, 1024 no resident-weight load
    unsigned long long* trace;          // [grid][4] s_memrealtime stamps (nullptr = off)
#endif
};

// One kernel configuration (template parameters of conv_mx).
struct MxConfig {
    int kind = 0;     // 0: conv_mx (staged weights, workgroup-synchronous stages)
                      // 1: conv_mxr (resident weights, per-wave pipelines); wm = waves, wn = 1
                      // 2: conv_rw (weights in VGPRs, shared patch ring; conv_rw.hip):
                      //    na = wn = 32-cout groups, wm = pixel groups, tw = tile width,
                      //    nbuf = patch slots
    int ks, s;        // kernel size (1 / 3), stride (1 / 2)
    int na, mb;       // per wave: na 32-cout A tiles x mb 32-pixel B tiles
    int wn, wm;       // waves along couts x along pixels
    int ncb;          // 16-channel blocks per stage
    int nbi = 0;      // conv_mxr: patch DMA instructions per wave per stage (template)
    int nbuf = 2;     // conv_mxr: patch buffers per wave (1: the next stage's DMA waits for this compute)
    int tw = 0;       // conv_rw: output tile width (template)
    int gdiv = 1;     // conv_rw: workgroups = (one per CU share) / gdiv (fewer weight-image loads)
    int nkc = 1;      // conv_rw: 64-channel K chunks, one wave each (mx_kchunks of the layer)
    int pc = 0;       // conv_rw: 1 = no per-tile workgroup barrier: slot hand-offs through LDS
                      //    counters, tiles issued nbuf - 2 ahead, the second half of the waves
                      //    started half a tile late (conv_rw.hip, "counter mode")
    int bn() const { return 32 * na * wn; }
    int nw() const { return wn * wm; }
};

// A planned layer: config + geometry + the LDS / DMA sizes the launcher needs.
struct MxPlan {
    MxConfig cfg{};
    int TH = 0, TW = 0, bc_log2 = 0, PC = 0, PR = 0;
    int nbi = 0, ains = 0;         // DMA instructions per wave per stage (B patch / A weights)
    int abytes = 0, bbytes = 0;    // LDS bytes per stage
    int lds = 0;                   // total dynamic LDS
    int sw_sh = 0, sw_mr = 0, conflicts = 0;
    int nst = 0, nslices = 0, ntasks = 0, ntw = 0, nth = 0;
    int grid = 0;
    int wstage = 0;                // bytes of one packed weight stage image
    bool ok = false;
};

// Layer shape as the planner sees it.
struct MxShape {
    int ks, s, cin, cout, Hi, Wi, Ho, Wo, B;
    int c0, c1;        // segment channel counts (c1 = 0: single segment)
    int up0, up1;
    int ldo = 0, ldr = 0;   // output / residual pixel strides (0: cout); conv_rw's 32-bit offsets
};

// conv_rw geometry of a configuration (stride, input channels, cout groups, pixel groups,
// B tiles per wave, tile width): waves, 16-B chunks per pixel, k-steps, tile pixels and
// rows, patch rows / cols, DMA instructions per wave per tile, bytes per patch slot
struct RwGeo {
    int nw, cpp, nks, tpx, th, pr, pc, nbi, nbr, slot;   // nbr: residual DMA instructions (res)
    int red;                                             // LDS bytes of the K-chunk partials
    int epi;                                             // LDS bytes of the epilogue staging tiles
};
RwGeo rw_geo(int S, int cin, int ncg, int npg, int mb, int tw, bool res, int nkc);
// K chunks of a layer's canonical order (1: the plain walk). Shape-dependent (kernel,
// stride, channels, output map) but batch-independent, so a batch-N forward equals N
// batch-1 forwards whatever plans the tuner picks.
inline int mx_kchunks(const MxShape& sh) {
    if (sh.ks != 3 || sh.c1 != 0 || sh.up0 != 0 || sh.cout % 64 || (long long)sh.Ho * sh.Wo > 1600) return 1;
    if (sh.s == 1 && (sh.cin == 128 || sh.cin == 256)) return sh.cin / 64;
    if (sh.s == 2 && sh.cin == 128) return 2;
    return 1;
}
MxPlan mx_plan_w(const MxShape& sh, const MxConfig& cfg, int num_cus);
void mx_candidates_w(const MxShape& sh, std::vector<MxConfig>& out);
std::vector<uint16_t> mx_pack_w(const MxPlan& pl, const MxShape& sh, const float* wf, int cin_logical,
                                const std::vector<int>& phys2log, bool bf16, int cout_logical);
int launch_rw(int dtype, const MxPlan& pl, const MxArgs& a, hipStream_t s);

// Candidate configurations for a layer (each with a feasible plan); the first is the
// heuristic default.
std::vector<MxPlan> mx_candidates(const MxShape& sh, int num_cus);
MxPlan mx_plan(const MxShape& sh, const MxConfig& cfg, int num_cus);

// Pack folded fp32 weights W[cout][cin_logical/g..][k][k] into the stage images of a
// plan. `phys2log[c]` maps a physical input channel to its logical channel (-1 = pad).
// Output: 16-bit values (bf16 if bf16, else fp16), size = nslices * nst * wstage / 2.
std::vector<uint16_t> mx_pack(const MxPlan& pl, const MxShape& sh, const float* wf, int cin_logical,
                              const std::vector<int>& phys2log, bool bf16, int cout_logical);

// Fill the runtime arguments (everything but pointers/strides the caller sets).
void mx_fill_args(const MxPlan& pl, const MxShape& sh, MxArgs& a);

int launch_mx(int dtype, const MxPlan& pl, const MxArgs& a, hipStream_t s);

}  // namespace yh
