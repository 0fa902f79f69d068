// Shared device-side types and launcher declarations for the gfx950 YOLOv11 path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace yh {

enum DType { F32 = 0, F16 = 1, BF16 = 2 };
inline int dtype_size(int dt) { return dt == F32 ? 4 : 2; }

enum Act { ACT_ID = 0, ACT_SILU = 1 };

// Dense conv as an implicit GEMM over NHWC activations.
//   GEMM rows M  = batch * Ho * Wo (output pixels)
//   GEMM cols N  = Cout (physical, multiple of 8)
//   reduction K  = KH * KW * Cin (Cin physical, multiple of 8), packed weights
//                  are [Coutp][Kp] with k = (kh*KW + kw)*Cin + ci, zero padded.
// The input may be the channel-concatenation of two NHWC views ("segments");
// a segment may be read through a nearest x2 upsample (up = 1), which is how
// DarkFPN's up+cat (nets/nn.py:203-209) is fused into the consumer's loader.
struct ConvArgs {
    const void* in0; int ldc0, c0, up0, h0, w0;   // segment 0: channels [0, c0)
    const void* in1; int ldc1, c1, up1, h1, w1;   // segment 1: channels [c0, c0+c1)
    int Hi, Wi, Ho, Wo, stride, pad, KH, KW, Cin, K, Kp, M;
    const void* w;       // packed weights, handle dtype
    const float* bias;   // [Coutp] fp32
    const int* ktab;     // [Kp/8]: (kh<<24)|(kw<<16)|ci, ci=0xffff for padding
    void* out; int ldo;  // output view base (channel offset applied), pixel stride
    const void* res; int ldr;  // optional residual view added after the activation
    int Cout;            // physical output channels written (multiple of 8)
    int act;
    int gm, gn;          // tile grid
    const void* zero;    // >= 16 zero bytes in device memory (source of padded taps)
    int ks;              // > 1: K split over the workgroup's waves (conv_gemm2k), set by
                         //      the engine's shape rule for 16-bit handles
};

// First layer: 3-channel NCHW input (the caller's tensor), 3x3 stride-2 conv.
struct FirstConvArgs {
    const void* const* io;  // io[0] = x (NCHW), read at kernel start (graph-replay friendly)
    int H, W, Ho, Wo, Cout, ldo, M;
    const float* w;      // [Cout][27] fp32 (ci, kh, kw)
    const float* bias;   // [Cout]
    void* out;
    int act;
    int in_u8;           // 1: x is uint8 (the loader's image tensor); the kernel applies
                         //    main.py:265-267's `x.to(dtype) / 255` while staging it
};

// Stem + net.p2.0 fused (nets/nn.py:160-163): the stem output stays in LDS.
struct Stem2Args {
    const void* const* io;   // io[0] = x (NCHW, 3 channels; uint8 when in_u8)
    int H, W, Hs, Ws, Ho, Wo, B;
    const float* w1;         // stem weights [27][c1p] fp32 (k = ci*9 + kh*3 + kw)
    const float* b1;         // stem bias [c1p]
    int c1, c1p, c2;         // stem couts, its padded stride in w1, p2.0 couts
    const void* prm;         // p2.0 fragments (c2/32 tiles x 9*c1/16 steps x 1 KB, MFMA lane order) + fp32 bias
    int prm_bias;            // byte offset of the bias in prm
    void* out; int ldo;      // p2.0 output view
    int in_u8;
    int ntw, nth;            // tiles per row / per column (stem2_tiles)
};
bool stem2_ok(int c1, int c2);
void stem2_tiles(int Ho, int Wo, int& ntw, int& nth);
int launch_stem2(int dtype, const Stem2Args& a, hipStream_t s);

// Depthwise 3x3 stride-1 conv on an NHWC view.
struct DwArgs {
    const void* in; int ldi;
    int H, W, C, M;
    const float* w;      // [9][C] fp32
    const float* bias;   // [C]
    void* out; int ldo;
    int act;
};

// SPPF: y1 = mp5(x), y2 = mp5(y1), y3 = mp5(y2) (nets/nn.py:90-94) from slice 0
// of a 4-slice concat buffer into slices 1..3.
struct PoolArgs {
    void* buf; int ldc, C, H, W, B;
};

// C2PSA attention (nets/nn.py:111-123) with the positional depthwise conv fused:
// out[:, h*dh + d] = softmax(q^T k * scale) v  +  pe(v)
struct AttnArgs {
    const void* qkv; int ldq;   // per head: [q(dk) | k(dk) | v(dh)]
    int T, Hs, Ws, heads, dk, dh;
    float scale;
    const float* pe_w;   // [9][heads*dh]
    const float* pe_b;   // [heads*dh]
    void* out; int ldo;
};

// Detect-head decode (nets/nn.py:255-270, DFL 222-225, make_anchors util.py:85-96).
struct DecodeArgs {
    const void* lvl[3]; int ldc; int H[3], W[3]; float stride[3];
    int nc, A, B;
    const void* const* io;  // io[1] = y (B, 4+nc, A)
    int a_lo;               // first anchor decoded (anchors [a_lo, A))
    int box;                // 0: class rows only (the box rows come from box_dfl)
};

// NMS (utils/util.py:123-169)
struct NmsArgs {
    const void* y; int B, A, nc;
    float conf;          // threshold, already rounded to the input dtype
    float iou;           // largest float <= iou threshold (so ovr > iou  <=>  ovr > thr)
    float max_wh;
    int max_det, max_nms;
    int* counts;               // [B] candidate counts (zeroed by nms_zero)
    unsigned* hist;            // [B][2048] coarse score-bin histogram (zeroed by the launcher)
    int bin_base;              // (fp32 bits >> 16) of the lowest bin
    float* dets; int* ndet;
    // first-batch scratch of the split greedy (nms.hip): per image a state record, the
    // decoded entries in score order and the lower-triangular IoU bitmask
    unsigned long long* state;  // [B][8]
    unsigned long long* gkeys;  // [B][4096]: the first batch's keys (unordered)
    float* ents;                // [B][3][4096][4]: offset box, plain box, (area, score, class, -)
    unsigned long long* mask;   // [B][64 * 64 * 65 / 2] words
#ifdef YH_ABLATION
    unsigned long long* trace;  // diagnostic builds only: [B][16] phase timestamps (s_memrealtime)
    int dbg;                    // diagnostic builds only: ablation bits (YH_NMS_DBG, nms.hip)
#endif
};

// Dense-conv kernel of the fp32 handle (conv.hip). The 16-bit handles run the
// conv_mx family (conv_mx.h).
enum ConvKernel { CONV_GEMM = 0 };

// Fused cls branch of the detect head (nets/nn.py:244-252), one launch for all levels:
//   DWConv 3x3 + SiLU -> Conv 1x1 + SiLU -> DWConv 3x3 + SiLU -> Conv 1x1 + SiLU
//   -> Conv2d 1x1 (+ bias)
// per TH x TW output tile, every intermediate in LDS (halo recomputed), bit-identical
// to the five separate launches (same per-channel FMA order, same MFMA K order, one
// rounding to the handle dtype per layer output).
struct HeadClsLevel {
    const void* x; int ldx, C0;      // level input (NHWC view), channels
    int H, W;
    void* y; int ldy;                // output view (the head tensor's cls slice)
    int aoff;                        // direct mode: the level's first anchor
    const float* dw1w; const float* dw1b; int dw1ld;   // [9][dw1ld] fp32, bias
    const void* pw1w; int pw1ld; const float* pw1b;    // [rows][pw1ld] dtype, bias
    const float* dw2w; const float* dw2b; int dw2ld;
    const void* pw2w; int pw2ld; const float* pw2b;
    const void* pw3w; int pw3ld; const float* pw3b;
    int TH, TW, ntw, tiles;          // output tile, tiles per row, tiles per image
    int wg0;                         // first workgroup of the level (one workgroup per tile)
};
struct HeadClsArgs {
    HeadClsLevel lv[3];
    int nlv, B, c3, nc;
    const void* zero;                // >= 16 zero bytes (source of out-of-image / padding chunks)
    // direct mode (io != nullptr): pw3's logits leave as sigmoid scores in rows 4.. of the
    // caller's y = io[1] (B, 4+nc, A) instead of the head tensor (the decode's class part)
    const void* const* io; int A;
};
#ifndef YH_HEAD_CLS_THREADS
#define YH_HEAD_CLS_THREADS 512
#endif
// 8-wave workgroups, two per CU (16 waves); 256 = the round-2 4-wave kernel (fragments
// preloaded a phase ahead), 7 % slower (profiles/r03_ops_hcls_{256,512}.txt)
constexpr int HEAD_CLS_THREADS = YH_HEAD_CLS_THREADS;
#ifndef YH_HEAD_CLS_LDS_KB
#define YH_HEAD_CLS_LDS_KB 80
#endif
constexpr int HEAD_CLS_LDS = YH_HEAD_CLS_LDS_KB * 1024;   // 80: two workgroups (16 waves) per CU, 8x16 tiles at 80x80
// LDS bytes of a tile's buffers; 0 if it does not fit
int head_cls_lds(int TH, int TW, int C0, int c3, int nc);
int launch_head_cls(int dtype, const HeadClsArgs& a, hipStream_t s);

// Fused C3k block (c3k.hip; nets/nn.py:52-63 CSPModule(c, c), c = 2 hh, two Residual(hh,
// e=1.0), hh = 32 or 64): every intermediate of a band of rows (+ the 4-row halo of the four
// 3x3 convs) in one workgroup's LDS. Maps whose bands of >= 4 rows keep <= 512 pixels (v11_n's
// 40x40 hh = 32 and 20x20 hh = 64 blocks at 640 x 640); bit-identical to the seven
// per-layer launches.
struct C3kArgs {
    const void* x; int ldx;          // block input (NHWC view, c channels)
    void* y; int ldy;                // block output view (c channels)
    int B, H, W;
    const void* prm;                 // packed parameters (c3k_offsets)
    int hh;                          // hidden channels (32 or 64)
    int bands;                       // row bands per image (set by launch_c3k: c3k_bands)
    int nbuf;                        // weight ring buffers (set by launch_c3k)
    unsigned long long* trace;       // micro benchmark builds (YH_ABLATION): per-workgroup stamps
};
int c3k_prm_bytes(int hh);
void c3k_offsets(int hh, int (&off)[9]);   // w1, w2, residual convs, w3, b1, b2, residual biases, b3, total
int c3k_lds(int H, int W, int hh);   // 0: no band split fits
int c3k_bands(int B, int H, int W, int hh);   // row bands per image (one workgroup each)
int c3k_region_px(int H, int W, int bands);   // LDS pixels of a band's region (band + 4-row halo)
int launch_c3k(int dtype, const C3kArgs& a, hipStream_t s);

// Box tail of the detect head, one launch for all levels: the last box conv (Conv2d 1x1
// + bias, nets/nn.py:241) with DFL (nn.py:222-225), make_anchors (utils/util.py:85-96) and
// dist2bbox (nn.py:264-268) in its epilogue, writing rows 0..3 of y = io[1]. Bit-identical
// to the conv launch + head_decode (same MFMA K order, logits rounded to the dtype first).
struct BoxDflLevel {
    const void* x; int ldx;          // box.l.1 output (NHWC), K = 16 * nk channels
    int H, W; float stride; int aoff;
    const void* w; int wld; const float* b;   // [64][wld] dtype weights, fp32 bias
    int wg0;                         // first workgroup of the level
};
struct BoxDflArgs {
    BoxDflLevel lv[3];
    int nlv, B, nk, nc, A;
    const void* const* io;
    int tpw;   // 32-pixel tiles per wave: 1, 2 or 4 (wg0 offsets are computed with it)
};
// Fused C3k2 block with one Residual bottleneck (nets/nn.py:66-80 with n = 1 and
// csp = False; Residual nn.py:42-49): conv1 1x1 (Cin -> 2c) -> split [a | b] ->
// b + conv3x3(conv3x3(b)) (c -> c/2 -> c) -> cat [a | b | r] -> conv2 1x1 (3c -> cout),
// every Conv with SiLU. A persistent workgroup walks TH x TW output tiles; the input tile
// (2-pixel halo) and every intermediate stay in LDS, the packed weights too. Bit-identical
// to the four conv_mx launches (same K order, one rounding per layer output, the residual
// added after the rounding and rounded again).
struct CspArgs {
    const void* x; int ldx;          // block input (NHWC view), Cin = 16 * ni channels
    void* y; int ldy;                // block output view, cout = 32 * no channels
    int H, W, B;
    const void* prm;                 // packed weight fragments + fp32 biases (csp_prm_bytes)
    int ni, nc, no;                  // Cin / 16, c / 16, cout / 32
    int TH, TW, ntw, tiles, ntiles;  // output tile, tiles per row / per image / in total
    const void* zero;                // >= 16 zero bytes
};
#ifndef YH_CSP_THREADS
#define YH_CSP_THREADS 1024
#endif
constexpr int CSP_THREADS = YH_CSP_THREADS;
// bytes of the packed parameter image (weight fragments in MFMA lane order + biases)
int csp_prm_bytes(int ni, int nc, int no);
// byte offsets of the parameter image: w1, w2, w3, w4 (fragments), b1, b2, b3, b4 (fp32), total
void csp_offsets(int ni, int nc, int no, int (&off)[9]);
// LDS bytes for a TH x TW tile, 0 if it does not fit or (ni, nc, no) is not instantiated
int csp_lds(int TH, int TW, int ni, int nc, int no);
int launch_csp(int dtype, const CspArgs& a, int grid, hipStream_t s);

constexpr int BOX_DFL_TPW = 2;       // 32-pixel tiles per wave (4 waves per workgroup; YH_BOXDFL_TPW: 1 / 2 / 4)
int launch_box_dfl(int dtype, const BoxDflArgs& a, hipStream_t s);

// The whole box branch of the detect head (boxc.hip), one launch for all levels: box.l.0 (3x3
// C0 -> 64) -> box.l.1 (3x3 64 -> 64) -> box.l.2 (1x1 64 -> 64 + bias) -> DFL + anchors +
// dist2bbox into rows 0..3 of y = io[1] (nets/nn.py:240-247, 222-225, 255-270), the two 64-channel
// intermediates only in LDS. Bit-identical to the per-layer launches + box_dfl.
struct BoxChainLevel {
    const void* x; int ldx, C0;      // box.l.0 input (NHWC view), its channels (64 / 128 / 256 / 512)
    int H, W;
    int TH, TW, ntw, tiles;          // output tile, tiles per row / per image (bx_tile)
    int nkc;                         // box.l.0's K chunks (mx_kchunks of its shape: 1 or C0 / 64)
    float stride; int aoff;          // the level's stride and first anchor
    const void* prm;                 // packed parameters (bx_prm_bytes(C0))
    int wg0;                         // first workgroup of the level (one per tile)
};
struct BoxChainArgs {
    BoxChainLevel lv[3];
    int nlv, B, nc, A;
    const void* const* io;
    const void* zero;                // >= 256 zero bytes
};
int bx_prm_bytes(int C0);
bool bx_ok(int C0);
bool bx_tile(int H, int W, int& TH, int& TW);
int launch_box_chain(int dtype, const BoxChainArgs& a, hipStream_t s);

// Pointwise chain (pwchain.hip): consecutive 1x1 convs of one map as one launch. A workgroup
// owns P consecutive pixels (flattened n, h, w) and runs the stages in order; a stage's input
// channels come in runs of whole 128-channel pieces, each from the LDS copy of an earlier
// stage's output or from a global view loaded into LDS in the prologue.
constexpr int PWC_THREADS = 512;
constexpr int PWC_MAX_STAGES = 6, PWC_MAX_RUNS = 4, PWC_MAX_LOADS = 6;
struct PwcRun {
    int lds;   // LDS byte offset of the run's first channel at pixel 0
    int ld;    // pixel stride of that LDS region (elements)
    int nkb;   // 16-channel blocks (a multiple of 8)
};
struct PwcStage {
    int K, N, act, nrun;
    PwcRun run[PWC_MAX_RUNS];
    const void* w; int wld;            // 16-bit weights in A-fragment order: fragment (a, kb) = 1 KB at
                                       // (a * (wld / 16) + kb) KB, lane-major (engine upload "pwfrag")
    const float* bias;                 // >= N floats
    int res_lds, res_ldl;              // residual in LDS (byte offset of channel 0, stride) or -1; a
                                       // residual no stage of the chain writes comes by the prologue
    void* out; int ldo;                // global output view (channel 0) and pixel stride
    int out_lds, out_ldl;              // LDS copy of the output (byte offset, stride) or -1
};
struct PwcLoad {
    const void* g; int ldg;            // global view (channel 0) and pixel stride (elements)
    int lds;                           // LDS byte offset; pixel stride nchunk + 1 16-B chunks
    int nchunk;                        // 16-B chunks (8 channels) per pixel
};
struct PwChainArgs {
    long long M;                       // pixels of the map (B * H * W)
    int P, nst, nload;
    int sink;                          // LDS byte offset of a scratch KB (weight warm-up DMAs)
    PwcStage st[PWC_MAX_STAGES];
    PwcLoad ld[PWC_MAX_LOADS];
    const void* zero;                  // >= 16 zero bytes
};
int launch_pw_chain(int dtype, const PwChainArgs& a, int lds, hipStream_t s);

// launchers (return hipError_t as int)
bool conv_kernel_ok(int dtype, int kern, const ConvArgs& a);
int launch_conv(int dtype, int kern, int BM, int BN, const ConvArgs& a, hipStream_t s);
int conv_lds_bytes(int dtype, int BM, int BN, int Kp);
int launch_first_conv(int dtype, const FirstConvArgs& a, int B, hipStream_t s);
int launch_dwconv(int dtype, const DwArgs& a, hipStream_t s);
int launch_sppf(int dtype, const PoolArgs& a, hipStream_t s);
int launch_attention(int dtype, const AttnArgs& a, int B, hipStream_t s);
int launch_decode(int dtype, const DecodeArgs& a, hipStream_t s);
int launch_set_io(void** io, const void* x, void* y, hipStream_t s);
int launch_nms(int dtype, const NmsArgs& a, hipStream_t s);

}  // namespace yh
