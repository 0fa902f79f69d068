// Host runtime of the gfx950 YOLOv11 path: builds the layer graph of a variant
// (mirroring the reference module tree, nets/nn.py:28-305), folds BatchNorm into
// the convs exactly like fuse_conv (nets/nn.py:8-25), packs weights for the
// implicit-GEMM kernels, owns the NHWC activation workspace, launches the
// kernels (optionally as one captured HIP graph) and exports the C ABI
// declared in include/yolo_hip.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "common.h"
#include "conv_mx.h"
#include "yolo_hip.h"


namespace yh {

static thread_local std::string g_err;

struct Fail : std::runtime_error {
    int code;
    Fail(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIPCHECK(expr)                                                                 \
    do {                                                                               \
        hipError_t e__ = (expr);                                                       \
        if (e__ != hipSuccess)                                                         \
            throw Fail(YH_EHIP, std::string(#expr) + ": " + hipGetErrorString(e__));   \
    } while (0)

static void require(bool ok, const std::string& msg, int code = YH_EINVAL) {
    if (!ok) throw Fail(code, msg);
}

static int round_up(int v, int m) { return (v + m - 1) / m * m; }

// ---------------------------------------------------------------- dtype casts
static uint16_t f2bf(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // NaN
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}
static uint16_t f2h(float f) {
    uint32_t x;
    std::memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u;
    const uint32_t ax = x & 0x7fffffffu;
    if (ax >= 0x7f800000u) return (uint16_t)(sign | 0x7c00u | (ax > 0x7f800000u ? 0x200u : 0u));
    if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);  // rounds to inf
    if (ax < 0x38800000u) {  // subnormal / zero in half
        float af;
        std::memcpy(&af, &ax, 4);
        const float scaled = af * 16777216.0f;  // 2^24: half subnormal unit = 2^-24
        const uint32_t m = (uint32_t)std::nearbyint(scaled);
        return (uint16_t)(sign | m);
    }
    uint32_t e = ((ax >> 23) - 112u) << 10;
    uint32_t m = (ax >> 13) & 0x3ffu;
    uint32_t h = e | m;
    const uint32_t rem = ax & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) ++h;
    return (uint16_t)(sign | h);
}

// ---------------------------------------------------------------- graph model
enum ConvKind { CK_DENSE = 0, CK_FIRST = 1, CK_DW = 2, CK_PE = 3 };
enum OpKind { OP_FIRST, OP_CONV, OP_DW, OP_SPPF, OP_ATTN, OP_DECODE, OP_HEADCLS, OP_BOXDFL, OP_CSP, OP_STEM2, OP_C3K,
              OP_BOXCHAIN, OP_PWCHAIN };
static const char* op_kind_name(OpKind k) {
    switch (k) {
        case OP_FIRST: return "stem";
        case OP_CONV: return "conv";
        case OP_DW: return "dwconv";
        case OP_SPPF: return "sppf";
        case OP_ATTN: return "attention";
        case OP_DECODE: return "decode";
        case OP_HEADCLS: return "head_cls";
        case OP_BOXDFL: return "box_dfl";
        case OP_CSP: return "c3k2";
        case OP_C3K: return "c3k";
        case OP_STEM2: return "stem_fused";
        case OP_BOXCHAIN: return "box_chain";
        case OP_PWCHAIN: return "pw_chain";
    }
    return "unknown";
}
enum OpClass { CL_CONV3 = 0, CL_CONV1 = 1, CL_FIRST = 2, CL_DW = 3, CL_SPPF = 4, CL_ATTN = 5, CL_DECODE = 6,
               CL_HEADCLS = 7, CL_BOXDFL = 8, CL_CSP = 9, CL_C3K = 10, CL_BOXCHAIN = 11, CL_PWCHAIN = 12, CL_N = 13 };

struct Tensor { int level; int C; };        // physical channels = pixel stride
struct View { int t = -1; int coff = 0; int C = 0; };

struct Seg { View v; int up = 0; };

struct ConvDesc {
    std::string name;
    ConvKind kind;
    int cout, cin, k, stride, groups, has_bias, act;
    std::vector<std::pair<int, int>> segs;   // (logical, physical) channel counts of the input
    int cin_p = 0, cout_p = 0, K = 0, Kp = 0, coutp_pad = 0;
    bool loaded = false;
    std::vector<float> wf, bf;  // folded fp32 weights (cout, cin/g, k, k) and bias (cout)
    void* w_dev = nullptr;
    float* b_dev = nullptr;
    int* ktab_dev = nullptr;
    std::vector<int> phys2log;                  // dense: physical input channel -> logical (-1 = pad)
    std::map<std::string, void*> mx_w;          // 16-bit dense: packed weights per conv_mx layout
};

struct Op {
    OpKind kind;
    int conv = -1;
    std::vector<Seg> in;
    View out, res;
    bool has_res = false;
    int heads = 0;
    View lvl[3];
    // OP_HEADCLS: per level (index = detect level 0..2) the five convs of the cls branch
    // (dw1, pw1, dw2, pw2, pw3), the level input and the head tensor's cls slice
    int hc[3][5] = {};
    View hx[3], hy[3];
    bool hlv[3] = {false, false, false};   // levels the fused op covers
    bool direct = false;                   // OP_HEADCLS: scores straight into y (decode folded in)
    // OP_BOXDFL: per level the last box conv and its input (the box.l.1 output)
    int bc[3] = {-1, -1, -1};
    View bx[3];
    // OP_DECODE: first level decoded, and whether the box rows are (false: box_dfl writes them)
    int dlo = 0;
    bool dbox = true;
    // OP_CSP: conv1, res_m.0.conv1, res_m.0.conv2, conv2 of a fused C3k2 block (in[0] -> out)
    // OP_STEM2: cs[0] = net.p2.0 (conv = the stem)
    int cs[4] = {-1, -1, -1, -1};
    // OP_C3K: conv1, conv2, res_m.0.conv1, res_m.0.conv2, res_m.1.conv1, res_m.1.conv2, conv3 of
    // a CSPModule, and the per-layer ops [alt0, alt1) it replaces at shapes where it fits
    int ck[7] = {-1, -1, -1, -1, -1, -1, -1};
    int alt0 = -1, alt1 = -1;
    // OP_BOXCHAIN: per level the box.l.0 / box.l.1 / box.l.2 convs (input hx[l]), the per-layer
    // ops it replaces at shapes where every level has a tile (bops: box.l.0 per level first)
    int bxc[3][3] = {{-1, -1, -1}, {-1, -1, -1}, {-1, -1, -1}};
    std::vector<int> alts;
    // OP_PWCHAIN: alts = the member 1x1 conv ops (stages, in order); per stage its input runs
    // (16-channel blocks in weight order: LDS region of an earlier stage's output, or a
    // prologue-loaded global view), its residual and whether its output is kept in LDS
    struct PwRun { int stage = -1; int coff = 0; int nch = 0; int load = -1; };   // coff: channel in the source
    struct PwStage { std::vector<PwRun> runs; int res_stage = -2; int res_coff = 0; int res_load = -1; bool keep = false; int lds = -1; };
    std::vector<PwStage> pws;
    std::vector<View> pwl;          // prologue loads (global views)
    std::vector<int> pwl_lds;       // their LDS byte offsets
    int pwP = 0, pwLds = 0;
    std::string label;
};

struct Workspace {
    int B = 0, H = 0, W = 0;
    void* base = nullptr;
    size_t bytes = 0;
    std::vector<size_t> off;  // per tensor
};

struct GraphKey {
    int B, H, W;
    int X = 0;   // input kind of a captured forward graph: 0 = handle dtype, 1 = uint8
    bool operator<(const GraphKey& o) const {
        return B != o.B ? B < o.B : (H != o.H ? H < o.H : (W != o.W ? W < o.W : X < o.X));
    }
};

// The library's few environment switches, read once per handle at yh_create
// (INTEGRATION.md lists them): YH_FUSE=0 turns every cross-layer fusion off (the
// bit-identity tests compare both), YH_CSP_TAIL=1 forces the C3k2 tail mode where
// the whole block would fit one launch (tested the same way), YH_CONV=<k> forces
// candidate plan k of every 16-bit dense conv, YH_TUNE_LOG=1 prints the tuner's timings,
// YH_C3K=0 keeps the C3k blocks as per-layer launches (compared bit for bit by the tests),
// YH_HCLS_WIDE=0 keeps a 256-channel level's cls branch (v11_n 20x20) as per-layer launches.
struct Options {
    bool fuse = true, csp_tail = false, tune_log = false, c3k = true, hcls_wide = true, box_chain = false, pw_chain = true;
    int conv_force = -1;
    static Options from_env() {
        Options o;
        if (const char* e = getenv("YH_FUSE")) o.fuse = atoi(e) != 0;
        if (const char* e = getenv("YH_BOXCHAIN")) o.box_chain = atoi(e) != 0;
        if (const char* e = getenv("YH_PWCHAIN")) o.pw_chain = atoi(e) != 0;
        if (const char* e = getenv("YH_CSP_TAIL")) o.csp_tail = atoi(e) != 0;
        if (const char* e = getenv("YH_C3K")) o.c3k = atoi(e) != 0;
        if (const char* e = getenv("YH_HCLS_WIDE")) o.hcls_wide = atoi(e) != 0;
        if (const char* e = getenv("YH_CONV")) o.conv_force = atoi(e);
        o.tune_log = getenv("YH_TUNE_LOG") != nullptr;
        return o;
    }
};

struct Net {
    yh_variant var;
    Options opt;
    int device, dtype, es;
    std::vector<Tensor> tensors;
    std::vector<ConvDesc> convs;
    std::vector<Op> ops;
    Workspace ws;
    void** io_dev = nullptr;      // {x, y}
    void* zero_dev = nullptr;     // 256 zero bytes: source of padded conv taps
    bool use_graph = true;
    std::map<GraphKey, hipGraphExec_t> graphs;
    hipStream_t cap_stream = nullptr;
    bool profile = false;
    std::vector<double> prof_ms;     // per launch unit of the profiled shape
    std::vector<int> prof_calls;
    GraphKey prof_key{0, 0, 0};
    std::vector<hipEvent_t> ev;
    int lastB = 0, lastH = 0, lastW = 0;
    // per-shape choice of dense-conv kernel for every op (ConvKernel; CONV_GEMM for
    // non-conv ops): timed once per (B, H, W) on the caller's stream, or forced by
    // YH_CONV=<kernel id>
    // 16-bit dense convs: the conv_mx plan chosen for every op at a shape (all plans of a
    // layer are bit-identical, the choice only changes speed), timed once per (B, H, W)
    // on the caller's stream or forced by yh_force_conv_kernel / YH_CONV=<candidate>
    struct MxChoice { MxPlan plan; const char* w = nullptr; std::string name; };
    std::map<GraphKey, std::vector<MxChoice>> conv_kern;
    const std::vector<MxChoice>* cur_kern = nullptr;
    int force_kern = -1;   // candidate index (testing); -1 = autotune
    int num_cus = 0;
    // launch units of the forward at the current shape (one op each)
    struct Unit { int first, last; bool level; };
    struct Plan {
        std::vector<Unit> units;
        std::vector<char> active;   // per op: launched at this shape (fused blocks pick per shape)
    };
    std::map<GraphKey, Plan> plans;
    const Plan* cur_plan = nullptr;

    // ---------------------------------------------------------- builder
    int tensor(int level, int C) {
        tensors.push_back({level, round_up(C, 8)});
        return (int)tensors.size() - 1;
    }
    View full(int t, int C = -1) {
        View v;
        v.t = t;
        v.coff = 0;
        v.C = C < 0 ? tensors[t].C : C;
        return v;
    }
    View slice(int t, int coff, int C) {
        require(coff % 8 == 0 && C % 8 == 0, "concat slice not a multiple of 8 channels");
        View v;
        v.t = t;
        v.coff = coff;
        v.C = C;
        return v;
    }
    int new_conv(const std::string& name, ConvKind kind, int cin, int cout, int k, int s, int g, int has_bias, int act) {
        ConvDesc d;
        d.name = name;
        d.kind = kind;
        d.cin = cin; d.cout = cout; d.k = k; d.stride = s; d.groups = g;
        d.has_bias = has_bias; d.act = act;
        convs.push_back(std::move(d));
        return (int)convs.size() - 1;
    }
    // dense conv op (k in {1,3}), input segments given as (view, logical channels, upsample)
    void dense(const std::string& name, const std::vector<Seg>& in, const std::vector<int>& logical, int cout, int k,
               int s, int act, View out, const View* res = nullptr, int has_bias = 0) {
        int cin = 0;
        for (int c : logical) cin += c;
        const int ci = new_conv(name, CK_DENSE, cin, cout, k, s, 1, has_bias, act);
        ConvDesc& d = convs[ci];
        for (size_t i = 0; i < in.size(); ++i) d.segs.push_back({logical[i], in[i].v.C});
        require(in.size() <= 2, "at most two concat segments");
        if (in.size() == 2) require(logical[0] == in[0].v.C && logical[0] % 8 == 0, "segment 0 must be 8-aligned");
        Op op;
        op.kind = OP_CONV;
        op.conv = ci;
        op.in = in;
        op.out = out;
        if (res) { op.res = *res; op.has_res = true; }
        op.label = name;
        ops.push_back(op);
    }
    View conv1(const std::string& name, View x, int xc, int cout, int act, View out, const View* res = nullptr) {
        dense(name, {Seg{x, 0}}, {xc}, cout, 1, 1, act, out, res);
        return out;
    }
    View conv3(const std::string& name, View x, int xc, int cout, int s, int act, View out, const View* res = nullptr) {
        dense(name, {Seg{x, 0}}, {xc}, cout, 3, s, act, out, res);
        return out;
    }

    // Residual (nn.py:42-49): out = x + conv2(conv1(x)), both 3x3 SiLU
    void residual(const std::string& p, View x, int ch, double e, View out, int level) {
        const int hid = (int)(ch * e);
        const int t = tensor(level, hid);
        conv3(p + ".conv1", x, ch, hid, 1, ACT_SILU, full(t));
        conv3(p + ".conv2", full(t), hid, ch, 1, ACT_SILU, out, &x);
    }
    // CSPModule / C3k (nn.py:52-63)
    // The residual chain a -> a' -> a'' runs through fresh tensors (not in place)
    // so that no region is rewritten after a 3x3 conv of another workgroup read
    // it; the last link
    // writes into the concat buffer.
    void cspmodule(const std::string& p, View x, int in_ch, int out_ch, View out, int level) {
        const int h = out_ch / 2;
        const int t = tensor(level, 2 * h);
        View a = slice(t, 0, h), b = slice(t, h, h);
        const int a0 = tensor(level, h), a1 = tensor(level, h);
        const int first = (int)ops.size();
        conv1(p + ".conv1", x, in_ch, h, ACT_SILU, full(a0));
        conv1(p + ".conv2", x, in_ch, h, ACT_SILU, b);
        residual(p + ".res_m.0", full(a0), h, 1.0, full(a1), level);
        residual(p + ".res_m.1", full(a1), h, 1.0, a, level);
        conv1(p + ".conv3", full(t), 2 * h, out_ch, ACT_SILU, out);
        // 16-bit handles: the whole block as one launch (c3k.hip) at shapes whose image fits
        // a workgroup's LDS (ensure_plan picks it or the seven launches above per shape)
        // c3k.hip moves 8 channels per 16-byte access at ptr(view) + 8 h: both views must start
        // on an 8-channel boundary (slice() enforces it today; checked here so the op never
        // depends on that)
        if (dtype != F32 && opt.fuse && opt.c3k && (in_ch == 64 || in_ch == 128) && out_ch == in_ch && x.C == in_ch &&
            x.coff % 8 == 0 && out.coff % 8 == 0) {
            Op op;
            op.kind = OP_C3K;
            op.label = p;
            for (int k = 0; k < 7; ++k) op.ck[k] = ops[first + k].conv;
            op.in = {Seg{x, 0}};
            op.out = out;
            op.alt0 = first;
            op.alt1 = (int)ops.size();
            ops.push_back(op);
        }
    }
    // CSP / C3k2 (nn.py:66-80); input may be a 2-segment (optionally upsampled) concat
    void csp(const std::string& p, const std::vector<Seg>& in, const std::vector<int>& logical, int out_ch, int n,
             bool use_c3k, int r, View out, int level) {
        const int c = out_ch / r;
        const bool tail = n == 1 && !use_c3k && fuse_csp_tail(c, out_ch, out) &&
                          (tail_first() || !fuse_csp(in, logical, c, out_ch, out));
        if (tail) {
            // conv1 as its own launch into a compact [a | b] tensor, then Residual + conv2 as
            // one launch (c3k2.hip tail mode)
            const int t1 = tensor(level, 2 * c);
            dense(p + ".conv1", in, logical, 2 * c, 1, 1, ACT_SILU, full(t1));
            Op op;
            op.kind = OP_CSP;
            op.label = p + ".tail";
            op.cs[1] = new_dense_conv(p + ".res_m.0.conv1", c, c / 2, 3, 0, ACT_SILU);
            op.cs[2] = new_dense_conv(p + ".res_m.0.conv2", c / 2, c, 3, 0, ACT_SILU);
            op.cs[3] = new_dense_conv(p + ".conv2", 3 * c, out_ch, 1, 0, ACT_SILU);
            op.in = {Seg{full(t1, 2 * c), 0}};
            op.out = out;
            ops.push_back(op);
            return;
        }
        if (n == 1 && !use_c3k && fuse_csp(in, logical, c, out_ch, out)) {
            // one launch for the whole block (c3k2.hip); the same four convs, loaded by name
            Op op;
            op.kind = OP_CSP;
            op.label = p;
            op.cs[0] = new_dense_conv(p + ".conv1", logical[0], 2 * c, 1, 0, ACT_SILU);
            op.cs[1] = new_dense_conv(p + ".res_m.0.conv1", c, c / 2, 3, 0, ACT_SILU);
            op.cs[2] = new_dense_conv(p + ".res_m.0.conv2", c / 2, c, 3, 0, ACT_SILU);
            op.cs[3] = new_dense_conv(p + ".conv2", 3 * c, out_ch, 1, 0, ACT_SILU);
            op.in = in;
            op.out = out;
            ops.push_back(op);
            return;
        }
        const int t = tensor(level, (2 + n) * c);
        dense(p + ".conv1", in, logical, 2 * c, 1, 1, ACT_SILU, slice(t, 0, 2 * c));
        for (int i = 0; i < n; ++i) {
            View src = slice(t, (1 + i) * c, c), dst = slice(t, (2 + i) * c, c);
            const std::string q = p + ".res_m." + std::to_string(i);
            if (!use_c3k) residual(q, src, c, 0.5, dst, level);
            else cspmodule(q, src, c, c, dst, level);
        }
        conv1(p + ".conv2", full(t), (2 + n) * c, out_ch, ACT_SILU, out);
    }
    // SPP / SPPF (nn.py:83-94)
    void sppf(const std::string& p, View x, int in_ch, int out_ch, View out, int level) {
        const int h = in_ch / 2;
        const int t = tensor(level, 4 * h);
        conv1(p + ".conv1", x, in_ch, h, ACT_SILU, slice(t, 0, h));
        Op op;
        op.kind = OP_SPPF;
        op.out = slice(t, 0, h);
        op.label = p + ".res_m";
        ops.push_back(op);
        conv1(p + ".conv2", full(t), 4 * h, out_ch, ACT_SILU, out);
    }
    // PSABlock (nn.py:126-136), in place on view x
    void psablock(const std::string& p, View x, int ch, int heads, int level) {
        const int dh = ch / heads, dk = dh / 2;
        require(dh == 64 && dk == 32, "PSA head dims must be dh=64, dk=32");
        const int qc = ch + 2 * dk * heads;
        const int tq = tensor(level, qc);
        conv1(p + ".conv1.qkv", x, ch, qc, ACT_ID, full(tq));
        const int ta = tensor(level, ch);
        const int pe = new_conv(p + ".conv1.conv1", CK_PE, ch, ch, 3, 1, ch, 0, ACT_ID);
        Op op;
        op.kind = OP_ATTN;
        op.conv = pe;
        op.in = {Seg{full(tq), 0}};
        op.out = full(ta);
        op.heads = heads;
        op.label = p + ".conv1";
        ops.push_back(op);
        conv1(p + ".conv1.conv2", full(ta), ch, ch, ACT_ID, x, &x);
        const int tf = tensor(level, 2 * ch);
        conv1(p + ".conv2.0", x, ch, 2 * ch, ACT_SILU, full(tf));
        conv1(p + ".conv2.1", full(tf), 2 * ch, ch, ACT_ID, x, &x);
    }
    // PSA / C2PSA (nn.py:139-148)
    void psa(const std::string& p, View x, int ch, int n, View out, int level) {
        const int half = ch / 2;
        const int t = tensor(level, 2 * half);
        conv1(p + ".conv1", x, ch, 2 * half, ACT_SILU, full(t));
        for (int i = 0; i < n; ++i) psablock(p + ".res_m." + std::to_string(i), slice(t, half, half), half, ch / 128, level);
        conv1(p + ".conv2", full(t), 2 * half, ch, ACT_SILU, out);
    }

    void build() {
        const int* w = var.width;
        const int* d = var.depth;
        const bool c0 = var.csp[0] != 0, c1 = var.csp[1] != 0;
        const int nc = var.num_classes;
        // ---- DarkNet (nn.py:151-189)
        const int t2 = tensor(2, w[2]);
        if (fuse_stem(w[0], w[1], w[2])) {
            // stem + net.p2.0 in one launch: the stem output never reaches HBM
            Op op;
            op.kind = OP_STEM2;
            op.conv = new_conv("net.p1.0", CK_FIRST, w[0], w[1], 3, 2, 1, 0, ACT_SILU);
            op.cs[0] = new_dense_conv("net.p2.0", w[1], w[2], 3, 0, ACT_SILU);
            convs[op.cs[0]].stride = 2;
            op.out = full(t2, w[2]);
            op.label = "net.p1.0+p2.0";
            ops.push_back(op);
        } else {
            const int t1 = tensor(1, w[1]);
            const int ci = new_conv("net.p1.0", CK_FIRST, w[0], w[1], 3, 2, 1, 0, ACT_SILU);
            Op op;
            op.kind = OP_FIRST;
            op.conv = ci;
            op.out = full(t1, w[1]);
            op.label = "net.p1.0";
            ops.push_back(op);
            conv3("net.p2.0", full(t1, w[1]), w[1], w[2], 2, ACT_SILU, full(t2, w[2]));
        }
        const int t2b = tensor(2, w[3]);
        csp("net.p2.1", {Seg{full(t2, w[2]), 0}}, {w[2]}, w[3], d[0], c0, 4, full(t2b, w[3]), 2);
        const int t3 = tensor(3, w[3]);
        conv3("net.p3.0", full(t2b, w[3]), w[3], w[3], 2, ACT_SILU, full(t3, w[3]));
        const int b3 = tensor(3, w[4]);
        csp("net.p3.1", {Seg{full(t3, w[3]), 0}}, {w[3]}, w[4], d[1], c0, 4, full(b3, w[4]), 3);
        const int t4 = tensor(4, w[4]);
        conv3("net.p4.0", full(b3, w[4]), w[4], w[4], 2, ACT_SILU, full(t4, w[4]));
        const int b4 = tensor(4, w[4]);
        csp("net.p4.1", {Seg{full(t4, w[4]), 0}}, {w[4]}, w[4], d[2], c1, 2, full(b4, w[4]), 4);
        const int t5 = tensor(5, w[5]);
        conv3("net.p5.0", full(b4, w[4]), w[4], w[5], 2, ACT_SILU, full(t5, w[5]));
        const int t5b = tensor(5, w[5]);
        csp("net.p5.1", {Seg{full(t5, w[5]), 0}}, {w[5]}, w[5], d[3], c1, 2, full(t5b, w[5]), 5);
        const int t5c = tensor(5, w[5]);
        sppf("net.p5.2", full(t5b, w[5]), w[5], w[5], full(t5c, w[5]), 5);
        // R = [h5(p4) | p5] (h6 input); backbone p5 is written into its slice 1
        const int R = tensor(5, w[4] + w[5]);
        View p5 = slice(R, w[4], w[5]);
        psa("net.p5.3", full(t5c, w[5]), w[5], d[4], p5, 5);
        // ---- DarkFPN (nn.py:192-209)
        const int Q = tensor(4, w[3] + w[4]);   // [h3(p3) | h1 out]
        View h1o = slice(Q, w[3], w[4]);
        csp("fpn.h1", {Seg{p5, 1}, Seg{full(b4, w[4]), 0}}, {w[5], w[4]}, w[4], d[5], c0, 2, h1o, 4);
        const int P3 = tensor(3, w[3]);
        csp("fpn.h2", {Seg{h1o, 1}, Seg{full(b3, w[4]), 0}}, {w[4], w[4]}, w[3], d[5], c0, 2, full(P3, w[3]), 3);
        conv3("fpn.h3", full(P3, w[3]), w[3], w[3], 2, ACT_SILU, slice(Q, 0, w[3]));
        const int P4 = tensor(4, w[4]);
        csp("fpn.h4", {Seg{full(Q), 0}}, {w[3] + w[4]}, w[4], d[5], c0, 2, full(P4, w[4]), 4);
        conv3("fpn.h5", full(P4, w[4]), w[4], w[4], 2, ACT_SILU, slice(R, 0, w[4]));
        const int P5 = tensor(5, w[5]);
        csp("fpn.h6", {Seg{full(R), 0}}, {w[4] + w[5]}, w[5], d[5], c1, 2, full(P5, w[5]), 5);
        // ---- Head (nn.py:228-270)
        const int boxc = std::max(64, w[3] / 4);
        const int clsc = std::max(std::max(80, w[3]), nc);
        const int ncp = round_up(nc, 8);
        const int xs[3] = {P3, P4, P5};
        const int xc[3] = {w[3], w[4], w[5]};
        int L[3];
        // per level, coarsest first: the 20x20 and 40x40 head branches join the
        // level program that computes P5 / P4; the 80x80 level runs last
        for (int l = 0; l < 3; ++l) L[l] = tensor(3 + l, 64 + ncp);
        // 16-bit handles run the cls branches of the levels that have an LDS tile as one
        // fused launch (head.hip), and fold the decode into the producers of the logits: the
        // box rows into box_dfl (last box conv + DFL), the fused levels' scores into
        // head_cls, the other levels' (a suffix) into a class-rows decode. YH_FUSE=0 keeps
        // the per-layer launches and the decode.
        bool fl[3];
        for (int l = 0; l < 3; ++l) fl[l] = fuse_head_cls(xc[l], clsc, nc);
        const bool fdec = fuse_decode(boxc, nc) && (fl[0] || !fl[1]) && (fl[1] || !fl[2]);
        bool fuse_any = false;
        Op hcop;
        hcop.kind = OP_HEADCLS;
        hcop.label = "head.cls";
        hcop.direct = fdec;
        Op bdop;
        bdop.kind = OP_BOXDFL;
        bdop.label = "head.box_dfl";
        int bop[3][2];   // per level: the ops of box.l.0 and box.l.1
        for (int l : {2, 1, 0}) {
            const int lvl = 3 + l;
            const std::string bp = "head.box." + std::to_string(l);
            const int tb1 = tensor(lvl, boxc), tb2 = tensor(lvl, boxc);
            bop[l][0] = (int)ops.size();
            conv3(bp + ".0", full(xs[l], xc[l]), xc[l], boxc, 1, ACT_SILU, full(tb1, boxc));
            bop[l][1] = (int)ops.size();
            conv3(bp + ".1", full(tb1, boxc), boxc, boxc, 1, ACT_SILU, full(tb2, boxc));
            if (fdec) {
                bdop.bc[l] = new_dense_conv(bp + ".2", boxc, 64, 1, 1, ACT_ID);
                bdop.bx[l] = full(tb2, boxc);
            } else {
                dense(bp + ".2", {Seg{full(tb2, boxc), 0}}, {boxc}, 64, 1, 1, ACT_ID, slice(L[l], 0, 64), nullptr, 1);
            }
            const std::string cp = "head.cls." + std::to_string(l);
            View o;
            o.t = L[l];
            o.coff = 64;
            o.C = ncp;
            if (fl[l]) {
                // the same five convs (weights are loaded by name), no per-layer ops
                fuse_any = hcop.hlv[l] = true;
                hcop.hc[l][0] = new_conv(cp + ".0", CK_DW, xc[l], xc[l], 3, 1, xc[l], 0, ACT_SILU);
                hcop.hc[l][1] = new_dense_conv(cp + ".1", xc[l], clsc, 1, 0, ACT_SILU);
                hcop.hc[l][2] = new_conv(cp + ".2", CK_DW, clsc, clsc, 3, 1, clsc, 0, ACT_SILU);
                hcop.hc[l][3] = new_dense_conv(cp + ".3", clsc, clsc, 1, 0, ACT_SILU);
                hcop.hc[l][4] = new_dense_conv(cp + ".4", clsc, nc, 1, 1, ACT_ID);
                hcop.hx[l] = full(xs[l], xc[l]);
                hcop.hy[l] = o;
                continue;
            }
            const int tc1 = tensor(lvl, xc[l]), tc2 = tensor(lvl, clsc), tc3 = tensor(lvl, clsc), tc4 = tensor(lvl, clsc);
            dw(cp + ".0", full(xs[l], xc[l]), xc[l], full(tc1, xc[l]));
            conv1(cp + ".1", full(tc1, xc[l]), xc[l], clsc, ACT_SILU, full(tc2, clsc));
            dw(cp + ".2", full(tc2, clsc), clsc, full(tc3, clsc));
            conv1(cp + ".3", full(tc3, clsc), clsc, clsc, ACT_SILU, full(tc4, clsc));
            dense(cp + ".4", {Seg{full(tc4, clsc), 0}}, {clsc}, nc, 1, 1, ACT_ID, o, nullptr, 1);
        }
        if (fuse_any) ops.push_back(hcop);
        if (fdec) ops.push_back(bdop);
        // 16-bit handles: the whole box branch of every level as one launch (boxc.hip) at shapes
        // where each level has a tile (ensure_plan picks it or the seven launches above)
        if (fdec && fuse_box_chain(boxc, xs, xc)) {
            Op bc;
            bc.kind = OP_BOXCHAIN;
            bc.label = "head.box";
            for (int l = 0; l < 3; ++l) {
                bc.bxc[l][0] = ops[bop[l][0]].conv;
                bc.bxc[l][1] = ops[bop[l][1]].conv;
                bc.bxc[l][2] = bdop.bc[l];
                bc.hx[l] = full(xs[l], xc[l]);
            }
            for (int l = 0; l < 3; ++l) bc.alts.push_back(bop[l][0]);
            for (int l = 0; l < 3; ++l) bc.alts.push_back(bop[l][1]);
            bc.alts.push_back((int)ops.size() - 1);   // box_dfl
            ops.push_back(bc);
        }
        Op dec;
        dec.kind = OP_DECODE;
        for (int l = 0; l < 3; ++l) dec.lvl[l] = full(L[l]);
        dec.label = "head.decode";
        dec.dbox = !fdec;
        dec.dlo = fdec ? (fl[2] ? 3 : fl[1] ? 2 : fl[0] ? 1 : 0) : 0;
        if (dec.dlo < 3) {
            if (fdec) dec.label = "head.decode_cls";
            ops.push_back(dec);
        }
        finalize_convs();
        fuse_pw_chains();
    }

    // ---- pointwise chains (pwchain.hip): maximal runs of consecutive 1x1 conv ops on one
    //      40x40-or-smaller map become one launch, inserted after the run's last op; the per-layer
    //      ops stay (inactive) for YH_PWCHAIN=0 and the parity tests
    void fuse_pw_chains() {
        if (dtype == F32 || !opt.fuse || !opt.pw_chain) return;
        for (size_t i = 0; i < ops.size();) {
            std::vector<char> taken(ops.size(), 0);   // per-layer alternatives of another fused op
            for (auto& o : ops) {
                for (int k = o.alt0; k >= 0 && k < o.alt1; ++k) taken[k] = 1;
                if (o.kind != OP_PWCHAIN)
                    for (int k : o.alts) taken[k] = 1;
            }
            auto eligible = [&](size_t k) {
                const Op& o = ops[k];
                if (o.kind != OP_CONV || taken[k]) return false;
                const ConvDesc& d = convs[o.conv];
                if (d.k != 1 || d.stride != 1 || d.cout % 32 || d.K % 128 || d.K > 1024 || d.cout > 1024) return false;
                const int lv = tensors[o.out.t].level;
                if (lv < 4 || o.out.coff % 8) return false;
                for (size_t si = 0; si < o.in.size(); ++si) {
                    const Seg& sg = o.in[si];
                    if (sg.up || tensors[sg.v.t].level != lv || d.segs[si].first != d.segs[si].second) return false;
                }
                if (o.has_res && (tensors[o.res.t].level != lv || o.res.C < d.cout)) return false;
                return true;
            };
            if (!eligible(i)) { ++i; continue; }
            const int lv = tensors[ops[i].out.t].level;
            size_t j = i + 1;
            while (j < ops.size() && j - i < (size_t)PWC_MAX_STAGES && eligible(j) && tensors[ops[j].out.t].level == lv) ++j;
            size_t made = 0;
            for (size_t e = j; e >= i + 2 && !made; --e)
                if (make_pw_chain(i, e)) made = e + 1;   // the chain op sits at e
            i = made ? made : i + 1;
        }
    }
    // the chain ops [i, e) as one OP_PWCHAIN inserted at e; false (nothing changed) if the stages'
    // sources do not split into whole 128-channel runs or the tile does not fit the LDS
    bool make_pw_chain(size_t i, size_t e) {
        const int n = (int)(e - i);
        Op ch;
        ch.kind = OP_PWCHAIN;
        ch.pws.resize(n);
        // the latest stage before k writing channel c of tensor t (-1: none)
        auto producer = [&](int k, int t, int c) {
            for (int q = k - 1; q >= 0; --q) {
                const View& o = ops[i + q].out;
                if (o.t == t && c >= o.coff && c < o.coff + convs[ops[i + q].conv].cout) return q;
            }
            return -1;
        };
        for (int k = 0; k < n; ++k) {
            const Op& o = ops[i + k];
            Op::PwStage& st = ch.pws[k];
            for (const Seg& sg : o.in) {
                const View& v = sg.v;
                for (int c = v.coff; c < v.coff + v.C;) {
                    const int q = producer(k, v.t, c);
                    int c1 = c + 8;
                    while (c1 < v.coff + v.C && producer(k, v.t, c1) == q) c1 += 8;
                    Op::PwRun r;
                    r.stage = q;
                    r.nch = c1 - c;
                    r.coff = q >= 0 ? c - ops[i + q].out.coff : c;
                    if (r.nch % 128) return false;
                    if (q < 0) {   // a global view: one prologue load per distinct view
                        View g;
                        g.t = v.t; g.coff = c; g.C = r.nch;
                        int li = -1;
                        for (size_t z = 0; z < ch.pwl.size(); ++z)
                            if (ch.pwl[z].t == g.t && ch.pwl[z].coff == g.coff && ch.pwl[z].C == g.C) li = (int)z;
                        if (li < 0) {
                            li = (int)ch.pwl.size();
                            ch.pwl.push_back(g);
                        }
                        r.load = li;
                    } else {
                        ch.pws[q].keep = true;
                    }
                    st.runs.push_back(r);
                    c = c1;
                }
            }
            if ((int)st.runs.size() > PWC_MAX_RUNS) return false;
            if (o.has_res) {
                const int cout = convs[o.conv].cout;
                const int q = producer(k, o.res.t, o.res.coff);
                for (int c = o.res.coff; c < o.res.coff + cout; c += 8)
                    if (producer(k, o.res.t, c) != q) return false;
                st.res_stage = q;
                if (q >= 0) {
                    st.res_coff = o.res.coff - ops[i + q].out.coff;
                    ch.pws[q].keep = true;
                } else {   // a global residual also comes in by the prologue (no VGPR load in the epilogue)
                    View g;
                    g.t = o.res.t; g.coff = o.res.coff; g.C = cout;
                    int li = -1;
                    for (size_t z = 0; z < ch.pwl.size(); ++z)
                        if (ch.pwl[z].t == g.t && ch.pwl[z].coff == g.coff && ch.pwl[z].C == g.C) li = (int)z;
                    if (li < 0) {
                        li = (int)ch.pwl.size();
                        ch.pwl.push_back(g);
                    }
                    st.res_load = li;
                }
            }
        }
        if ((int)ch.pwl.size() > PWC_MAX_LOADS) return false;
        // LDS: the kept stage outputs (pixel stride cout + 8), then the loads (stride C + 8,
        // whole 1 KB LDS-DMA instructions)
        auto layout = [&](int P) {
            int off = 0;
            for (int k = 0; k < n; ++k) {
                Op::PwStage& st = ch.pws[k];
                st.lds = -1;
                if (!st.keep) continue;
                st.lds = off;
                off += (P * (convs[ops[i + k].conv].cout + 8) * 2 + 15) & ~15;
            }
            ch.pwl_lds.assign(ch.pwl.size(), 0);
            for (size_t z = 0; z < ch.pwl.size(); ++z) {
                off = (off + 1023) & ~1023;
                ch.pwl_lds[z] = off;
                off += (P * (ch.pwl[z].C + 8) * 2 + 1023) & ~1023;
            }
            off = (off + 1023) & ~1023;
            return off + 1024;   // the weight warm-up DMAs' sink (pw_chain)
        };
        int P = 64, lds = layout(64);
        if (lds > 160 * 1024) {
            P = 32;
            lds = layout(32);
        }
        if (lds > 160 * 1024) return false;
        ch.pwP = P;
        ch.pwLds = lds;
        for (int k = 0; k < n; ++k) ch.alts.push_back((int)(i + k));
        ch.label = ops[i].label + " +" + std::to_string(n - 1);
        ch.out = ops[e - 1].out;
        // insert at e: op indices >= e move up by one
        for (auto& o : ops) {
            if (o.alt0 >= (int)e) o.alt0++;
            if (o.alt1 >= (int)e) o.alt1++;
            for (int& k : o.alts)
                if (k >= (int)e) k++;
        }
        ops.insert(ops.begin() + e, ch);
        return true;
    }
    // a dense conv with a single unsegmented input and no op of its own (fused ops)
    int new_dense_conv(const std::string& name, int cin, int cout, int k, int has_bias, int act) {
        const int ci = new_conv(name, CK_DENSE, cin, cout, k, 1, 1, has_bias, act);
        convs[ci].segs.push_back({cin, round_up(cin, 8)});
        return ci;
    }
    // the stem and net.p2.0 run fused (conv.hip stem_fused) on 16-bit handles for the
    // instantiated widths (v11_n 16 -> 32, v11_s 32 -> 64)
    bool fuse_stem(int c0, int c1, int c2) const {
        if (dtype == F32 || !opt.fuse) return false;
        return c0 == 3 && stem2_ok(c1, c2);
    }
    // packed p2.0 parameters of the fused stem: fragments (tile a, step k = cb*9 + tap,
    // lane, j) in MFMA lane order with conv_mx's row permutation, then the fp32 bias
    const void* stem2_params(const Op& op, int& bias_off) {
        ConvDesc& d = convs[op.cs[0]];
        const int nt = d.cout / 32, nk = 9 * (d.cin / 16);
        bias_off = nt * nk * 1024;
        auto it = d.mx_w.find("stem2");
        if (it != d.mx_w.end()) return it->second;
        require(d.loaded, "weights of " + d.name + " not loaded", YH_ESTATE);
        std::vector<uint8_t> img((size_t)bias_off + (size_t)d.cout * 4, 0);
        uint16_t* dst = reinterpret_cast<uint16_t*>(img.data());
        for (int a = 0; a < nt; ++a)
            for (int k = 0; k < nk; ++k)
                for (int lane = 0; lane < 64; ++lane)
                    for (int j = 0; j < 8; ++j) {
                        const int R = lane & 31, hh = lane >> 5;
                        const int co = 32 * a + 16 * ((R >> 2) & 1) + (R & 3) + 4 * (R >> 3);
                        const int cb = k / 9, tap = k - cb * 9, ch = 16 * cb + 8 * hh + j;
                        const float v = d.wf[((size_t)co * d.cin + ch) * 9 + tap];
                        dst[((size_t)(a * nk + k) * 64 + lane) * 8 + j] = dtype == BF16 ? f2bf(v) : f2h(v);
                    }
        float* bd = reinterpret_cast<float*>(img.data() + bias_off);
        for (int i = 0; i < d.cout; ++i) bd[i] = d.bf[i];
        void* dev = nullptr;
        HIPCHECK(hipMalloc(&dev, img.size()));
        HIPCHECK(hipMemcpy(dev, img.data(), img.size(), hipMemcpyHostToDevice));
        d.mx_w.emplace("stem2", dev);
        return dev;
    }
    // a C3k2 block with one Residual runs fused (c3k2.hip) on 16-bit handles when its input
    // is one plain view of 16-channel blocks and (Cin, c, cout) has an instantiated kernel
    bool fuse_csp(const std::vector<Seg>& in, const std::vector<int>& logical, int c, int out_ch, View out) const {
        if (dtype == F32 || !opt.fuse) return false;
        if (in.size() != 1 || in[0].up || in[0].v.C != logical[0] || logical[0] % 16 || c % 16 || out_ch % 32) return false;
        if (out.coff % 8 || in[0].v.coff % 8) return false;
        int TH, TW;
        return csp_tile(logical[0] / 16, c / 16, out_ch / 32, 1 << 30, 1 << 30, TH, TW);
    }
    bool fuse_csp_tail(int c, int out_ch, View out) const {
        if (dtype == F32 || !opt.fuse) return false;
        if (c % 16 || out_ch % 32 || out.coff % 8) return false;
        int TH, TW;
        return csp_tile(0, c / 16, out_ch / 32, 1 << 30, 1 << 30, TH, TW);
    }
    // tail mode even where the whole block fits one launch (Options::csp_tail, tests)
    bool tail_first() const { return opt.csp_tail; }
    static bool csp_tile(int ni, int nc, int no, int H, int W, int& TH, int& TW) {
        // YH_CSP_TILE=<TH>x<TW> (experiments): that tile first where it fits one workgroup
        if (const char* e = getenv("YH_CSP_TILE")) {
            int th = 0, tw = 0;
            if (sscanf(e, "%dx%d", &th, &tw) == 2 && th > 0 && tw > 0 && th <= H && tw <= W &&
                csp_lds(th, tw, ni, nc, no) > 0) {
                TH = th;
                TW = tw;
                return true;
            }
        }
        // 16-wave workgroups (one per CU): the largest tile that fits (8 x 32 / 16 x 16 against
        // 8-wave 8 x 16 pairs: bench +2.5 %, net.p3.1 65 -> 62 us, fpn.h2.tail 40 -> 37 us);
        // 8-wave ones: the largest tile of >= 64 pixels that leaves room for a second workgroup
        // per CU, else the largest that fits (measured: net.p3.1 at 2x4 tiles, two per CU,
        // 263 us against 68 us at 8x16, one per CU)
        static const int cand[][2] = {{8, 32}, {16, 16}, {8, 16}, {8, 8}, {4, 16}, {4, 8}, {2, 8}, {2, 4}};
        const bool wide = CSP_THREADS >= 1024;
        for (int lim : {80 * 1024, 160 * 1024})
            for (auto& c : cand) {
                if (wide && lim == 80 * 1024) break;
                if (!wide && c[0] * c[1] > 128) continue;
                if (c[0] > H || c[1] > W || (lim == 80 * 1024 && c[0] * c[1] < 64)) continue;
                const int b = csp_lds(c[0], c[1], ni, nc, no);
                if (b > 0 && b <= lim) {
                    TH = c[0];
                    TW = c[1];
                    return true;
                }
            }
        return false;
    }
    // packed parameter image of a fused C3k2 op (cached in conv1's mx_w; the other three
    // convs hold a marker, so reloading any of the four rebuilds it)
    const void* csp_params(const Op& op) {
        // tail mode (no conv1 in the op): the cache lives in the Residual's first conv
        const int k0 = op.cs[0] >= 0 ? 0 : 1;
        ConvDesc& d0 = convs[op.cs[k0]];
        auto it = d0.mx_w.find("csp");
        bool ok = it != d0.mx_w.end();
        for (int k = k0 + 1; k < 4; ++k) ok = ok && convs[op.cs[k]].mx_w.count("csp_dep");
        if (ok) return it->second;
        if (it != d0.mx_w.end()) {
            (void)hipFree(it->second);
            d0.mx_w.erase(it);
        }
        for (int k = k0; k < 4; ++k) require(convs[op.cs[k]].loaded, "weights of " + convs[op.cs[k]].name + " not loaded", YH_ESTATE);
        const ConvDesc &r1 = convs[op.cs[1]], &r2 = convs[op.cs[2]], &c2 = convs[op.cs[3]];
        const int ni = k0 == 0 ? convs[op.cs[0]].cin / 16 : 0, nc = r1.cin / 16, no = c2.cout / 32, nh = (nc + 1) / 2;
        int off[9];
        csp_offsets(ni, nc, no, off);
        std::vector<uint8_t> img((size_t)off[8], 0);
        // fragment (tile a, step k, lane, j): cout row permuted so lane half hh holds couts
        // 32a + 16hh .. +15; K value 8hh + j of step k = (block cb, tap)
        auto frags = [&](int o, const ConvDesc& d, int ntile, int nk) {
            const int kk2 = d.k * d.k;
            uint16_t* dst = reinterpret_cast<uint16_t*>(img.data() + o);
            for (int a = 0; a < ntile; ++a)
                for (int k = 0; k < nk; ++k)
                    for (int lane = 0; lane < 64; ++lane)
                        for (int j = 0; j < 8; ++j) {
                            const int R = lane & 31, hh = lane >> 5;
                            const int co = 32 * a + 16 * ((R >> 2) & 1) + (R & 3) + 4 * (R >> 3);
                            const int cb = k / kk2, tap = k - cb * kk2, ch = 16 * cb + 8 * hh + j;
                            float v = 0.f;
                            if (co < d.cout && ch < d.cin) v = d.wf[((size_t)co * d.cin + ch) * kk2 + tap];
                            dst[((size_t)(a * nk + k) * 64 + lane) * 8 + j] = dtype == BF16 ? f2bf(v) : f2h(v);
                        }
        };
        if (ni) frags(off[0], convs[op.cs[0]], nc, ni);
        frags(off[1], r1, 1, 9 * nc);
        frags(off[2], r2, nh, 9 * nh);
        frags(off[3], c2, no, 3 * nc);
        auto biases = [&](int o, const ConvDesc& d) {
            float* dst = reinterpret_cast<float*>(img.data() + o);
            for (int i = 0; i < d.cout; ++i) dst[i] = d.bf[i];
        };
        if (ni) biases(off[4], convs[op.cs[0]]);
        biases(off[5], r1);
        biases(off[6], r2);
        biases(off[7], c2);
        void* dev = nullptr;
        HIPCHECK(hipMalloc(&dev, img.size()));
        HIPCHECK(hipMemcpy(dev, img.data(), img.size(), hipMemcpyHostToDevice));
        d0.mx_w.emplace("csp", dev);
        for (int k = k0 + 1; k < 4; ++k) convs[op.cs[k]].mx_w.emplace("csp_dep", nullptr);
        return dev;
    }
    // packed parameters of a fused C3k block (c3k.hip layout), cached with its first conv
    const void* c3k_params(const Op& op) {
        ConvDesc& d0 = convs[op.ck[0]];
        auto it = d0.mx_w.find("c3k");
        bool ok = it != d0.mx_w.end();
        for (int k = 1; k < 7; ++k) ok = ok && convs[op.ck[k]].mx_w.count("c3k_dep");
        if (ok) return it->second;
        if (it != d0.mx_w.end()) {
            (void)hipFree(it->second);
            d0.mx_w.erase(it);
        }
        for (int k = 0; k < 7; ++k) require(convs[op.ck[k]].loaded, "weights of " + convs[op.ck[k]].name + " not loaded", YH_ESTATE);
        // hidden channels hh = conv1's couts (32 or 64): NT3 = hh / 32 tiles of conv1 / conv2 /
        // the 3x3 convs over hh / 8 (1x1) or 9 hh / 16 (3x3) K steps, conv3: hh / 16 tiles
        const int hh = convs[op.ck[0]].cout, nt3 = hh / 32, nk1 = hh / 8, nk3 = 9 * hh / 16;
        int off[9];
        c3k_offsets(hh, off);
        std::vector<uint8_t> img((size_t)off[8], 0);
        // fragment (tile a, step k, lane, j); rows: lane half hh of tile a holds couts
        // 32a + 16hh .. +15 (c3k2.hip's order), or with bits 2 and 3 of the row swapped (rho:
        // conv2, whose accumulators become conv3's B fragments)
        auto frags = [&](int o, const ConvDesc& d, int ntile, int nk, bool rho) {
            const int kk2 = d.k * d.k;
            uint16_t* dst = reinterpret_cast<uint16_t*>(img.data() + o);
            for (int a = 0; a < ntile; ++a)
                for (int k = 0; k < nk; ++k)
                    for (int lane = 0; lane < 64; ++lane)
                        for (int j = 0; j < 8; ++j) {
                            const int R = lane & 31, hh = lane >> 5;
                            const int co = rho ? 32 * a + ((R & 0x13) | ((R & 4) << 1) | ((R & 8) >> 1))
                                               : 32 * a + 16 * ((R >> 2) & 1) + (R & 3) + 4 * (R >> 3);
                            const int cb = k / kk2, tap = k - cb * kk2, ch = 16 * cb + 8 * hh + j;
                            float v = 0.f;
                            if (co < d.cout && ch < d.cin) v = d.wf[((size_t)co * d.cin + ch) * kk2 + tap];
                            dst[((size_t)(a * nk + k) * 64 + lane) * 8 + j] = dtype == BF16 ? f2bf(v) : f2h(v);
                        }
        };
        frags(off[0], convs[op.ck[0]], nt3, nk1, false);
        frags(off[1], convs[op.ck[1]], nt3, nk1, true);
        for (int r = 0; r < 4; ++r) frags(off[2] + r * nt3 * nk3 * 1024, convs[op.ck[2 + r]], nt3, nk3, false);
        frags(off[3], convs[op.ck[6]], hh / 16, nk1, false);
        auto biases = [&](int o, const ConvDesc& d) {
            float* dst = reinterpret_cast<float*>(img.data() + o);
            for (int i = 0; i < d.cout; ++i) dst[i] = d.bf[i];
        };
        biases(off[4], convs[op.ck[0]]);
        biases(off[5], convs[op.ck[1]]);
        for (int r = 0; r < 4; ++r) biases(off[6] + r * hh * 4, convs[op.ck[2 + r]]);
        biases(off[7], convs[op.ck[6]]);
        void* dev = nullptr;
        HIPCHECK(hipMalloc(&dev, img.size()));
        HIPCHECK(hipMemcpy(dev, img.data(), img.size(), hipMemcpyHostToDevice));
        d0.mx_w.emplace("c3k", dev);
        for (int k = 1; k < 7; ++k) convs[op.ck[k]].mx_w.emplace("c3k_dep", nullptr);
        return dev;
    }
    // the box branch runs as one launch (boxc.hip) for 64 box channels and level inputs of
    // 64 / 128 / 256 / 512 channels (plain views)
    bool fuse_box_chain(int boxc, const int (&xs)[3], const int (&xc)[3]) const {
        if (dtype == F32 || !opt.fuse || !opt.box_chain || boxc != 64) return false;
        for (int l = 0; l < 3; ++l)
            if (!bx_ok(xc[l]) || tensors[xs[l]].C != xc[l]) return false;
        return true;
    }
    // packed parameters of one level of the box chain (boxc.hip layout), cached with box.l.0
    const void* box_chain_params(const Op& op, int l) {
        ConvDesc& d0 = convs[op.bxc[l][0]];
        auto it = d0.mx_w.find("bxc");
        bool ok = it != d0.mx_w.end();
        for (int k = 1; k < 3; ++k) ok = ok && convs[op.bxc[l][k]].mx_w.count("bxc_dep");
        if (ok) return it->second;
        if (it != d0.mx_w.end()) {
            (void)hipFree(it->second);
            d0.mx_w.erase(it);
        }
        for (int k = 0; k < 3; ++k) require(convs[op.bxc[l][k]].loaded, "weights of " + convs[op.bxc[l][k]].name + " not loaded", YH_ESTATE);
        const ConvDesc &c0 = convs[op.bxc[l][0]], &c1 = convs[op.bxc[l][1]], &c2 = convs[op.bxc[l][2]];
        const int C0 = c0.cin, ncb = C0 / 16;
        require(c0.cout == 64 && c1.cin == 64 && c1.cout == 64 && c2.cin == 64 && c2.cout == 64 && c2.k == 1,
                "box chain: conv shapes");
        std::vector<uint8_t> img((size_t)bx_prm_bytes(C0), 0);
        uint16_t* dst = reinterpret_cast<uint16_t*>(img.data());
        auto cvt = [&](float v) { return dtype == BF16 ? f2bf(v) : f2h(v); };
        const size_t item = 18 * 1024 / 2;   // ring item (uint16 units)
        for (int lane = 0; lane < 64; ++lane) {
            const int R = lane & 31, hh = lane >> 5;
            for (int a = 0; a < 2; ++a) {
                // conv_mx's rows (lane half hh: couts 16 hh ..) and c3k's permuted rows (registers
                // 8 jj .. of tile a = channels 32 a + 16 jj + 8 hh ..: the 1x1's B fragments)
                const int co0 = 32 * a + 16 * ((R >> 2) & 1) + (R & 3) + 4 * (R >> 3);
                const int co1 = 32 * a + ((R & 0x13) | ((R & 4) << 1) | ((R & 8) >> 1));
                const int co2 = 32 * ((R >> 2) & 1) + 16 * a + (R & 3) + 4 * (R >> 3);   // box_dfl's rows
                for (int j = 0; j < 8; ++j) {
                    for (int cb = 0; cb < ncb; ++cb)
                        for (int t = 0; t < 9; ++t)
                            dst[cb * item + ((size_t)(a * 9 + t) * 64 + lane) * 8 + j] =
                                cvt(c0.wf[((size_t)co0 * C0 + 16 * cb + 8 * hh + j) * 9 + t]);
                    for (int kb = 0; kb < 4; ++kb) {
                        for (int t = 0; t < 9; ++t)
                            dst[(ncb + kb) * item + ((size_t)(a * 9 + t) * 64 + lane) * 8 + j] =
                                cvt(c1.wf[((size_t)co1 * 64 + 16 * kb + 8 * hh + j) * 9 + t]);
                        dst[(ncb + 4) * item + ((size_t)(a * 4 + kb) * 64 + lane) * 8 + j] =
                            cvt(c2.wf[(size_t)co2 * 64 + 16 * kb + 8 * hh + j]);
                    }
                }
            }
        }
        float* bd = reinterpret_cast<float*>(img.data() + img.size() - 3 * 64 * 4);
        for (int i = 0; i < 64; ++i) {
            bd[i] = c0.bf[i];
            bd[64 + i] = c1.bf[i];
            bd[128 + i] = c2.bf[i];
        }
        void* dev = nullptr;
        HIPCHECK(hipMalloc(&dev, img.size()));
        HIPCHECK(hipMemcpy(dev, img.data(), img.size(), hipMemcpyHostToDevice));
        d0.mx_w.emplace("bxc", dev);
        for (int k = 1; k < 3; ++k) convs[op.bxc[l][k]].mx_w.emplace("bxc_dep", nullptr);
        return dev;
    }
    BoxChainArgs box_chain_args(const Op& op, int B, int H, int W) {
        BoxChainArgs a{};
        a.B = B;
        a.nc = var.num_classes;
        a.A = anchor_off(3, H, W);
        a.io = (const void* const*)io_dev;
        a.zero = zero_dev;
        int wg = 0;
        // workgroup order: the coarsest level, whose tiles are the longest, first (142 vs 148 us)
        for (int k = 0; k < 3; ++k) {
            const int l = 2 - k;
            BoxChainLevel& v = a.lv[a.nlv++];
            const int lv = tensors[op.hx[l].t].level;
            v.x = ptr(op.hx[l]);
            v.ldx = ldc(op.hx[l]);
            v.C0 = convs[op.bxc[l][0]].cin;
            v.H = H >> lv;
            v.W = W >> lv;
            require(bx_tile(v.H, v.W, v.TH, v.TW), "head.box: no tile");
            v.ntw = (v.W + v.TW - 1) / v.TW;
            v.tiles = v.ntw * ((v.H + v.TH - 1) / v.TH);
            // box.l.0's canonical K order at this shape (conv_mx.h mx_kchunks)
            ConvArgs ca{};
            int BM, BN;
            conv_args(ops[op.alts[l]], B, H, W, ca, BM, BN);
            v.nkc = mx_kchunks(mx_shape(ca, B));
            v.stride = (float)(1 << lv);
            v.aoff = anchor_off(l, H, W);
            v.prm = box_chain_params(op, l);
            v.wg0 = wg;
            wg += B * v.tiles;
        }
        return a;
    }
    // the decode folds into box_dfl + head_cls / a class-rows decode (16-bit handles; the
    // box branch's last conv has 4 or 6 16-channel K blocks)
    bool fuse_decode(int boxc, int nc) const {
        if (dtype == F32 || !opt.fuse) return false;
        return (boxc == 64 || boxc == 96) && nc % 4 == 0;
    }
    // first anchor of detect level l (0..2) for an H x W input (make_anchors order)
    static int anchor_off(int l, int H, int W) {
        int a = 0;
        for (int k = 0; k < l; ++k) a += (H >> (3 + k)) * (W >> (3 + k));
        return a;
    }
    // a level's cls branch is fused when it has 16-channel blocks, 4-channel class groups
    // and an LDS tile next to its resident weights
    bool fuse_head_cls(int C0, int c3, int nc) const {
        if (dtype == F32 || !opt.fuse) return false;
        if (c3 % 16 || nc % 4 || C0 % 16) return false;
        if (C0 > 128 && !opt.hcls_wide) return false;
        int TH, TW;
        return head_cls_tile(C0, c3, nc, 1 << 30, 1 << 30, TH, TW);
    }
    // output tile of one level of the fused cls branch: the largest candidate whose
    // workgroup (resident weights + one tile's buffers) fits the LDS
    static bool head_cls_tile(int C0, int c3, int nc, int H, int W, int& TH, int& TW) {
        static const int cand[][2] = {{16, 16}, {8, 32}, {8, 16}, {8, 8}, {4, 16}, {4, 8}, {8, 4}, {4, 4}, {2, 8}, {2, 4}, {2, 2}};
        for (auto& c : cand) {
            if (c[0] > H || c[1] > W) continue;
            if (head_cls_lds(c[0], c[1], C0, c3, nc) > 0) {
                TH = c[0];
                TW = c[1];
                return true;
            }
        }
        return false;
    }

    void dw(const std::string& name, View x, int ch, View out) {
        const int ci = new_conv(name, CK_DW, ch, ch, 3, 1, ch, 0, ACT_SILU);
        Op op;
        op.kind = OP_DW;
        op.conv = ci;
        op.in = {Seg{x, 0}};
        op.out = out;
        op.label = name;
        ops.push_back(op);
    }

    void finalize_convs() {
        for (auto& d : convs) {
            if (d.kind == CK_DENSE) {
                d.cin_p = 0;
                for (auto& s : d.segs) d.cin_p += s.second;
                d.K = d.k * d.k * d.cin_p;
                d.Kp = round_up(d.K, 64);
                d.cout_p = round_up(d.cout, 8);
                d.coutp_pad = round_up(d.cout_p, 128);
            } else {
                d.cin_p = round_up(d.cin, 8);
                d.cout_p = round_up(d.cout, 8);
                d.coutp_pad = d.cout_p;
            }
        }
    }

    // ---------------------------------------------------------- weights
    void load_conv(int idx, const float* w, const float* b, const float* g, const float* be, const float* mu,
                   const float* var_, double eps) {
        require(idx >= 0 && idx < (int)convs.size(), "conv index out of range");
        ConvDesc& d = convs[idx];
        const int cpg = d.cin / d.groups;
        const size_t per = (size_t)cpg * d.k * d.k;
        d.wf.assign(w, w + per * d.cout);
        d.bf.assign(d.cout, 0.0f);
        if (b) for (int o = 0; o < d.cout; ++o) d.bf[o] = b[o];
        if (g) {
            // fuse_conv (nets/nn.py:8-25), fp32 throughout:
            //   s = gamma / sqrt(eps + var); W' = s * W; b' = s * b + (beta - gamma*mean / sqrt(var + eps))
            const float epsf = (float)eps;
            for (int o = 0; o < d.cout; ++o) {
                const float den = std::sqrt(var_[o] + epsf);
                const float s = g[o] / den;
                for (size_t i = 0; i < per; ++i) d.wf[o * per + i] = s * d.wf[o * per + i];
                const float bnorm = be[o] - (g[o] * mu[o]) / den;
                d.bf[o] = s * d.bf[o] + bnorm;
            }
        }
        upload(d);
        d.loaded = true;
    }

    void upload(ConvDesc& d) {
        free_conv(d);
        std::vector<float> bias(d.coutp_pad, 0.0f);
        for (int o = 0; o < d.cout; ++o) bias[o] = d.bf[o];
        HIPCHECK(hipMalloc(&d.b_dev, bias.size() * 4));
        HIPCHECK(hipMemcpy(d.b_dev, bias.data(), bias.size() * 4, hipMemcpyHostToDevice));
        if (d.kind == CK_DENSE) {
            // packed [coutp_pad][Kp], k = (kh*KW + kw)*cin_p + ci_phys
            std::vector<float> wp((size_t)d.coutp_pad * d.Kp, 0.0f);
            std::vector<int> ktab(d.Kp / 8, 0xffff);
            // physical -> logical channel map
            std::vector<int> phys2log(d.cin_p, -1);
            int lo = 0, ph = 0;
            for (auto& s : d.segs) {
                for (int c = 0; c < s.first; ++c) phys2log[ph + c] = lo + c;
                lo += s.first;
                ph += s.second;
            }
            d.phys2log = phys2log;
            const size_t per = (size_t)d.cin * d.k * d.k;
            for (int kh = 0; kh < d.k; ++kh)
                for (int kw = 0; kw < d.k; ++kw)
                    for (int cp = 0; cp < d.cin_p; ++cp) {
                        const int kk = (kh * d.k + kw) * d.cin_p + cp;
                        if (cp % 8 == 0) ktab[kk / 8] = (kh << 24) | (kw << 16) | cp;
                        const int cl = phys2log[cp];
                        if (cl < 0) continue;
                        for (int o = 0; o < d.cout; ++o)
                            wp[(size_t)o * d.Kp + kk] = d.wf[o * per + (size_t)cl * d.k * d.k + kh * d.k + kw];
                    }
            d.w_dev = to_device(wp);
            if (d.k == 1 && dtype != F32 && d.Kp % 16 == 0) {
                // the same 16-bit weights in MFMA A-fragment order for pw_chain: fragment (a, kb) =
                // couts 32a .. 32a + 31 x k 16kb .. 16kb + 15 as 64 lanes x 16 B (lane l: cout 32a +
                // (l & 31), k 16kb + 8 (l >> 5) .. + 7), one contiguous KB, so a wave's fragment load
                // is one coalesced KB instead of 32 strided rows
                const int na = (d.cout + 31) / 32, nkb = d.Kp / 16;
                std::vector<float> fr((size_t)na * 32 * d.Kp, 0.0f);
                for (int a = 0; a < na; ++a)
                    for (int kb = 0; kb < nkb; ++kb)
                        for (int l = 0; l < 64; ++l)
                            for (int e = 0; e < 8; ++e) {
                                const int o = a * 32 + (l & 31), k = kb * 16 + 8 * (l >> 5) + e;
                                fr[(((size_t)a * nkb + kb) * 64 + l) * 8 + e] = o < d.coutp_pad ? wp[(size_t)o * d.Kp + k] : 0.0f;
                            }
                d.mx_w["pwfrag"] = to_device(fr);
            }
            HIPCHECK(hipMalloc(&d.ktab_dev, ktab.size() * 4));
            HIPCHECK(hipMemcpy(d.ktab_dev, ktab.data(), ktab.size() * 4, hipMemcpyHostToDevice));
        } else if (d.kind == CK_FIRST) {
            // transposed [27][cout_p]: k = ci*9 + kh*3 + kw
            std::vector<float> wp((size_t)d.cout_p * 27, 0.0f);
            for (int o = 0; o < d.cout; ++o)
                for (int k = 0; k < 27; ++k) wp[(size_t)k * d.cout_p + o] = d.wf[(size_t)o * 27 + k];
            HIPCHECK(hipMalloc(&d.w_dev, wp.size() * 4));
            HIPCHECK(hipMemcpy(d.w_dev, wp.data(), wp.size() * 4, hipMemcpyHostToDevice));
        } else {  // depthwise / pe: [9][C] fp32
            std::vector<float> wp((size_t)9 * d.cout_p, 0.0f);
            for (int c = 0; c < d.cout; ++c)
                for (int t = 0; t < 9; ++t) wp[(size_t)t * d.cout_p + c] = d.wf[(size_t)c * 9 + t];
            HIPCHECK(hipMalloc(&d.w_dev, wp.size() * 4));
            HIPCHECK(hipMemcpy(d.w_dev, wp.data(), wp.size() * 4, hipMemcpyHostToDevice));
        }
    }

    void* to_device(const std::vector<float>& v) {
        void* p = nullptr;
        if (dtype == F32) {
            HIPCHECK(hipMalloc(&p, v.size() * 4));
            HIPCHECK(hipMemcpy(p, v.data(), v.size() * 4, hipMemcpyHostToDevice));
        } else {
            std::vector<uint16_t> h(v.size());
            for (size_t i = 0; i < v.size(); ++i) h[i] = dtype == BF16 ? f2bf(v[i]) : f2h(v[i]);
            HIPCHECK(hipMalloc(&p, h.size() * 2));
            HIPCHECK(hipMemcpy(p, h.data(), h.size() * 2, hipMemcpyHostToDevice));
        }
        return p;
    }

    static void free_conv(ConvDesc& d) {
        for (auto& kv : d.mx_w) (void)hipFree(kv.second);
        d.mx_w.clear();
        if (d.w_dev) (void)hipFree(d.w_dev);
        if (d.b_dev) (void)hipFree(d.b_dev);
        if (d.ktab_dev) (void)hipFree(d.ktab_dev);
        d.w_dev = nullptr;
        d.b_dev = nullptr;
        d.ktab_dev = nullptr;
    }

    // ---------------------------------------------------------- workspace
    // Tensors are laid out coarsest level first, so the 40x40 / 20x20 tensors and
    // the 80x80 inputs of the level program sit in the first bytes of the
    // workspace (it addresses them by 32-bit offsets).
    size_t ws_bytes_for(int B, int H, int W, std::vector<size_t>* offs) const {
        size_t total = 0;
        if (offs) offs->assign(tensors.size(), 0);
        for (int lvl = 5; lvl >= 0; --lvl)
            for (size_t i = 0; i < tensors.size(); ++i) {
                const Tensor& t = tensors[i];
                if (t.level != lvl) continue;
                const size_t b = (size_t)B * (H >> t.level) * (W >> t.level) * t.C * es;
                if (offs) (*offs)[i] = total;
                total += (b + 255) & ~(size_t)255;
            }
        return total;
    }
    size_t tensor_end(int t) const {
        return ws.off[t] + (size_t)ws.B * (ws.H >> tensors[t].level) * (ws.W >> tensors[t].level) * tensors[t].C * es;
    }
    void reserve(int B, int H, int W) {
        require(B > 0 && H > 0 && W > 0 && H % 32 == 0 && W % 32 == 0, "input height/width must be positive multiples of 32");
        if (ws.base && ws.B == B && ws.H == H && ws.W == W) return;
        std::vector<size_t> offs;
        const size_t need = ws_bytes_for(B, H, W, &offs);
        if (!ws.base || need > ws.bytes) {
            drop_graphs();
            if (ws.base) HIPCHECK(hipFree(ws.base));
            ws.base = nullptr;
            const hipError_t e = hipMalloc(&ws.base, need);
            if (e != hipSuccess) throw Fail(YH_ENOMEM, "workspace allocation failed");
            ws.bytes = need;
        } else if (ws.B != B || ws.H != H || ws.W != W) {
            drop_graphs();
        }
        ws.off = offs;
        ws.B = B;
        ws.H = H;
        ws.W = W;
    }
    char* ptr(const View& v) const {
        return (char*)ws.base + ws.off[v.t] + (size_t)v.coff * es;
    }
    int ldc(const View& v) const { return tensors[v.t].C; }

    void drop_graphs() {
        // A graph exec (and the plans / workspace it points into) must not be destroyed
        // while a replay is still in flight; a multi-branch exec destroyed mid-replay
        // left libamdhip64 to segfault in a later hipGraphLaunch.
        if (!graphs.empty() || !plans.empty()) {
            (void)hipSetDevice(device);
            (void)hipDeviceSynchronize();
        }
        for (auto& kv : graphs) (void)hipGraphExecDestroy(kv.second);
        graphs.clear();
        free_plans();
    }

    // ---------------------------------------------------------- launches
    static void pick_tile(long long M, int cout, int& BM, int& BN) {
        BN = cout <= 16 ? 16 : cout <= 32 ? 32 : cout <= 64 ? 64 : 128;
        const long long gn = (cout + BN - 1) / BN;
        BM = 64;
        for (int bm : {256, 128}) {
            if (((M + bm - 1) / bm) * gn >= 1024) { BM = bm; break; }
        }
    }

    void conv_args(const Op& op, int B, int H, int W, ConvArgs& a, int& BM, int& BN) const {
        const ConvDesc& d = convs[op.conv];
        const Tensor& to = tensors[op.out.t];
        const int lvl_in = tensors[op.in[0].v.t].level - op.in[0].up;
        a.Hi = H >> lvl_in; a.Wi = W >> lvl_in;
        a.Ho = H >> to.level; a.Wo = W >> to.level;
        a.stride = d.stride; a.pad = d.k / 2; a.KH = d.k; a.KW = d.k;
        for (size_t si = 0; si < op.in.size(); ++si) {
            const Seg& sg = op.in[si];
            const Tensor& ts = tensors[sg.v.t];
            const int hh = H >> ts.level, ww = W >> ts.level;
            if (si == 0) { a.in0 = ptr(sg.v); a.ldc0 = ts.C; a.c0 = sg.v.C; a.up0 = sg.up; a.h0 = hh; a.w0 = ww; }
            else { a.in1 = ptr(sg.v); a.ldc1 = ts.C; a.c1 = sg.v.C; a.up1 = sg.up; a.h1 = hh; a.w1 = ww; }
        }
        if (op.in.size() == 1) { a.in1 = a.in0; a.ldc1 = a.ldc0; a.c1 = 0; a.up1 = 0; a.h1 = a.h0; a.w1 = a.w0; }
        a.Cin = d.cin_p; a.K = d.K; a.Kp = d.Kp;
        a.M = B * a.Ho * a.Wo;
        a.w = d.w_dev; a.bias = d.b_dev; a.ktab = d.ktab_dev;
        a.out = ptr(op.out); a.ldo = to.C;
        if (op.has_res) { a.res = ptr(op.res); a.ldr = ldc(op.res); }
        a.Cout = d.cout_p;
        a.act = d.act;
        pick_tile(a.M, a.Cout, BM, BN);
        a.gm = (a.M + BM - 1) / BM;
        a.gn = (a.Cout + BN - 1) / BN;
        a.zero = zero_dev;
        a.ks = 1;
    }

    DwArgs dw_args(const Op& op, int B, int H, int W) const {
        const ConvDesc& d = convs[op.conv];
        const Tensor& ti = tensors[op.in[0].v.t];
        DwArgs a{};
        a.in = ptr(op.in[0].v); a.ldi = ti.C;
        a.H = H >> ti.level; a.W = W >> ti.level; a.C = d.cout_p; a.M = B * a.H * a.W;
        a.w = (const float*)d.w_dev; a.bias = d.b_dev;
        a.out = ptr(op.out); a.ldo = ldc(op.out); a.act = d.act;
        return a;
    }
    PoolArgs pool_args(const Op& op, int B, int H, int W) const {
        const Tensor& t = tensors[op.out.t];
        PoolArgs a{};
        a.buf = ptr(op.out); a.ldc = t.C; a.C = op.out.C; a.H = H >> t.level; a.W = W >> t.level; a.B = B;
        return a;
    }
    AttnArgs attn_args(const Op& op, int H, int W) const {
        const ConvDesc& d = convs[op.conv];
        const Tensor& tq = tensors[op.in[0].v.t];
        AttnArgs a{};
        a.qkv = ptr(op.in[0].v); a.ldq = tq.C;
        a.Hs = H >> tq.level; a.Ws = W >> tq.level; a.T = a.Hs * a.Ws;
        a.heads = op.heads; a.dk = 32; a.dh = 64;
        a.scale = (float)std::pow(32.0, -0.5);
        a.pe_w = (const float*)d.w_dev; a.pe_b = d.b_dev;
        a.out = ptr(op.out); a.ldo = ldc(op.out);
        return a;
    }

    // ---------------------------------------------------------- conv_mx (16-bit dense convs)
    MxShape mx_shape(const ConvArgs& a, int B) const {
        MxShape sh{};
        sh.ks = a.KH; sh.s = a.stride; sh.cin = a.Cin; sh.cout = a.Cout;
        sh.Hi = a.Hi; sh.Wi = a.Wi; sh.Ho = a.Ho; sh.Wo = a.Wo; sh.B = B;
        sh.c0 = a.c1 ? a.c0 : a.Cin; sh.c1 = a.c1; sh.up0 = a.up0; sh.up1 = a.up1;
        sh.ldo = a.ldo; sh.ldr = a.res ? a.ldr : 0;
        return sh;
    }
    static std::string mx_name(const MxPlan& p) {
        char b[96];
        if (p.cfg.kind == 2)
            snprintf(b, sizeof(b), "rw_g%d_p%d_mb%d_ns%d_t%dx%d%s%s", p.cfg.na, p.cfg.wm, p.cfg.mb, p.cfg.nbuf, p.TH, p.TW,
                     p.cfg.gdiv == 2 ? "_d2" : p.cfg.gdiv == 4 ? "_d4" : "", p.cfg.pc ? "_cm" : "");
        else
            snprintf(b, sizeof(b), "%s_na%d_mb%d_w%dx%d_ncb%d_t%dx%d", p.cfg.kind ? "mxr" : "mx", p.cfg.na, p.cfg.mb,
                     p.cfg.wn, p.cfg.wm, p.cfg.ncb, p.TH, p.TW);
        return b;
    }
    // packed weights of conv `ci` in the layout of plan `p` (cached per layout)
    const char* mx_weights(int ci, const MxPlan& p, const MxShape& sh) {
        ConvDesc& d = convs[ci];
        char k[96];
        snprintf(k, sizeof(k), "%d/%d/%d/%d/%d/%d/%d/%d", p.cfg.kind, p.cfg.ks, p.cfg.na, p.cfg.wn, p.cfg.ncb, p.nst,
                 p.nslices, p.wstage);
        auto it = d.mx_w.find(k);
        if (it != d.mx_w.end()) return (const char*)it->second;
        require(d.loaded, "weights of " + d.name + " not loaded", YH_ESTATE);
        const std::vector<uint16_t> pk = mx_pack(p, sh, d.wf.data(), d.cin, d.phys2log, dtype == BF16, d.cout);
        void* dev = nullptr;
        HIPCHECK(hipMalloc(&dev, pk.size() * 2));
        HIPCHECK(hipMemcpy(dev, pk.data(), pk.size() * 2, hipMemcpyHostToDevice));
        d.mx_w.emplace(k, dev);
        return (const char*)dev;
    }
    int launch_mx_op(const Op& op, const MxPlan& pl, int B, int H, int W, hipStream_t s) {
        ConvArgs a{};
        int BM, BN;
        conv_args(op, B, H, W, a, BM, BN);
        const MxShape sh = mx_shape(a, B);
        MxArgs m{};
        mx_fill_args(pl, sh, m);
        m.in0 = (const char*)a.in0;
        m.in1 = a.c1 ? (const char*)a.in1 : nullptr;
        m.ldc0 = a.ldc0; m.ldc1 = a.ldc1;
        m.hs0 = a.h0; m.ws0 = a.w0; m.hs1 = a.h1; m.ws1 = a.w1;
        m.w = mx_weights(op.conv, pl, sh);
        m.bias = a.bias;
        m.out = (char*)a.out; m.ldo = a.ldo;
        m.res = (const char*)a.res; m.ldr = a.ldr;
        m.act = a.act;
        m.zero = (const char*)zero_dev;
        return launch_mx(dtype, pl, m, s);
    }

    // input bytes a plan stages per output pixel and cout slice, relative to one read of the
    // input: the tile's patch over its outputs (halo, stride) times the cout slices
    static double patch_reads(const MxPlan& pl) {
        const double out = (double)pl.TH * pl.TW;
        const double in = (double)pl.PR * pl.PC / (pl.cfg.ks == 3 && pl.cfg.s == 2 ? 4.0 : 1.0);
        return in / out * pl.nslices;
    }

    // Pick the conv_mx plan of every dense conv for this shape: one plain forward with
    // each layer's default plan (realistic activations in the workspace), then every
    // candidate plan of every layer timed over 3 launches after a warm-up launch, each
    // right after the forward's preceding op (in situ; the input's cache state of the
    // forward: back-to-back launches of one layer favoured plans that re-read a
    // MALL-resident input, e.g. net.p3.0's 32-B-per-stage plan at 2x HBM traffic). The
    // candidates are bit-identical (one reduction order), so the choice only changes
    // speed. Runs outside any graph capture; the next forward recomputes everything.
    void ensure_tuned(int B, int H, int W, hipStream_t s) {
        if (dtype == F32) return;   // conv_gemm only
        const GraphKey key{B, H, W};
        auto it = conv_kern.find(key);
        if (it != conv_kern.end()) { cur_kern = &it->second; return; }
        if (!num_cus) HIPCHECK(hipDeviceGetAttribute(&num_cus, hipDeviceAttributeMultiprocessorCount, device));
        const int forced = force_kern >= 0 ? force_kern : opt.conv_force;
        const bool tune_log = opt.tune_log;
        std::vector<MxChoice> ch(ops.size());
        std::vector<std::vector<MxPlan>> cands(ops.size());
        for (size_t i = 0; i < ops.size(); ++i) {
            if (ops[i].kind != OP_CONV) continue;
            ConvArgs a{};
            int BM, BN;
            conv_args(ops[i], B, H, W, a, BM, BN);
            cands[i] = mx_candidates(mx_shape(a, B), num_cus);
            require(!cands[i].empty(), "no conv_mx plan for " + ops[i].label);
            const int pick = forced >= 0 ? std::min(forced, (int)cands[i].size() - 1) : 0;
            ch[i].plan = cands[i][pick];
            ch[i].name = mx_name(ch[i].plan);
        }
        auto& slot = conv_kern[key];
        slot = ch;
        cur_kern = &slot;
        if (forced >= 0) return;
        run_ops(B, H, W, s);
        hipEvent_t e0, e1;
        HIPCHECK(hipEventCreate(&e0));
        HIPCHECK(hipEventCreate(&e1));
        const std::vector<char>& act = cur_plan->active;
        for (size_t i = 0; i < ops.size(); ++i) {
            if (ops[i].kind != OP_CONV || cands[i].size() < 2 || !act[i]) continue;
            int prev = (int)i - 1;
            while (prev >= 0 && !act[prev]) --prev;
            // two interleaved rounds over the candidates, each candidate's faster round kept: one
            // disturbed measurement (another lane's kernels, a clock step) no longer decides a
            // layer's plan for the life of the engine (a bench's roofline forward once read its
            // 3x3 family 17 % slower than the same library's next run)
            std::vector<float> t_ms(cands[i].size(), 3.0e38f);
            for (int round = 0; round < 2; ++round)
            for (size_t c = 0; c < cands[i].size(); ++c) {
                const MxPlan& pl = cands[i][c];
                int rc = launch_mx_op(ops[i], pl, B, H, W, s);
                float ms = 0.f;
                if (prev >= 0) {
                    // in situ: each timed launch right after the op that precedes it in the
                    // forward, so the input's cache state (just written, L2 / MALL warm, the
                    // layer's other operands cold) is the forward's, not a back-to-back loop's
                    for (int r = 0; r < 3 && rc == 0; ++r) {
                        launch_op((size_t)prev, B, H, W, s);
                        HIPCHECK(hipEventRecord(e0, s));
                        rc = launch_mx_op(ops[i], pl, B, H, W, s);
                        HIPCHECK(hipEventRecord(e1, s));
                        HIPCHECK(hipEventSynchronize(e1));
                        float t = 0.f;
                        HIPCHECK(hipEventElapsedTime(&t, e0, e1));
                        ms += t;
                    }
                } else {
                    HIPCHECK(hipEventRecord(e0, s));
                    for (int r = 0; r < 3 && rc == 0; ++r) rc = launch_mx_op(ops[i], pl, B, H, W, s);
                    HIPCHECK(hipEventRecord(e1, s));
                    HIPCHECK(hipEventSynchronize(e1));
                    HIPCHECK(hipEventElapsedTime(&ms, e0, e1));
                }
                if (rc != 0) throw Fail(YH_EHIP, "tuning launch of " + ops[i].label + " failed");
                if (tune_log)
                    fprintf(stderr, "[yh tune] %-36s %-40s %8.2f us\n", ops[i].label.c_str(), mx_name(pl).c_str(),
                            ms * 1e3f / 3);
                t_ms[c] = std::min(t_ms[c], ms);
            }
            // pick after every candidate is timed: the fastest, except that for 3x3 layers a plan
            // within 3 % of the fastest that re-reads fewer input bytes (halo and cout-slice
            // re-reads) wins - stable choices, less HBM pressure beside the other lanes
            // YH_TUNE_CU=1 (experiment): rank by CU-time (time x CUs the grid occupies) instead of
            // time: with lanes overlapping, a plan that leaves CUs to the other lanes can win
            if (getenv("YH_TUNE_CU"))
                for (size_t c = 0; c < cands[i].size(); ++c)
                    t_ms[c] *= (float)std::min(cands[i][c].grid, num_cus) / (float)num_cus;
            const float best = *std::min_element(t_ms.begin(), t_ms.end());
            size_t pick = 0;
            for (size_t c = 0; c < cands[i].size(); ++c) {
                const MxPlan &pc = cands[i][c], &pp = cands[i][pick];
                const bool near = pc.cfg.ks == 3 && t_ms[c] <= best * 1.03f;
                const bool near_p = pp.cfg.ks == 3 && t_ms[pick] <= best * 1.03f;
                bool better;
                if (near && near_p) {
                    const double rc_ = patch_reads(pc), rp = patch_reads(pp);
                    better = rc_ < rp || (rc_ == rp && t_ms[c] < t_ms[pick]);
                } else {
                    better = (near && !near_p) || (!near_p && t_ms[c] < t_ms[pick]);
                }
                if (better) pick = c;
            }
            slot[i].plan = cands[i][pick];
            slot[i].name = mx_name(cands[i][pick]);
        }
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    }

    PwChainArgs pw_chain_args(const Op& op, int B, int H, int W) {
        PwChainArgs a{};
        const int lv = tensors[op.out.t].level;
        a.M = (long long)B * (H >> lv) * (W >> lv);
        a.P = op.pwP;
        a.nst = (int)op.pws.size();
        a.nload = (int)op.pwl.size();
        // YH_PWC_WARM=0 (read when the arguments are built): no L2 warm-up in the prologue
        const char* ew = getenv("YH_PWC_WARM");
        a.sink = ew && atoi(ew) == 0 ? -1 : op.pwLds - 1024;
        a.zero = zero_dev;
        for (int z = 0; z < a.nload; ++z) {
            PwcLoad& L = a.ld[z];
            L.g = ptr(op.pwl[z]);
            L.ldg = ldc(op.pwl[z]);
            L.lds = op.pwl_lds[z];
            L.nchunk = op.pwl[z].C / 8;
        }
        for (int k = 0; k < a.nst; ++k) {
            const Op& o = ops[op.alts[k]];
            const ConvDesc& d = convs[o.conv];
            const Op::PwStage& ps = op.pws[k];
            PwcStage& st = a.st[k];
            st.K = d.K;
            st.N = d.cout;
            st.act = d.act;
            st.nrun = (int)ps.runs.size();
            for (int r = 0; r < st.nrun; ++r) {
                const Op::PwRun& pr = ps.runs[r];
                PwcRun& R = st.run[r];
                R.nkb = pr.nch / 16;
                if (pr.stage >= 0) {
                    const int ld = convs[ops[op.alts[pr.stage]].conv].cout + 8;
                    R.lds = op.pws[pr.stage].lds + pr.coff * 2;
                    R.ld = ld;
                } else {
                    R.lds = op.pwl_lds[pr.load];
                    R.ld = op.pwl[pr.load].C + 8;
                }
            }
            // A-fragment-ordered copy (upload: "pwfrag"); wld = Kp gives its k-blocks per A tile
            auto itw = d.mx_w.find("pwfrag");
            require(itw != d.mx_w.end(), "pw_chain: no fragment-ordered weights for " + d.name);
            st.w = itw->second;
            st.wld = d.Kp;
            st.bias = d.b_dev;
            st.res_lds = -1;
            if (o.has_res) {
                if (ps.res_stage >= 0) {
                    st.res_lds = op.pws[ps.res_stage].lds + ps.res_coff * 2;
                    st.res_ldl = convs[ops[op.alts[ps.res_stage]].conv].cout + 8;
                } else {
                    st.res_lds = op.pwl_lds[ps.res_load];
                    st.res_ldl = op.pwl[ps.res_load].C + 8;
                }
            }
            st.out = ptr(o.out);
            st.ldo = ldc(o.out);
            st.out_lds = ps.keep ? ps.lds : -1;
            st.out_ldl = d.cout + 8;
        }
        return a;
    }

    HeadClsArgs head_cls_args(const Op& op, int B, int H, int W) {
        HeadClsArgs a{};
        a.B = B;
        a.nc = var.num_classes;
        int l0 = 0;
        while (!op.hlv[l0]) ++l0;
        a.c3 = convs[op.hc[l0][1]].cout;
        // workgroup order: levels 0, 1, 2 (issuing the 20x20 level first was 1.5-3 us slower,
        // profiles/r03_ops_hcls_order.txt)
        int lvls[3], nl = 0;
        for (int l = 0; l < 3; ++l)
            if (op.hlv[l]) lvls[nl++] = l;
        for (int k = 0; k < nl; ++k) {
            const int l = lvls[k];
            HeadClsLevel& v = a.lv[a.nlv++];
            const Tensor& t = tensors[op.hx[l].t];
            v.H = H >> t.level;
            v.W = W >> t.level;
            v.x = ptr(op.hx[l]);
            v.ldx = ldc(op.hx[l]);
            v.C0 = op.hx[l].C;
            v.y = ptr(op.hy[l]);
            v.ldy = ldc(op.hy[l]);
            v.aoff = anchor_off(l, H, W);
            const ConvDesc &d1 = convs[op.hc[l][0]], &p1 = convs[op.hc[l][1]], &d2 = convs[op.hc[l][2]],
                           &p2 = convs[op.hc[l][3]], &p3 = convs[op.hc[l][4]];
            require(d1.loaded && p1.loaded && d2.loaded && p2.loaded && p3.loaded, "head.cls weights not loaded");
            v.dw1w = (const float*)d1.w_dev; v.dw1b = d1.b_dev; v.dw1ld = d1.cout_p;
            v.pw1w = p1.w_dev; v.pw1ld = p1.Kp; v.pw1b = p1.b_dev;
            v.dw2w = (const float*)d2.w_dev; v.dw2b = d2.b_dev; v.dw2ld = d2.cout_p;
            v.pw2w = p2.w_dev; v.pw2ld = p2.Kp; v.pw2b = p2.b_dev;
            v.pw3w = p3.w_dev; v.pw3ld = p3.Kp; v.pw3b = p3.b_dev;
            require(head_cls_tile(v.C0, a.c3, a.nc, v.H, v.W, v.TH, v.TW), "head.cls: no LDS tile");
            v.ntw = (v.W + v.TW - 1) / v.TW;
            v.tiles = v.ntw * ((v.H + v.TH - 1) / v.TH);
        }
        a.zero = zero_dev;
        if (op.direct) {
            a.io = (const void* const*)io_dev;
            a.A = anchor_off(3, H, W);
        }
        // one workgroup per tile, levels in lvls order
        int wg = 0;
        for (int k = 0; k < nl; ++k) {
            a.lv[k].wg0 = wg;
            wg += B * a.lv[k].tiles;
        }
        return a;
    }

    BoxDflArgs box_dfl_args(const Op& op, int B, int H, int W) {
        BoxDflArgs a{};
        a.B = B;
        a.nc = var.num_classes;
        a.A = anchor_off(3, H, W);
        a.io = (const void* const*)io_dev;
        a.nk = op.bx[0].C / 16;
        // tiles per wave (YH_BOXDFL_TPW: 1 / 2 / 4, read when the arguments are built)
        const char* et = getenv("YH_BOXDFL_TPW");
        a.tpw = BOX_DFL_TPW;
        if (et && (atoi(et) == 1 || atoi(et) == 2 || atoi(et) == 4)) a.tpw = atoi(et);
        int wg = 0;
        for (int l = 0; l < 3; ++l) {
            BoxDflLevel& v = a.lv[a.nlv++];
            const ConvDesc& d = convs[op.bc[l]];
            require(d.loaded, "head.box weights not loaded");
            require(d.cin == 16 * a.nk && d.cout == 64 && d.cout_p >= 64, "box_dfl: conv shape");
            const int lv = tensors[op.bx[l].t].level;
            v.x = ptr(op.bx[l]);
            v.ldx = ldc(op.bx[l]);
            v.H = H >> lv;
            v.W = W >> lv;
            v.stride = (float)(1 << lv);
            v.aoff = anchor_off(l, H, W);
            v.w = d.w_dev;
            v.wld = d.Kp;
            v.b = d.b_dev;
            v.wg0 = wg;
            const long long tiles = ((long long)B * v.H * v.W + 31) / 32;
            wg += (int)((tiles + 4 * a.tpw - 1) / (4 * a.tpw));
        }
        return a;
    }

    void launch_op(size_t oi, int B, int H, int W, hipStream_t s) {
        const Op& op = ops[oi];
        int rc = 0;
        switch (op.kind) {
            case OP_FIRST: {
                const ConvDesc& d = convs[op.conv];
                FirstConvArgs a{};
                a.io = (const void* const*)io_dev;
                a.H = H; a.W = W; a.Ho = H >> 1; a.Wo = W >> 1;
                a.Cout = d.cout_p;
                a.ldo = ldc(op.out);
                a.M = B * a.Ho * a.Wo;
                a.w = (const float*)d.w_dev;
                a.bias = d.b_dev;
                a.out = ptr(op.out);
                a.act = d.act;
                a.in_u8 = in_u8;
                rc = launch_first_conv(dtype, a, B, s);
                break;
            }
            case OP_CONV: {
                if (dtype != F32) {
                    require(cur_kern != nullptr, "conv plans not chosen", YH_ESTATE);
                    rc = launch_mx_op(op, (*cur_kern)[oi].plan, B, H, W, s);
                    break;
                }
                ConvArgs a{};
                int BM, BN;
                conv_args(op, B, H, W, a, BM, BN);
                rc = launch_conv(dtype, CONV_GEMM, BM, BN, a, s);
                break;
            }
            case OP_DW: rc = launch_dwconv(dtype, dw_args(op, B, H, W), s); break;
            case OP_SPPF: rc = launch_sppf(dtype, pool_args(op, B, H, W), s); break;
            case OP_ATTN: rc = launch_attention(dtype, attn_args(op, H, W), B, s); break;
            case OP_HEADCLS: {
                rc = launch_head_cls(dtype, head_cls_args(op, B, H, W), s);
                break;
            }
            case OP_DECODE: {
                DecodeArgs a{};
                for (int l = 0; l < 3; ++l) {
                    const Tensor& t = tensors[op.lvl[l].t];
                    a.lvl[l] = ptr(op.lvl[l]);
                    a.H[l] = H >> t.level; a.W[l] = W >> t.level;
                    a.stride[l] = (float)(1 << t.level);
                    a.ldc = t.C;
                }
                a.nc = var.num_classes;
                a.A = a.H[0] * a.W[0] + a.H[1] * a.W[1] + a.H[2] * a.W[2];
                a.B = B;
                a.io = (const void* const*)io_dev;
                a.a_lo = anchor_off(op.dlo, H, W);
                a.box = op.dbox ? 1 : 0;
                rc = launch_decode(dtype, a, s);
                break;
            }
            case OP_BOXDFL: rc = launch_box_dfl(dtype, box_dfl_args(op, B, H, W), s); break;
            case OP_BOXCHAIN: rc = launch_box_chain(dtype, box_chain_args(op, B, H, W), s); break;
            case OP_PWCHAIN: rc = launch_pw_chain(dtype, pw_chain_args(op, B, H, W), op.pwLds, s); break;
            case OP_STEM2: {
                const ConvDesc& d = convs[op.conv];
                Stem2Args a{};
                a.io = (const void* const*)io_dev;
                a.H = H; a.W = W; a.Hs = H >> 1; a.Ws = W >> 1; a.Ho = H >> 2; a.Wo = W >> 2; a.B = B;
                a.w1 = (const float*)d.w_dev;
                a.b1 = d.b_dev;
                a.c1 = d.cout; a.c1p = d.cout_p; a.c2 = convs[op.cs[0]].cout;
                a.prm = stem2_params(op, a.prm_bias);
                a.out = ptr(op.out);
                a.ldo = ldc(op.out);
                a.in_u8 = in_u8;
                stem2_tiles(a.Ho, a.Wo, a.ntw, a.nth);
                rc = launch_stem2(dtype, a, s);
                break;
            }
            case OP_CSP: {
                CspArgs a{};
                const View& xv = op.in[0].v;
                const int lv = tensors[xv.t].level;
                a.x = ptr(xv);
                a.ldx = ldc(xv);
                a.y = ptr(op.out);
                a.ldy = ldc(op.out);
                a.H = H >> lv;
                a.W = W >> lv;
                a.B = B;
                a.prm = csp_params(op);
                a.ni = op.cs[0] >= 0 ? convs[op.cs[0]].cin / 16 : 0;
                a.nc = convs[op.cs[1]].cin / 16;
                a.no = convs[op.cs[3]].cout / 32;
                require(csp_tile(a.ni, a.nc, a.no, a.H, a.W, a.TH, a.TW), op.label + ": no LDS tile");
                a.ntw = (a.W + a.TW - 1) / a.TW;
                a.tiles = a.ntw * ((a.H + a.TH - 1) / a.TH);
                a.ntiles = B * a.tiles;
                a.zero = zero_dev;
                if (!num_cus) HIPCHECK(hipDeviceGetAttribute(&num_cus, hipDeviceAttributeMultiprocessorCount, device));
                // two workgroups per CU when the LDS allows (measured: net.p2.1 138 -> 103 us at b32)
                {
                    // persistent workgroups: as many as are resident at once (two per CU where the
                    // LDS allows)
                    const int lds = csp_lds(a.TH, a.TW, a.ni, a.nc, a.no);
                    const int per_cu = CSP_THREADS < 1024 && lds > 0 && lds <= 80 * 1024 ? 2 : 1;
                    rc = launch_csp(dtype, a, std::min(a.ntiles, per_cu * num_cus), s);
                }
                break;
            }
            case OP_C3K: {
                C3kArgs a{};
                const View& xv = op.in[0].v;
                const int lv = tensors[xv.t].level;
                a.x = ptr(xv);
                a.ldx = ldc(xv);
                a.y = ptr(op.out);
                a.ldy = ldc(op.out);
                a.H = H >> lv;
                a.W = W >> lv;
                a.B = B;
                a.prm = c3k_params(op);
                a.hh = convs[op.ck[0]].cout;
                rc = launch_c3k(dtype, a, s);
                break;
            }
        }
        if (rc != 0) throw Fail(YH_EHIP, "launch of " + op.label + " failed: " + hipGetErrorString((hipError_t)rc));
    }

    // ---------------------------------------------------------- launch units
    // One launch unit per op (the unit layer stays for the profiling / segment APIs).
    void free_plans() {
        plans.clear();
        cur_plan = nullptr;
    }
    void ensure_plan(int B, int H, int W) {
        const GraphKey key{B, H, W};
        auto it = plans.find(key);
        if (it != plans.end()) { cur_plan = &it->second; return; }
        Plan pl;
        // a fused C3k block runs where bands of its map fit a workgroup's LDS (c3k_lds), its
        // seven per-layer launches everywhere else
        pl.active.assign(ops.size(), 1);
        for (size_t i = 0; i < ops.size(); ++i) {
            if (ops[i].kind != OP_BOXCHAIN) continue;
            bool fits = true;
            for (int l = 0; l < 3; ++l) {
                const int lv = tensors[ops[i].hx[l].t].level;
                int th, tw;
                fits = fits && bx_tile(H >> lv, W >> lv, th, tw);
            }
            if (fits)
                for (int k : ops[i].alts) pl.active[k] = 0;
            else
                pl.active[i] = 0;
        }
        // a pointwise chain reads every stage's weights once per workgroup: kept where that is at
        // most 160 MB per launch (v11_n b32: 52-90 MB, 104 -> 77 us for its three chains),
        // per-layer launches above (v11_s b64 1.4 GB: the chains ran 2.2x slower,
        // profiles/r05_pw_chain_configs.txt)
        for (size_t i = 0; i < ops.size(); ++i) {
            if (ops[i].kind != OP_PWCHAIN) continue;
            const int lv = tensors[ops[i].out.t].level;
            const long long M = (long long)B * (H >> lv) * (W >> lv);
            const double grid = (double)((M + ops[i].pwP - 1) / ops[i].pwP);
            double wb = 0;
            for (int k : ops[i].alts) wb += (double)convs[ops[k].conv].cout * convs[ops[k].conv].K * es;
            if (wb * grid <= 160e6)
                for (int k : ops[i].alts) pl.active[k] = 0;
            else
                pl.active[i] = 0;
        }
        for (size_t i = 0; i < ops.size(); ++i) {
            if (ops[i].kind != OP_C3K) continue;
            const int lv = tensors[ops[i].out.t].level;
            if (c3k_lds(H >> lv, W >> lv, convs[ops[i].ck[0]].cout) > 0)
                for (int k = ops[i].alt0; k < ops[i].alt1; ++k) pl.active[k] = 0;
            else
                pl.active[i] = 0;
        }
        for (size_t i = 0; i < ops.size(); ++i)
            if (pl.active[i]) pl.units.push_back(Unit{(int)i, (int)i + 1, false});
        cur_plan = &plans.emplace(key, std::move(pl)).first->second;
    }
    void launch_unit(const Unit& u, int B, int H, int W, hipStream_t s) {
        for (int k = u.first; k < u.last; ++k) launch_op(k, B, H, W, s);
    }

    void run_ops(int B, int H, int W, hipStream_t s) {
        if (!cur_plan) {
            for (size_t i = 0; i < ops.size(); ++i) launch_op(i, B, H, W, s);
            return;
        }
        for (auto& u : cur_plan->units) launch_unit(u, B, H, W, s);
    }

    int in_u8 = 0;   // the current forward's input kind (see GraphKey::X)
    void forward(const void* x, int B, int H, int W, void* y, hipStream_t s, int x_u8 = 0) {
        in_u8 = x_u8;
        for (auto& d : convs) require(d.loaded, "weights of " + d.name + " not loaded", YH_ESTATE);
        reserve(B, H, W);
        HIPCHECK(hipSetDevice(device));
        require(launch_set_io(io_dev, x, y, s) == 0, "set_io launch failed", YH_EHIP);
        ensure_plan(B, H, W);
        ensure_tuned(B, H, W, s);
        lastB = B; lastH = H; lastW = W;
        if (profile) {   // HIP events around every launch unit, on the caller's stream
            const size_t nu = cur_plan->units.size();
            if (ev.size() < 2 * nu) {
                for (auto e : ev) (void)hipEventDestroy(e);
                ev.assign(2 * nu, nullptr);
                for (auto& e : ev) HIPCHECK(hipEventCreate(&e));
            }
            if (prof_key.B != B || prof_key.H != H || prof_key.W != W) {
                prof_ms.assign(nu, 0.0);
                prof_calls.assign(nu, 0);
                prof_key = GraphKey{B, H, W};
            }
            for (size_t i = 0; i < nu; ++i) {
                HIPCHECK(hipEventRecord(ev[2 * i], s));
                launch_unit(cur_plan->units[i], B, H, W, s);
                HIPCHECK(hipEventRecord(ev[2 * i + 1], s));
            }
            HIPCHECK(hipEventSynchronize(ev[2 * nu - 1]));
            for (size_t i = 0; i < nu; ++i) {
                float ms = 0.f;
                HIPCHECK(hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]));
                prof_ms[i] += ms;
                prof_calls[i] += 1;
            }
            return;
        }
        if (!use_graph) {
            run_ops(B, H, W, s);
            return;
        }
        const GraphKey key{B, H, W, in_u8};
        auto it = graphs.find(key);
        if (it == graphs.end()) {
            // one eager pass first: every kernel of the plan is then loaded and has its
            // function attributes (dynamic-LDS limits) set outside any stream capture
            run_ops(B, H, W, s);
            if (!cap_stream) HIPCHECK(hipStreamCreateWithFlags(&cap_stream, hipStreamNonBlocking));
            hipGraph_t g = nullptr;
            HIPCHECK(hipStreamBeginCapture(cap_stream, hipStreamCaptureModeThreadLocal));
            try {
                run_ops(B, H, W, cap_stream);
            } catch (...) {
                (void)hipStreamEndCapture(cap_stream, &g);
                if (g) (void)hipGraphDestroy(g);
                throw;
            }
            HIPCHECK(hipStreamEndCapture(cap_stream, &g));
            hipGraphExec_t ex = nullptr;
            HIPCHECK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
            (void)hipGraphDestroy(g);
            it = graphs.emplace(key, ex).first;
        }
        HIPCHECK(hipGraphLaunch(it->second, s));
    }

    // ---------------------------------------------------------- per-op accounting
    OpClass op_class(const Op& op) const {
        switch (op.kind) {
            case OP_FIRST: return CL_FIRST;
            case OP_CONV: return convs[op.conv].k == 3 ? CL_CONV3 : CL_CONV1;
            case OP_DW: return CL_DW;
            case OP_SPPF: return CL_SPPF;
            case OP_ATTN: return CL_ATTN;
            case OP_DECODE: return CL_DECODE;
            case OP_HEADCLS: return CL_HEADCLS;
            case OP_BOXDFL: return CL_BOXDFL;
            case OP_CSP: return CL_CSP;
            case OP_STEM2: return CL_FIRST;
            case OP_C3K: return CL_C3K;
            case OP_BOXCHAIN: return CL_BOXCHAIN;
            case OP_PWCHAIN: return CL_PWCHAIN;
        }
        return CL_CONV1;
    }
    // algorithmic bytes (each operand read once, output written once) and flops per call
    void op_cost(const Op& op, int B, int H, int W, double& bytes, double& flops) const {
        bytes = 0; flops = 0;
        auto px = [&](int level) { return (double)B * (H >> level) * (W >> level); };
        switch (op.kind) {
            case OP_FIRST: {
                const ConvDesc& d = convs[op.conv];
                const double out = px(1);
                bytes = (double)B * 3 * H * W * es + out * d.cout * es + d.cout * 27.0 * 4;
                flops = 2.0 * out * d.cout * 27;
                break;
            }
            case OP_CONV: {
                const ConvDesc& d = convs[op.conv];
                const double out = px(tensors[op.out.t].level);
                for (size_t si = 0; si < op.in.size(); ++si) {
                    const Seg& sg = op.in[si];
                    bytes += px(tensors[sg.v.t].level) * d.segs[si].first * es;
                }
                bytes += out * d.cout * es + (double)d.cout * d.cin * d.k * d.k * es;
                if (op.has_res) bytes += out * d.cout * es;
                flops = 2.0 * out * d.cout * d.cin * d.k * d.k;
                break;
            }
            case OP_DW: {
                const ConvDesc& d = convs[op.conv];
                const double n = px(tensors[op.out.t].level);
                bytes = 2.0 * n * d.cout * es;
                flops = 2.0 * n * d.cout * 9;
                break;
            }
            case OP_SPPF: {
                const double n = px(tensors[op.out.t].level);
                bytes = 6.0 * n * op.out.C * es;
                flops = 3.0 * n * op.out.C * 25;
                break;
            }
            case OP_ATTN: {
                const double T = (double)(H >> tensors[op.out.t].level) * (W >> tensors[op.out.t].level);
                const double C = op.heads * 64.0;
                bytes = (double)B * T * (op.heads * 128.0 + C) * es;
                flops = (double)B * op.heads * (2.0 * T * T * (32 + 64)) + 2.0 * B * T * C * 9;
                break;
            }
            case OP_HEADCLS: {
                // the level inputs read once, the class logits written once, weights once
                for (int l = 0; l < 3; ++l) {
                    if (!op.hlv[l]) continue;
                    const double n = px(tensors[op.hx[l].t].level);
                    const int C0 = op.hx[l].C;
                    const ConvDesc& p1 = convs[op.hc[l][1]];
                    const int c3 = p1.cout, nc = convs[op.hc[l][4]].cout;
                    bytes += n * C0 * es + n * nc * es + (9.0 * (C0 + c3) * 4) +
                             ((double)C0 * c3 + (double)c3 * c3 + (double)c3 * nc) * es;
                    flops += 2.0 * n * (9.0 * C0 + (double)C0 * c3 + 9.0 * c3 + (double)c3 * c3 + (double)c3 * nc);
                }
                break;
            }
            case OP_DECODE: {
                double A = 0, cin = 0;
                for (int l = 0; l < 3; ++l) {
                    A += px(tensors[op.lvl[l].t].level);
                    cin = tensors[op.lvl[l].t].C;
                }
                (void)cin;
                if (op.dbox) {
                    bytes = A * (64 + var.num_classes) * es + A * (4 + var.num_classes) * es;
                    flops = A * (64 * 4.0 + var.num_classes * 4.0);
                } else {
                    A = 0;
                    for (int l = op.dlo; l < 3; ++l) A += px(tensors[op.lvl[l].t].level);
                    bytes = 2.0 * A * var.num_classes * es;
                    flops = A * var.num_classes * 4.0;
                }
                break;
            }
            case OP_STEM2: {
                // the image read once, p2.0's output written once, both weights once
                const ConvDesc& d = convs[op.conv];
                const ConvDesc& d2 = convs[op.cs[0]];
                const double s1 = px(1), o2 = px(2);
                bytes = (double)B * 3 * H * W * (in_u8 ? 1 : es) + o2 * d2.cout * es + d.cout * 27.0 * 4 +
                        (double)d2.cout * d2.cin * 9 * es;
                flops = 2.0 * s1 * d.cout * 27 + 2.0 * o2 * d2.cout * d2.cin * 9;
                break;
            }
            case OP_CSP: {
                // block input read once, block output written once, the four convs' weights once
                const double n = px(tensors[op.out.t].level);
                bytes = n * op.in[0].v.C * es + n * convs[op.cs[3]].cout * es;
                for (int k = 0; k < 4; ++k) {
                    if (op.cs[k] < 0) continue;   // tail mode: conv1 is its own op
                    const ConvDesc* d = &convs[op.cs[k]];
                    const double macs = (double)d->cout * d->cin * d->k * d->k;
                    bytes += macs * es;
                    flops += 2.0 * n * macs;
                }
                break;
            }
            case OP_C3K: {
                // block input read once (conv1 and conv2 share it), block output written once,
                // the seven convs' weights once
                const double n = px(tensors[op.out.t].level);
                bytes = n * op.in[0].v.C * es + n * convs[op.ck[6]].cout * es;
                for (int k = 0; k < 7; ++k) {
                    const ConvDesc& d = convs[op.ck[k]];
                    const double macs = (double)d.cout * d.cin * d.k * d.k;
                    bytes += macs * es;
                    flops += 2.0 * n * macs;
                }
                break;
            }
            case OP_PWCHAIN: {
                // the prologue's global inputs (incl. the global residuals) read once, every stage's
                // output written (all stay materialised), each stage's weights once
                const double n = px(tensors[op.out.t].level);
                for (const View& v : op.pwl) bytes += n * v.C * es;
                for (size_t k = 0; k < op.pws.size(); ++k) {
                    const Op& o = ops[op.alts[k]];
                    const ConvDesc& d = convs[o.conv];
                    bytes += n * d.cout * es + (double)d.cout * d.cin * es;
                    flops += 2.0 * n * d.cout * d.cin;
                }
                break;
            }
            case OP_BOXCHAIN: {
                // the level inputs read once, 4 box rows written, the three convs' weights once
                for (int l = 0; l < 3; ++l) {
                    const double n = px(tensors[op.hx[l].t].level);
                    const int C0 = convs[op.bxc[l][0]].cin;
                    const double macs = 64.0 * C0 * 9 + 64.0 * 64 * 9 + 64.0 * 64;
                    bytes += n * C0 * es + n * 4 * es + macs * es + 3 * 64 * 4.0;
                    flops += 2.0 * n * macs + n * 64 * 4.0;
                }
                break;
            }
            case OP_BOXDFL: {
                // the box.l.1 outputs read once, 4 box rows written, weights once per level
                for (int l = 0; l < 3; ++l) {
                    const double n = px(tensors[op.bx[l].t].level);
                    const int K = op.bx[l].C;
                    bytes += n * K * es + n * 4 * es + 64.0 * K * es + 64 * 4.0;
                    flops += 2.0 * n * 64 * K + n * 64 * 4.0;
                }
                break;
            }
        }
    }

    // ---------------------------------------------------------- parity taps (tests only)
    // The workspace operands of an op, in a fixed order (yh_debug_op_desc lists them):
    // inputs first, then outputs. `logical` = channels the op reads / writes of the view.
    struct Operand { std::string role; View v; int up = 0; int logical = 0; };
    std::vector<Operand> operands(const Op& op) const {
        std::vector<Operand> r;
        auto add = [&](const std::string& role, const View& v, int up, int logical) {
            Operand o;
            o.role = role; o.v = v; o.up = up; o.logical = logical;
            r.push_back(o);
        };
        switch (op.kind) {
            case OP_CONV: {
                const ConvDesc& d = convs[op.conv];
                for (size_t si = 0; si < op.in.size(); ++si)
                    add("in" + std::to_string(si), op.in[si].v, op.in[si].up, d.segs[si].first);
                if (op.has_res) add("res", op.res, 0, d.cout);
                add("out", op.out, 0, d.cout);
                break;
            }
            case OP_FIRST: case OP_STEM2: add("out", op.out, 0, op.out.C); break;
            case OP_DW: case OP_ATTN: case OP_CSP: case OP_C3K:
                add("in0", op.in[0].v, op.in[0].up, op.in[0].v.C);
                add("out", op.out, 0, op.out.C);
                break;
            case OP_SPPF: {
                View o = op.out;
                o.coff += op.out.C;
                o.C = 3 * op.out.C;
                add("in0", op.out, 0, op.out.C);
                add("out", o, 0, o.C);
                break;
            }
            case OP_HEADCLS:
                for (int l = 0; l < 3; ++l)
                    if (op.hlv[l]) add("x" + std::to_string(l), op.hx[l], 0, op.hx[l].C);
                if (!op.direct)
                    for (int l = 0; l < 3; ++l)
                        if (op.hlv[l]) add("y" + std::to_string(l), op.hy[l], 0, var.num_classes);
                break;
            case OP_BOXDFL:
                for (int l = 0; l < 3; ++l) add("x" + std::to_string(l), op.bx[l], 0, op.bx[l].C);
                break;
            case OP_BOXCHAIN:
                for (int l = 0; l < 3; ++l) add("x" + std::to_string(l), op.hx[l], 0, op.hx[l].C);
                break;
            case OP_DECODE:
                for (int l = 0; l < 3; ++l) add("L" + std::to_string(l), op.lvl[l], 0, 64 + var.num_classes);
                break;
            case OP_PWCHAIN:
                // per stage s<k>.in<i> / s<k>.res (inputs, read before the chain runs), then the
                // outputs no later stage overwrites (s<k>.out)
                for (size_t k = 0; k < op.alts.size(); ++k) {
                    const Op& o = ops[op.alts[k]];
                    const ConvDesc& d = convs[o.conv];
                    const std::string p = "s" + std::to_string(k) + ".";
                    for (size_t si = 0; si < o.in.size(); ++si) add(p + "in" + std::to_string(si), o.in[si].v, 0, d.segs[si].first);
                    if (o.has_res) add(p + "res", o.res, 0, d.cout);
                }
                for (size_t k = 0; k < op.alts.size(); ++k)
                    if (pw_final(op, (int)k)) {
                        const Op& o = ops[op.alts[k]];
                        add("s" + std::to_string(k) + ".out", o.out, 0, convs[o.conv].cout);
                    }
                break;
        }
        return r;
    }
    // stage k's output is not overwritten by a later stage of the chain
    bool pw_final(const Op& op, int k) const {
        const Op& o = ops[op.alts[k]];
        const int c0 = o.out.coff, c1 = c0 + convs[o.conv].cout;
        for (size_t q = k + 1; q < op.alts.size(); ++q) {
            const Op& w = ops[op.alts[q]];
            const int w0 = w.out.coff, w1 = w0 + convs[w.conv].cout;
            if (w.out.t == o.out.t && w0 < c1 && c0 < w1) return false;
        }
        return true;
    }
    // the convs an op computes, in the op's order (-1: none in that place, e.g. tail-mode conv1)
    std::vector<int> op_convs(const Op& op) const {
        switch (op.kind) {
            case OP_CONV: case OP_FIRST: case OP_DW: case OP_ATTN: return {op.conv};
            case OP_STEM2: return {op.conv, op.cs[0]};
            case OP_CSP: return {op.cs[0], op.cs[1], op.cs[2], op.cs[3]};
            case OP_C3K: return std::vector<int>(op.ck, op.ck + 7);
            case OP_HEADCLS: {
                std::vector<int> r;
                for (int l = 0; l < 3; ++l)
                    for (int k = 0; k < 5; ++k) r.push_back(op.hlv[l] ? op.hc[l][k] : -1);
                return r;
            }
            case OP_BOXDFL: return {op.bc[0], op.bc[1], op.bc[2]};
            case OP_BOXCHAIN: {
                std::vector<int> r;
                for (int l = 0; l < 3; ++l)
                    for (int k = 0; k < 3; ++k) r.push_back(op.bxc[l][k]);
                return r;
            }
            case OP_PWCHAIN: {
                std::vector<int> r;
                for (int k : op.alts) r.push_back(ops[k].conv);
                return r;
            }
            case OP_SPPF: case OP_DECODE: return {};
        }
        return {};
    }
    std::string op_desc(int oi, int B, int H, int W) const {
        const Op& op = ops[oi];
        auto it = plans.find(GraphKey{B, H, W});
        const int active = it == plans.end() ? -1 : it->second.active[oi];
        std::string s = "{\"index\": " + std::to_string(oi) + ", \"kind\": \"" + op_kind_name(op.kind) +
                        "\", \"label\": \"" + op.label + "\", \"active\": " + std::to_string(active) +
                        ", \"heads\": " + std::to_string(op.heads) + ", \"direct\": " + std::to_string(op.direct ? 1 : 0) +
                        ", \"dlo\": " + std::to_string(op.dlo) + ", \"dbox\": " + std::to_string(op.dbox ? 1 : 0) +
                        ", \"convs\": [";
        const std::vector<int> cv = op_convs(op);
        for (size_t i = 0; i < cv.size(); ++i) {
            if (i) s += ", ";
            if (cv[i] < 0) { s += "null"; continue; }
            const ConvDesc& d = convs[cv[i]];
            s += "{\"name\": \"" + d.name + "\", \"k\": " + std::to_string(d.k) + ", \"s\": " + std::to_string(d.stride) +
                 ", \"g\": " + std::to_string(d.groups) + ", \"act\": " + std::to_string(d.act) + ", \"cin\": " +
                 std::to_string(d.cin) + ", \"cout\": " + std::to_string(d.cout) + ", \"bias\": " +
                 std::to_string(d.has_bias) + "}";
        }
        s += "], \"operands\": [";
        const std::vector<Operand> od = operands(op);
        for (size_t i = 0; i < od.size(); ++i) {
            const int lv = tensors[od[i].v.t].level;
            s += std::string(i ? ", " : "") + "{\"role\": \"" + od[i].role + "\", \"H\": " + std::to_string(H >> lv) +
                 ", \"W\": " + std::to_string(W >> lv) + ", \"C\": " + std::to_string(od[i].v.C) + ", \"logical\": " +
                 std::to_string(od[i].logical) + ", \"up\": " + std::to_string(od[i].up) + "}";
        }
        s += "]";
        if (op.kind == OP_PWCHAIN) {
            // per stage: its input runs in weight order (seg = input segment, off = channel within
            // it; src = -1: that device operand, else the output of stage src from channel soff) and
            // its residual source (-2 none, -1 the s<k>.res operand, else a stage's output)
            s += ", \"stages\": [";
            for (size_t k = 0; k < op.pws.size(); ++k) {
                const Op& o = ops[op.alts[k]];
                const Op::PwStage& ps = op.pws[k];
                s += std::string(k ? ", " : "") + "{\"runs\": [";
                int si = 0, soff = 0;
                for (size_t r = 0; r < ps.runs.size(); ++r) {
                    const Op::PwRun& pr = ps.runs[r];
                    while (soff >= o.in[si].v.C) {
                        soff -= o.in[si].v.C;
                        ++si;
                    }
                    s += std::string(r ? ", " : "") + "{\"seg\": " + std::to_string(si) + ", \"off\": " +
                         std::to_string(soff) + ", \"n\": " + std::to_string(pr.nch) + ", \"src\": " +
                         std::to_string(pr.stage) + ", \"soff\": " + std::to_string(pr.stage >= 0 ? pr.coff : 0) + "}";
                    soff += pr.nch;
                }
                s += "], \"res\": " + std::to_string(o.has_res ? ps.res_stage : -2) + ", \"res_off\": " +
                     std::to_string(ps.res_coff) + ", \"final\": " + std::to_string(pw_final(op, (int)k) ? 1 : 0) + "}";
            }
            s += "]";
        }
        s += "}";
        return s;
    }
    // the active ops in [first, last) of the forward at (B, H, W), launched eagerly on s
    void debug_run(const void* x, int x_u8, int B, int H, int W, void* y, int first, int last, hipStream_t s) {
        in_u8 = x_u8;
        for (auto& d : convs) require(d.loaded, "weights of " + d.name + " not loaded", YH_ESTATE);
        require(ws.base && ws.B == B && ws.H == H && ws.W == W, "yh_debug_run_ops: run yh_forward at this shape first",
                YH_ESTATE);
        require(first >= 0 && first <= last && last <= (int)ops.size(), "op range out of bounds");
        HIPCHECK(hipSetDevice(device));
        require(launch_set_io(io_dev, x, y, s) == 0, "set_io launch failed", YH_EHIP);
        ensure_plan(B, H, W);
        ensure_tuned(B, H, W, s);
        for (int i = first; i < last; ++i)
            if (cur_plan->active[i]) launch_op((size_t)i, B, H, W, s);
    }
    // operand `slot` of op `oi` copied out of the workspace as a dense (B, h, w, C) array
    void debug_operand(int oi, int slot, void* dst, size_t dst_bytes, hipStream_t s) const {
        require(oi >= 0 && oi < (int)ops.size(), "op index out of range");
        const std::vector<Operand> od = operands(ops[oi]);
        require(slot >= 0 && slot < (int)od.size(), "operand slot out of range");
        require(ws.base != nullptr, "no workspace yet", YH_ESTATE);
        const View& v = od[slot].v;
        const int lv = tensors[v.t].level;
        const size_t rows = (size_t)ws.B * (ws.H >> lv) * (ws.W >> lv);
        // the caller sizes dst from a desc made at some (batch, H, W): a desc of another shape
        // (or a later reserve() at a larger one) must not turn into an out-of-bounds write
        require(dst_bytes == rows * (size_t)v.C * es, "yh_debug_operand: dst size " + std::to_string(dst_bytes) +
                " B does not match the operand at the workspace shape (" + std::to_string(rows * (size_t)v.C * es) +
                " B)");
        HIPCHECK(hipMemcpy2DAsync(dst, (size_t)v.C * es, ptr(v), (size_t)ldc(v) * es, (size_t)v.C * es, rows,
                                  hipMemcpyDeviceToDevice, s));
    }

    ~Net() {
        drop_graphs();
        free_plans();
        for (auto& d : convs) free_conv(d);
        if (ws.base) (void)hipFree(ws.base);
        if (io_dev) (void)hipFree(io_dev);
        if (zero_dev) (void)hipFree(zero_dev);
        if (cap_stream) (void)hipStreamDestroy(cap_stream);
        for (auto e : ev) (void)hipEventDestroy(e);
    }
};

}  // namespace yh

struct yh_handle {
    yh::Net net;
};

using yh::Fail;

namespace {

template <typename F>
int guarded(F&& f) {
    try {
        f();
        yh::g_err.clear();
        return YH_OK;
    } catch (const Fail& e) {
        yh::g_err = e.what();
        return e.code;
    } catch (const std::exception& e) {
        yh::g_err = e.what();
        return YH_EINVAL;
    } catch (...) {
        yh::g_err = "unknown error";
        return YH_EINVAL;
    }
}

}  // namespace

extern "C" {

int yh_abi_version(void) { return YH_ABI_VERSION; }

const char* yh_last_error(void) { return yh::g_err.c_str(); }

int yh_create(const yh_variant* v, int device, int dtype, yh_handle** out) {
    return guarded([&] {
        yh::require(v && out, "null argument");
        yh::require(dtype == YH_F32 || dtype == YH_F16 || dtype == YH_BF16, "dtype must be YH_F32, YH_F16 or YH_BF16");
        yh::require(v->num_classes > 0, "num_classes must be positive");
        for (int i = 1; i < 6; ++i) yh::require(v->width[i] > 0 && v->width[i] % 8 == 0, "widths must be multiples of 8");
        yh::require(v->width[0] == 3, "input channels (width[0]) must be 3");
        for (int i = 0; i < 6; ++i) yh::require(v->depth[i] >= 1, "depths must be >= 1");
        int ndev = 0;
        HIPCHECK(hipGetDeviceCount(&ndev));
        yh::require(device >= 0 && device < ndev, "device ordinal out of range");
        HIPCHECK(hipSetDevice(device));
        std::unique_ptr<yh_handle> h(new yh_handle());
        yh::Net& n = h->net;
        n.var = *v;
        n.opt = yh::Options::from_env();
        n.device = device;
        n.dtype = dtype;
        n.es = yh::dtype_size(dtype);
        n.build();
        HIPCHECK(hipMalloc(&n.io_dev, 2 * sizeof(void*)));
        HIPCHECK(hipMalloc(&n.zero_dev, 256));
        HIPCHECK(hipMemset(n.zero_dev, 0, 256));
        *out = h.release();
    });
}

void yh_destroy(yh_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->net.device);
    delete h;
}

int yh_conv_count(const yh_handle* h) { return h ? (int)h->net.convs.size() : YH_EINVAL; }

int yh_conv_info(const yh_handle* h, int index, const char** name, int* cout, int* cin_per_group, int* ksize,
                 int* groups, int* has_bias) {
    return guarded([&] {
        yh::require(h && index >= 0 && index < (int)h->net.convs.size(), "conv index out of range");
        const yh::ConvDesc& d = h->net.convs[index];
        if (name) *name = d.name.c_str();
        if (cout) *cout = d.cout;
        if (cin_per_group) *cin_per_group = d.cin / d.groups;
        if (ksize) *ksize = d.k;
        if (groups) *groups = d.groups;
        if (has_bias) *has_bias = d.has_bias;
    });
}

int yh_load_conv(yh_handle* h, int index, const float* weight, const float* bias, const float* bn_gamma,
                 const float* bn_beta, const float* bn_mean, const float* bn_var, double bn_eps) {
    return guarded([&] {
        yh::require(h && weight, "null argument");
        yh::require(!bn_gamma || (bn_beta && bn_mean && bn_var), "BatchNorm needs gamma, beta, mean and var");
        HIPCHECK(hipSetDevice(h->net.device));
        h->net.load_conv(index, weight, bias, bn_gamma, bn_beta, bn_mean, bn_var, bn_eps);
        h->net.drop_graphs();   // captured graphs and level programs hold the old weight pointers
    });
}

int yh_num_anchors(const yh_handle* h, int height, int width, int* anchors) {
    return guarded([&] {
        yh::require(h && anchors, "null argument");
        yh::require(height > 0 && width > 0 && height % 32 == 0 && width % 32 == 0, "height/width must be multiples of 32");
        int a = 0;
        for (int l = 3; l <= 5; ++l) a += (height >> l) * (width >> l);
        *anchors = a;
    });
}

int yh_workspace_bytes(const yh_handle* h, int batch, int height, int width, size_t* bytes) {
    return guarded([&] {
        yh::require(h && bytes, "null argument");
        yh::require(batch > 0 && height % 32 == 0 && width % 32 == 0, "bad shape");
        *bytes = h->net.ws_bytes_for(batch, height, width, nullptr);
    });
}

int yh_reserve(yh_handle* h, int batch, int height, int width) {
    return guarded([&] {
        yh::require(h, "null handle");
        HIPCHECK(hipSetDevice(h->net.device));
        h->net.reserve(batch, height, width);
    });
}

int yh_forward(yh_handle* h, const void* x, int batch, int height, int width, void* y, void* stream) {
    return guarded([&] {
        yh::require(h && x && y, "null argument");
        yh::require(batch > 0, "batch must be positive");
        HIPCHECK(hipSetDevice(h->net.device));
        h->net.forward(x, batch, height, width, y, (hipStream_t)stream);
    });
}

int yh_forward_u8(yh_handle* h, const void* x, int batch, int height, int width, void* y, void* stream) {
    return guarded([&] {
        yh::require(h && x && y, "null argument");
        yh::require(batch > 0, "batch must be positive");
        HIPCHECK(hipSetDevice(h->net.device));
        h->net.forward(x, batch, height, width, y, (hipStream_t)stream, 1);
    });
}

// workspace: candidate keys [B][A*nc] u64 | counts [B] | histograms [B][2048] | the split greedy's
// first-batch scratch (yh::NmsArgs::state / gkeys / ents / mask), 256-byte aligned sections
namespace {
constexpr size_t NMS_STATE_B = 64, NMS_GK_B = 4096 * 8, NMS_ENTS_B = 3 * 4096 * 16, NMS_MASK_B = 64 * 64 * 65 / 2 * 8;
size_t nms_al(size_t v) { return (v + 255) & ~(size_t)255; }
// [counts B x i32][hist B x 2048 u32][state][gkeys][ents][mask] (no per-candidate key list: the
// keys are made from the scores where they are needed, nms.hip for_pairs)
size_t nms_off_hist(int B, int nc, int A) { (void)nc; (void)A; return nms_al((size_t)B * 4); }
size_t nms_off_state(int B, int nc, int A) { return nms_al(nms_off_hist(B, nc, A) + (size_t)B * 2048 * 4); }
size_t nms_off_gk(int B, int nc, int A) { return nms_al(nms_off_state(B, nc, A) + (size_t)B * NMS_STATE_B); }
size_t nms_off_ents(int B, int nc, int A) { return nms_al(nms_off_gk(B, nc, A) + (size_t)B * NMS_GK_B); }
size_t nms_off_mask(int B, int nc, int A) { return nms_al(nms_off_ents(B, nc, A) + (size_t)B * NMS_ENTS_B); }
}  // namespace

size_t yh_nms_workspace_bytes(int batch, int num_classes, int anchors) {
    if (batch <= 0 || num_classes <= 0 || anchors <= 0) return 0;
    return nms_off_mask(batch, num_classes, anchors) + (size_t)batch * NMS_MASK_B;
}

#ifdef YH_ABLATION
// Diagnostic builds only (make EXTRA=-DYH_ABLATION; not in the ABI header):
// yh_debug_nms_trace(buf) makes later yh_nms calls record per-image phase timestamps
// into the device buffer buf ([batch][16] u64, s_memrealtime ticks at 100 MHz).
static unsigned long long* nms_trace = nullptr;
extern "C" int yh_debug_nms_trace(void* device_buf) {
    nms_trace = (unsigned long long*)device_buf;
    return 0;
}
#endif

int yh_nms(int dtype, const void* y, int batch, int num_classes, int anchors, float conf_threshold,
           double iou_threshold, int max_det, int max_nms, float max_wh, void* workspace, size_t workspace_bytes,
           float* dets, int* counts, void* stream) {
    return guarded([&] {
        yh::require(y && dets && counts && workspace, "null argument");
        yh::require(dtype == YH_F32 || dtype == YH_F16 || dtype == YH_BF16, "bad dtype");
        yh::require(batch > 0 && anchors > 0 && num_classes > 0, "bad shape");
        yh::require(max_det > 0 && max_det <= 1024, "max_det must be in [1, 1024]");
        yh::require(max_nms > 0, "max_nms must be positive");
        yh::require(conf_threshold >= 0.0f, "conf_threshold must be >= 0");
        yh::require((long long)anchors * num_classes < (1ll << 26), "anchors * classes exceeds 2^26");
        yh::require(workspace_bytes >= yh_nms_workspace_bytes(batch, num_classes, anchors), "NMS workspace too small");
        yh::NmsArgs a{};
        a.y = y; a.B = batch; a.A = anchors; a.nc = num_classes;
        // compare in the input dtype: torch rounds the Python-float threshold to
        // the tensor dtype before comparing (util.py:130,147)
        float conf = conf_threshold;
        if (dtype == YH_F16) {
            const uint16_t hb = yh::f2h(conf);
            const uint32_t ex = (hb >> 10) & 0x1f, mt = hb & 0x3ff;
            conf = ex == 0 ? std::ldexp((float)mt, -24)
                 : ex == 31 ? INFINITY : std::ldexp((float)(mt | 0x400), (int)ex - 25);
        } else if (dtype == YH_BF16) {
            const uint32_t u = (uint32_t)yh::f2bf(conf) << 16;
            std::memcpy(&conf, &u, 4);
        }
        a.conf = conf;
        // largest float <= iou_threshold: for any float ovr, ovr > thr (double) <=> ovr > a.iou
        float t = (float)iou_threshold;
        if ((double)t > iou_threshold) t = std::nextafter(t, -INFINITY);
        a.iou = t;
        a.max_wh = max_wh;
        a.max_det = max_det;
        a.max_nms = max_nms;
#ifdef YH_ABLATION
        a.trace = nms_trace;
        a.dbg = getenv("YH_NMS_DBG") ? atoi(getenv("YH_NMS_DBG")) : 0;
#endif
        a.counts = (int*)workspace;
        a.hist = (unsigned*)((char*)workspace + nms_off_hist(batch, num_classes, anchors));
        a.state = (unsigned long long*)((char*)workspace + nms_off_state(batch, num_classes, anchors));
        a.gkeys = (unsigned long long*)((char*)workspace + nms_off_gk(batch, num_classes, anchors));
        a.ents = (float*)((char*)workspace + nms_off_ents(batch, num_classes, anchors));
        a.mask = (unsigned long long*)((char*)workspace + nms_off_mask(batch, num_classes, anchors));
        {   // lowest bin at the threshold (or 2047 bins below 1.0 for tiny thresholds)
            uint32_t cb;
            std::memcpy(&cb, &a.conf, 4);
            const int one = 0x3F80;
            a.bin_base = std::max((int)(cb >> 16), one - 2047);
        }
        a.dets = dets;
        a.ndet = counts;
        const int rc = yh::launch_nms(dtype, a, (hipStream_t)stream);
        if (rc != 0) throw Fail(YH_EHIP, std::string("NMS launch failed: ") + hipGetErrorString((hipError_t)rc));
    });
}

int yh_unit_count(const yh_handle* h, int batch, int height, int width) {
    if (!h) return YH_EINVAL;
    auto it = h->net.plans.find(yh::GraphKey{batch, height, width});
    if (it == h->net.plans.end()) return YH_ESTATE;
    return (int)it->second.units.size();
}

int yh_unit_info(const yh_handle* h, int index, int batch, int height, int width, int* first_op, int* num_ops,
                 int* is_level, double* ms_total, int* calls) {
    return guarded([&] {
        yh::require(h, "null handle");
        const yh::Net& n = h->net;
        auto it = n.plans.find(yh::GraphKey{batch, height, width});
        yh::require(it != n.plans.end(), "no forward has run at this shape yet", YH_ESTATE);
        const auto& us = it->second.units;
        yh::require(index >= 0 && index < (int)us.size(), "unit index out of range");
        const bool prof_here = n.prof_key.B == batch && n.prof_key.H == height && n.prof_key.W == width;
        if (first_op) *first_op = us[index].first;
        if (num_ops) *num_ops = us[index].last - us[index].first;
        if (is_level) *is_level = us[index].level ? 1 : 0;
        if (ms_total) *ms_total = prof_here && index < (int)n.prof_ms.size() ? n.prof_ms[index] : 0.0;
        if (calls) *calls = prof_here && index < (int)n.prof_calls.size() ? n.prof_calls[index] : 0;
    });
}

int yh_set_graph(yh_handle* h, int enable) {
    return guarded([&] {
        yh::require(h, "null handle");
        h->net.use_graph = enable != 0;
    });
}

int yh_profile_enable(yh_handle* h, int enable) {
    return guarded([&] {
        yh::require(h, "null handle");
        h->net.profile = enable != 0;
    });
}

int yh_profile_reset(yh_handle* h) {
    return guarded([&] {
        yh::require(h, "null handle");
        std::fill(h->net.prof_ms.begin(), h->net.prof_ms.end(), 0.0);
        std::fill(h->net.prof_calls.begin(), h->net.prof_calls.end(), 0);
    });
}

int yh_force_conv_kernel(yh_handle* h, int kernel) {
    return guarded([&] {
        yh::require(h, "null handle");
        yh::require(kernel >= -1, "conv plan index out of range");
        h->net.force_kern = kernel;
        h->net.conv_kern.clear();
        h->net.cur_kern = nullptr;
        h->net.drop_graphs();
    });
}

int yh_debug_op_desc(const yh_handle* h, int index, int batch, int height, int width, char* buf, size_t size) {
    int len = 0;
    const int rc = guarded([&] {
        yh::require(h && index >= 0 && index < (int)h->net.ops.size(), "op index out of range");
        const std::string s = h->net.op_desc(index, batch, height, width);
        yh::require(buf && size > s.size(), "buffer too small");
        std::memcpy(buf, s.c_str(), s.size() + 1);
        len = (int)s.size();
    });
    return rc == YH_OK ? len : rc;
}

int yh_debug_run_ops(yh_handle* h, const void* x, int x_u8, int batch, int height, int width, void* y, int first,
                     int last, void* stream) {
    return guarded([&] {
        yh::require(h && x && y, "null argument");
        h->net.debug_run(x, x_u8, batch, height, width, y, first, last, (hipStream_t)stream);
    });
}

int yh_debug_operand(const yh_handle* h, int index, int slot, void* dst, size_t dst_bytes, void* stream) {
    return guarded([&] {
        yh::require(h && dst, "null argument");
        HIPCHECK(hipSetDevice(h->net.device));
        h->net.debug_operand(index, slot, dst, dst_bytes, (hipStream_t)stream);
    });
}

int yh_op_count(const yh_handle* h) { return h ? (int)h->net.ops.size() : YH_EINVAL; }

int yh_op_kernel(const yh_handle* h, int index, int batch, int height, int width, const char** name) {
    return guarded([&] {
        yh::require(h && index >= 0 && index < (int)h->net.ops.size(), "op index out of range");
        const yh::Net& n = h->net;
        const yh::Op& op = n.ops[index];
        if (op.kind != yh::OP_CONV) {
            if (name) *name = yh::op_kind_name(op.kind);
            return;
        }
        if (n.dtype == yh::F32) {
            if (name) *name = "gemm_f32";
            return;
        }
        auto it = n.conv_kern.find(yh::GraphKey{batch, height, width});
        yh::require(it != n.conv_kern.end(), "no forward has run at this shape yet", YH_ESTATE);
        if (name) *name = it->second[index].name.c_str();
    });
}

int yh_op_info(const yh_handle* h, int index, int batch, int height, int width, const char** label, int* op_class,
               double* bytes, double* flops, double* ms_total, int* calls) {
    return guarded([&] {
        yh::require(h && index >= 0 && index < (int)h->net.ops.size(), "op index out of range");
        const yh::Net& n = h->net;
        const yh::Op& op = n.ops[index];
        if (label) *label = op.label.c_str();
        if (op_class) *op_class = (int)n.op_class(op);
        double b = 0, f = 0;
        n.op_cost(op, batch, height, width, b, f);
        if (bytes) *bytes = b;
        if (flops) *flops = f;
        // profiled time of the op's own launch unit; 0 calls for ops fused into a level program
        double ms = 0.0;
        int nc = 0;
        auto it = n.plans.find(yh::GraphKey{batch, height, width});
        const bool prof_here = n.prof_key.B == batch && n.prof_key.H == height && n.prof_key.W == width;
        if (it != n.plans.end() && prof_here) {
            const auto& us = it->second.units;
            for (size_t u = 0; u < us.size() && u < n.prof_ms.size(); ++u)
                if (!us[u].level && us[u].first == index) { ms = n.prof_ms[u]; nc = n.prof_calls[u]; }
        }
        if (ms_total) *ms_total = ms;
        if (calls) *calls = nc;
    });
}

}  // extern "C"
