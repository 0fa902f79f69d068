// Micro benchmark + correctness check of the conv_mx plans on the v11_n / v11_s
// layer shapes. Every candidate plan of a layer is checked against a naive fp32
// reference kernel (same bf16 inputs / weights) and against the first plan bit for
// bit (the family shares one reduction order), then timed with HIP events.
//   build: make -C tools/micro mx_bench      run: tools/micro/mx_bench [filter]
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <algorithm>

#include "conv_mx.h"

using namespace yh;

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

__global__ void fill_rand(__bf16* p, long long n, unsigned seed, float scale) {
    long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    for (; i < n; i += (long long)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u ^ seed;
        x ^= x >> 15; x *= 2246822519u; x ^= x >> 13; x *= 3266489917u; x ^= x >> 16;
        p[i] = (__bf16)(((x & 0xffff) / 32768.0f - 1.0f) * scale);
    }
}

// naive reference: out[m][co] (fp32, after bias + act) from NHWC bf16 input (single
// segment or two segments with nearest upsample), fp32 weights [co][ci][k][k]
struct RefArgs {
    const __bf16* in0; const __bf16* in1; int ldc0, ldc1, c0, cin, up0, up1, hs0, ws0, hs1, ws1;
    int Hi, Wi, Ho, Wo, B, ks, s, cout, act;
    const float* w; const float* bias; const __bf16* res; int ldr; float* out;
};
__global__ void conv_ref(RefArgs a) {
    long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    long long M = (long long)a.B * a.Ho * a.Wo;
    if (idx >= M * a.cout) return;
    int co = (int)(idx % a.cout);
    long long m = idx / a.cout;
    int n = (int)(m / (a.Ho * a.Wo));
    int r = (int)(m % (a.Ho * a.Wo));
    int ho = r / a.Wo, wo = r % a.Wo;
    float acc = 0.f;
    int pad = a.ks / 2;
    for (int kh = 0; kh < a.ks; ++kh)
        for (int kw = 0; kw < a.ks; ++kw) {
            int hi = ho * a.s - pad + kh, wi = wo * a.s - pad + kw;
            if (hi < 0 || hi >= a.Hi || wi < 0 || wi >= a.Wi) continue;
            for (int ci = 0; ci < a.cin; ++ci) {
                float x;
                if (ci < a.c0) {
                    long long pix = ((long long)n * a.hs0 + (hi >> a.up0)) * a.ws0 + (wi >> a.up0);
                    x = (float)a.in0[pix * a.ldc0 + ci];
                } else {
                    long long pix = ((long long)n * a.hs1 + (hi >> a.up1)) * a.ws1 + (wi >> a.up1);
                    x = (float)a.in1[pix * a.ldc1 + ci - a.c0];
                }
                float wv = (float)(__bf16)a.w[((long long)co * a.cin + ci) * a.ks * a.ks + kh * a.ks + kw];
                acc += x * wv;
            }
        }
    float v = acc + a.bias[co];
    if (a.act) v = v / (1.f + expf(-v));
    v = (float)(__bf16)v;
    if (a.res) v += (float)a.res[m * a.ldr + co];
    a.out[m * a.cout + co] = v;
}

struct Layer {
    const char* name;
    int ks, s, cin, cout, Ho, Wo, res;
    int c0, c1, up0;   // 2-segment 1x1 inputs (c1 > 0)
};

int main(int argc, char** argv) {
    const char* filt = argc > 1 ? argv[1] : nullptr;
    const int B = argc > 2 ? atoi(argv[2]) : 32;
    const int iters = 20;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int ncu = prop.multiProcessorCount;
    // v11_n @640 layer shapes; Ho/Wo are output sizes
    std::vector<Layer> layers = {
        {"p2.0 3x3s2 16-32 @160", 3, 2, 16, 32, 160, 160, 0, 16, 0, 0},
        {"p2.1.res.c1 3x3 16-8 @160", 3, 1, 16, 8, 160, 160, 0, 16, 0, 0},
        {"p2.1.res.c2 3x3 8-16 @160 +res", 3, 1, 8, 16, 160, 160, 1, 8, 0, 0},
        {"p3.0 3x3s2 64-64 @80", 3, 2, 64, 64, 80, 80, 0, 64, 0, 0},
        {"p3.1.res.c1 3x3 32-16 @80", 3, 1, 32, 16, 80, 80, 0, 32, 0, 0},
        {"p3.1.res.c2 3x3 16-32 @80 +res", 3, 1, 16, 32, 80, 80, 1, 16, 0, 0},
        {"p4.0 3x3s2 128-128 @40", 3, 2, 128, 128, 40, 40, 0, 128, 0, 0},
        {"p4 c3k 3x3 32-32 @40", 3, 1, 32, 32, 40, 40, 0, 32, 0, 0},
        {"h1.res.c1 3x3 64-32 @40", 3, 1, 64, 32, 40, 40, 0, 64, 0, 0},
        {"h1.res.c2 3x3 32-64 @40 +res", 3, 1, 32, 64, 40, 40, 1, 32, 0, 0},
        {"p5 c3k.c2 3x3 64-64 @20 +res", 3, 1, 64, 64, 20, 20, 1, 64, 0, 0},
        {"p5.0 3x3s2 128-256 @20", 3, 2, 128, 256, 20, 20, 0, 128, 0, 0},
        {"p5 c3k 3x3 64-64 @20", 3, 1, 64, 64, 20, 20, 0, 64, 0, 0},
        {"h3 3x3s2 64-64 @40", 3, 2, 64, 64, 40, 40, 0, 64, 0, 0},
        {"h5 3x3s2 128-128 @20", 3, 2, 128, 128, 20, 20, 0, 128, 0, 0},
        {"box0.0 3x3 64-64 @80", 3, 1, 64, 64, 80, 80, 0, 64, 0, 0},
        {"box1.0 3x3 128-64 @40", 3, 1, 128, 64, 40, 40, 0, 128, 0, 0},
        {"box2.0 3x3 256-64 @20", 3, 1, 256, 64, 20, 20, 0, 256, 0, 0},
        {"p2.1.conv1 1x1 32-32 @160", 1, 1, 32, 32, 160, 160, 0, 32, 0, 0},
        {"p2.1.conv2 1x1 48-64 @160", 1, 1, 48, 64, 160, 160, 0, 48, 0, 0},
        {"p3.1.conv2 1x1 96-128 @80", 1, 1, 96, 128, 80, 80, 0, 96, 0, 0},
        {"h2.conv1 1x1 up128+128-64 @80", 1, 1, 256, 64, 80, 80, 0, 128, 128, 1},
        {"cls0.1 1x1 64-80 @80", 1, 1, 64, 80, 80, 80, 0, 64, 0, 0},
        {"cls0.3 1x1 80-80 @80", 1, 1, 80, 80, 80, 80, 0, 80, 0, 0},
        {"p5.2.conv2 1x1 512-256 @20", 1, 1, 512, 256, 20, 20, 0, 512, 0, 0},
        {"h1.conv1 1x1 up256+128-128 @40", 1, 1, 384, 128, 40, 40, 0, 256, 128, 1},
        // v11_x @1280 (C5, run with B = 16)
        {"x p2.0 3x3s2 96-192 @320", 3, 2, 96, 192, 320, 320, 0, 96, 0, 0},
        {"x p3.0 3x3s2 192-384 @160", 3, 2, 192, 384, 160, 160, 0, 192, 0, 0},
        {"x p4.0 3x3s2 384-768 @80", 3, 2, 384, 768, 80, 80, 0, 384, 0, 0},
        {"x box0.0 3x3 192-96 @160", 3, 1, 192, 96, 160, 160, 0, 192, 0, 0},
        {"x p2.1.conv2 1x1 480-192 @320", 1, 1, 480, 192, 320, 320, 0, 480, 0, 0},
    };
    __bf16* zero;
    CK(hipMalloc(&zero, 4096));
    CK(hipMemset(zero, 0, 4096));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (const Layer& L : layers) {
        if (filt && !strstr(L.name, filt)) continue;
        MxShape sh{};
        sh.ks = L.ks; sh.s = L.s; sh.cin = L.cin; sh.cout = L.cout;
        sh.Ho = L.Ho; sh.Wo = L.Wo; sh.Hi = L.Ho * L.s; sh.Wi = L.Wo * L.s; sh.B = B;
        sh.c0 = L.c1 ? L.c0 : L.cin; sh.c1 = L.c1; sh.up0 = L.c1 ? L.up0 : 0; sh.up1 = 0;
        sh.ldo = L.cout; sh.ldr = L.res ? L.cout : 0;
        const int hs0 = sh.up0 ? sh.Hi / 2 : sh.Hi, ws0 = sh.up0 ? sh.Wi / 2 : sh.Wi;
        const long long npx0 = (long long)B * hs0 * ws0, npx1 = (long long)B * sh.Hi * sh.Wi;
        const int ldc0 = sh.c0, ldc1 = L.c1 ? L.c1 : 8;
        __bf16 *in0, *in1 = nullptr, *out, *res = nullptr;
        const long long M = (long long)B * sh.Ho * sh.Wo;
        CK(hipMalloc(&in0, npx0 * ldc0 * 2));
        fill_rand<<<1024, 256>>>(in0, npx0 * ldc0, 1u, 1.0f);
        if (L.c1) {
            CK(hipMalloc(&in1, npx1 * ldc1 * 2));
            fill_rand<<<1024, 256>>>(in1, npx1 * ldc1, 2u, 1.0f);
        }
        CK(hipMalloc(&out, M * L.cout * 2));
        if (L.res) {
            CK(hipMalloc(&res, M * L.cout * 2));
            fill_rand<<<1024, 256>>>(res, M * L.cout, 3u, 1.0f);
        }
        // weights fp32 [co][ci][k][k], fan-in scaled
        const int taps = L.ks * L.ks;
        std::vector<float> wf((size_t)L.cout * L.cin * taps), bias(((L.cout + 127) / 128) * 128, 0.f);
        unsigned sd = 12345;
        const float sc = 1.7f / std::sqrt((float)(L.cin * taps));
        for (auto& v : wf) { sd = sd * 1664525u + 1013904223u; v = ((sd >> 8) / 8388608.0f - 1.0f) * sc; }
        for (int i = 0; i < L.cout; ++i) { sd = sd * 1664525u + 1013904223u; bias[i] = ((sd >> 8) / 8388608.0f - 1.0f) * 0.2f; }
        float *wd, *bd, *refo;
        CK(hipMalloc(&wd, wf.size() * 4));
        CK(hipMemcpy(wd, wf.data(), wf.size() * 4, hipMemcpyHostToDevice));
        CK(hipMalloc(&bd, bias.size() * 4));
        CK(hipMemcpy(bd, bias.data(), bias.size() * 4, hipMemcpyHostToDevice));
        CK(hipMalloc(&refo, M * L.cout * 4));
        RefArgs ra{in0, in1, ldc0, ldc1, sh.c0, L.cin, sh.up0, 0, hs0, ws0, sh.Hi, sh.Wi, sh.Hi, sh.Wi, sh.Ho, sh.Wo, B,
                   L.ks, L.s, L.cout, 1, wd, bd, res, L.cout, refo};
        const long long nref = M * L.cout;
        conv_ref<<<(unsigned)((nref + 255) / 256), 256>>>(ra);
        CK(hipDeviceSynchronize());
        std::vector<float> ref(nref);
        CK(hipMemcpy(ref.data(), refo, nref * 4, hipMemcpyDeviceToHost));
        std::vector<int> phys2log(L.cin);
        for (int c = 0; c < L.cin; ++c) phys2log[c] = c;
        const double bytes = (double)(npx0 * sh.c0 + (L.c1 ? npx1 * L.c1 : 0)) * 2 + (double)M * L.cout * 2 * (L.res ? 2 : 1) +
                             (double)wf.size() * 2;
        const double flops = 2.0 * M * L.cout * L.cin * taps;
        printf("== %s  B=%d  %.1f MB  %.2f GFLOP\n", L.name, B, bytes / 1e6, flops / 1e9);
        std::vector<uint16_t> first;
        auto cands = mx_candidates(sh, ncu);
        for (const MxPlan& pl : cands) {
            auto pk = mx_pack(pl, sh, wf.data(), L.cin, phys2log, true, L.cout);
            char* wdev;
            CK(hipMalloc(&wdev, pk.size() * 2));
            CK(hipMemcpy(wdev, pk.data(), pk.size() * 2, hipMemcpyHostToDevice));
            MxArgs a{};
            mx_fill_args(pl, sh, a);
            a.in0 = (const char*)in0; a.in1 = L.c1 ? (const char*)in1 : nullptr;
            a.ldc0 = ldc0; a.ldc1 = ldc1;
            a.hs0 = hs0; a.ws0 = ws0; a.hs1 = sh.Hi; a.ws1 = sh.Wi;
            a.w = wdev; a.bias = bd; a.out = (char*)out; a.ldo = L.cout;
            a.res = (const char*)res; a.ldr = L.cout; a.act = 1; a.zero = (const char*)zero;
            CK(hipMemset(out, 0xff, M * L.cout * 2));
            int rc = launch_mx(BF16, pl, a, 0);
            CK(hipDeviceSynchronize());
            if (rc) { printf("  launch failed %d\n", rc); continue; }
            std::vector<uint16_t> got(nref);
            CK(hipMemcpy(got.data(), out, nref * 2, hipMemcpyDeviceToHost));
            double maxd = 0, maxr = 0;
            long long bad = 0;
            for (long long i = 0; i < nref; ++i) {
                uint32_t u = (uint32_t)got[i] << 16;
                float g;
                memcpy(&g, &u, 4);
                const double d = std::fabs((double)g - ref[i]);
                if (!(d <= 0.02 + 0.02 * std::fabs(ref[i]))) ++bad;
                if (d > maxd || d != d) maxd = d;
            }
            bool ident = true;
            if (first.empty()) first = got;
            else ident = first == got;
            for (int r = 0; r < 3; ++r) launch_mx(BF16, pl, a, 0);
            CK(hipEventRecord(e0, 0));
            for (int r = 0; r < iters; ++r) launch_mx(BF16, pl, a, 0);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / iters;
            std::vector<int> modes;
            std::vector<float> dms;
            if (const char* ab = getenv("MX_ABL")) {
                for (const char* q = ab; *q;) {
                    modes.push_back(atoi(q));
                    while (*q && *q != ',') ++q;
                    if (*q == ',') ++q;
                }
                for (int md : modes) {
                    MxArgs b = a;
                    b.dbg = md;
                    for (int r = 0; r < 2; ++r) launch_mx(BF16, pl, b, 0);
                    CK(hipEventRecord(e0, 0));
                    for (int r = 0; r < iters; ++r) launch_mx(BF16, pl, b, 0);
                    CK(hipEventRecord(e1, 0));
                    CK(hipEventSynchronize(e1));
                    float t = 0;
                    CK(hipEventElapsedTime(&t, e0, e1));
                    dms.push_back(t * 1e3f / iters);
                }
            }
            printf("  %s na%d mb%d wn%d wm%d ncb%d  task %dx%d bc%d nbi%d ains%d lds%6d grid%5d conf%4d | %8.2f us %7.0f GB/s %6.0f TF | maxd %.3g bad %lld %s\n",
                   pl.cfg.kind == 2 ? (pl.cfg.pc ? (pl.cfg.nbuf == 3 ? "C3" : pl.cfg.nbuf == 4 ? "C4" : "C5") : pl.cfg.nbuf == 2 ? "W2" : pl.cfg.nbuf == 3 ? "W3" : pl.cfg.nbuf == 4 ? "W4" : "W5") : pl.cfg.kind ? "R" : "S", pl.cfg.na, pl.cfg.mb, pl.cfg.wn, pl.cfg.wm, pl.cfg.ncb, pl.TH, pl.TW, 1 << pl.bc_log2, pl.nbi, pl.ains,
                   pl.lds, pl.grid, pl.conflicts, us, bytes / us * 1e-3, flops / us * 1e-6, maxd, bad,
                   ident ? "ident" : "DIFF");
            if (getenv("MX_TRACE")) {
                unsigned long long* tr;
                CK(hipMalloc(&tr, (size_t)pl.grid * 4 * 8));
                CK(hipMemset(tr, 0, (size_t)pl.grid * 4 * 8));
                MxArgs b = a;
                b.trace = tr;
                b.dbg = atoi(getenv("MX_TRACE"));
                launch_mx(BF16, pl, b, 0);
                launch_mx(BF16, pl, b, 0);
                CK(hipDeviceSynchronize());
                std::vector<unsigned long long> h((size_t)pl.grid * 4);
                CK(hipMemcpy(h.data(), tr, h.size() * 8, hipMemcpyDeviceToHost));
                unsigned long long t0 = ~0ull, tend = 0;
                std::vector<double> setup, first, loop, start;
                for (int g = 0; g < pl.grid; ++g) {
                    if (!h[g * 4 + 3]) continue;
                    t0 = std::min(t0, h[g * 4]);
                    tend = std::max(tend, h[g * 4 + 3]);
                }
                for (int g = 0; g < pl.grid; ++g) {
                    if (!h[g * 4 + 3]) continue;
                    start.push_back((h[g * 4] - t0) * 0.01);
                    setup.push_back((h[g * 4 + 1] - h[g * 4]) * 0.01);
                    first.push_back((h[g * 4 + 2] - h[g * 4 + 1]) * 0.01);
                    loop.push_back((h[g * 4 + 3] - h[g * 4 + 2]) * 0.01);
                }
                auto st = [](std::vector<double> v, const char* nm) {
                    std::sort(v.begin(), v.end());
                    if (v.empty()) return;
                    printf("  %s min %.2f med %.2f max %.2f", nm, v[0], v[v.size() / 2], v.back());
                };
                printf("      trace(us): span %.2f |", (tend - t0) * 0.01);
                st(start, "start"); st(setup, "setup"); st(first, "first"); st(loop, "loop");
                printf("\n");
                CK(hipFree(tr));
            }
            if (!modes.empty()) {
                printf("      ablation:");
                for (size_t k = 0; k < modes.size(); ++k) printf("  dbg%d %.2f", modes[k], dms[k]);
                printf(" us\n");
            }
            (void)maxr;
            CK(hipFree(wdev));
        }
        CK(hipFree(in0)); if (in1) CK(hipFree(in1)); CK(hipFree(out)); if (res) CK(hipFree(res));
        CK(hipFree(wd)); CK(hipFree(bd)); CK(hipFree(refo));
    }
    return 0;
}
