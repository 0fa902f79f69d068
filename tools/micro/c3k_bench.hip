// Fused C3k block (csrc/c3k.hip) in isolation: average duration per launch (HIP events) and
// the per-workgroup phase times from the kernel's stamps (YH_ABLATION build; stamps are
// s_memrealtime, 100 MHz). Random weights / inputs (timing only, no numerics).
//   ./c3k_bench [B H W hh] ...   (default: v11_n's 640 x 640 batch-32 blocks)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "common.h"

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

static unsigned short bf(float v) {
    unsigned u;
    memcpy(&u, &v, 4);
    return (unsigned short)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
}

static void run(int B, int H, int W, int hh) {
    const int c = 2 * hh;
    int off[9];
    yh::c3k_offsets(hh, off);
    std::vector<unsigned char> prm((size_t)off[8]);
    srand(1);
    auto* w16 = reinterpret_cast<unsigned short*>(prm.data());
    for (int i = 0; i < off[4] / 2; ++i) w16[i] = bf(((rand() & 1023) - 512) / 8192.f);
    auto* bias = reinterpret_cast<float*>(prm.data() + off[4]);
    for (int i = 0; i < (off[8] - off[4]) / 4; ++i) bias[i] = 0.01f * ((i % 7) - 3);
    std::vector<unsigned short> x((size_t)B * H * W * c);
    for (auto& v : x) v = bf(((rand() & 1023) - 512) / 512.f);
    void *dp, *dx, *dy;
    unsigned long long* dt;
    CK(hipMalloc(&dp, prm.size()));
    CK(hipMalloc(&dx, x.size() * 2));
    CK(hipMalloc(&dy, x.size() * 2));
    CK(hipMemcpy(dp, prm.data(), prm.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dx, x.data(), x.size() * 2, hipMemcpyHostToDevice));
    yh::C3kArgs a{};
    a.x = dx; a.ldx = c; a.y = dy; a.ldy = c; a.B = B; a.H = H; a.W = W; a.prm = dp; a.hh = hh;
    const int bands = yh::c3k_bands(B, H, W, hh);
    const int nwg = B * bands;
    CK(hipMalloc(&dt, (size_t)nwg * 24 * 8));
    CK(hipMemset(dt, 0, (size_t)nwg * 24 * 8));
    for (int r = 0; r < 3; ++r) CK((hipError_t)yh::launch_c3k(yh::BF16, a, 0));
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 50;
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) CK((hipError_t)yh::launch_c3k(yh::BF16, a, 0));
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    a.trace = dt;
    CK((hipError_t)yh::launch_c3k(yh::BF16, a, 0));
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> tr((size_t)nwg * 24);
    CK(hipMemcpy(tr.data(), dt, tr.size() * 8, hipMemcpyDeviceToHost));
    const int nitems = hh == 64 ? 18 : 5;
    printf("B=%d %dx%d hh=%d: %d bands (rows %d, region %d px), %d workgroups: %.2f us per launch\n", B, H, W, hh, bands,
           (H + bands - 1) / bands, yh::c3k_region_px(H, W, bands), nwg, ms * 1000.f / reps);
    unsigned long long t0 = ~0ull, tmax = 0;
    for (int g = 0; g < nwg; ++g)
        if (tr[g * 24]) t0 = std::min(t0, tr[g * 24]), tmax = std::max(tmax, tr[g * 24 + 3 + nitems]);
    auto med = [&](int k0, int k1) {
        std::vector<double> v;
        for (int g = 0; g < nwg; ++g)
            if (tr[g * 24 + k1] && tr[g * 24 + k0]) v.push_back((double)(tr[g * 24 + k1] - tr[g * 24 + k0]) * 0.01);
        if (v.empty()) return 0.0;
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
    };
    std::vector<double> st;
    for (int g = 0; g < nwg; ++g)
        if (tr[g * 24]) st.push_back((double)(tr[g * 24] - t0) * 0.01);
    std::sort(st.begin(), st.end());
    printf("  span %.2f us | start skew med %.2f max %.2f | per workgroup (median): total %.2f prologue %.2f phaseA %.2f\n",
           (tmax - t0) * 0.01, st[st.size() / 2], st.back(), med(0, 3 + nitems), med(0, 1), med(1, 2));
    printf("  items:");
    printf(" %.2f", med(2, 3));
    for (int i = 0; i < nitems; ++i) printf(" %.2f", med(3 + i, 4 + i));
    printf("\n");
    CK(hipFree(dp)); CK(hipFree(dx)); CK(hipFree(dy)); CK(hipFree(dt));
}

int main(int argc, char** argv) {
    if (argc >= 5) {
        for (int i = 1; i + 3 < argc; i += 4) run(atoi(argv[i]), atoi(argv[i + 1]), atoi(argv[i + 2]), atoi(argv[i + 3]));
    } else {
        run(32, 20, 20, 64);
        run(32, 40, 40, 32);
        run(32, 40, 40, 64);
    }
    return 0;
}
