// Write-pattern calibration for the K = 32 1x1 convs (net.p2.1.conv1: 32 channels in,
// 32 channels out into the C3k2 concat buffer, whose pixel stride is 48 channels).
// Each thread copies one 16-B chunk: 64 B read per pixel (contiguous), 64 B written
// per pixel at an output pixel stride of LDO channels. Algorithmic bytes are the same
// for every LDO; LDO = 32 is fully contiguous, 48 leaves every 96-B pixel with a
// 32-B hole (the partial-line case), 64 a 64-B hole.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/write_pattern.hip -o tools/micro/write_pattern
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int B = 32, H = 160, W = 160, CIN = 32, COUT = 32;

__global__ __launch_bounds__(256) void k_copy(const uint4* in, uint4* out, int ldo8) {
    const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long npx = (long long)B * H * W;
    if (t >= npx * (COUT / 8)) return;
    const long long px = t / (COUT / 8);
    const int c = (int)(t % (COUT / 8));
    uint4 v = in[px * (CIN / 8) + c];
    v.x ^= 0x5a5a5a5au;
    out[px * ldo8 + c] = v;
}

// 4 chunks per thread, all loads issued before the stores (more bytes in flight per wave)
__global__ __launch_bounds__(256) void k_copy4(const uint4* in, uint4* out, int ldo8) {
    const long long npx = (long long)B * H * W;
    const long long n = npx * (COUT / 8);
    const long long t0 = ((long long)blockIdx.x * 256) * 4 + threadIdx.x;
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const long long t = t0 + u * 256;
        v[u] = t < n ? in[(t / (COUT / 8)) * (CIN / 8) + t % (COUT / 8)] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const long long t = t0 + u * 256;
        v[u].x ^= 0x5a5a5a5au;
        if (t < n) out[(t / (COUT / 8)) * ldo8 + t % (COUT / 8)] = v[u];
    }
}

int main() {
    const long long npx = (long long)B * H * W;
    uint4 *in, *out;
    if (hipMalloc(&in, npx * CIN * 2) != hipSuccess || hipMalloc(&out, npx * 64 * 2) != hipSuccess) return 1;
    (void)hipMemset(in, 1, npx * CIN * 2);
    (void)hipMemset(out, 0, npx * 64 * 2);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const long long nthr = npx * (COUT / 8);
    const dim3 grid((unsigned)((nthr + 255) / 256));
    const double bytes = (double)npx * (CIN + COUT) * 2;
    const int ldos[] = {32, 48, 64};
    for (int ldo : ldos) {
        for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k_copy, grid, dim3(256), 0, 0, in, out, ldo / 8);
        const int reps = 20;
        (void)hipEventRecord(e0, 0);
        for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_copy, grid, dim3(256), 0, 0, in, out, ldo / 8);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double us = ms * 1e3 / reps;
        printf("ldo %2d ch: %7.2f us  %6.0f GB/s (64 B read + 64 B written per pixel, %.1f MB)\n", ldo, us,
               bytes / us / 1e3, bytes / 1e6);
        const dim3 grid4((unsigned)((nthr + 1023) / 1024));
        for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k_copy4, grid4, dim3(256), 0, 0, in, out, ldo / 8);
        (void)hipEventRecord(e0, 0);
        for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_copy4, grid4, dim3(256), 0, 0, in, out, ldo / 8);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double us4 = ms * 1e3 / reps;
        printf("ldo %2d ch, 4 chunks/thread: %7.2f us  %6.0f GB/s\n", ldo, us4, bytes / us4 / 1e3);
    }
    (void)hipFree(in);
    (void)hipFree(out);
    return 0;
}
