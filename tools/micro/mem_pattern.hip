// Memory-pattern calibration for the 160x160 bottleneck conv (net.p2.1.res_m.0.conv1:
// 16 of 32 channels in, 8 channels out, B=32): how fast can the data alone move?
//   a) stream: every input chunk read once, one 16-B output per pixel
//   b) taps:   the 3x3 neighbourhood of every pixel read (9 loads / pixel / chunk)
//   hipcc --offload-arch=gfx950 -O3 tools/micro/mem_pattern.hip -o tools/micro/mem_pattern
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int B = 32, H = 160, W = 160, LDI = 32, CIN = 16, LDO = 8;

__global__ __launch_bounds__(256) void k_stream(const uint4* in, uint4* out) {
    const long long px = (long long)blockIdx.x * 256 + threadIdx.x;
    if (px >= (long long)B * H * W) return;
    const uint4* p = in + px * (LDI / 8);
    uint4 a = p[0], b = p[1];
    out[px] = make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
}

__global__ __launch_bounds__(256) void k_taps(const uint4* in, uint4* out) {
    const long long px = (long long)blockIdx.x * 256 + threadIdx.x;
    if (px >= (long long)B * H * W) return;
    const int n = (int)(px / (H * W)), r = (int)(px % (H * W)), h = r / W, w = r % W;
    uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int kh = -1; kh <= 1; ++kh)
#pragma unroll
        for (int kw = -1; kw <= 1; ++kw) {
            const int hh = min(max(h + kh, 0), H - 1), ww = min(max(w + kw, 0), W - 1);
            const uint4* p = in + (((long long)n * H + hh) * W + ww) * (LDI / 8);
            uint4 a = p[0], b = p[1];
            acc.x ^= a.x ^ b.x; acc.y ^= a.y ^ b.y; acc.z ^= a.z ^ b.z; acc.w ^= a.w ^ b.w;
        }
    out[px] = acc;
}

int main() {
    const long long npx = (long long)B * H * W;
    uint4 *in, *out;
    hipMalloc(&in, npx * LDI * 2);
    hipMalloc(&out, npx * LDO * 2);
    hipMemset(in, 1, npx * LDI * 2);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const dim3 g((unsigned)((npx + 255) / 256));
    const double bytes = npx * (CIN * 2.0 + LDO * 2.0);
    for (int rep = 0; rep < 2; ++rep) {
        float ms;
        hipLaunchKernelGGL(k_stream, g, dim3(256), 0, 0, in, out);
        hipEventRecord(e0, 0);
        for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k_stream, g, dim3(256), 0, 0, in, out);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("stream: %.2f us  %.0f GB/s (algorithmic %.1f MB)\n", ms * 100, bytes / (ms * 1e-4) / 1e9, bytes / 1e6);
        hipLaunchKernelGGL(k_taps, g, dim3(256), 0, 0, in, out);
        hipEventRecord(e0, 0);
        for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k_taps, g, dim3(256), 0, 0, in, out);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("taps:   %.2f us  %.0f GB/s algorithmic\n", ms * 100, bytes / (ms * 1e-4) / 1e9);
    }
    return 0;
}
