// Bare MFMA throughput on this box: v_mfma_f32_16x16x32_bf16 with register operands,
// 8 independent accumulators per wave, W waves per SIMD. Prints TFLOP/s per config.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/mfma_peak.hip -o tools/micro/mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

__global__ __launch_bounds__(256) void mfma32_loop(float* out, int iters) {
    bf16x8 a, b;
    for (int i = 0; i < 8; ++i) {
        a[i] = (__bf16)(0.001f * (threadIdx.x + i));
        b[i] = (__bf16)(0.002f * (threadIdx.x - i));
    }
    f32x16 acc[4];
    for (int i = 0; i < 4; ++i)
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[i], 0, 0, 0);
    }
    float s = 0.f;
    for (int i = 0; i < 4; ++i)
        for (int r = 0; r < 16; ++r) s += acc[i][r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void mfma_loop(float* out, int iters) {
    bf16x8 a, b;
    for (int i = 0; i < 8; ++i) {
        a[i] = (__bf16)(0.001f * (threadIdx.x + i));
        b[i] = (__bf16)(0.002f * (threadIdx.x - i));
    }
    f32x4 acc[8];
    for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[i], 0, 0, 0);
    }
    float s = 0.f;
    for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    int dev = 0, ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    float* out;
    const int maxblocks = ncu * 8;
    hipMalloc(&out, (size_t)maxblocks * 256 * sizeof(float));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 4096;
    for (int bpc : {1, 2, 4}) {   // 256-thread blocks per CU -> 1, 2, 4 waves per SIMD
        const int blocks = ncu * bpc;
        hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, 0, out, 64);
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, 0, out, iters);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0.f;
        hipEventElapsedTime(&ms, e0, e1);
        const double flops = (double)blocks * 4 * iters * 8 * 16.0 * 16.0 * 32.0 * 2.0;
        printf("16x16x32 bf16: CUs %d, %d waves/SIMD: %.1f TFLOP/s (%.3f ms)\n", ncu, bpc, flops / (ms * 1e-3) / 1e12, ms);
        hipLaunchKernelGGL(mfma32_loop, dim3(blocks), dim3(256), 0, 0, out, 64);
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(mfma32_loop, dim3(blocks), dim3(256), 0, 0, out, iters);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        const double f32 = (double)blocks * 4 * iters * 4 * 32.0 * 32.0 * 16.0 * 2.0;
        printf("32x32x16 bf16: CUs %d, %d waves/SIMD: %.1f TFLOP/s (%.3f ms)\n", ncu, bpc, f32 / (ms * 1e-3) / 1e12, ms);
    }
    hipFree(out);
    return 0;
}
