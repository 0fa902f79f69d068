// Latency of one scalar kernel-argument load vs one scalar load of device memory
// (s_memrealtime stamps, 100 MHz), measured in the first and a repeated access.
#include <hip/hip_runtime.h>
#include <cstdio>
struct Big { int v[64]; unsigned long long* out; const int* dev; };
__global__ void probe(const Big p) {
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int a = p.v[5];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    int b = p.v[40];
    asm volatile("" :: "s"(a));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
    int c = __builtin_amdgcn_readfirstlane(p.dev[blockIdx.x & 7]);
    asm volatile("s_waitcnt lgkmcnt(0) vmcnt(0)" ::: "memory");
    unsigned long long t3 = __builtin_amdgcn_s_memrealtime();
    int d = __builtin_amdgcn_readfirstlane(p.dev[(blockIdx.x & 7) + 8]);
    asm volatile("s_waitcnt lgkmcnt(0) vmcnt(0)" ::: "memory");
    unsigned long long t4 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        p.out[blockIdx.x * 5 + 0] = t1 - t0;
        p.out[blockIdx.x * 5 + 1] = t2 - t1;
        p.out[blockIdx.x * 5 + 2] = t3 - t2;
        p.out[blockIdx.x * 5 + 3] = t4 - t3;
        p.out[blockIdx.x * 5 + 4] = a + b + c + d;
    }
}
int main() {
    Big b{};
    for (int i = 0; i < 64; ++i) b.v[i] = i;
    int* dev;
    hipMalloc(&dev, 64 * 4);
    hipMemset(dev, 0, 256);
    hipMalloc(&b.out, 512 * 5 * 8);
    b.dev = dev;
    for (int rep = 0; rep < 3; ++rep) {
        probe<<<512, 64>>>(b);
        hipDeviceSynchronize();
        unsigned long long h[512 * 5];
        hipMemcpy(h, b.out, sizeof(h), hipMemcpyDeviceToHost);
        double s[4] = {0, 0, 0, 0}, mx[4] = {0, 0, 0, 0};
        for (int g = 0; g < 512; ++g)
            for (int k = 0; k < 4; ++k) { s[k] += h[g * 5 + k]; if (h[g * 5 + k] > mx[k]) mx[k] = h[g * 5 + k]; }
        printf("rep %d (us, mean/max over 512 WGs): karg1 %.3f/%.3f karg2 %.3f/%.3f dev1 %.3f/%.3f dev2 %.3f/%.3f\n", rep,
               s[0] / 512 * 0.01, mx[0] * 0.01, s[1] / 512 * 0.01, mx[1] * 0.01, s[2] / 512 * 0.01, mx[2] * 0.01,
               s[3] / 512 * 0.01, mx[3] * 0.01);
    }
    return 0;
}
