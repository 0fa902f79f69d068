// Per-CU load throughput of the two ways a conv stages its input patch:
//   mode 0: global_load_lds_dwordx4 (LDS-DMA, what conv_mx / conv_mxr use)
//   mode 2: global_load_dwordx4 into VGPRs only (folded into a checksum)
// Every wave streams 1 KB pieces (64 lanes x 16 B) over a buffer of `bytes` (small: L2 /
// MALL resident; large: HBM), keeping `depth` pieces in flight. Prints GB/s chip-wide and
// bytes per cycle per CU at the measured shader clock.
//   build: hipcc --offload-arch=gfx950 -O3 dma_rate.hip -o dma_rate     run: ./dma_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

__device__ __forceinline__ void glds(const void* src, unsigned lds_addr) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds_addr) : "memory");
}

template <int MODE, int DEPTH>
__global__ __launch_bounds__(512) void stream(const uint4* buf, long long pieces, int iters, unsigned* sink) {
    extern __shared__ __attribute__((aligned(1024))) uint4 sm[];
    typedef __attribute__((address_space(3))) uint4* lp;
    const unsigned lds0 = (unsigned)(size_t)(lp)sm;
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long long gw = (long long)blockIdx.x * (blockDim.x >> 6) + wv, nw = (long long)gridDim.x * (blockDim.x >> 6);
    unsigned acc = 0;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            const long long pc = (gw + (long long)(it * DEPTH + d) * nw) & (pieces - 1);   // pieces: power of 2
            const uint4* src = buf + pc * 64 + lane;
            const unsigned dst = lds0 + (unsigned)((wv * DEPTH + d) * 1024);
            if constexpr (MODE == 0) {
                glds(src, dst);
            } else {
                const uint4 v = *src;
                acc ^= v.x ^ v.y ^ v.z ^ v.w;
            }
        }
        if constexpr (MODE == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

template <int MODE, int DEPTH>
double run(const uint4* buf, long long bytes, int grid, int block, int iters, unsigned* sink) {
    const long long pieces = bytes / 1024;
    const int lds = (block / 64) * DEPTH * 1024;
    auto k = &stream<MODE, DEPTH>;
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    hipLaunchKernelGGL(k, dim3(grid), dim3(block), lds, 0, buf, pieces, iters, sink);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(block), lds, 0, buf, pieces, iters, sink);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double moved = 5.0 * grid * (block / 64) * (double)iters * DEPTH * 1024;
    return moved / (ms * 1e-3) / 1e9;   // GB/s
}

int main() {
    int ncu = 0, clk = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    CK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0));
    const long long big = 1ll << 30;
    uint4* buf;
    unsigned* sink;
    CK(hipMalloc(&buf, big));
    CK(hipMemset(buf, 1, big));
    CK(hipMalloc(&sink, 64));
    printf("CUs %d, max shader clock %.2f GHz\n", ncu, clk / 1e6);
    const long long sizes[2] = {2ll << 20, big};
    const char* names[3] = {"LDS-DMA", "", "load only"};
    for (long long sz : sizes) {
        for (int waves : {4, 8}) {
            const int grid = ncu, block = 64 * waves, iters = sz > (64ll << 20) ? 64 : 256;
            double g[3][2];
            g[0][0] = run<0, 4>(buf, sz, grid, block, iters, sink);
            g[0][1] = run<0, 8>(buf, sz, grid, block, iters / 2, sink);
            g[2][0] = run<2, 4>(buf, sz, grid, block, iters, sink);
            g[2][1] = run<2, 8>(buf, sz, grid, block, iters / 2, sink);
            for (int m = 0; m < 3; m += 2)
                printf("buffer %5lld MB  %d waves/CU  %-14s depth 4: %7.0f GB/s (%5.1f B/clk/CU @2.1GHz)  depth 8: %7.0f GB/s (%5.1f)\n",
                       sz >> 20, waves, names[m], g[m][0], g[m][0] * 1e9 / (ncu * 2.1e9), g[m][1],
                       g[m][1] * 1e9 / (ncu * 2.1e9));
        }
    }
    return 0;
}
