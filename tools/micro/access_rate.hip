// Chip-wide rate of the two per-lane access shapes the dense convs use on NHWC tiles of
// 64 channels (128 B per pixel), against fully coalesced ones (every wave-instruction
// covering whole 128-B lines):
//   store "lane-pixel" : mx_epi's shape - lane (l32, h) owns pixel l32 of a 32-pixel tile
//                        and 32 of its couts; one instruction writes 16 B at
//                        pix*128 + h*64 + c*16 (32 lines touched, 32 B each)
//   store "coalesced"  : instruction c writes bytes [c*1024, c*1024+1024) of the tile
//   LDS-DMA "2 lanes/px": a 16-channel stage of a patch: lane -> pixel lane/2, chunk lane&1
//                        (32 B of each of 32 lines per instruction)
//   LDS-DMA "8 lanes/px": lane -> pixel lane/8, chunk lane&7 (8 whole lines per instruction)
// Buffers: 26.2 MB (v11_n b32 80x80x64 bf16: MALL-resident when repeated) and 1 GB (HBM).
//   hipcc --offload-arch=gfx950 -O3 access_rate.hip -o access_rate
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

// one tile = 32 pixels x 128 B = 4 KB; MODE 0/1 stores (lane-pixel / coalesced), 2/3 LDS-DMA
// loads (2 lanes per pixel x 4 stages / 8 lanes per pixel x 4 instructions)
template <int MODE>
__global__ __launch_bounds__(512) void tiles(char* buf, long long ntiles, int depth) {
    extern __shared__ __attribute__((aligned(1024))) uint4 sm[];
    typedef __attribute__((address_space(3))) uint4* lp;
    const unsigned lds0 = (unsigned)(size_t)(lp)sm;
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long long gw = (long long)blockIdx.x * (blockDim.x >> 6) + wv, nw = (long long)gridDim.x * (blockDim.x >> 6);
    const int l32 = lane & 31, h = lane >> 5;
    const uint4 v = make_uint4(lane, 1, 2, 3);
    int inflight = 0;
    for (long long t = gw; t < ntiles; t += nw) {
        char* base = buf + t * 4096;
        if constexpr (MODE == 0) {
#pragma unroll
            for (int c = 0; c < 4; ++c) *reinterpret_cast<uint4*>(base + l32 * 128 + h * 64 + c * 16) = v;
        } else if constexpr (MODE == 1) {
#pragma unroll
            for (int c = 0; c < 4; ++c) *reinterpret_cast<uint4*>(base + c * 1024 + lane * 16) = v;
        } else if constexpr (MODE == 2) {
#pragma unroll
            for (int st = 0; st < 4; ++st)
                glds(base + (lane >> 1) * 128 + st * 32 + (lane & 1) * 16, lds0 + (unsigned)((wv * 4 + st) * 1024));
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                glds(base + i * 1024 + lane * 16, lds0 + (unsigned)((wv * 4 + i) * 1024));
        }
        if (++inflight == depth) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            inflight = 0;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int MODE>
float run(char* buf, long long bytes, int wpc, int depth, int reps) {
    const long long ntiles = bytes / 4096;
    const int block = 64 * wpc;
    auto k = &tiles<MODE>;
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    const int lds = wpc * 4 * 1024;
    hipLaunchKernelGGL(k, dim3(256), dim3(block), lds, 0, buf, ntiles, depth);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(256), dim3(block), lds, 0, buf, ntiles, depth);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1000.f / reps;
}

int main() {
    const long long big = 1ll << 30, small = 32ll * 6400 * 128;
    char* buf;
    CK(hipMalloc(&buf, big));
    CK(hipMemset(buf, 1, big));
    const char* names[4] = {"store lane-pixel (32 B / line / instr)", "store coalesced", "LDS-DMA 2 lanes/px (32 B / line)",
                            "LDS-DMA 8 lanes/px (whole lines)"};
    for (long long bytes : {small, big}) {
        for (int wpc : {4, 8}) {
            for (int depth : {2, 8}) {
                float us[4];
                const int reps = bytes == big ? 5 : 50;
                us[0] = run<0>(buf, bytes, wpc, depth, reps);
                us[1] = run<1>(buf, bytes, wpc, depth, reps);
                us[2] = run<2>(buf, bytes, wpc, depth, reps);
                us[3] = run<3>(buf, bytes, wpc, depth, reps);
                for (int m = 0; m < 4; ++m)
                    printf("%6.1f MB  %d waves/CU  depth %d  %-40s %9.2f us  %7.0f GB/s\n", bytes / 1e6, wpc, depth, names[m],
                           us[m], bytes / (us[m] * 1e3));
            }
        }
    }
    CK(hipFree(buf));
    return 0;
}
