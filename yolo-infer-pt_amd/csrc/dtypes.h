// Device-side dtype traits: storage types, 8-element chunk moves, MFMA step.
#pragma once
#include <hip/hip_runtime.h>

namespace yh {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

// A "chunk" = 8 consecutive channels of one pixel = 16 B for 2-byte types, 32 B for f32.
template <typename T> struct Chunk { uint4 v[sizeof(T) / 2]; };

template <typename T>
__device__ __forceinline__ Chunk<T> ld_chunk(const T* p) {
    Chunk<T> c;
    const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 2); ++i) c.v[i] = q[i];
    return c;
}
template <typename T>
__device__ __forceinline__ void st_chunk(T* p, const Chunk<T>& c) {
    uint4* q = reinterpret_cast<uint4*>(p);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 2); ++i) q[i] = c.v[i];
}
template <typename T>
__device__ __forceinline__ Chunk<T> zero_chunk() {
    Chunk<T> c;
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 2); ++i) c.v[i] = make_uint4(0, 0, 0, 0);
    return c;
}

template <typename T> __device__ __forceinline__ float tof(T v) { return (float)v; }
template <typename T> __device__ __forceinline__ T fromf(float v) { return (T)v; }
// v rounded to T and back (the value a T store followed by a load would give)
template <typename T> __device__ __forceinline__ float fromf_round(float v) { return tof(fromf<T>(v)); }

template <typename T>
__device__ __forceinline__ void chunk_to_f(const Chunk<T>& c, float (&f)[8]) {
    const T* e = reinterpret_cast<const T*>(&c);
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = tof(e[i]);
}
template <typename T>
__device__ __forceinline__ Chunk<T> f_to_chunk(const float (&f)[8]) {
    Chunk<T> c;
    T* e = reinterpret_cast<T*>(&c);
#pragma unroll
    for (int i = 0; i < 8; ++i) e[i] = fromf<T>(f[i]);
    return c;
}

// SiLU: exact-rounded exp/div on the f32 (parity) path, hardware exp/rcp on 16-bit paths.
template <typename T> __device__ __forceinline__ float silu(float x) {
#ifdef YH_SILU_EXPERIMENT   // cost experiment only (wrong values): SiLU without transcendentals
    return x * fmaf(x, 0.25f, 0.5f);
#else
    return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x));
#endif
}
template <> __device__ __forceinline__ float silu<float>(float x) { return x / (1.0f + expf(-x)); }

// One 16(rows) x 16(cols) x 32(k) MFMA step. a/b point at a lane's 8 consecutive
// k values of its row (A) / column (B). For f32 the 32-deep step is eight exact
// f32 MFMAs (16x16x4); the k permutation is the same for A and B, so the sum is
// over the same 32 products.
typedef double f64x4 __attribute__((ext_vector_type(4)));

// One 16x16 x K=32-bytes-of-operands MFMA step of conv_gemm. acc_t is the accumulator
// type; finish() adds the bias and rounds to float. The 16-bit paths accumulate in
// fp32 (16x16x32); the fp32 (parity) path runs v_mfma_f64_16x16x4f64 on the fp32
// operands widened to fp64: the products are exact and the K sums carry no fp32
// rounding, so a layer's only fp32 rounding is its output's (a sequential fp32 chain
// over K = 576..2304 made the fp32 forward several times noisier than the reference's
// blocked CPU sums).
template <typename T> struct Mma;
template <> struct Mma<__bf16> {
    typedef f32x4 acc_t;
    static __device__ __forceinline__ float finish(float a, float b) { return a + b; }
    // output row (cout within the 16-tile) of accumulator register r in lane group q = lane / 16
    static __device__ __forceinline__ int row(int q, int r) { return 4 * q + r; }
    static __device__ __forceinline__ void step(f32x4& acc, const uint4* a, const uint4* b) {
        bf16x8 av = __builtin_bit_cast(bf16x8, a[0]);
        bf16x8 bv = __builtin_bit_cast(bf16x8, b[0]);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
    }
};
template <> struct Mma<_Float16> {
    typedef f32x4 acc_t;
    static __device__ __forceinline__ float finish(float a, float b) { return a + b; }
    // output row (cout within the 16-tile) of accumulator register r in lane group q = lane / 16
    static __device__ __forceinline__ int row(int q, int r) { return 4 * q + r; }
    static __device__ __forceinline__ void step(f32x4& acc, const uint4* a, const uint4* b) {
        f16x8 av = __builtin_bit_cast(f16x8, a[0]);
        f16x8 bv = __builtin_bit_cast(f16x8, b[0]);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, bv, acc, 0, 0, 0);
    }
};
template <> struct Mma<float> {
    typedef f64x4 acc_t;
    static __device__ __forceinline__ float finish(double a, float b) { return (float)(a + (double)b); }
    // v_mfma_f64_16x16x4f64 interleaves the rows: register r of lane group q holds row q + 4 r
    static __device__ __forceinline__ int row(int q, int r) { return q + 4 * r; }
    static __device__ __forceinline__ void step(f64x4& acc, const uint4* a, const uint4* b) {
        const float* af = reinterpret_cast<const float*>(a);
        const float* bf = reinterpret_cast<const float*>(b);
#pragma unroll
        for (int kk = 0; kk < 8; ++kk)
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64((double)af[kk], (double)bf[kk], acc, 0, 0, 0);
    }
};

// The caller's output tensor reached through io[] (a pointer loaded from device memory, so the
// compiler cannot infer its address space): as a global pointer its stores are global_store,
// counted in vmcnt only. Through the generic pointer they are flat stores, which also count in
// lgkmcnt - every later LDS wait of the wave would then wait for them to reach memory - and the
// pointer itself is re-loaded (waiting on vmcnt(0)) at every store it may alias.
template <typename T> using gptr = __attribute__((address_space(1))) T*;
template <typename T> __device__ __forceinline__ gptr<T> io_global(const void* p) { return (gptr<T>)(const_cast<void*>(p)); }
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
template <typename T>
__device__ __forceinline__ void st_chunk(gptr<T> p, const Chunk<T>& c) {
    const gptr<u32x4v> q = (gptr<u32x4v>)p;
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 2); ++i) q[i] = __builtin_bit_cast(u32x4v, c.v[i]);
}

// lane l's x from lane l ^ 32 (the other wave half) by gfx950's v_permlane32_swap: a VALU
// exchange, not an LDS round trip as a ds_bpermute shuffle
__device__ __forceinline__ float xor32_swap(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    // r[0] = the low half's values in both halves, r[1] = the high half's
    return __uint_as_float((threadIdx.x & 32) ? r[0] : r[1]);
#else
    return x;
#endif
}

// XCD-aware bijective remap of a 1-D block id: blocks b and b+8 share an XCD
// (round-robin dispatch), so give each XCD a contiguous range of logical ids.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + (bid >> 3);
}

// Touch every 64-B line of a kernel's argument block (the first `bytes` <= 1 KB of the kernarg
// segment) with 16 scalar loads issued back to back and one wait, so the kernel's later argument
// reads hit the scalar cache: a large argument struct read with data-dependent indices otherwise
// pays one L2 round trip per line, one after another (pw_chain's prologue: ~4 us of such chains).
// One asm block: the compiler's own scheduling split the loads over three waits.
template <int bytes>
__device__ __forceinline__ void touch_kernargs() {
    static_assert(bytes > 0 && bytes <= 1024, "touch_kernargs: at most 16 lines");
#if defined(__HIP_DEVICE_COMPILE__)
    constexpr int last = ((bytes - 1) / 64) * 64;
#define YH_KL(i) ((i) * 64 < last ? (i) * 64 : last)
    unsigned r[16];
    asm volatile(
        "s_load_dword %0, %16, %17\n\ts_load_dword %1, %16, %18\n\ts_load_dword %2, %16, %19\n\t"
        "s_load_dword %3, %16, %20\n\ts_load_dword %4, %16, %21\n\ts_load_dword %5, %16, %22\n\t"
        "s_load_dword %6, %16, %23\n\ts_load_dword %7, %16, %24\n\ts_load_dword %8, %16, %25\n\t"
        "s_load_dword %9, %16, %26\n\ts_load_dword %10, %16, %27\n\ts_load_dword %11, %16, %28\n\t"
        "s_load_dword %12, %16, %29\n\ts_load_dword %13, %16, %30\n\ts_load_dword %14, %16, %31\n\t"
        "s_load_dword %15, %16, %32\n\ts_waitcnt lgkmcnt(0)"
        : "=&s"(r[0]), "=&s"(r[1]), "=&s"(r[2]), "=&s"(r[3]), "=&s"(r[4]), "=&s"(r[5]), "=&s"(r[6]), "=&s"(r[7]),
          "=&s"(r[8]), "=&s"(r[9]), "=&s"(r[10]), "=&s"(r[11]), "=&s"(r[12]), "=&s"(r[13]), "=&s"(r[14]),
          "=&s"(r[15])
        : "s"(__builtin_amdgcn_kernarg_segment_ptr()), "n"(YH_KL(0)), "n"(YH_KL(1)), "n"(YH_KL(2)), "n"(YH_KL(3)),
          "n"(YH_KL(4)), "n"(YH_KL(5)), "n"(YH_KL(6)), "n"(YH_KL(7)), "n"(YH_KL(8)), "n"(YH_KL(9)), "n"(YH_KL(10)),
          "n"(YH_KL(11)), "n"(YH_KL(12)), "n"(YH_KL(13)), "n"(YH_KL(14)), "n"(YH_KL(15))
        : "memory");
#undef YH_KL
#endif
}

}  // namespace yh
