// fp32 accumulation error of v_mfma_f32_16x16x4f32 vs a VALU fmaf chain, against
// exact (fp64) dot products: mean signed error (bias) and mean / max |error| in
// units of the fp32 ulp of the result. Used to track down the fp32 forward's noise.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void mfma_dot(const float* A, const float* B, float* C, int K) {
    // one wave: C[16][16] = A[16][K] . B[K][16] (row-major A, B[k][n])
    const int lane = threadIdx.x;
    const int r = lane & 15, kq = lane >> 4;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < K; k0 += 4) {
        const float a = A[r * K + k0 + kq];
        const float b = B[(k0 + kq) * 16 + r];
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
    }
    // acc[i] = C[row = 4*(lane>>4) + i][col = lane & 15]
    for (int i = 0; i < 4; ++i) C[(4 * kq + i) * 16 + r] = acc[i];
}

__global__ void valu_dot(const float* A, const float* B, float* C, int K) {
    const int t = threadIdx.x;   // 256 threads: one output each
    const int m = t >> 4, n = t & 15;
    float acc = 0.f;
    for (int k = 0; k < K; ++k) acc = fmaf(A[m * K + k], B[k * 16 + n], acc);
    C[m * 16 + n] = acc;
}

int main() {
    const int Ks[] = {64, 576, 1152, 2304};
    for (int K : Ks) {
        std::vector<float> a(16 * K), b(K * 16);
        unsigned s = 1234567u;
        auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) / 8388608.0f - 1.0f); };
        for (auto& v : a) v = rnd();
        for (auto& v : b) v = rnd() * 0.1f + 0.05f;   // biased: partial sums drift like conv outputs
        float *da, *db, *dc1, *dc2;
        hipMalloc(&da, a.size() * 4); hipMalloc(&db, b.size() * 4);
        hipMalloc(&dc1, 256 * 4); hipMalloc(&dc2, 256 * 4);
        hipMemcpy(da, a.data(), a.size() * 4, hipMemcpyHostToDevice);
        hipMemcpy(db, b.data(), b.size() * 4, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(mfma_dot, dim3(1), dim3(64), 0, 0, da, db, dc1, K);
        hipLaunchKernelGGL(valu_dot, dim3(1), dim3(256), 0, 0, da, db, dc2, K);
        std::vector<float> c1(256), c2(256);
        hipMemcpy(c1.data(), dc1, 1024, hipMemcpyDeviceToHost);
        hipMemcpy(c2.data(), dc2, 1024, hipMemcpyDeviceToHost);
        double bias[2] = {0, 0}, mabs[2] = {0, 0}, mx[2] = {0, 0};
        for (int m = 0; m < 16; ++m)
            for (int n = 0; n < 16; ++n) {
                double ex = 0;
                for (int k = 0; k < K; ++k) ex += (double)a[m * K + k] * b[k * 16 + n];
                const double ulp = std::ldexp(1.0, std::ilogb((float)ex) - 23);
                const float got[2] = {c1[m * 16 + n], c2[m * 16 + n]};
                for (int q = 0; q < 2; ++q) {
                    const double e = ((double)got[q] - ex) / ulp;
                    bias[q] += e / 256; mabs[q] += std::fabs(e) / 256; mx[q] = std::fmax(mx[q], std::fabs(e));
                }
            }
        printf("K=%5d  mfma_f32_16x16x4f32: bias %+7.2f ulp  mean|e| %6.2f  max %7.2f   |  valu fmaf chain: bias %+7.2f  mean|e| %6.2f  max %7.2f\n",
               K, bias[0], mabs[0], mx[0], bias[1], mabs[1], mx[1]);
        hipFree(da); hipFree(db); hipFree(dc1); hipFree(dc2);
    }
    return 0;
}
