// Lane layout of v_mfma_f64_16x16x4f64: A[i][k] = (k == 0) * (i + 1), B[k][j] = (k == 0) * (100 + j)
// with the f32 16x16x4 operand mapping (lane -> row/col lane % 16, k = lane / 16); prints
// which (i, j) each lane's accumulator register r holds (value = (i + 1) * (100 + j)).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));
__global__ void k(double* out) {
    const int lane = threadIdx.x;
    const double a = (lane / 16 == 0) ? (double)(lane % 16 + 1) : 0.0;
    const double b = (lane / 16 == 0) ? (double)(100 + lane % 16) : 0.0;
    f64x4 acc = {0, 0, 0, 0};
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    for (int r = 0; r < 4; ++r) out[lane * 4 + r] = acc[r];
}
int main() {
    double* d;
    (void)hipMalloc(&d, 256 * 8);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    double h[256];
    (void)hipMemcpy(h, d, 256 * 8, hipMemcpyDeviceToHost);
    for (int lane = 0; lane < 64; ++lane) {
        printf("lane %2d:", lane);
        for (int r = 0; r < 4; ++r) {
            const double v = h[lane * 4 + r];
            int fi = -1, fj = -1;
            for (int i = 0; i < 16; ++i)
                for (int j = 0; j < 16; ++j)
                    if ((i + 1) * (100 + j) == v) { fi = i; fj = j; }
            printf("  r%d=(%d,%d)", r, fi, fj);
        }
        printf("\n");
    }
    return 0;
}
