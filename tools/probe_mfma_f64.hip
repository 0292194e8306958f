// Probe of the v_mfma_f64_16x16x4f64 operand layout (exact integer data): D = C + A B with
// A 16x4, B 4x16.  Assumed maps (cdna_hip_programming.md): A lane l -> A[l & 15][l >> 4],
// B lane l -> B[l >> 4][l & 15], C/D lane l reg i -> [(l >> 4) + 4 i][l & 15].
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ void k(double *out) {
    const int l = threadIdx.x;
    const double a = (double)((l & 15) * 10 + (l >> 4));        // A[r][k] = 10 r + k
    const double b = (double)((l >> 4) * 100 + (l & 15) + 1);   // B[k][c] = 100 k + c + 1
    d4 c;
    for (int i = 0; i < 4; ++i) c[i] = (double)(((l >> 4) + 4 * i) * 1000 + (l & 15));   // C[r][c] = 1000 r + c
    d4 d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    for (int i = 0; i < 4; ++i) out[((l >> 4) + 4 * i) * 16 + (l & 15)] = d[i];
}
int main() {
    double *o;
    hipMalloc(&o, 256 * 8);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o);
    double h[256];
    hipMemcpy(h, o, sizeof(h), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int r = 0; r < 16; ++r)
        for (int cc = 0; cc < 16; ++cc) {
            double ref = 1000.0 * r + cc;
            for (int kk = 0; kk < 4; ++kk) ref += (10.0 * r + kk) * (100.0 * kk + cc + 1);
            if (h[r * 16 + cc] != ref) ++bad;
        }
    printf("mfma_f64_16x16x4 layout probe: %d mismatches of 256\n", bad);
    return bad != 0;
}
