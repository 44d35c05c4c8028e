#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
// A [16][128] fp8, B [16][128] fp8 (row = n, k contiguous); C[m][n] = sum_k A[m][k] B[n][k]
__global__ void k(const unsigned char* A, const unsigned char* B, float* C, int variant) {
  int l = threadIdx.x;
  v8i a, b;
  unsigned char* pa = (unsigned char*)&a;
  unsigned char* pb = (unsigned char*)&b;
  for (int j = 0; j < 32; ++j) {
    int kk;
    if (variant == 0) kk = 32 * (l >> 4) + j;                     // contiguous 32 per lane group
    else kk = 8 * (l >> 4) + (j & 7) + 32 * (j >> 3);              // 4 x (8-byte pieces of the 16x16x32 layout)
    pa[j] = A[(l & 15) * 128 + kk];
    pb[j] = B[(l & 15) * 128 + kk];
  }
  v4f c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(b, a, c, 0, 0, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
  // (B,A) swapped like the framework: lane owns row m = lane&15? check both
  for (int r = 0; r < 4; ++r) C[l * 4 + r] = c[r];
}
static float e4m3(unsigned char v) {
  int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
  float f = e == 0 ? ldexpf((float)m, -9) : ldexpf(1.f + m / 8.f, e - 7);
  return s ? -f : f;
}
int main() {
  unsigned char hA[16 * 128], hB[16 * 128];
  srand(1);
  for (int i = 0; i < 16 * 128; ++i) { hA[i] = (unsigned char)(rand() % 0x70); hB[i] = (unsigned char)(rand() % 0x70) | ((rand() & 1) << 7); }
  unsigned char *dA, *dB; float* dC;
  hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dC, 256 * 4);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice); hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  for (int variant = 0; variant < 2; ++variant) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC, variant);
    float hC[256];
    hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
    // framework convention: lane owns n = ..., acc[r]: with (B,A) swapped, C/D col = lane&15 -> m, row = 4*(lane>>4)+r -> n
    double err = 0, ref = 0;
    for (int l = 0; l < 64; ++l) for (int r = 0; r < 4; ++r) {
      int m = l & 15, n = 4 * (l >> 4) + r;
      double s = 0; for (int kk = 0; kk < 128; ++kk) s += (double)e4m3(hA[m * 128 + kk]) * e4m3(hB[n * 128 + kk]);
      err = fmax(err, fabs(s - hC[l * 4 + r])); ref = fmax(ref, fabs(s));
    }
    printf("variant %d: max err %g (ref max %g)\n", variant, err, ref);
  }
  return 0;
}
