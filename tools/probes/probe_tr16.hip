// Determine the lane mapping of ds_read_b64_tr_b16 on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short v4s __attribute__((ext_vector_type(4)));
__global__ void k(int* out) {
  __shared__ unsigned short lds[64 * 64];
  for (int i = threadIdx.x; i < 64 * 64; i += 64) lds[i] = (unsigned short)((i / 64) * 256 + (i % 64));
  __syncthreads();
  int l = threadIdx.x;
  int row = l / 4, col = (l % 4) * 4;  // lane l supplies row l/4, cols 4*(l%4)..+3
  v4s r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(lds + row * 64 + col));
  for (int j = 0; j < 4; ++j) out[l * 4 + j] = (unsigned short)r[j];
}
int main() {
  int* d; hipMalloc(&d, 64 * 4 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  int h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int j = 0; j < 4; ++j) printf(" (r%2d,c%2d)", h[l * 4 + j] / 256, h[l * 4 + j] % 256);
    printf("\n");
  }
  return 0;
}
