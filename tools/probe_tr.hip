// Probe ds_read_b64_tr_b16 semantics: LDS[r][c] = r*256 + c (16-bit), 16 rows x 64 cols.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s4 __attribute__((ext_vector_type(4)));
__global__ void k(short* out, int mode) {
  __shared__ __attribute__((aligned(16))) short lds[64 * 64];
  for (int i = threadIdx.x; i < 64 * 64; i += 64) lds[i] = (short)((i / 64) * 256 + (i % 64));
  __syncthreads();
  const int lane = threadIdx.x;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  // mode 0: guide layout: lane 4q+p -> row q (+4*(g>>1)), cols 16*(g&1) + 4p
  int row = 4 * (g >> 1) + q, col = 16 * (g & 1) + 4 * p;
  typedef __attribute__((address_space(3))) s4 L;
  s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((L*)(lds + row * 64 + col));
  for (int j = 0; j < 4; ++j) out[lane * 4 + j] = v[j];
}
int main() {
  short* d; hipMalloc(&d, 64 * 4 * 2);
  k<<<1, 64>>>(d, 0);
  short h[256]; hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int j = 0; j < 4; ++j) printf(" (r%d,c%d)", h[l*4+j] / 256, h[l*4+j] % 256);
    printf("\n");
  }
  return 0;
}
