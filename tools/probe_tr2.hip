// Probe the attention kernel's swizzled image + rd_tr helper (HD=64) against expectations.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s16x4 __attribute__((ext_vector_type(4)));
template <int HD> __device__ int swz(int r) {
  if constexpr (HD >= 128) return ((r & 3) << 2) | ((r >> 2) & 3);
  else return (((r >> 1) & 1) << 2) | ((r >> 2) & 3);
}
template <int HD> __device__ void rd_tr(const short* img, int rbase, int c0, int lane, short* out) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3, hh = lane >> 5;
  const int c = c0 + 16 * (g & 1) + 4 * pp;
  const int ch = c >> 3, within = c & 7;
  const int ra = rbase + 4 * hh + q, rb = ra + 8;
  typedef __attribute__((address_space(3))) s16x4 L;
  s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((L*)(img + ra * HD + 8 * (ch ^ swz<HD>(ra)) + within));
  s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((L*)(img + rb * HD + 8 * (ch ^ swz<HD>(rb)) + within));
  for (int j = 0; j < 4; ++j) { out[j] = a[j]; out[4 + j] = b[j]; }
}
template <int HD> __global__ void k(short* out) {
  __shared__ __attribute__((aligned(16))) short lds[64 * HD];
  // row-major image with swizzled 16B chunks: element (r, c) stored at r*HD + 8*((c>>3)^swz(r)) + (c&7)
  for (int i = threadIdx.x; i < 64 * HD; i += 64) {
    int r = i / HD, c = i % HD;
    lds[r * HD + 8 * ((c >> 3) ^ swz<HD>(r)) + (c & 7)] = (short)(r * 256 + c);
  }
  __syncthreads();
  short o[8];
  rd_tr<HD>(lds, 16, 32, threadIdx.x, o);  // k-step rows 16.., d-tile 1
  for (int j = 0; j < 8; ++j) out[threadIdx.x * 8 + j] = o[j];
}
int main() {
  short* d; (void)hipMalloc(&d, 64 * 8 * 2);
  short h[512];
  k<64><<<1, 64>>>(d); (void)hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l) for (int j = 0; j < 8; ++j) {
    int hh = l >> 5; int er = 16 + 8 * (j >> 2) + 4 * hh + (j & 3), ec = 32 + (l & 31);
    int gr = h[l*8+j] / 256, gc = h[l*8+j] % 256;
    if (gr != er || gc != ec) { if (bad < 20) printf("HD64 lane %d j %d: got (r%d,c%d) want (r%d,c%d)\n", l, j, gr, gc, er, ec); bad++; }
  }
  printf("HD64 bad=%d\n", bad);
  k<128><<<1, 64>>>(d); (void)hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
  bad = 0;
  for (int l = 0; l < 64; ++l) for (int j = 0; j < 8; ++j) {
    int hh = l >> 5; int er = 16 + 8 * (j >> 2) + 4 * hh + (j & 3), ec = 32 + (l & 31);
    int gr = h[l*8+j] / 256, gc = h[l*8+j] % 256;
    if (gr != er || gc != ec) { if (bad < 20) printf("HD128 lane %d j %d: got (r%d,c%d) want (r%d,c%d)\n", l, j, gr, gc, er, ec); bad++; }
  }
  printf("HD128 bad=%d\n", bad);
  return 0;
}
