// Probe the operand lane map of v_mfma_scale_f32_32x32x64_f8f6f4 with fp8 (e4m3) inputs:
// try candidate k(lane, byte) maps, compare against a CPU matmul with exact small values.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void k(const uint8_t* a, const uint8_t* b, float* c) {
  const int l = threadIdx.x;
  i32x8 av, bv;
  for (int i = 0; i < 8; ++i) {
    av[i] = *reinterpret_cast<const int*>(a + l * 32 + 4 * i);
    bv[i] = *reinterpret_cast<const int*>(b + l * 32 + 4 * i);
  }
  f32x16 acc = {};
  acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, acc, 0, 0, 0, 127, 0, 127);
  for (int r = 0; r < 16; ++r) c[l * 16 + r] = acc[r];
}

static uint8_t enc(int v) {  // e4m3: 0, +-1, +-2, 3
  switch (v) { case 0: return 0; case 1: return 0x38; case 2: return 0x40; case 3: return 0x44;
    case -1: return 0xB8; case -2: return 0xC0; default: return 0; }
}
static int kmap(int h, int l, int t) {
  const int hh = l >> 5;
  switch (h) {
    case 0: return 32 * hh + t;
    case 1: return 8 * hh + 16 * (t >> 3) + (t & 7);
    case 2: return 16 * hh + 32 * (t >> 4) + (t & 15);
    case 3: return 4 * hh + 8 * (t >> 2) + (t & 3);
    default: return 0;
  }
}
int main() {
  int A[32][64], B[64][32];
  unsigned s = 12345;
  auto rnd = [&]() { s = s * 1103515245u + 12345u; return (int)((s >> 16) % 6) - 2; };  // -2..3
  for (int i = 0; i < 32; ++i) for (int k = 0; k < 64; ++k) A[i][k] = rnd();
  for (int k = 0; k < 64; ++k) for (int j = 0; j < 32; ++j) B[k][j] = rnd();
  float Cref[32][32];
  for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) {
    float acc = 0; for (int k = 0; k < 64; ++k) acc += A[i][k] * B[k][j]; Cref[i][j] = acc; }
  uint8_t *da, *db; float* dc;
  (void)hipMalloc(&da, 2048); (void)hipMalloc(&db, 2048); (void)hipMalloc(&dc, 64 * 16 * 4);
  for (int h = 0; h < 4; ++h) {
    uint8_t ha[2048], hb[2048];
    for (int l = 0; l < 64; ++l) for (int t = 0; t < 32; ++t) {
      const int kk = kmap(h, l, t);
      ha[l * 32 + t] = enc(A[l & 31][kk]);
      hb[l * 32 + t] = enc(B[kk][l & 31]);
    }
    (void)hipMemcpy(da, ha, 2048, hipMemcpyHostToDevice);
    (void)hipMemcpy(db, hb, 2048, hipMemcpyHostToDevice);
    k<<<1, 64>>>(da, db, dc);
    float hc[1024];
    (void)hipMemcpy(hc, dc, 4096, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l) for (int r = 0; r < 16; ++r) {
      const int col = l & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
      if (hc[l * 16 + r] != Cref[row][col]) bad++;
    }
    printf("hypothesis %d: mismatches %d / 1024\n", h, bad);
  }
  return 0;
}
