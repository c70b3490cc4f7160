// LDS tile images + MFMA operand reads shared by the MFMA GEMM kernels (grouped MoE GEMM in
// moe.hip, implicit-GEMM convolution in conv.hip).
//
// Two tile images per operand:
//  * K-contiguous  [rows][BK]  -- 8-byte units XOR-swizzled by row group (kc_off), read as
//    two 8-byte halves per lane in the permuted k order of ld_kc;
//  * K-strided     [BK][cols]  -- 16-byte chunks XOR-swizzled by k row (ks_off), read with
//    ds_read_b64_tr_b16 (ld_ks) so the MFMA sees a k-major fragment without a register transpose.
// Both feed v_mfma_f32_32x32x16_bf16 with the same (permuted) k order on A and B, so any mix of
// images is consistent.
#pragma once
#include "spa_common.h"

namespace spa {

typedef short s16x4_t __attribute__((ext_vector_type(4)));

template <int BK>
__device__ __forceinline__ int kc_off(int r, int u) {
  constexpr int P = 128 / BK;              // rows per 256-byte (64-bank) span
  constexpr int NU = BK / 4;               // 8-byte units per row
  return r * BK + 4 * (u ^ ((r / P) & (NU - 1)));
}
template <int L>
__device__ __forceinline__ int ks_off(int r, int ch) {   // 16B chunk ch of k-row r, row length L
  return r * L + 8 * (ch ^ (((r & 3) << 2) | ((r >> 2) & 3)));
}
// MFMA operand with permuted k order: k = 16s + 4hh + {0..3}, 16s + 8 + 4hh + {0..3}
template <int BK>
__device__ __forceinline__ bf16x8 ld_kc(const bf16* t, int row, int s, int hh) {
  const bf16x4 a = *reinterpret_cast<const bf16x4*>(t + kc_off<BK>(row, 4 * s + hh));
  const bf16x4 b = *reinterpret_cast<const bf16x4*>(t + kc_off<BK>(row, 4 * s + 2 + hh));
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}
template <int L>
__device__ __forceinline__ bf16x8 ld_ks(const bf16* t, int col0, int s, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3, hh = lane >> 5;
  const int c = col0 + 16 * (g & 1) + 4 * pp;
  const int ra = 16 * s + 4 * hh + q, rb = ra + 8;
  typedef __attribute__((address_space(3))) s16x4_t LT;
  const s16x4_t a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LT*)(t + ks_off<L>(ra, c >> 3) + (c & 7)));
  const s16x4_t b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LT*)(t + ks_off<L>(rb, c >> 3) + (c & 7)));
  const bf16x4 av = __builtin_bit_cast(bf16x4, a), bv = __builtin_bit_cast(bf16x4, b);
  return __builtin_shufflevector(av, bv, 0, 1, 2, 3, 4, 5, 6, 7);
}


// fast unsigned division by a runtime constant (n < 2^31): q = (umulhi(n, m) + n) >> s
struct FastDiv {
  unsigned m;
  int s, d;
};
inline FastDiv make_fastdiv(int d) {
  int s = 0;
  while ((1LL << s) < d) ++s;
  const unsigned m = (unsigned)(((1ULL << 32) * ((1ULL << s) - d)) / d + 1);
  return FastDiv{m, s, d};
}
__device__ __forceinline__ int fdiv(int n, const FastDiv& f) {
  return (int)((__umulhi((unsigned)n, f.m) + (unsigned)n) >> f.s);
}

}  // namespace spa
