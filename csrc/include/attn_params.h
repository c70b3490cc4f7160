// Flash-attention kernel parameters shared by attention.hip and attention_bwd4.hip (the dK/dV
// kernel built with the max-ILP machine scheduler in its own translation unit).
#pragma once
#include "attn_common.h"

namespace spa {

struct AttnParams {
  const bf16* q; const bf16* k; const bf16* v; const bf16* o; const bf16* dout;
  bf16* out; bf16* dq; bf16* dk; bf16* dv;
  float* lse; const float* lse_in; float* delta; float* dqacc;  // dqacc: fused bwd fp32 dQ [B,Tq,H,HD]
  int B, H, Hkv, Tq, Tk;
  long sqb, sqt, sqh, skb, skt, skh, svb, svt, svh, sob, sot, soh;
  long sdob, sdot, sdoh;
  long sdqb, sdqt, sdqh, sdkb, sdkt, sdkh, sdvb, sdvt, sdvh;
  float scale;       // softmax scale (natural)
  float scale_log2;  // scale * log2(e)
  int causal_off;    // key j visible to query i iff j <= i + causal_off
  // dK/dV q-head split (small Hkv x key-block grids, e.g. MQA): hsplit blocks per key block,
  // each summing G/hsplit q-heads into fp32 partials dkacc/dvacc [hsplit, B, Tk, Hkv, HD]
  int hsplit;
  float* dkacc; float* dvacc;
  // fused dropout on P (DROP kernels): keep iff hash(seed, b, h, q, key) >> 8 >= drop_thr
  unsigned seed_lo, seed_hi, drop_thr;
  float drop_scale;  // 1 / (1 - p)
  const int64_t* seed_ptr;  // device seed (graph-safe: a fresh mask per HIP-graph replay) or null
  // profiling only (SPA_ATTN_STAMP): per-wave s_memtime segment sums of the dK/dV loop, or null
  long long* stamp;
  int xcd;  // query-parallel kernels: XCD-aware block order (q_block_map)
};

// dK^T / dV^T accumulator (rows d = 32dt + (r&3) + 8(r>>2) + 4hh, column = key) -> global:
// bf16 (dk scaled) when the block owns all q-heads of its kv-head, else fp32 partials.
template <int HD>
__device__ __forceinline__ void store_kv_grad(const AttnParams& p, const f32x16 (&acc)[HD / 32], bool is_k,
                                              int b, int hk, int key, int split, int hh) {
  if (key >= p.Tk) return;
  constexpr int DT = HD / 32;
  if (p.hsplit == 1) {
    bf16* dst = is_k ? p.dk + b * p.sdkb + (long)key * p.sdkt + hk * p.sdkh
                     : p.dv + b * p.sdvb + (long)key * p.sdvt + hk * p.sdvh;
    const float sc = is_k ? p.scale : 1.f;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 w;
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = (bf16)(acc[dt][4 * g + i] * sc);
        *reinterpret_cast<bf16x4*>(dst + 32 * dt + 8 * g + 4 * hh) = w;
      }
  } else {
    float* dst = (is_k ? p.dkacc : p.dvacc) +
                 ((((long)split * p.B + b) * p.Tk + key) * p.Hkv + hk) * HD;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4 w;
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = acc[dt][4 * g + i];
        *reinterpret_cast<f32x4*>(dst + 32 * dt + 8 * g + 4 * hh) = w;
      }
  }
}


// attention_bwd4.hip: one-wave-per-SIMD dK/dV for head dim 128
void launch_dkdv4_128(const AttnParams& p, bool causal, int grid, hipStream_t st);

}  // namespace spa
