// Flash-attention kernel parameters and device helpers shared by the attention kernels.
#pragma once
#include "attn_common.h"

// debug build (spa_debug.h): the (batch, row, head) a block derived from its tile ids, checked
// against the problem at every global store (`if (SPA_DBG_BRH(...)) *dst = ...`); `true` otherwise
#define SPA_DBG_BRH(b, r, R, h, H) (SPA_DBG_OK(b, p.B) & SPA_DBG_OK(r, R) & SPA_DBG_OK(h, H))

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
  // dS-materialising backward (attn_bwd_dkdv3_kernel<.., DSOUT> -> attn_bwd_dq_ds_kernel): the
  // bf16 dS of every 32-query x 32-key block in consumer order, ds_kvstride elements per (b, kv-head),
  // block (qt, kt) of q-head g at ds_index(); ds_nqt / ds_nkt = 32-row tiles of Tq / Tk
  bf16* dsbuf;
  long ds_kvstride;
  int ds_nqt, ds_nkt;
  // key-split query-parallel kernels (few (b, head) pairs, e.g. TP-sharded MQA): ksplit blocks per
  // query block, each over a contiguous share of its key tiles, writing fp32 partials -- forward:
  // unnormalised O rows at part [ksplit, B, H, Tq, part_ld] plus (m, l) pairs at mlpart
  // [ksplit, B, H, Tq, 2], merged by attn_fwd_merge_kernel; dQ: unscaled dQ rows at part
  // [ksplit, B, Tq, H, part_ld], summed by attn_dq_reduce_kernel. vhalf: the forward's V / O
  // column offset per blockIdx.y (head dim 256 run as two 128-column halves in one launch).
  int ksplit;
  float* part;
  float* mlpart;
  int part_ld;
  int vhalf;
  // attn_bwd_dkdv5_kernel: row constants [B*H][2][rowk_ld] = -lse*log2(e) | -delta per query row
  // (rowk_ld = Tq rounded up to 64, zeros past Tq), DMA'd into LDS with each Q / dO tile
  float* rowk;
  int rowk_ld;
};

// host launcher of the dK/dV v5 path (csrc/kernels/attention_dkdv5.hip): rowk pass + dK/dV kernel
void launch_dkdv5(AttnParams& p, bool causal, hipStream_t st);
// host launcher of the short-sequence fused backward (csrc/kernels/attention_short.hip)
void launch_bwd_short(AttnParams& p, bool causal, hipStream_t st);

// 2 KiB dS block index inside one (b, kv-head) region, in the order the dQ pass streams it: per
// 64-query block qb its key steps kt (causal Tq == Tk: kt <= 2qb + 1, non-causal: all nkt), per
// step the G q-heads of the group, per head the two 32-query halves t. A dQ block (4 waves = 4 heads
// of one qb at G = 4) then reads one contiguous 16 KiB piece per key step. The t = 0 block of the
// causal last step (kt = 2qb + 1 > qt) is a hole: never written, never used.
__device__ __forceinline__ long ds_index(int qt, int kt, int g, int G, int nkt, bool causal) {
  const int qb = qt >> 1, t = qt & 1;
  const long step = causal ? (long)qb * (qb + 1) + kt : (long)qb * nkt + kt;
  return (step * G + g) * 2 + t;
}
// elements per (b, kv-head) region
inline long ds_kv_elems(int nq64, int nkt, int G, bool causal) {
  return 1024L * 2 * G * (causal ? (long)nq64 * (nq64 + 1) : (long)nq64 * nkt);
}
// 16-B chunk slot of (producer half s, lane half h, key k) in a 2 KiB dS block: the 8 bf16 of a
// chunk are the dS of key k for queries 16s + 8(j>>2) + 4h + (j&3), j = 0..7 (the dK/dV kernel's
// packed-accumulator order). Slot = (k>>2)*16 + (2s+h)*4 + (k&3): every 32-lane half of the
// consumer's transposed reads (4 keys k>>2-aligned x all (s, h)) then covers 16 distinct slots
// mod 16 = one whole bank row, conflict-free.
__device__ __forceinline__ int ds_slot(int s, int h, int k) { return (k >> 2) * 16 + (2 * s + h) * 4 + (k & 3); }

// dK^T / dV^T accumulator (rows d = 32dt + (r&3) + 8(r>>2) + 4hh, column = key) -> global:
// bf16 (dk scaled) when the block owns all q-heads of its kv-head, else fp32 partials.
// NDT < HD / 32: the accumulator holds the 32-dim tiles dt0 .. dt0 + NDT - 1 only (a role's share).
template <int HD, int NDT = HD / 32>
__device__ __forceinline__ void store_kv_grad(const AttnParams& p, const f32x16 (&acc)[NDT], bool is_k,
                                              int b, int hk, int key, int split, int hh, int dt0 = 0) {
  if (key >= p.Tk) return;
  if (!(SPA_DBG_BRH(b, key, p.Tk, hk, p.Hkv) & SPA_DBG_OK(split, p.hsplit))) return;
  static_assert(NDT <= HD / 32, "store_kv_grad: more tiles than the head dim");
  constexpr int DT = NDT;
  if (p.hsplit == 1) {
    bf16* dst = (is_k ? p.dk + b * p.sdkb + (long)key * p.sdkt + hk * p.sdkh
                      : p.dv + b * p.sdvb + (long)key * p.sdvt + hk * p.sdvh) + 32 * dt0;
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
                 ((((long)split * p.B + b) * p.Tk + key) * p.Hkv + hk) * HD + 32 * dt0;
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


}  // namespace spa
