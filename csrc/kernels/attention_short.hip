// Short-sequence fused attention backward (ViT-B/16: T = 197, head dim 64), in its own translation
// unit so that it gets its own device flags (no SLP vectorisation, see below). Launched from
// attn_bwd (attention.hip) through launch_bwd_short.
#include "attn_common.h"
#include "attn_params.h"

SPA_DEBUG_TU("attention_short.hip")

namespace spa {

// ---------------------------------------------------------------------------
// Short-sequence fused backward (Tq, Tk <= 256, head dim 64, one q-head per kv-head): ViT-B/16
// (vision transformer/ViT.ipynb:208,221; T = 197). One block = 8 waves = one (batch, head).
// The whole sequence's Q, K, V and dO sit in four LDS images (128 KB), so dQ, dK and dV come
// out of one launch with no atomics, no delta pass and one barrier:
//   A  wave w loads rows 32w..32w+31 of q, k, v, dO and o into registers, writes its rows of the
//      four images (zeros past T) and the row constants -lse2 / -delta of its queries.
//   B  dQ of the wave's 32 queries: query on the lane, the dq kernel's body over the K / V images.
//   C  dK / dV of the wave's 32 keys: key on the lane, the dkdv kernel's body over the Q / dO
//      images, with this wave's own K / V rows (already in registers) as the B operands.
// The split kernels at T = 197 pay two prologues per (b, h), re-read K / V (dq) and Q / dO
// (dkdv) from HBM and leave a 69-key second key block: 0.43 ms there vs 0.30-0.32 ms here at
// B 256 (profiles/r2_attn_short_v1.txt). A persistent variant prefetching the next pair's rows
// under B and C spilled 14-37 VGPRs at 2 waves/SIMD and was not kept.
// Round 5 (this file): both tile loops fully unrolled (T <= 256: 8 tiles), so every LDS operand
// address is a per-lane base plus an immediate (the rolled loops re-added 8-29 tile offsets per
// iteration), and the TU is compiled without SLP vectorisation (_build.py EXTRA_FLAGS): hipcc
// paired the P * dP products into v_pk_mul_f32 behind 12 v_mov / v_alignbit shuffles per tile --
// VALU the kernel is bound by (VALU/MFMA 11.7, profiles/r4_vit_b16_step_and_attn_pmc.txt).
// ---------------------------------------------------------------------------
template <int HD, bool CAUSAL>
__global__ __launch_bounds__(512) void attn_bwd_short_kernel(AttnParams p) {
  constexpr int NW = 8, TMAX = 32 * NW, KS = HD / 16, DT = HD / 32, IMG = TMAX * HD;
  static_assert(HD == 64, "short backward: the four images fit LDS at head dim 64");
  __shared__ __attribute__((aligned(16))) bf16 smem[4 * IMG];           // Q | K | V | dO
  __shared__ __attribute__((aligned(16))) float rowl[TMAX], rowd[TMAX];  // -lse2, -delta per query
  bf16* Qi = smem;
  bf16* Ki = smem + IMG;
  bf16* Vi = smem + 2 * IMG;
  bf16* Di = smem + 3 * IMG;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int h = blockIdx.x % p.H, b = blockIdx.x / p.H;  // H == Hkv
  SPA_DBG_CHECK(b, p.B);
  SPA_DBG_ASSERT(p.Tq <= TMAX && p.Tk <= TMAX, p.Tq, TMAX);
  const int r0 = __builtin_amdgcn_readfirstlane(wave * 32);
  const int row = r0 + l32;
  const float c = p.scale_log2;

  bf16x8 qf[KS], df[KS], kf[KS], vf[KS];
  float dlt = 0.f;
  {
    const bool qv = row < p.Tq, kv = row < p.Tk;
    const bf16* qp = p.q + b * p.sqb + (long)row * p.sqt + h * p.sqh + 8 * hh;
    const bf16* dp = p.dout + b * p.sdob + (long)row * p.sdot + h * p.sdoh + 8 * hh;
    const bf16* op = p.o + b * p.sob + (long)row * p.sot + h * p.soh + 8 * hh;
    const bf16* kp = p.k + b * p.skb + (long)row * p.skt + h * p.skh + 8 * hh;
    const bf16* vp = p.v + b * p.svb + (long)row * p.svt + h * p.svh + 8 * hh;
    bf16x8 of[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      qf[s] = qv ? *reinterpret_cast<const bf16x8*>(qp + 16 * s) : zero8();
      df[s] = qv ? *reinterpret_cast<const bf16x8*>(dp + 16 * s) : zero8();
      of[s] = qv ? *reinterpret_cast<const bf16x8*>(op + 16 * s) : zero8();
      kf[s] = kv ? *reinterpret_cast<const bf16x8*>(kp + 16 * s) : zero8();
      vf[s] = kv ? *reinterpret_cast<const bf16x8*>(vp + 16 * s) : zero8();
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      // row = this lane's row; chunk 2s+hh holds d = 16s + 8hh .. +8 (the fragments' own layout)
      const int o = img_off<HD>(row, 2 * s + hh);
      *reinterpret_cast<bf16x8*>(Qi + o) = qf[s];
      *reinterpret_cast<bf16x8*>(Ki + o) = kf[s];
      *reinterpret_cast<bf16x8*>(Vi + o) = vf[s];
      *reinterpret_cast<bf16x8*>(Di + o) = df[s];
#pragma unroll
      for (int j = 0; j < 8; ++j) dlt += (float)of[s][j] * (float)df[s][j];
    }
    dlt = halfsum(dlt);
    if (hh == 0) {
      rowl[row] = qv ? -p.lse_in[((long)b * p.H + h) * p.Tq + row] * 1.4426950408889634f : -INFINITY;
      rowd[row] = qv ? -dlt : 0.f;
    }
  }
  __syncthreads();
  LdsOff<HD> off;
  off.init(lane);

  // ---- B: dQ of queries r0..r0+31 (S^T = K Q^T, dP^T = V dO^T - delta, dQ^T += K^T dS^T)
  if (r0 < p.Tq) {
    const float nlse2 = rowl[row];
    f32x16 acc[DT];
#pragma unroll
    for (int i = 0; i < DT; ++i) acc[i] = splat16(0.f);
    const int kend = CAUSAL ? min(p.Tk, r0 + 32 + p.causal_off) : p.Tk;
    const int nkt = kend > 0 ? cdiv(kend, 32) : 0;
    // one key tile; MASK only where the tile reaches past Tk or the causal diagonal (a uniform
    // branch between the two bodies: a predicated mask on every unrolled tile cost 48 VALU each)
    auto tile = [&](const int t, auto maskc) {
      constexpr bool MASK = decltype(maskc)::value;
      const bf16* Ks = Ki + 32 * t * HD;
      const bf16* Vs = Vi + 32 * t * HD;
      f32x16 s = mfma32(ld_row(Ks, off.row[0]), qf[0], splat16(0.f));
#pragma unroll
      for (int ks = 1; ks < KS; ++ks) s = mfma32(ld_row(Ks, off.row[ks]), qf[ks], s);
      f32x16 dp = mfma32(ld_row(Vs, off.row[0]), df[0], splat16(-dlt));
#pragma unroll
      for (int ks = 1; ks < KS; ++ks) dp = mfma32(ld_row(Vs, off.row[ks]), df[ks], dp);
      if constexpr (MASK) {
        const int ks0 = 32 * t;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = ks0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if (key >= p.Tk || (CAUSAL && key > row + p.causal_off)) s[r] = -INFINITY;
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) s[r] = fexp2(fmaf(s[r], c, nlse2)) * dp[r];
      const bf16x8 sa = pack_acc(s, 0), sb = pack_acc(s, 1);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        acc[dt] = mfma32(ld_tr(Ks, off.tra[dt], off.trb[dt]), sa, acc[dt]);
        acc[dt] = mfma32(ld_tr(Ks + 16 * HD, off.tra[dt], off.trb[dt]), sb, acc[dt]);
      }
    };
#pragma unroll
    for (int t = 0; t < TMAX / 32; ++t) {
      if (t >= nkt) break;
      const bool need = (32 * t + 32 > p.Tk) || (CAUSAL && 32 * t + 31 > r0 + p.causal_off);
      if (__builtin_amdgcn_readfirstlane(need)) tile(t, IC<1>{});
      else tile(t, IC<0>{});
    }
    if (row < p.Tq && SPA_DBG_BRH(b, row, p.Tq, h, p.H)) {
      bf16* o = p.dq + b * p.sdqb + (long)row * p.sdqt + h * p.sdqh;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          bf16x4 w;
#pragma unroll
          for (int i = 0; i < 4; ++i) w[i] = (bf16)(acc[dt][4 * g + i] * p.scale);
          *reinterpret_cast<bf16x4*>(o + 32 * dt + 8 * g + 4 * hh) = w;
        }
    }
  }

  // ---- C: dK / dV of keys r0..r0+31 (S = Q K^T, dP = dO V^T - delta, dV^T += dO^T P,
  //         dK^T += Q^T dS); rows of s / dp are queries 32t + 8g + 4hh + i (r = 4g + i)
  if (r0 < p.Tk) {
    f32x16 dkt[DT], dvt[DT];
#pragma unroll
    for (int i = 0; i < DT; ++i) dkt[i] = dvt[i] = splat16(0.f);
    const int qs = CAUSAL ? max(0, r0 - p.causal_off) : 0;
    const int nqt = cdiv(p.Tq, 32);
#pragma unroll
    for (int t = 0; t < TMAX / 32; ++t) {
      if (t < qs / 32) continue;
      if (t >= nqt) break;
      const bf16* Qs = Qi + 32 * t * HD;
      const bf16* Ds = Di + 32 * t * HD;
      f32x16 dp;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 dv = *reinterpret_cast<const f32x4*>(rowd + 32 * t + 8 * g + 4 * hh);
#pragma unroll
        for (int i = 0; i < 4; ++i) dp[4 * g + i] = dv[i];
      }
      f32x16 s = mfma32(ld_row(Qs, off.row[0]), kf[0], splat16(0.f));
#pragma unroll
      for (int ks = 1; ks < KS; ++ks) s = mfma32(ld_row(Qs, off.row[ks]), kf[ks], s);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) dp = mfma32(ld_row(Ds, off.row[ks]), vf[ks], dp);
      const int qt0 = 32 * t;
      if (CAUSAL && qt0 + p.causal_off < r0 + 31) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int qq = qt0 + 8 * (r >> 2) + 4 * hh + (r & 3);
          if (row > qq + p.causal_off) s[r] = -INFINITY;
        }
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 lv = *reinterpret_cast<const f32x4*>(rowl + 32 * t + 8 * g + 4 * hh);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * g + i;
          const float pr = fexp2(fmaf(s[r], c, lv[i]));  // queries >= Tq: -lse2 = -inf -> 0
          s[r] = pr;
          dp[r] = pr * dp[r];
        }
      }
      const bf16x8 pa = pack_acc(s, 0), pb = pack_acc(s, 1), sa = pack_acc(dp, 0), sb = pack_acc(dp, 1);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        dvt[dt] = mfma32(ld_tr(Ds, off.tra[dt], off.trb[dt]), pa, dvt[dt]);
        dvt[dt] = mfma32(ld_tr(Ds + 16 * HD, off.tra[dt], off.trb[dt]), pb, dvt[dt]);
      }
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        dkt[dt] = mfma32(ld_tr(Qs, off.tra[dt], off.trb[dt]), sa, dkt[dt]);
        dkt[dt] = mfma32(ld_tr(Qs + 16 * HD, off.tra[dt], off.trb[dt]), sb, dkt[dt]);
      }
    }
    store_kv_grad<HD>(p, dkt, true, b, h, row, 0, hh);
    store_kv_grad<HD>(p, dvt, false, b, h, row, 0, hh);
  }
}

// host side: one block per (b, h) (H == Hkv), Tq, Tk <= 256
void launch_bwd_short(AttnParams& p, bool causal, hipStream_t st) {
  p.hsplit = 1;
  if (causal) attn_bwd_short_kernel<64, true><<<p.B * p.H, 512, 0, st>>>(p);
  else attn_bwd_short_kernel<64, false><<<p.B * p.H, 512, 0, st>>>(p);
}

}  // namespace spa
