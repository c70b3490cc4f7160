// One-wave-per-SIMD dK/dV backward kernel (head dim 128), split from attention.hip so that this
// translation unit alone is built with the max-ILP machine scheduler (solvingpapers_amd/_build.py
// EXTRA_FLAGS): it issues every operand read of a chain before the chain, where the default
// scheduler re-used one register quad and waited out each LDS round trip.
#include "attn_params.h"

namespace spa {

// ---------------------------------------------------------------------------
// Backward dK/dV, one wave per SIMD with the whole register file (dkdv4, HD 128).
//
// Why: the paired kernel (dkdv3) holds 2 waves per SIMD and sits at the 256-register cap, so
// hipcc re-uses ONE register quad for every LDS operand of a chain -- ds_read, wait, MFMA,
// ds_read, wait, MFMA -- and each 32-cycle MFMA waits out a full LDS round trip. Here each
// SIMD runs one wave of 4 (256 threads, __launch_bounds__(256, 1): up to 512 registers), and
// every wave does all four products of its 32 keys with whole operand sets in registers:
//   per 32-row query sub-tile: Q rows (8 x b128) and dO rows (8 x b128) read up front ->
//   S chain (8 MFMA) and dP chain (8 MFMA) back to back -> the dO^T / Q^T transposed operands
//   (32 x tr_b64) issued before the softmax VALU -> dV^T (8 MFMA) and dK^T (8 MFMA) chains.
// Row constants start the accumulators: S = Q (c K)^T - lse2 with K pre-scaled by
// c = scale * log2(e) in registers (P = exp2(S) needs no FMA) and dP = dO V^T - delta.
// Q / dO tiles (64 rows) and their lse / delta are register-staged two tiles ahead through a
// 3-slot LDS ring (one barrier per tile). Causal: heaviest key blocks first; diagonal tiles
// masked. Built with the max-ILP machine scheduler (its own translation unit, see _build.py):
// the default one reuses one register quad per operand chain and waits on every LDS read.
// ---------------------------------------------------------------------------
template <int HD, bool CAUSAL>
__global__ __launch_bounds__(256, 1) void attn_bwd_dkdv4_kernel(AttnParams p) {
  static_assert(HD == 128, "dkdv4: head dim 128 (register budget sized for it)");
  constexpr int BMQ = 64, BNK = 128, KS = HD / 16, DT = HD / 32;
  constexpr int TQB = BMQ * HD * 2;                    // bytes of one 64-row image
  constexpr int SLOT = 2 * TQB + 2 * BMQ * 4;          // Q | dO | lse[64] | delta[64]
  // ONE LDS array: a second __shared__ object can make hipcc drain the DMA queue at ds_reads
  __shared__ __attribute__((aligned(1024))) char smem[3 * SLOT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5;
  const int nbh = p.Hkv * p.B;
  const int bh = blockIdx.x % nbh;
  const int rest = blockIdx.x / nbh;                   // causal: low key blocks (heaviest) first
  const int split = rest % p.hsplit, kb = rest / p.hsplit;
  const int hk = bh % p.Hkv, b = bh / p.Hkv;
  const int Gs = p.H / p.Hkv / p.hsplit;
  const int h0 = hk * (p.H / p.Hkv) + split * Gs;
  const int kw0 = __builtin_amdgcn_readfirstlane(kb * BNK + wave * 32);
  const int key = kw0 + (lane & 31);
  const bool kvalid = key < p.Tk;
  const float c = p.scale_log2;

  // K (pre-scaled by c) and V fragments of this lane's key: the B operands of S and dP
  bf16x8 kf[KS], vf[KS];
  {
    const bf16* kp = p.k + b * p.skb + (long)key * p.skt + hk * p.skh + 8 * hh;
    const bf16* vp = p.v + b * p.svb + (long)key * p.svt + hk * p.svh + 8 * hh;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      bf16x8 kr = kvalid ? *reinterpret_cast<const bf16x8*>(kp + 16 * s) : zero8();
#pragma unroll
      for (int j = 0; j < 8; ++j) kr[j] = (bf16)((float)kr[j] * c);
      kf[s] = kr;
      vf[s] = kvalid ? *reinterpret_cast<const bf16x8*>(vp + 16 * s) : zero8();
    }
  }
  f32x16 dkt[DT], dvt[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) { dkt[i] = splat16(0.f); dvt[i] = splat16(0.f); }

  int qstart = 0, wave_qstart = 0;
  if (CAUSAL) {
    qstart = max(0, kb * BNK - p.causal_off);
    wave_qstart = max(0, kw0 - p.causal_off);
  }
  const int t0 = qstart / BMQ;
  const int ntq = p.Tq > 0 ? cdiv(p.Tq, BMQ) : 0;
  const int nper = ntq - t0 > 0 ? ntq - t0 : 0;       // q-tiles per head
  const int total = nper * Gs;                          // (head, q-tile) iterations

  // register-staged tile loads (global -> 32 VGPRs -> ds_write, TileLoader): LDS-DMA would need
  // no registers, but hipcc waits vmcnt(0) before every ds_read_b64_tr_b16 while any LDS-DMA is
  // in flight (it cannot tell the DMA's slot from the one being read), which drains a prefetch
  // issued two tiles ahead on every sub-tile
  TileLoader<HD, BMQ, 256> lq_, ld_;
  lq_.init(p.sqt, tid);
  ld_.init(p.sdot, tid);
  float rl = 0.f, rd = 0.f;                            // raw row constants (tid < 64)
  int f_hg = 0, f_tq = 0;                              // (head group, q-tile) of the next fetch
  auto fetch = [&]() {
    const int h = h0 + f_hg;
    const int qq0 = (t0 + f_tq) * BMQ;
    lq_.load(p.q + b * p.sqb + h * p.sqh, p.sqt, qq0, p.Tq);
    ld_.load(p.dout + b * p.sdob + h * p.sdoh, p.sdot, qq0, p.Tq);
    if (tid < BMQ) {
      const long r = ((long)b * p.H + h) * p.Tq + min(qq0 + tid, p.Tq - 1);
      rl = p.lse_in[r];
      rd = p.delta[r];
    }
    if (++f_tq == nper) { f_tq = 0; ++f_hg; }
  };
  auto commit = [&](const int slot) {
    char* sl = smem + slot * SLOT;
    lq_.store(reinterpret_cast<bf16*>(sl));
    ld_.store(reinterpret_cast<bf16*>(sl + TQB));
    if (tid < BMQ) {                                   // rows >= Tq: zero Q / dO rows -> no effect
      reinterpret_cast<float*>(sl + 2 * TQB)[tid] = rl;
      reinterpret_cast<float*>(sl + 2 * TQB)[BMQ + tid] = rd;
    }
  };
  if (total > 0) {
    fetch();
    commit(0);
    if (total > 1) fetch();
  }
  __syncthreads();
  LdsOff<HD> off;
  off.init(lane);
  int c_tq = 0;                                        // q-tile index of the tile being computed
  // A 64-row tile = two 32-row query sub-tiles t, each: chains (S = Q (cK)^T and dP = dO V^T,
  // 16 MFMA) -> softmax VALU (P, dS) -> dV^T += dO^T P, dK^T += Q^T dS (16 MFMA). The sub-tiles
  // are interleaved -- chains(0), chains(1), softmax(0), dVdK(0), softmax(1), dVdK(1) -- in one
  // basic block, so the max-ILP scheduler can put each softmax's VALU beside MFMAs that do not
  // depend on it (the other sub-tile's chains / products) instead of idling the matrix pipe.
  struct Acc2 { f32x16 s, dp; };
  struct Ops4 { bf16x8 pa, pb, sa, sb; };
  auto chains = [&](const char* sl, const int t) {
    const bf16* Qs = reinterpret_cast<const bf16*>(sl);
    const bf16* Ds = reinterpret_cast<const bf16*>(sl + TQB);
    bf16x8 qa[KS], da[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qa[ks] = ld_row(Qs + 32 * t * HD, off.row[ks]);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) da[ks] = ld_row(Ds + 32 * t * HD, off.row[ks]);
    // chains start from zero (inline-0 accumulator): each element is read once by the VALU
    Acc2 r;
    r.s = mfma32(qa[0], kf[0], splat16(0.f));
#pragma unroll
    for (int ks = 1; ks < KS; ++ks) r.s = mfma32(qa[ks], kf[ks], r.s);
    r.dp = mfma32(da[0], vf[0], splat16(0.f));
#pragma unroll
    for (int ks = 1; ks < KS; ++ks) r.dp = mfma32(da[ks], vf[ks], r.dp);
    return r;
  };
  auto softmax = [&](const char* sl, const int qt0, const int t, const Acc2& a) {
    const float* lse = reinterpret_cast<const float*>(sl + 2 * TQB);
    const float* dlt = lse + BMQ;
    // register r <-> query row 32t + 8g + 4hh + i (r = 4g + i); P = exp2(S' - lse2),
    // dS = P (dP - delta). Causal: row offsets below d are masked (d <= 0 off the diagonal; a
    // branch-free select -- a wave-uniform branch made hipcc re-home the dK/dV accumulators)
    const int d = key - qt0 - 4 * hh - p.causal_off;
    f32x16 pr, ds;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 lv = *reinterpret_cast<const f32x4*>(lse + 32 * t + 8 * g + 4 * hh);
      const f32x4 dv = *reinterpret_cast<const f32x4*>(dlt + 32 * t + 8 * g + 4 * hh);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 4 * g + i;
        float e = fexp2(fmaf(lv[i], -1.4426950408889634f, a.s[r]));
        if (CAUSAL && (i + 8 * g) < d) e = 0.f;
        pr[r] = e;
        ds[r] = e * (a.dp[r] - dv[i]);
      }
    }
    return Ops4{pack_acc(pr, 0), pack_acc(pr, 1), pack_acc(ds, 0), pack_acc(ds, 1)};
  };
  auto products = [&](const char* sl, const int t, const Ops4& o) {
    const bf16* Qs = reinterpret_cast<const bf16*>(sl);
    const bf16* Ds = reinterpret_cast<const bf16*>(sl + TQB);
    bf16x8 dtr[2 * DT], qtr[2 * DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      dtr[2 * dt] = ld_tr(Ds + 32 * t * HD, off.tra[dt], off.trb[dt]);
      dtr[2 * dt + 1] = ld_tr(Ds + (32 * t + 16) * HD, off.tra[dt], off.trb[dt]);
      qtr[2 * dt] = ld_tr(Qs + 32 * t * HD, off.tra[dt], off.trb[dt]);
      qtr[2 * dt + 1] = ld_tr(Qs + (32 * t + 16) * HD, off.tra[dt], off.trb[dt]);
    }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      dvt[dt] = mfma32(dtr[2 * dt], o.pa, dvt[dt]);
      dvt[dt] = mfma32(dtr[2 * dt + 1], o.pb, dvt[dt]);
      dkt[dt] = mfma32(qtr[2 * dt], o.sa, dkt[dt]);
      dkt[dt] = mfma32(qtr[2 * dt + 1], o.sb, dkt[dt]);
    }
  };
  auto compute = [&](const int it, auto slotc) {
    constexpr int SL = decltype(slotc)::value;
    const char* sl = smem + SL * SLOT;
    const int qq0 = (t0 + c_tq) * BMQ;
    if (++c_tq == nper) c_tq = 0;
    if (kw0 >= p.Tk || (CAUSAL && qq0 + BMQ - 1 < wave_qstart)) return;
    const Acc2 a0 = chains(sl, 0);
    const Acc2 a1 = chains(sl, 1);
    const Ops4 o0 = softmax(sl, qq0, 0, a0);
    products(sl, 0, o0);
    const Ops4 o1 = softmax(sl, qq0 + 32, 1, a1);
    products(sl, 1, o1);
  };
  // interval it (tile it in slot it % 3): commit tile it+1 (fetched one interval ago) into slot
  // (it+1) % 3 -- last read in interval it-2 --, fetch tile it+2 into registers, compute tile it
  auto step = [&](const int it, auto slotc) {
    constexpr int SL = decltype(slotc)::value;
    if (it + 1 < total) {
      commit((SL + 1) % 3);
      if (it + 2 < total) fetch();
    }
    compute(it, slotc);
    __syncthreads();
  };
  for (int it = 0; it < total; it += 3) {
    step(it, IC<0>{});
    if (it + 1 < total) step(it + 1, IC<1>{});
    if (it + 2 < total) step(it + 2, IC<2>{});
  }
  store_kv_grad<HD>(p, dkt, true, b, hk, key, split, hh);
  store_kv_grad<HD>(p, dvt, false, b, hk, key, split, hh);
}


void launch_dkdv4_128(const AttnParams& p, bool causal, int grid, hipStream_t st) {
  if (causal) attn_bwd_dkdv4_kernel<128, true><<<grid, 256, 0, st>>>(p);
  else attn_bwd_dkdv4_kernel<128, false><<<grid, 256, 0, st>>>(p);
}

}  // namespace spa
