// Flash attention (forward + backward) for gfx950 on MFMA v_mfma_f32_32x32x16_bf16.
//
// Covers the attention variants of the catalogue with one kernel family:
//   causal MHA (gpt/gpt-jax.ipynb:344-353), GQA with RoPE'd q/k
//   (llama3/LLaMA-jax.ipynb:809-829 — no materialised repeat_kv: q-head h reads
//   kv-head h / (H/Hkv)), MQA (gemma/gemma.ipynb:238-256, Hkv = 1) and ViT
//   non-causal self-attention (vision transformer/ViT.ipynb:208,221; T = 197 tails).
//
// Design (wave64, 32x32x16 MFMA):
//  * Every product is arranged so the QUERY (fwd, dQ) or the KEY (dK/dV) sits on
//    the MFMA lane:  S^T = K Q^T,  O^T = V^T P^T  (fwd);  S = Q K^T, dV^T = dO^T P,
//    dK^T = Q^T dS  (dkdv);  dQ^T = K^T dS^T  (dq). The softmax state is then
//    lane-local, and P / dS feed the next MFMA straight from the accumulator
//    registers (their k order is permuted: element j of half h = row
//    16s + 8(j>>2) + 4h + (j&3); the other operand is read with the same order).
//  * The other operand of those "transposed" products (V^T, dO^T, Q^T, K^T) is read
//    with ds_read_b64_tr_b16 from the SAME row-major LDS image that the row
//    products read with ds_read_b128 — one image per tensor, written with 16-byte
//    stores. Images use 16-byte-chunk XOR swizzles chosen so both read kinds are
//    bank-conflict free (HD>=128: ch ^ ((r&3)<<2 | (r>>2)&3); HD=64: ch ^ ((r>>1&1)<<2 | (r>>2)&3)).
//  * Double-buffered K/V (or Q/dO) LDS tiles with register prefetch two tiles
//    ahead: one barrier per tile. Tiles come in through buffer loads whose
//    descriptor range ends at the last valid row, so ragged tails read zeros from
//    the hardware range check instead of per-lane branches.
//  * VALU budget (the loops are VALU-issue bound at 2 waves/SIMD, measured
//    SQ_INSTS_VALU ~10x SQ_INSTS_MFMA before this layout): bare v_exp_f32
//    (__builtin_amdgcn_exp2f, no denormal range reduction), one v_fma per score
//    (scale and max folded), masks only on the diagonal / tail tiles, the row max
//    combined across the two lane halves with v_permlane32_swap, the online-softmax
//    rescale deferred until some row max grew by more than 2^8 (T13: P <= 256 in
//    bf16, l and O in fp32), and the bwd row constants (-lse, -delta) preloaded
//    into the accumulators instead of zeros.
//  * Causal: heavy blocks first; waves skip tiles entirely above their diagonal.
//  * Backward = two deterministic kernels (no float atomics): dq (query-parallel,
//    also produces delta = rowsum(dO*O)) then dkdv (key-parallel, loops the GQA
//    group's q-heads so dK/dV of a kv-head are summed in registers). An optional
//    fused variant (dkdv<..., FUSEDQ>) adds dQ += dS K with fp32 atomics.
//  * q/k and v may have different head dims (HDK, HDV): DeepSeek-V3 MLA trains with
//    q/k = 128 nope + 64 rope = 192 and v = 128, run here with no zero padding (KS = HDK/16
//    k-steps for S, HDV/32 output tiles for O; a 192-wide row is staged in a 256-wide LDS
//    row so one swizzle serves every image).
//  * Attention-probability dropout (gpt/gpt-jax.ipynb:351, gemma/gemma.ipynb:248,
//    deepseekv3/deepseekv3.ipynb:1186) is fused: the keep mask of element (b, h, q, key) is a
//    32-bit counter hash of (seed, b, h, q, key), regenerated bit-identically by the forward
//    (query on the lane) and by both backward kernels (key on the lane) -- no (T, T) mask is
//    ever stored. P's row sum (the softmax normaliser, the lse) is taken BEFORE the mask;
//    O = (P * M / (1-p)) V, and the backward uses dS = P * (M * dP / (1-p) - delta) with
//    delta = rowsum(dO * O) unchanged.
// q/k/v/o and grads are addressed with (batch, seq, head) strides so the kernels
// read/write a fused [B, T, H + 2*Hkv, hd] qkv buffer in place.
#include "attn_common.h"
#include "attn_params.h"

SPA_DEBUG_TU("attention.hip")

namespace spa {



// ---- dropout counter hash (bit-identical in ops/attention.py dropout_keep_mask) ------
__device__ __forceinline__ unsigned mix32(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
// per (b, h) stream
__device__ __forceinline__ unsigned drop_base(const AttnParams& p, int b, int h) {
  unsigned lo = p.seed_lo, hi = p.seed_hi;
  if (p.seed_ptr) {
    const uint64_t sd = (uint64_t)*p.seed_ptr;
    lo = (unsigned)(sd & 0xffffffffu);
    hi = (unsigned)(sd >> 32);
  }
  return mix32(lo ^ mix32(hi + (unsigned)(b * p.H + h) * 0x9E3779B9U));
}
__device__ __forceinline__ bool drop_keep(unsigned base, int q, int key, unsigned thr) {
  return (mix32(base + (unsigned)q * 0x85EBCA6BU + (unsigned)key * 0xC2B2AE35U) >> 8) >= thr;
}



// Query-parallel block -> (q-block, batch, q-head). Default: q-block major over (b, h), heaviest
// causal q-blocks first. XCD-aware (p.xcd, needs B*Hkv % 8 == 0): the hardware hands block i to
// XCD i % 8, so logical tile L = (i % 8) * (grid / 8) + i / 8 gives each XCD a contiguous chunk
// of an order that is (b, kv-head) major: every q-head of a GQA group, and every q-block of it,
// runs on the XCD whose private L2 already holds that kv-head's K / V (LLaMA3-8B: one kv-head per
// XCD). Within an XCD the q-blocks still go heaviest first.
__device__ __forceinline__ void q_block_map(const AttnParams& p, int nqb, bool causal, int& qb, int& b, int& h,
                                            int bi, int nblk) {
  const int G = p.H / p.Hkv;
  if (p.xcd) {
    const int cpx = nblk / 8;
    const int L = (bi % 8) * cpx + bi / 8;
    const int per_unit = nqb * G;
    const int u = L / per_unit, rem = L % per_unit;
    const int qr = rem / G, g = rem % G;
    qb = causal ? nqb - 1 - qr : qr;
    b = u / p.Hkv;
    h = (u % p.Hkv) * G + g;
  } else {
    const int nbh = p.H * p.B;
    const int bh = bi % nbh;
    qb = bi / nbh;
    if (causal) qb = nqb - 1 - qb;  // heaviest q-blocks first
    h = bh % p.H;
    b = bh / p.H;
  }
}

// ---------------------------------------------------------------------------
// Forward: block = NW waves x 32 query rows; K/V tiles of BN keys.
// ---------------------------------------------------------------------------
template <int HDK, int HDV> constexpr int attn_bn() { return (HDK >= 256 || HDV >= 256) ? 32 : 64; }

#ifndef FWD_PV_SCHED
#define FWD_PV_SCHED 1
#endif
template <int HDK, int HDV, int NW, bool CAUSAL, bool DROP>
__global__ __launch_bounds__(NW * 64) void attn_fwd_kernel(AttnParams p) {
  constexpr int BN = attn_bn<HDK, HDV>(), NSUB = BN / 32, BM = 32 * NW, KS = HDK / 16, DT = HDV / 32;
  constexpr int NT = NW * 64, IK = img_w<HDK>(), IV = img_w<HDV>();
  constexpr int TK = BN * IK, TV = BN * IV, TB = TK + TV;
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * TB];  // [buf][K|V]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lq = lane & 31, hh = lane >> 5;
  const int nqb = cdiv(p.Tq, BM);
  // key split (p.ksplit > 1): block -> (query block, split si); si covers a contiguous share of
  // the query block's key tiles and writes fp32 partials (see AttnParams)
  const int si = blockIdx.x % p.ksplit;
  int qb, b, h;
  q_block_map(p, nqb, CAUSAL, qb, b, h, blockIdx.x / p.ksplit, gridDim.x / p.ksplit);
  const int hk = h / (p.H / p.Hkv);
  SPA_DBG_CHECK(qb, nqb);
  SPA_DBG_CHECK(hk, p.Hkv);
  (void)SPA_DBG_BRH(b, 0, 1, h, p.H);
  const int q0 = __builtin_amdgcn_readfirstlane(qb * BM + wave * 32);
  const int q = q0 + lq;
  const float c = p.scale_log2;
  const int vcol = blockIdx.y * p.vhalf;   // this launch slice's V / O columns
  unsigned dbase = 0;
  if constexpr (DROP) dbase = drop_base(p, b, h);

  bf16x8 qf[KS];
  {
    const bf16* qp = p.q + b * p.sqb + (long)q * p.sqt + h * p.sqh + 8 * hh;
#pragma unroll
    for (int s = 0; s < KS; ++s) qf[s] = q < p.Tq ? *reinterpret_cast<const bf16x8*>(qp + 16 * s) : zero8();
  }
  f32x16 o[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) o[i] = splat16(0.f);
  float m = -1e30f, l = 0.f;

  int kend = p.Tk;
  if (CAUSAL) kend = min(p.Tk, qb * BM + BM + p.causal_off);
  // a wave past the last query row (T = 197: rows 224..255 of a 256-row block) skips all MFMA
  // work but keeps staging tiles and meeting the block's barriers
  const int wave_kend = q0 >= p.Tq ? 0 : CAUSAL ? min(p.Tk, q0 + 32 + p.causal_off) : p.Tk;
  const int ntiles_all = kend > 0 ? cdiv(kend, BN) : 0;
  const int kper = cdiv(ntiles_all, p.ksplit);
  const int jbeg = min(ntiles_all, si * kper);
  const int ntiles = min(ntiles_all, jbeg + kper) - jbeg;
  const int kb0 = jbeg * BN;

  const bf16* kbase = p.k + b * p.skb + hk * p.skh;
  const bf16* vbase = p.v + b * p.svb + hk * p.svh + vcol;
  TileLoader<HDK, BN, NT> lk;
  TileLoader<HDV, BN, NT> lv;
  lk.init(p.skt, tid);
  lv.init(p.svt, tid);
  if (ntiles > 0) {
    lk.load(kbase, p.skt, kb0, p.Tk);
    lv.load(vbase, p.svt, kb0, p.Tk);
    lk.store(smem);
    lv.store(smem + TK);
    if (ntiles > 1) { lk.load(kbase, p.skt, kb0 + BN, p.Tk); lv.load(vbase, p.svt, kb0 + BN, p.Tk); }
  }
  __syncthreads();
  LdsOff<IK> offk;
  LdsOff<IV> offv;
  offk.init(lane);
  offv.init(lane);
  // causal / tail mask of one 32-key sub-tile (keys k0..k0+31): only on diagonal / tail
  // tiles, and kept apart from the softmax so the O-rescale code exists once (two merged
  // copies made hipcc re-home all of O with 64 v_mov per sub-tile)
  auto mask = [&](f32x16& s, const int k0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = k0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
      if (key >= p.Tk || (CAUSAL && key > q + p.causal_off)) s[r] = -INFINITY;
    }
  };
  // scores -> probabilities for one 32-key sub-tile: each sub-tile is its own online-softmax step
  auto softmax = [&](f32x16& s) {
    float mx = s[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, s[r]);
    const float mxs = halfmax(mx) * c;
    // per-lane (exec-masked) rescale: both lane halves of a row take the same decision.
    // A wave-uniform branch here made hipcc re-home all of O (64 v_mov per sub-tile).
    if (mxs > m + kRescaleThr) {
      const float alpha = fexp2(m - mxs);
      l *= alpha;
#pragma unroll
      for (int i = 0; i < DT; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[i][r] *= alpha;
      m = mxs;
    }
    const float nm = -m;
    float ls = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float e = fexp2(fmaf(s[r], c, nm));
      s[r] = e;
      ls += e;
    }
    l += ls;
  };
  // P -> P * M / (1-p): after the row sum, so the normaliser (and the lse) is the undropped one
  auto dropout = [&](f32x16& s, const int k0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = k0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
      s[r] = drop_keep(dbase, q, key, p.drop_thr) ? s[r] * p.drop_scale : 0.f;
    }
  };
  // body(j, buffer) with the buffer a compile-time constant (loop unrolled x2) so
  // every LDS address is a precomputed lane offset + an immediate
  auto body = [&](const int j, auto bufc) {
    constexpr int BUF = decltype(bufc)::value;
    const int k0 = kb0 + j * BN;
    const bf16* Ks = smem + BUF * TB;
    const bf16* Vs = Ks + TK;
    if (j + 1 < ntiles) {
      bf16* Kn = smem + (1 - BUF) * TB;
      lk.store(Kn);
      lv.store(Kn + TK);
      if (j + 2 < ntiles) { lk.load(kbase, p.skt, k0 + 2 * BN, p.Tk); lv.load(vbase, p.svt, k0 + 2 * BN, p.Tk); }
    }
#pragma unroll
    for (int t = 0; t < NSUB; ++t) {
      const int ks0 = k0 + 32 * t;
      if (ks0 < wave_kend) {
        // every K-row operand read issued before the chain (sched_group_barrier: DS reads, then
        // MFMAs): hipcc's default order re-used one register quad and waited out each LDS read
        bf16x8 kr[KS];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) kr[ks] = ld_row(Ks + 32 * t * IK, offk.row[ks]);
        f32x16 s = mfma32(kr[0], qf[0], splat16(0.f));
#pragma unroll
        for (int ks = 1; ks < KS; ++ks) s = mfma32(kr[ks], qf[ks], s);
        __builtin_amdgcn_sched_group_barrier(0x100, KS, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, KS, 0);
        const bool need_mask = (ks0 + 32 > p.Tk) || (CAUSAL && ks0 + 31 > q0 + p.causal_off);
        if (need_mask) mask(s, ks0);
        softmax(s);
        if constexpr (DROP) dropout(s, ks0);
        const bf16x8 pa = pack_acc(s, 0), pb = pack_acc(s, 1);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          o[dt] = mfma32(ld_tr(Vs + 32 * t * IV, offv.tra[dt], offv.trb[dt]), pa, o[dt]);
          o[dt] = mfma32(ld_tr(Vs + (32 * t + 16) * IV, offv.tra[dt], offv.trb[dt]), pb, o[dt]);
        }
        if (FWD_PV_SCHED) chain_sched<2 * DT, 2, 3>();
      }
    }
    __syncthreads();
  };
  // the loop's prefetch is conditional (no loads on the last tiles), so hipcc cannot count the
  // q-fragment loads of the prologue past it and waited vmcnt(0) -- draining the prefetch just
  // issued -- at every tile's first MFMA. An empty asm that USES the fragments makes it wait for
  // them here, once (an asm s_waitcnt is invisible to its waitcnt pass)
#pragma unroll
  for (int s = 0; s < KS; ++s) asm volatile("" ::"v"(qf[s]));
  for (int j = 0; j < ntiles; j += 2) {
    body(j, IC<0>{});
    if (j + 1 < ntiles) body(j + 1, IC<1>{});
  }
  l = halfsum(l);
  if (p.ksplit > 1) {      // fp32 partial: unnormalised O and the (m, l) softmax state
    if (q < p.Tq && SPA_DBG_OK(si, p.ksplit)) {
      const long row = (((long)si * p.B + b) * p.H + h) * p.Tq + q;
      SPA_DBG_CHECK(row, (long)p.ksplit * p.B * p.H * p.Tq);
      float* dst = p.part + row * p.part_ld + vcol;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          f32x4 w;
#pragma unroll
          for (int i = 0; i < 4; ++i) w[i] = o[dt][4 * g + i];
          *reinterpret_cast<f32x4*>(dst + 32 * dt + 8 * g + 4 * hh) = w;
        }
      if (hh == 0 && blockIdx.y == 0) {
        float2 ml;
        ml.x = m;
        ml.y = l;
        reinterpret_cast<float2*>(p.mlpart)[row] = ml;
      }
    }
    return;
  }
  const float inv = l > 0.f ? 1.f / l : 0.f;
  if (q < p.Tq && SPA_DBG_BRH(b, q, p.Tq, h, p.H)) {
    bf16* op = p.out + b * p.sob + (long)q * p.sot + h * p.soh + vcol;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 w;
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = (bf16)(o[dt][4 * g + i] * inv);
        *reinterpret_cast<bf16x4*>(op + 32 * dt + 8 * g + 4 * hh) = w;
      }
    if (hh == 0 && p.lse)
      p.lse[((long)b * p.H + h) * p.Tq + q] = (l > 0.f) ? (m + __log2f(l)) * 0.69314718055994531f : INFINITY;
  }
}

// ---------------------------------------------------------------------------
// Forward at head dim 256 (Gemma MQA), S computed once per row group: 8 waves = 4 row groups of
// 32 queries x 2 roles. The leader (waves 0-3) holds its rows' Q fragments, computes S = K Q^T
// and the online softmax, writes P (bf16, MFMA-operand order) and the per-row rescale factor to
// LDS, and accumulates O columns 0..127; the follower (waves 4-7, the leader's SIMD partner)
// rescales and accumulates O columns 128..255 from that P. Against the split-V launch (two column
// halves that each recompute S: 1.5x the MFMA work, 24 KB of LDS reads per wave per tile) this
// is 1x the MFMA work and 136 KB of LDS reads per CU per 32-key tile instead of 192 KB.
// One barrier per interval, V lagging K by one tile:
//   interval j, leader:   O[:, :128]  += V(j-1)^T P(j-1)  |  S(j) -> softmax -> P(j), alpha(j) -> LDS
//   interval j, follower: O[:, 128:] *= alpha(j-1);  O[:, 128:] += V(j-1)^T P(j-1)
// K(j) and V(j-1) are resident in interval j (2-deep rings each), which commits K(j+1) and V(j).
// Key split (p.ksplit) as attn_fwd_kernel: fp32 partials of both column halves + (m, l).
// ---------------------------------------------------------------------------
template <bool CAUSAL>
__global__ __launch_bounds__(512) void attn_fwd256p_kernel(AttnParams p) {
  constexpr int HD = 256, BN = 32, BM = 128, KS = HD / 16, DH = 4, NT = 512;
  constexpr int TI = BN * HD;                 // one 32-key K or V image (elements)
  constexpr int PS = 4 * 2 * 64 * 8;          // one P slot: [group][half][lane][8]
  __shared__ __attribute__((aligned(16))) bf16 smem[4 * TI + 2 * PS];   // K[2] | V[2] | P[2]
  __shared__ __attribute__((aligned(16))) float arow[2][4][64];        // [slot][group][lane] alpha
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave & 3, role = wave >> 2;
  const int lq = lane & 31, hh = lane >> 5;
  const int nqb = cdiv(p.Tq, BM);
  const int si = blockIdx.x % p.ksplit;
  int qb, b, h;
  q_block_map(p, nqb, CAUSAL, qb, b, h, blockIdx.x / p.ksplit, gridDim.x / p.ksplit);
  const int hk = h / (p.H / p.Hkv);
  SPA_DBG_CHECK(qb, nqb);
  SPA_DBG_CHECK(hk, p.Hkv);
  (void)SPA_DBG_BRH(b, 0, 1, h, p.H);
  const int q0 = __builtin_amdgcn_readfirstlane(qb * BM + grp * 32);
  const int q = q0 + lq;
  const float c = p.scale_log2;

  int kend = p.Tk;
  if (CAUSAL) kend = min(p.Tk, qb * BM + BM + p.causal_off);
  const int wave_kend = q0 >= p.Tq ? 0 : CAUSAL ? min(p.Tk, q0 + 32 + p.causal_off) : p.Tk;
  const int ntiles_all = kend > 0 ? cdiv(kend, BN) : 0;
  const int kper = cdiv(ntiles_all, p.ksplit);
  const int jbeg = min(ntiles_all, si * kper);
  const int ntiles = min(ntiles_all, jbeg + kper) - jbeg;
  const int kb0 = jbeg * BN;

  const bf16* kbase = p.k + b * p.skb + hk * p.skh;
  const bf16* vbase = p.v + b * p.svb + hk * p.svh;
  TileLoader<HD, BN, NT> lk, lv;
  lk.init(p.skt, tid);
  lv.init(p.svt, tid);
  if (ntiles > 0) {
    lk.load(kbase, p.skt, kb0, p.Tk);
    lk.store(smem);
    lv.load(vbase, p.svt, kb0, p.Tk);
    if (ntiles > 1) lk.load(kbase, p.skt, kb0 + BN, p.Tk);
  }
  bf16x8 qf[KS];
  if (role == 0) {
    const bf16* qp = p.q + b * p.sqb + (long)q * p.sqt + h * p.sqh + 8 * hh;
#pragma unroll
    for (int s = 0; s < KS; ++s) qf[s] = q < p.Tq ? *reinterpret_cast<const bf16x8*>(qp + 16 * s) : zero8();
  }
  __syncthreads();
  LdsOff<HD> off;
  off.init(lane);
  f32x16 o[DH];
#pragma unroll
  for (int i = 0; i < DH; ++i) o[i] = splat16(0.f);
  float m = -1e30f, l = 0.f;
  bf16* pme = smem + 4 * TI + grp * (2 * 64 * 8) + lane * 8;   // + slot * PS + half * 512

  auto interval = [&](const int j, auto bufc, auto rolec) {
    constexpr int BUF = decltype(bufc)::value, ROLE = decltype(rolec)::value;
    if (j + 1 < ntiles) lk.store(smem + (1 - BUF) * TI);          // K(j+1)
    if (j < ntiles) lv.store(smem + (2 + BUF) * TI);              // V(j)
    if (j + 2 < ntiles) lk.load(kbase, p.skt, kb0 + (j + 2) * BN, p.Tk);
    if (j + 1 < ntiles) lv.load(vbase, p.svt, kb0 + (j + 1) * BN, p.Tk);
    const bf16* Vp = smem + (3 - BUF) * TI;                        // V(j-1)
    const bf16* pr = pme + (1 - BUF) * PS;                         // P(j-1)
    if (j >= 1 && kb0 + (j - 1) * BN < wave_kend) {
      if constexpr (ROLE == 1) {
        const float al = arow[1 - BUF][grp][lane];
#pragma unroll
        for (int i = 0; i < DH; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[i][r] *= al;
      }
      const bf16x8 pa = *reinterpret_cast<const bf16x8*>(pr);
      const bf16x8 pb = *reinterpret_cast<const bf16x8*>(pr + 512);
#pragma unroll
      for (int dt = 0; dt < DH; ++dt) {
        o[dt] = mfma32(ld_tr(Vp, off.tra[dt + DH * ROLE], off.trb[dt + DH * ROLE]), pa, o[dt]);
        o[dt] = mfma32(ld_tr(Vp + 16 * HD, off.tra[dt + DH * ROLE], off.trb[dt + DH * ROLE]), pb, o[dt]);
      }
      chain_sched<2 * DH, 2, 3, 2>();
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (ROLE == 0) {
      const int k0 = kb0 + j * BN;
      if (j < ntiles && k0 < wave_kend) {
        const bf16* Ks = smem + BUF * TI;
        bf16x8 kr[KS];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) kr[ks] = ld_row(Ks, off.row[ks]);
        f32x16 s = mfma32(kr[0], qf[0], splat16(0.f));
#pragma unroll
        for (int ks = 1; ks < KS; ++ks) s = mfma32(kr[ks], qf[ks], s);
        __builtin_amdgcn_sched_group_barrier(0x100, KS, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, KS, 0);
        if ((k0 + 32 > p.Tk) || (CAUSAL && k0 + 31 > q0 + p.causal_off)) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = k0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
            if (key >= p.Tk || (CAUSAL && key > q + p.causal_off)) s[r] = -INFINITY;
          }
        }
        float mx = s[0];
#pragma unroll
        for (int r = 1; r < 16; ++r) mx = fmaxf(mx, s[r]);
        const float mxs = halfmax(mx) * c;
        float al = 1.f;
        if (mxs > m + kRescaleThr) {
          al = fexp2(m - mxs);
          l *= al;
#pragma unroll
          for (int i = 0; i < DH; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) o[i][r] *= al;
          m = mxs;
        }
        const float nm = -m;
        float ls = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = fexp2(fmaf(s[r], c, nm));
          s[r] = e;
          ls += e;
        }
        l += ls;
        bf16* pw = pme + BUF * PS;
        *reinterpret_cast<bf16x8*>(pw) = pack_acc(s, 0);
        *reinterpret_cast<bf16x8*>(pw + 512) = pack_acc(s, 1);
        arow[BUF][grp][lane] = al;
      }
    }
    __syncthreads();
  };
  if (role == 0) {
#pragma unroll
    for (int s = 0; s < KS; ++s) asm volatile("" ::"v"(qf[s]));
    for (int j = 0; j <= ntiles; j += 2) {
      interval(j, IC<0>{}, IC<0>{});
      if (j + 1 <= ntiles) interval(j + 1, IC<1>{}, IC<0>{});
    }
  } else {
    for (int j = 0; j <= ntiles; j += 2) {
      interval(j, IC<0>{}, IC<1>{});
      if (j + 1 <= ntiles) interval(j + 1, IC<1>{}, IC<1>{});
    }
  }
  // the follower takes the row sum from its leader (arow is free after the last barrier)
  if (role == 0) {
    l = halfsum(l);
    arow[0][grp][lane] = l;
  }
  __syncthreads();
  if (role == 1) l = arow[0][grp][lane];
  const int vcol = role * 128;
  if (p.ksplit > 1) {
    if (q < p.Tq && SPA_DBG_OK(si, p.ksplit)) {
      const long row = (((long)si * p.B + b) * p.H + h) * p.Tq + q;
      SPA_DBG_CHECK(row, (long)p.ksplit * p.B * p.H * p.Tq);
      float* dst = p.part + row * p.part_ld + vcol;
#pragma unroll
      for (int dt = 0; dt < DH; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          f32x4 w;
#pragma unroll
          for (int i = 0; i < 4; ++i) w[i] = o[dt][4 * g + i];
          *reinterpret_cast<f32x4*>(dst + 32 * dt + 8 * g + 4 * hh) = w;
        }
      if (hh == 0 && role == 0) {
        float2 ml;
        ml.x = m;
        ml.y = l;
        reinterpret_cast<float2*>(p.mlpart)[row] = ml;
      }
    }
    return;
  }
  const float inv = l > 0.f ? 1.f / l : 0.f;
  if (q < p.Tq && SPA_DBG_BRH(b, q, p.Tq, h, p.H)) {
    bf16* op = p.out + b * p.sob + (long)q * p.sot + h * p.soh + vcol;
#pragma unroll
    for (int dt = 0; dt < DH; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 w;
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = (bf16)(o[dt][4 * g + i] * inv);
        *reinterpret_cast<bf16x4*>(op + 32 * dt + 8 * g + 4 * hh) = w;
      }
    if (hh == 0 && role == 0 && p.lse)
      p.lse[((long)b * p.H + h) * p.Tq + q] = (l > 0.f) ? (m + __log2f(l)) * 0.69314718055994531f : INFINITY;
  }
}

// ---------------------------------------------------------------------------
// Backward dQ (query-parallel; also writes delta = rowsum(dO*O)).
//   S^T = K Q^T ; P^T = exp2(S^T*c - lse2) ; dP^T = V dO^T - delta ; dS^T = P^T dP^T
//   dQ^T += K^T dS^T   (K^T via tr reads of the K image)
// DROP: dP^T = M * (V dO^T) / (1-p) - delta  (the accumulator starts at 0, not -delta)
// ---------------------------------------------------------------------------
template <int HDK, int HDV, int NW, bool CAUSAL, bool DROP>
__global__ __launch_bounds__(NW * 64) void attn_bwd_dq_kernel(AttnParams p) {
  constexpr int BN = attn_bn<HDK, HDV>(), NSUB = BN / 32, BM = 32 * NW, KSK = HDK / 16, KSV = HDV / 16;
  constexpr int DT = HDK / 32, NT = NW * 64, IK = img_w<HDK>(), IV = img_w<HDV>();
  constexpr int TK = BN * IK, TV = BN * IV, TB = TK + TV;
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * TB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lq = lane & 31, hh = lane >> 5;
  const int nqb = cdiv(p.Tq, BM);
  const int si = blockIdx.x % p.ksplit;     // key split: see the forward kernel
  int qb, b, h;
  q_block_map(p, nqb, CAUSAL, qb, b, h, blockIdx.x / p.ksplit, gridDim.x / p.ksplit);
  const int hk = h / (p.H / p.Hkv);
  SPA_DBG_CHECK(qb, nqb);
  SPA_DBG_CHECK(hk, p.Hkv);
  (void)SPA_DBG_BRH(b, 0, 1, h, p.H);
  const int q0 = __builtin_amdgcn_readfirstlane(qb * BM + wave * 32);
  const int q = q0 + lq;
  const bool qvalid = q < p.Tq;
  const float c = p.scale_log2;
  unsigned dbase = 0;
  if constexpr (DROP) dbase = drop_base(p, b, h);

  bf16x8 qf[KSK], df[KSV];
  float dlt = 0.f;
  {
    const bf16* qp = p.q + b * p.sqb + (long)q * p.sqt + h * p.sqh + 8 * hh;
    const bf16* dp = p.dout + b * p.sdob + (long)q * p.sdot + h * p.sdoh + 8 * hh;
    const bf16* op = p.o + b * p.sob + (long)q * p.sot + h * p.soh + 8 * hh;
#pragma unroll
    for (int s = 0; s < KSK; ++s) qf[s] = qvalid ? *reinterpret_cast<const bf16x8*>(qp + 16 * s) : zero8();
#pragma unroll
    for (int s = 0; s < KSV; ++s) {
      df[s] = qvalid ? *reinterpret_cast<const bf16x8*>(dp + 16 * s) : zero8();
      const bf16x8 ov = qvalid ? *reinterpret_cast<const bf16x8*>(op + 16 * s) : zero8();
#pragma unroll
      for (int j = 0; j < 8; ++j) dlt += (float)ov[j] * (float)df[s][j];
    }
    dlt = halfsum(dlt);
  }
  const long srow = ((long)b * p.H + h) * p.Tq + q;
  if (qvalid && hh == 0 && si == 0 && SPA_DBG_OK(srow, (long)p.B * p.H * p.Tq)) p.delta[srow] = dlt;
  const float nlse2 = qvalid ? -p.lse_in[srow] * 1.4426950408889634f : -INFINITY;
  f32x16 acc[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) acc[i] = splat16(0.f);

  int kend = p.Tk;
  if (CAUSAL) kend = min(p.Tk, qb * BM + BM + p.causal_off);
  // a wave past the last query row (T = 197: rows 224..255 of a 256-row block) skips all MFMA
  // work but keeps staging tiles and meeting the block's barriers
  const int wave_kend = q0 >= p.Tq ? 0 : CAUSAL ? min(p.Tk, q0 + 32 + p.causal_off) : p.Tk;
  const int ntiles_all = kend > 0 ? cdiv(kend, BN) : 0;
  const int kper = cdiv(ntiles_all, p.ksplit);
  const int jbeg = min(ntiles_all, si * kper);
  const int ntiles = min(ntiles_all, jbeg + kper) - jbeg;
  const int kb0 = jbeg * BN;
  const bf16* kbase = p.k + b * p.skb + hk * p.skh;
  const bf16* vbase = p.v + b * p.svb + hk * p.svh;
  TileLoader<HDK, BN, NT> lk;
  TileLoader<HDV, BN, NT> lv;
  lk.init(p.skt, tid);
  lv.init(p.svt, tid);
  if (ntiles > 0) {
    lk.load(kbase, p.skt, kb0, p.Tk);
    lv.load(vbase, p.svt, kb0, p.Tk);
    lk.store(smem);
    lv.store(smem + TK);
    if (ntiles > 1) { lk.load(kbase, p.skt, kb0 + BN, p.Tk); lv.load(vbase, p.svt, kb0 + BN, p.Tk); }
  }
  __syncthreads();
  LdsOff<IK> offk;
  LdsOff<IV> offv;
  offk.init(lane);
  offv.init(lane);
  auto mask = [&](f32x16& s, const int k0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = k0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
      if (key >= p.Tk || (CAUSAL && key > q + p.causal_off)) s[r] = -INFINITY;
    }
  };
  // one 32-key sub-tile: s <- dS^T = P^T (dP^T - delta)   (dp already carries -delta)
  auto dsoft = [&](f32x16& s, const f32x16& dp) {
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = fexp2(fmaf(s[r], c, nlse2)) * dp[r];
  };
  auto body = [&](const int j, auto bufc) {
    constexpr int BUF = decltype(bufc)::value;
    const int k0 = kb0 + j * BN;
    const bf16* Ks = smem + BUF * TB;
    const bf16* Vs = Ks + TK;
    if (j + 1 < ntiles) {
      bf16* Kn = smem + (1 - BUF) * TB;
      lk.store(Kn);
      lv.store(Kn + TK);
      if (j + 2 < ntiles) { lk.load(kbase, p.skt, k0 + 2 * BN, p.Tk); lv.load(vbase, p.svt, k0 + 2 * BN, p.Tk); }
    }
#pragma unroll
    for (int t = 0; t < NSUB; ++t) {
      const int ks0 = k0 + 32 * t;
      if (ks0 < wave_kend) {
        // K rows up front, V rows issued between the S MFMAs (sched_group_barrier), so neither
        // chain waits out an LDS round trip per MFMA
        bf16x8 kr[KSK], vr[KSV];
#pragma unroll
        for (int ks = 0; ks < KSK; ++ks) kr[ks] = ld_row(Ks + 32 * t * IK, offk.row[ks]);
#pragma unroll
        for (int ks = 0; ks < KSV; ++ks) vr[ks] = ld_row(Vs + 32 * t * IV, offv.row[ks]);
        f32x16 s = mfma32(kr[0], qf[0], splat16(0.f));
#pragma unroll
        for (int ks = 1; ks < KSK; ++ks) s = mfma32(kr[ks], qf[ks], s);
        f32x16 dp = mfma32(vr[0], df[0], splat16(DROP ? 0.f : -dlt));
#pragma unroll
        for (int ks = 1; ks < KSV; ++ks) dp = mfma32(vr[ks], df[ks], dp);
        constexpr int KMIN = KSK < KSV ? KSK : KSV;
        __builtin_amdgcn_sched_group_barrier(0x100, KSK, 0);
#pragma unroll
        for (int ks = 0; ks < KMIN; ++ks) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        if constexpr (KSK > KSV) __builtin_amdgcn_sched_group_barrier(0x008, KSK - KSV, 0);
        if constexpr (KSV > KSK) __builtin_amdgcn_sched_group_barrier(0x100, KSV - KSK, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, KSV, 0);
        if constexpr (DROP) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = ks0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
            dp[r] = (drop_keep(dbase, q, key, p.drop_thr) ? dp[r] * p.drop_scale : 0.f) - dlt;
          }
        }
        const bool need_mask = (ks0 + 32 > p.Tk) || (CAUSAL && ks0 + 31 > q0 + p.causal_off);
        if (need_mask) mask(s, ks0);
        dsoft(s, dp);
        const bf16x8 sa = pack_acc(s, 0), sb = pack_acc(s, 1);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          acc[dt] = mfma32(ld_tr(Ks + 32 * t * IK, offk.tra[dt], offk.trb[dt]), sa, acc[dt]);
          acc[dt] = mfma32(ld_tr(Ks + (32 * t + 16) * IK, offk.tra[dt], offk.trb[dt]), sb, acc[dt]);
        }
        if (FWD_PV_SCHED) chain_sched<2 * DT, 2, 3>();
      }
    }
    __syncthreads();
  };
  for (int j = 0; j < ntiles; j += 2) {
    body(j, IC<0>{});
    if (j + 1 < ntiles) body(j + 1, IC<1>{});
  }
  if (qvalid && !SPA_DBG_BRH(b, q, p.Tq, h, p.H)) return;
  if (qvalid && p.ksplit > 1) {   // fp32 partial (unscaled), summed by attn_dq_reduce_kernel
    float* dst = p.part + ((((long)si * p.B + b) * p.Tq + q) * p.H + h) * p.part_ld;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4 w;
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = acc[dt][4 * g + i];
        *reinterpret_cast<f32x4*>(dst + 32 * dt + 8 * g + 4 * hh) = w;
      }
  } else if (qvalid) {
    bf16* op = p.dq + b * p.sdqb + (long)q * p.sdqt + h * p.sdqh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 w;
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = (bf16)(acc[dt][4 * g + i] * p.scale);
        *reinterpret_cast<bf16x4*>(op + 32 * dt + 8 * g + 4 * hh) = w;
      }
  }
}

// ---------------------------------------------------------------------------
// Key-split merges. Forward: per row, M = max_s m_s, w_s = 2^(m_s - M), O = sum_s w_s O_s /
// sum_s w_s l_s (m in the kernel's log2-scaled units), lse = (M + log2 L) ln 2. dQ: sum of the
// partials times the softmax scale. One thread per 8 columns of a row.
// ---------------------------------------------------------------------------
template <int HDV>
__global__ __launch_bounds__(256) void attn_fwd_merge_kernel(AttnParams p) {
  constexpr int CPR = HDV / 8;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const long rows = (long)p.B * p.H * p.Tq;
  if (idx >= rows * CPR) return;
  const long row = idx / CPR;                 // (b, h, q)
  const int c8 = (int)(idx % CPR) * 8;
  const int q = (int)(row % p.Tq);
  const int bh = (int)(row / p.Tq), h = bh % p.H, b = bh / p.H;
  const float2* ml = reinterpret_cast<const float2*>(p.mlpart);
  float M = -INFINITY;
  for (int s = 0; s < p.ksplit; ++s) {
    const float2 v = ml[(long)s * rows + row];
    if (v.y > 0.f) M = fmaxf(M, v.x);
  }
  float L = 0.f, acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0.f;
  for (int s = 0; s < p.ksplit; ++s) {
    const float2 v = ml[(long)s * rows + row];
    if (!(v.y > 0.f)) continue;
    const float w = exp2f(v.x - M);
    L += w * v.y;
    const float* src = p.part + ((long)s * rows + row) * p.part_ld + c8;
    const f32x4 a = *reinterpret_cast<const f32x4*>(src), bq = *reinterpret_cast<const f32x4*>(src + 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc[i] += w * a[i];
      acc[4 + i] += w * bq[i];
    }
  }
  const float inv = L > 0.f ? 1.f / L : 0.f;
  bf16x8 o;
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = (bf16)(acc[i] * inv);
  if (!SPA_DBG_BRH(b, q, p.Tq, h, p.H)) return;
  *reinterpret_cast<bf16x8*>(p.out + b * p.sob + (long)q * p.sot + h * p.soh + c8) = o;
  if (c8 == 0 && p.lse) p.lse[row] = L > 0.f ? (M + __log2f(L)) * 0.69314718055994531f : INFINITY;
}

template <int HDK>
__global__ __launch_bounds__(256) void attn_dq_reduce_kernel(AttnParams p) {
  constexpr int CPR = HDK / 8;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const long rows = (long)p.B * p.Tq * p.H;
  if (idx >= rows * CPR) return;
  const long row = idx / CPR;                 // (b, q, h)
  const int c8 = (int)(idx % CPR) * 8;
  const int h = (int)(row % p.H);
  const long bq = row / p.H;
  const int q = (int)(bq % p.Tq), b = (int)(bq / p.Tq);
  float acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0.f;
  for (int s = 0; s < p.ksplit; ++s) {
    const float* src = p.part + ((long)s * rows + row) * p.part_ld + c8;
    const f32x4 a = *reinterpret_cast<const f32x4*>(src), bb = *reinterpret_cast<const f32x4*>(src + 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc[i] += a[i];
      acc[4 + i] += bb[i];
    }
  }
  bf16x8 o;
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = (bf16)(acc[i] * p.scale);
  if (!SPA_DBG_BRH(b, q, p.Tq, h, p.H)) return;
  *reinterpret_cast<bf16x8*>(p.dq + b * p.sdqb + (long)q * p.sdqt + h * p.sdqh + c8) = o;
}

// ---------------------------------------------------------------------------
// Backward dK/dV: key-block parallel (4 waves x 32 keys), key on the lane.
//   S = Q K^T, dP = dO V^T - delta   (A = Q / dO row reads, B = K / V fragments in regs;
//                                     the dP accumulator starts at -delta of its row)
//   dV^T += dO^T P, dK^T += Q^T dS   (A = tr reads of the Q / dO images, B = accumulators)
// Loops over the q-heads sharing this kv-head (GQA) so the group sum stays in regs.
// DROP: dV^T += dO^T (P M / (1-p)); dS = P (M dP / (1-p) - delta), M regenerated by hash.
// ---------------------------------------------------------------------------
template <int HDK, int HDV, bool CAUSAL, int MT, bool FUSEDQ, bool DROP, bool DSOUT = false>
__global__ __launch_bounds__(256) void attn_bwd_dkdv_kernel(AttnParams p) {
  // MT 32-row q sub-tiles per iteration (more MFMA work per barrier / LDS fill)
  constexpr int BMQ = 32 * MT, BNK = 128, KSK = HDK / 16, KSV = HDV / 16, DTK = HDK / 32, DTV = HDV / 32;
  constexpr int NT = 256, IK = img_w<HDK>(), IV = img_w<HDV>();
  constexpr int TQ = BMQ * IK, TD = BMQ * IV, TB = TQ + TD;
  static_assert(!FUSEDQ || HDK == HDV, "fused dQ path: equal head dims only");
  // FUSEDQ: dQ computed here too (dQ += dS K over this block's 128 keys, fp32 atomics into
  // p.dqacc) -> 5 MFMA products per tile instead of 7 for the split dq + dkdv kernels.
  // dS crosses LDS once ([key][q] image, transposed reads), K sits in a [key][d] image.
  constexpr int KIMG = FUSEDQ ? BNK * IK : 8, DSIMG = FUSEDQ ? BNK * 64 : 8;
  // VLDS (head dim 256, one wave per SIMD): the V fragments of the block's 128 keys live in an
  // LDS image instead of 64 VGPRs, which leaves the registers to request every chain's LDS
  // operands ahead (chain_sched); without them hipcc re-used one operand quad per chain and
  // waited out each LDS read before each MFMA (a bare 1-wave SIMD has nothing to overlap it)
  constexpr bool VLDS = HDK == 256 && HDV == 256 && !FUSEDQ && !DROP;
  constexpr int VIMG = VLDS ? BNK * IV : 8;
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * TB + KIMG + DSIMG + VIMG];  // [buf][Q|dO] | K | dS | V
  bf16* kimg = smem + 2 * TB;
  bf16* dsimg = kimg + KIMG;
  bf16* vimg = dsimg + DSIMG + (long)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * 32 * IV;  // this wave's keys
  __shared__ __attribute__((aligned(16))) float rowc[2][2 * BMQ];  // [buf][-lse2 | -delta]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lk = lane & 31, hh = lane >> 5;
  const int nbh = p.Hkv * p.B;
  const int bh = blockIdx.x % nbh;
  const int rest = blockIdx.x / nbh;  // causal: low key blocks are heaviest, launched first
  const int split = rest % p.hsplit, kb = rest / p.hsplit;
  const int hk = bh % p.Hkv, b = bh / p.Hkv;
  SPA_DBG_CHECK(b, p.B);
  SPA_DBG_CHECK(split, p.hsplit);
  const int G = p.H / p.Hkv;             // q-heads sharing this kv-head
  const int h0 = hk * G;
  const int kw0 = __builtin_amdgcn_readfirstlane(kb * BNK + wave * 32);
  const int key = kw0 + lk;
  const bool kvalid = key < p.Tk;
  const float c = p.scale_log2;

  bf16x8 kf[KSK], vf[KSV];
  {
    const bf16* kp = p.k + b * p.skb + (long)key * p.skt + hk * p.skh + 8 * hh;
    const bf16* vp = p.v + b * p.svb + (long)key * p.svt + hk * p.svh + 8 * hh;
#pragma unroll
    for (int s = 0; s < KSK; ++s) {
      kf[s] = kvalid ? *reinterpret_cast<const bf16x8*>(kp + 16 * s) : zero8();
      if constexpr (FUSEDQ)   // row = this lane's key; chunk 2s+hh holds d = 16s + 8hh .. +8
        *reinterpret_cast<bf16x8*>(kimg + img_off<IK>(wave * 32 + lk, 2 * s + hh)) = kf[s];
    }
#pragma unroll
    for (int s = 0; s < KSV; ++s) {
      vf[s] = kvalid ? *reinterpret_cast<const bf16x8*>(vp + 16 * s) : zero8();
      if constexpr (VLDS) *reinterpret_cast<bf16x8*>(vimg + img_off<IV>(lk, 2 * s + hh)) = vf[s];
    }
  }
  f32x16 dkt[DTK], dvt[DTV];
#pragma unroll
  for (int i = 0; i < DTK; ++i) dkt[i] = splat16(0.f);
#pragma unroll
  for (int i = 0; i < DTV; ++i) dvt[i] = splat16(0.f);

  int qstart = 0, wave_qstart = 0;
  if (CAUSAL) {
    qstart = max(0, kb * BNK - p.causal_off);
    wave_qstart = max(0, kw0 - p.causal_off);
  }
  const int t0 = qstart / BMQ;
  const int ntq = p.Tq > 0 ? cdiv(p.Tq, BMQ) : 0;
  const int nper = ntq - t0 > 0 ? ntq - t0 : 0;  // q-tiles per head
  // (head, q-tile) iterations of the whole group, in hsplit contiguous shares (whole heads when
  // hsplit divides G); this block runs [ib, ib + total) into its own fp32 partial
  const int tot_all = nper * G;
  const int iper = cdiv(tot_all, p.hsplit);
  const int ib = min(tot_all, split * iper);
  const int total = min(tot_all, ib + iper) - ib;
  TileLoader<HDK, BMQ, NT> lq_;
  TileLoader<HDV, BMQ, NT> ld_;
  lq_.init(p.sqt, tid);
  ld_.init(p.sdot, tid);
  // per-thread row constants of the prefetched tile (tid < BMQ): raw loads, transformed only at
  // commit time so the loads stay in flight (an immediate use would wait vmcnt(0) on the whole
  // Q / dO tile prefetch issued just before)
  float rl = 0.f, rd = 0.f;
  bool rv = false;
  auto fetch = [&](int it) {
    it += ib;
    const int hg = it / nper, tq = t0 + it % nper;
    const int h = h0 + hg;
    const int qq0 = tq * BMQ;
    lq_.load(p.q + b * p.sqb + h * p.sqh, p.sqt, qq0, p.Tq);
    ld_.load(p.dout + b * p.sdob + h * p.sdoh, p.sdot, qq0, p.Tq);
    if (tid < BMQ) {
      const int qq = qq0 + tid;
      const long rbase = ((long)b * p.H + h) * p.Tq;
      rv = qq < p.Tq;
      const long r = rbase + min(qq, p.Tq - 1);
      rl = p.lse_in[r];
      rd = p.delta[r];
    }
  };
  auto commit_tile = [&](int buf) {
    lq_.store(smem + buf * TB);
    ld_.store(smem + buf * TB + TQ);
    if (tid < BMQ) {
      rowc[buf][tid] = rv ? -rl * 1.4426950408889634f : -INFINITY;
      rowc[buf][BMQ + tid] = rv ? -rd : 0.f;
    }
  };
  if (total > 0) {
    fetch(0);
    commit_tile(0);
    if (total > 1) fetch(1);
  }
  __syncthreads();
  LdsOff<IK> offk;
  LdsOff<IV> offv;
  offk.init(lane);
  offv.init(lane);
  // rows of s/dp[t] are queries qq0 + 32t + 8g + 4hh + i (r = 4g + i); column = key (lane)
  // one 32-query sub-tile (rows qt0 + 8g + 4hh + i): s <- P, dp <- dS = P (dP - delta)
  auto mask = [&](f32x16& s, const int qt0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qq = qt0 + 8 * (r >> 2) + 4 * hh + (r & 3);
      if (key > qq + p.causal_off) s[r] = -INFINITY;
    }
  };
  auto dsoft = [&](f32x16& s, f32x16& dp, const float* rc) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 lv = *reinterpret_cast<const f32x4*>(rc + 8 * g + 4 * hh);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 4 * g + i;
        const float pr = fexp2(fmaf(s[r], c, lv[i]));  // rows >= Tq: -lse2 = -inf -> 0
        s[r] = pr;
        dp[r] = pr * dp[r];
      }
    }
  };
  auto body = [&](const int it, auto bufc) {
    constexpr int BUF = decltype(bufc)::value;
    const int tq = t0 + (it + ib) % nper;
    const int qq0 = tq * BMQ;
    const bf16* Qs = smem + BUF * TB;
    const bf16* Ds = Qs + TQ;
    const float* rc = rowc[BUF];
    if (it + 1 < total) {
      commit_tile(1 - BUF);
      if (it + 2 < total) fetch(it + 2);
    }
    const bool active = kw0 < p.Tk && !(CAUSAL && qq0 + BMQ - 1 < wave_qstart);
    if (active) {
      unsigned dbase = 0;
      if constexpr (DROP) dbase = drop_base(p, b, h0 + (it + ib) / nper);
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        // dP accumulator starts at -delta of each row (register r <-> query row 8g+4hh+i);
        // with dropout at 0 (delta is subtracted after the mask)
        f32x16 dp;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 dv = *reinterpret_cast<const f32x4*>(rc + BMQ + 32 * t + 8 * g + 4 * hh);
#pragma unroll
          for (int i = 0; i < 4; ++i) dp[4 * g + i] = DROP ? 0.f : dv[i];
        }
        f32x16 s = mfma32(ld_row(Qs + 32 * t * IK, offk.row[0]), kf[0], splat16(0.f));
#pragma unroll
        for (int ks = 1; ks < KSK; ++ks) s = mfma32(ld_row(Qs + 32 * t * IK, offk.row[ks]), kf[ks], s);
        if constexpr (VLDS) chain_sched<KSK, 1, 3, 4>();        // + the 4 delta reads
#pragma unroll
        for (int ks = 0; ks < KSV; ++ks)
          dp = mfma32(ld_row(Ds + 32 * t * IV, offv.row[ks]), VLDS ? ld_row(vimg, offv.row[ks]) : vf[ks], dp);
        if constexpr (VLDS) chain_sched<KSV, 2, 2>();
        const int qt0 = qq0 + 32 * t;
        unsigned keep = 0xffffu;  // bit r: element r kept by dropout
        if constexpr (DROP) {
          keep = 0;
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4 dv = *reinterpret_cast<const f32x4*>(rc + BMQ + 32 * t + 8 * g + 4 * hh);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int r = 4 * g + i;
              const bool kp = drop_keep(dbase, qt0 + 8 * g + 4 * hh + i, key, p.drop_thr);
              keep |= (unsigned)kp << r;
              dp[r] = (kp ? dp[r] * p.drop_scale : 0.f) + dv[i];
            }
          }
        }
        const bool need_mask = CAUSAL && qt0 + p.causal_off < kw0 + 31;
        if (need_mask) mask(s, qt0);
        dsoft(s, dp, rc + 32 * t);
        if constexpr (DROP) {
#pragma unroll
          for (int r = 0; r < 16; ++r) s[r] = ((keep >> r) & 1) ? s[r] * p.drop_scale : 0.f;
        }
        const bf16x8 pa = pack_acc(s, 0), pb = pack_acc(s, 1), sa = pack_acc(dp, 0), sb = pack_acc(dp, 1);
        if constexpr (DSOUT) {   // bf16 dS of this 32 x 32 block -> p.dsbuf (ds_slot layout, see dkdv3)
          const int qt = qt0 >> 5, kt = kw0 >> 5;
          if ((!CAUSAL || kt <= qt) && qt < p.ds_nqt && kt < p.ds_nkt) {
            const __amdgpu_buffer_rsrc_t dsr = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(p.dsbuf + ((long)b * p.Hkv + hk) * p.ds_kvstride), 0, (int)(p.ds_kvstride * 2), 0x00020000);
            const int bo = (int)(ds_index(qt, kt, (it + ib) / nper, G, p.ds_nkt, CAUSAL) * 2048);
            SPA_DBG_CHECK(bo / 2048, p.ds_kvstride / 1024);
            const int vo = 16 * ds_slot(0, hh, lk);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, sa), dsr, vo, bo, 0);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, sb), dsr, vo + 128, bo, 0);
          }
        }
        if constexpr (FUSEDQ) {
          // dS rows of this wave's 32 keys -> [key][q] image (registers 4g..4g+3 = 4 consecutive q)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            bf16x4 w4;
#pragma unroll
            for (int i = 0; i < 4; ++i) w4[i] = (bf16)dp[4 * g + i];
            *reinterpret_cast<bf16x4*>(dsimg + img_off<64>(wave * 32 + lk, 4 * t + g) + 4 * hh) = w4;
          }
        }
#pragma unroll
        for (int dt = 0; dt < DTV; ++dt) {
          dvt[dt] = mfma32(ld_tr(Ds + 32 * t * IV, offv.tra[dt], offv.trb[dt]), pa, dvt[dt]);
          dvt[dt] = mfma32(ld_tr(Ds + (32 * t + 16) * IV, offv.tra[dt], offv.trb[dt]), pb, dvt[dt]);
        }
        if constexpr (VLDS) chain_sched<2 * DTV, 2, 2>();
#pragma unroll
        for (int dt = 0; dt < DTK; ++dt) {
          dkt[dt] = mfma32(ld_tr(Qs + 32 * t * IK, offk.tra[dt], offk.trb[dt]), sa, dkt[dt]);
          dkt[dt] = mfma32(ld_tr(Qs + (32 * t + 16) * IK, offk.tra[dt], offk.trb[dt]), sb, dkt[dt]);
        }
        if constexpr (VLDS) chain_sched<2 * DTK, 2, 2>();
      }
    } else if constexpr (FUSEDQ) {
      // masked-out wave: its keys contribute nothing to dQ this tile
      bf16x4 z4;
#pragma unroll
      for (int i = 0; i < 4; ++i) z4[i] = (bf16)0.f;
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<bf16x4*>(dsimg + img_off<64>(wave * 32 + lk, 4 * t + g) + 4 * hh) = z4;
    }
    if constexpr (FUSEDQ) {
      __syncthreads();  // dS image complete
      const int h = h0 + (it + ib) / nper;
#pragma unroll
      for (int tile = wave; tile < MT * DTK; tile += 4) {
        const int tq = tile / DTK, td = tile % DTK;
        const int q0 = qq0 + 32 * tq;
        if (CAUSAL && q0 + 31 + p.causal_off < kb * BNK) continue;   // every key of the block is masked
        if (q0 >= p.Tq) continue;
        f32x16 acc = splat16(0.f);
#pragma unroll
        for (int kk = 0; kk < BNK / 16; ++kk)
          acc = mfma32(rd_tr<64>(dsimg, 16 * kk, 32 * tq, lane), rd_tr<IK>(kimg, 16 * kk, 32 * td, lane), acc);
        float* dst = p.dqacc + ((long)b * p.Tq * p.H + h) * HDK + 32 * td + lk;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int qq = q0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if (qq < p.Tq && SPA_DBG_BRH(b, qq, p.Tq, h, p.H)) atomicAdd(dst + (long)qq * p.H * HDK, acc[r]);
        }
      }
    }
    __syncthreads();
  };
  for (int it = 0; it < total; it += 2) {
    body(it, IC<0>{});
    if (it + 1 < total) body(it + 1, IC<1>{});
  }
  store_kv_grad<HDK>(p, dkt, true, b, hk, key, split, hh);
  store_kv_grad<HDV>(p, dvt, false, b, hk, key, split, hh);
}

// ---------------------------------------------------------------------------
// Backward dK/dV, paired waves, software-pipelined (no dropout): 8 waves = 4 pairs x 32 keys (128
// keys per block), key on the lane. Splitting the four products of a key column over two waves
// halves each wave's live registers, which puts two waves on every SIMD: role A holds K and dV^T,
// role B holds V and dK^T of the pair's 32 keys, and role A produces P one interval ahead of its
// consumers, so every interval has ONE block barrier and the same MFMA count per role:
//   interval k, role A:  dV^T += dO(k-1)^T P(k-1)          |  S(k) = Q(k) K^T -> P(k) -> LDS
//   interval k, role B:  dP(k-1) = dO(k-1) V^T - delta;  dS = P(k-1) dP(k-1);  dK^T += Q(k-1)^T dS
// (a two-phase variant with a barrier per role left each role idle about a third of the time at
// those barriers by s_memtime stamps, profiles/r2_attn_dkdv_stamps.txt, and was removed). Nothing
// but the accumulators is carried across intervals: P travels through a 2-deep bf16 LDS ring
// in MFMA-operand order (role A re-reads its own P for dV). Q / dO tiles live in a 3-deep LDS
// ring (tiles k-1 and k are read while k+1 is committed); lse / delta travel with their tile.
// ---------------------------------------------------------------------------
#ifndef DKDV3_SCHED
#define DKDV3_SCHED 0   // 1: chain_sched hints (no effect at 256 VGPRs: one operand register quad; kept for experiments)
#endif
#ifndef DKDV3_DVS_SCHED
#define DKDV3_DVS_SCHED 1   // DVS (hd 256): chain_sched on both roles' dV^T chains
#endif
// SPA_DKDV3_STAMP=1 (a profiling build, never the shipped one: each s_memtime read drains the
// LDS counter): per-wave s_memtime segment sums of the interval loop into p.stamp when the host
// sets it (SPA_ATTN_STAMP=1), [blocks * 8 waves, 8] int64: staging, compute 1 (A: dV^T; B: dP,
// dS), compute 2 (A: S -> P; B: dK^T), barrier wait, epilogue, intervals, whole wave, 0
#ifndef SPA_DKDV3_STAMP
#define SPA_DKDV3_STAMP 0
#endif
#if SPA_DKDV3_STAMP
#define DK3_TICK(i)                                                   \
  do {                                                                \
    const long long tn_ = (long long)__builtin_amdgcn_s_memtime();    \
    seg[i] += tn_ - ts_;                                              \
    ts_ = tn_;                                                        \
  } while (0)
#else
#define DK3_TICK(i) \
  do {              \
  } while (0)
#endif
// DSOUT: role B also stores the bf16 dS of each live 32 x 32 block to p.dsbuf (ds_slot layout),
// the operand of the separate dQ = dS K pass (attn_bwd_dq_ds_kernel) that replaces the dq
// kernel's recomputation of S and dP.
// HDK != HDV (MLA's q/k 192, v 128): role A's fragments / accumulator span HDK / HDV and role B's
// HDV / HDK; the Q and dO images keep their own widths; 32-query intervals (MT = 1) past head dim
// 128, where a 3-deep ring of 64-query tiles would not fit the LDS.
// DVS (head dim 256, Gemma MQA; with DSOUT): no dK here -- dK = dS^T Q is its own streaming pass over
// the stored dS (attn_bwd_dk_ds256_kernel) -- and the dV^T accumulator is split between the roles:
// role A: K fragments + dV^T dims 0..127 (S 16 MFMAs + dV 8 per interval), role B: V fragments +
// dV^T dims 128..255 (dP 16 + dV 8). 64 fragment + 64 accumulator registers per role, where one
// role of the full kernel (fragments + a 256-dim accumulator) spilled 103-130 dwords at 2 waves/SIMD.
template <int HDK, int HDV, bool CAUSAL, bool DSOUT = false, bool DVS = false>
__global__ __launch_bounds__(512) void attn_bwd_dkdv3_kernel(AttnParams p) {
  static_assert(!DVS || (DSOUT && HDK == HDV), "dkdv3 DVS: the dS-materialising square-head form only");
  constexpr int MT = (HDK > 128 || HDV > 128) ? 1 : 2, BMQ = 32 * MT, BNK = 128, NT = 512;
  constexpr int KSK = HDK / 16, KSV = HDV / 16, DTK = HDK / 32, DTV = HDV / 32;
  constexpr int KSX = KSK > KSV ? KSK : KSV, DTX = DVS ? DTV / 2 : (DTK > DTV ? DTK : DTV);
  constexpr int IWK = img_w<HDK>(), IWV = img_w<HDV>();
  constexpr int TQ = BMQ * IWK, TB = TQ + BMQ * IWV, PSLOT = 4 * MT * 2 * 64 * 8;
  __shared__ __attribute__((aligned(16))) bf16 smem[3 * TB];     // [ring][Q | dO]
  __shared__ __attribute__((aligned(16))) bf16 pimg[2 * PSLOT];  // [slot][pair][t][half][lane][8]
  __shared__ __attribute__((aligned(16))) float rowc[3][2 * BMQ]; // [ring][-lse2 | -delta]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pair = wave & 3, role = wave >> 2;
  const int hh = lane >> 5;
  const int nbh = p.Hkv * p.B;
  const int bh = blockIdx.x % nbh;
  const int rest = blockIdx.x / nbh;
  const int split = rest % p.hsplit, kb = rest / p.hsplit;
  const int hk = bh % p.Hkv, b = bh / p.Hkv;
  SPA_DBG_CHECK(b, p.B);
  SPA_DBG_CHECK(split, p.hsplit);
  const int Gs = p.H / p.Hkv / p.hsplit;
  const int h0 = hk * (p.H / p.Hkv) + split * Gs;
  const int kw0 = __builtin_amdgcn_readfirstlane(kb * BNK + pair * 32);
  const int key = kw0 + (lane & 31);
  const bool kvalid = key < p.Tk;
  const float c = p.scale_log2;
#if SPA_DKDV3_STAMP
  long long seg[5] = {0, 0, 0, 0, 0};
  const long long t_start = (long long)__builtin_amdgcn_s_memtime();
  long long ts_ = t_start;
#endif

  bf16x8 xf[KSX];  // A: K fragments (KSK), B: V fragments (KSV) of this lane's key
  {
    const bf16* xp = role == 0 ? p.k + b * p.skb + (long)key * p.skt + hk * p.skh + 8 * hh
                               : p.v + b * p.svb + (long)key * p.svt + hk * p.svh + 8 * hh;
    const int nks = role == 0 ? KSK : KSV;
#pragma unroll
    for (int s = 0; s < KSX; ++s) xf[s] = kvalid && s < nks ? *reinterpret_cast<const bf16x8*>(xp + 16 * s) : zero8();
  }
  f32x16 acc[DTX];  // A: dV^T (DTV), B: dK^T (DTK); DVS: A / B dV^T dims 0.. / HDV/2.. (DTV/2 each)
#pragma unroll
  for (int i = 0; i < DTX; ++i) acc[i] = splat16(0.f);

  int qstart = 0, wave_qstart = 0;
  if (CAUSAL) {
    qstart = max(0, kb * BNK - p.causal_off);
    wave_qstart = max(0, kw0 - p.causal_off);
  }
  const int t0 = qstart / BMQ;
  const int ntq = p.Tq > 0 ? cdiv(p.Tq, BMQ) : 0;
  const int nper = ntq - t0 > 0 ? ntq - t0 : 0;
  const int total = nper * Gs;
  TileLoader<HDK, BMQ, NT> lq_;
  TileLoader<HDV, BMQ, NT> ld_;
  lq_.init(p.sqt, tid);
  ld_.init(p.sdot, tid);
  float rl = 0.f, rd = 0.f;   // raw row constants of the prefetched tile (transformed at commit)
  bool rv = false;
  // the row constants are loaded and committed by threads tid < BMQ (role A's wave 0); ROWS = 0
  // leaves them out of role B's copy of the loop entirely, so no rl / rd load is pending there
  // (one was, in a register hipcc reused: a vmcnt(0) before role B's first dP MFMA)
  auto fetch = [&](int it, auto rowsc) {
    const int h = h0 + it / nper;
    const int qq0 = (t0 + it % nper) * BMQ;
    lq_.load(p.q + b * p.sqb + h * p.sqh, p.sqt, qq0, p.Tq);
    ld_.load(p.dout + b * p.sdob + h * p.sdoh, p.sdot, qq0, p.Tq);
    if (decltype(rowsc)::value && tid < BMQ) {
      const int qq = qq0 + tid;
      const long r = ((long)b * p.H + h) * p.Tq + min(qq, p.Tq - 1);
      rv = qq < p.Tq;
      rl = p.lse_in[r];
      rd = p.delta[r];
    }
  };
  auto commit_tile = [&](int slot, auto rowsc) {
    lq_.store(smem + slot * TB);
    ld_.store(smem + slot * TB + TQ);
    if (decltype(rowsc)::value && tid < BMQ) {
      rowc[slot][tid] = rv ? -rl * 1.4426950408889634f : -INFINITY;
      rowc[slot][BMQ + tid] = rv ? -rd : 0.f;
    }
  };
  auto tile_active = [&](int it) {
    const int qq0 = (t0 + it % nper) * BMQ;
    return kw0 < p.Tk && !(CAUSAL && qq0 + BMQ - 1 < wave_qstart);
  };
  if (total > 0) {
    fetch(0, IC<1>{});
    commit_tile(0, IC<1>{});
    if (total > 1) fetch(1, IC<1>{});
  }
  __syncthreads();
  LdsOff<IWK> offk;   // Q image
  LdsOff<IWV> offv;   // dO image
  offk.init(lane);
  offv.init(lane);
  bf16* pme = pimg + pair * (MT * 2 * 64 * 8) + lane * 8;   // + slot * PSLOT + (t * 2 + half) * 512
  bool prev_act = false;
  // interval k (slot SC = k % 3): tiles k-1 (slot (SC+2)%3) and k (slot SC) resident; commits k+1
  // ROLE is a compile-time constant and each role runs its own copy of the interval loop (same
  // barrier count): with one loop branching on the role per interval, the accumulators of the
  // two roles met in phi nodes and hipcc re-homed all 64 of them (32 v_mov_b64) every interval
  auto interval = [&](const int k, auto slotc, auto rolec) {
    constexpr int SC = decltype(slotc)::value, SP = (SC + 2) % 3;
    constexpr int ROLE = decltype(rolec)::value;
    // unconditional staging (past the end: the slot of tile k - 2, no longer read, and a re-fetch
    // of the last tile): a conditional prefetch made hipcc merge the load registers through
    // copies that waited vmcnt(0) right behind the loads
    commit_tile((SC + 1) % 3, IC<ROLE == 0>{});
    fetch(min(k + 2, total - 1), IC<ROLE == 0>{});
    DK3_TICK(0);
    const bool cur = k < total && tile_active(k);
    const bf16* Qc = smem + SC * TB;
    const bf16* Qp = smem + SP * TB;
    const bf16* Dp = Qp + TQ;
    const bf16* pr = pme + ((k + 1) & 1) * PSLOT;        // P(k-1)
    if constexpr (ROLE == 0) {
      if (prev_act) {                                    // dV^T += dO(k-1)^T P(k-1)
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          const bf16x8 pa = *reinterpret_cast<const bf16x8*>(pr + (t * 2 + 0) * 512);
          const bf16x8 pb = *reinterpret_cast<const bf16x8*>(pr + (t * 2 + 1) * 512);
#pragma unroll
          for (int dt = 0; dt < (DVS ? DTX : DTV); ++dt) {
            acc[dt] = mfma32(ld_tr(Dp + 32 * t * IWV, offv.tra[dt], offv.trb[dt]), pa, acc[dt]);
            acc[dt] = mfma32(ld_tr(Dp + (32 * t + 16) * IWV, offv.tra[dt], offv.trb[dt]), pb, acc[dt]);
          }
          if (DKDV3_SCHED || (DVS && DKDV3_DVS_SCHED)) chain_sched<2 * (DVS ? DTX : DTV), 2, 2, 2>();
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      DK3_TICK(1);
      if (cur) {                                         // S(k) -> P(k) -> LDS slot k & 1
        const int qq0 = (t0 + k % nper) * BMQ;
        const float* rc = rowc[SC];
        bf16* pw = pme + (k & 1) * PSLOT;
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          f32x16 s = mfma32(ld_row(Qc + 32 * t * IWK, offk.row[0]), xf[0], splat16(0.f));
#pragma unroll
          for (int ks = 1; ks < KSK; ++ks) s = mfma32(ld_row(Qc + 32 * t * IWK, offk.row[ks]), xf[ks], s);
          if (DKDV3_SCHED) chain_sched<KSK, 1, 2>();
          const int qt0 = qq0 + 32 * t;
          if (CAUSAL && qt0 + p.causal_off < kw0 + 31) {
            const int d = key - qt0 - 4 * hh - p.causal_off;   // row offsets below d are masked
#pragma unroll
            for (int r = 0; r < 16; ++r)
              if ((r & 3) + 8 * (r >> 2) < d) s[r] = -INFINITY;
          }
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4 lv = *reinterpret_cast<const f32x4*>(rc + 32 * t + 8 * g + 4 * hh);
#pragma unroll
            for (int i = 0; i < 4; ++i) s[4 * g + i] = fexp2(fmaf(s[4 * g + i], c, lv[i]));
          }
          *reinterpret_cast<bf16x8*>(pw + (t * 2 + 0) * 512) = pack_acc(s, 0);
          *reinterpret_cast<bf16x8*>(pw + (t * 2 + 1) * 512) = pack_acc(s, 1);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      DK3_TICK(2);
    } else {
      if (!prev_act) {
        prev_act = cur;
        __syncthreads();
        DK3_TICK(3);
        return;
      }
      // tile k-1: dP, dS, dK^T
      const bf16* Dpr = Dp;
      const float* rc = rowc[SP];
      // DSOUT: one scalar buffer descriptor per (b, q-head) and scalar block offsets; the only
      // per-lane part (the chunk slot) is recomputed at the store (this kernel is at 256 VGPRs)
      int qtp = 0, hp = 0;
      if constexpr (DSOUT) {
        hp = h0 + (k - 1) / nper;
        qtp = (t0 + (k - 1) % nper) * (BMQ / 32);
      }
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        f32x16 dp;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 dv = *reinterpret_cast<const f32x4*>(rc + BMQ + 32 * t + 8 * g + 4 * hh);
#pragma unroll
          for (int i = 0; i < 4; ++i) dp[4 * g + i] = dv[i];
        }
#pragma unroll
        for (int ks = 0; ks < KSV; ++ks) dp = mfma32(ld_row(Dpr + 32 * t * IWV, offv.row[ks]), xf[ks], dp);
        if (DKDV3_SCHED) chain_sched<KSV, 1, 2, 4>();     // + the 4 delta reads
        const bf16x8 pa = *reinterpret_cast<const bf16x8*>(pr + (t * 2 + 0) * 512);
        const bf16x8 pb = *reinterpret_cast<const bf16x8*>(pr + (t * 2 + 1) * 512);
        f32x16 ds;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          ds[r] = (float)pa[r] * dp[r];
          ds[8 + r] = (float)pb[r] * dp[8 + r];
        }
        const bf16x8 sa = pack_acc(ds, 0), sb = pack_acc(ds, 1);
        if constexpr (DSOUT) {
          const int qt = qtp + t, kt = kw0 >> 5;
          if ((!CAUSAL || kt <= qt) && qt < p.ds_nqt && kt < p.ds_nkt) {
            const __amdgpu_buffer_rsrc_t dsr = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(p.dsbuf + ((long)b * p.Hkv + hk) * p.ds_kvstride), 0, (int)(p.ds_kvstride * 2), 0x00020000);
            const int bo = (int)(ds_index(qt, kt, hp - hk * (p.H / p.Hkv), p.H / p.Hkv, p.ds_nkt, CAUSAL) * 2048);
            SPA_DBG_CHECK(bo / 2048, p.ds_kvstride / 1024);
            const int vo = 16 * ds_slot(0, (int)(__lane_id() >> 5), (int)(__lane_id() & 31));
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, sa), dsr, vo, bo, 0);        // s = 0
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, sb), dsr, vo + 128, bo, 0);  // s = 1: slot + 8
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        DK3_TICK(1);
        if constexpr (DVS) {   // dV^T dims HDV/2.. += dO(k-1)^T P(k-1) (role A holds dims 0..)
#pragma unroll
          for (int dt = 0; dt < DTX; ++dt) {
            acc[dt] = mfma32(ld_tr(Dpr + 32 * t * IWV, offv.tra[DTX + dt], offv.trb[DTX + dt]), pa, acc[dt]);
            acc[dt] = mfma32(ld_tr(Dpr + (32 * t + 16) * IWV, offv.tra[DTX + dt], offv.trb[DTX + dt]), pb, acc[dt]);
          }
          if (DKDV3_DVS_SCHED) chain_sched<2 * DTX, 2, 2>();
        } else {
#pragma unroll
          for (int dt = 0; dt < DTK; ++dt) {
            acc[dt] = mfma32(ld_tr(Qp + 32 * t * IWK, offk.tra[dt], offk.trb[dt]), sa, acc[dt]);
            acc[dt] = mfma32(ld_tr(Qp + (32 * t + 16) * IWK, offk.tra[dt], offk.trb[dt]), sb, acc[dt]);
          }
          if (DKDV3_SCHED) chain_sched<2 * DTK, 2, 2, 2>();  // + the P(k-1) reads
        }
        __builtin_amdgcn_sched_barrier(0);
        DK3_TICK(2);
      }
    }
    prev_act = cur;
    __syncthreads();
    DK3_TICK(3);
  };
  // as in the forward: the prefetch is conditional, so hipcc could not count the fragment loads
  // of the prologue past it and waited vmcnt(0) -- the Q / dO prefetch just issued -- before
  // role A's first S MFMA of every interval; an empty asm using the fragments waits for them here, once
#pragma unroll
  for (int s = 0; s < KSX; ++s) asm volatile("" ::"v"(xf[s]));
  if (role == 0) {
    for (int k = 0; k <= total; k += 3) {
      interval(k, IC<0>{}, IC<0>{});
      if (k + 1 <= total) interval(k + 1, IC<1>{}, IC<0>{});
      if (k + 2 <= total) interval(k + 2, IC<2>{}, IC<0>{});
    }
  } else {
    for (int k = 0; k <= total; k += 3) {
      interval(k, IC<0>{}, IC<1>{});
      if (k + 1 <= total) interval(k + 1, IC<1>{}, IC<1>{});
      if (k + 2 <= total) interval(k + 2, IC<2>{}, IC<1>{});
    }
  }
  if constexpr (DVS) {
    store_kv_grad<HDV>(p, acc, false, b, hk, key, split, hh, role * DTX);
  } else if constexpr (HDK == HDV) {
    store_kv_grad<HDK>(p, acc, role == 1, b, hk, key, split, hh);
  } else {
    if (role == 1) {
      f32x16 ak[DTK];
#pragma unroll
      for (int i = 0; i < DTK; ++i) ak[i] = acc[i];
      store_kv_grad<HDK>(p, ak, true, b, hk, key, split, hh);
    } else {
      f32x16 av[DTV];
#pragma unroll
      for (int i = 0; i < DTV; ++i) av[i] = acc[i];
      store_kv_grad<HDV>(p, av, false, b, hk, key, split, hh);
    }
  }
#if SPA_DKDV3_STAMP
  DK3_TICK(4);
  if (p.stamp != nullptr && lane < 8) {   // one value per lane: vector stores
    long long v = 0;
#pragma unroll
    for (int i = 0; i < 5; ++i) v = lane == i ? seg[i] : v;
    v = lane == 5 ? (long long)(total + 1) : lane == 6 ? ts_ - t_start : v;
    p.stamp[((long)blockIdx.x * 8 + wave) * 8 + lane] = v;
  }
#endif
}

// ---------------------------------------------------------------------------
// Backward dQ from the materialised dS (after attn_bwd_dkdv3_kernel<HD, CAUSAL, true>):
//   dQ^T[d][q] = sum_key K^T[d][key] dS^T[key][q]
// One product instead of the dq kernel's three (S = Q K^T, dP = dO V^T recomputed, then dS K), at
// the price of writing and reading dS once (bf16, 2 KiB per live 32 x 32 block: 2.2 GB at the
// LLaMA3-8B shape) -- so this pass streams HBM rather than the matrix pipe.
// Block = 4 waves = 4 (q-head, 64-query) units of one (batch, kv-head): with GQA group G the units
// run heads fastest (G = 4: the four q-heads of one 64-query block), so the K tile of each 32-key
// step is staged once for all of them. Per step every wave DMAs its two 2 KiB dS blocks (its
// 64 queries) and a quarter of the K tile straight into LDS (buffer_load ... lds): 3 slots, two
// steps in flight, one counted vmcnt + one barrier per step; no vmcnt(0) of hipcc's own (the DMA is inline asm: hipcc's waitcnt pass, which cannot tell the DMA's
// LDS bytes from the ds_reads', would otherwise drain it before every step's reads). dS^T fragments come out of the ds_slot image with ds_read_b64_tr_b16
// (conflict-free), K^T fragments out of the swizzled K image (same reads as the dq kernel).
// Non-live blocks (above the causal diagonal, or a missing unit) are loaded through a zero-range
// descriptor (zeros, same DMA count per step) and skipped by the MFMAs.
// ---------------------------------------------------------------------------
template <int HD, bool CAUSAL, bool NT>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_ds_kernel(AttnParams p) {
  static_assert(HD == 128, "dq_ds: head dim 128 (K tile = 4 KiB-row images of 256 B)");
  constexpr int DT = HD / 32, KIMG = 32 * HD, WSLOT = 2 * 1024, SLOT = KIMG + 4 * WSLOT, NSLOT = 3;
  __shared__ __attribute__((aligned(16))) bf16 smem[NSLOT * SLOT];   // [slot][K | 4 waves x 2 dS blocks]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5;
  const int G = p.H / p.Hkv;
  const int nq64 = cdiv(p.Tq, 64);
  const int upkv = nq64 * G;
  const int wgpkv = cdiv(upkv, 4);
  const int nbkv = p.B * p.Hkv;
  const int bkv = blockIdx.x % nbkv;                            // = XCD group when B*Hkv == 8
  const int w = CAUSAL ? wgpkv - 1 - (int)(blockIdx.x / nbkv) : (int)(blockIdx.x / nbkv);  // heaviest first
  const int b = bkv / p.Hkv, hk = bkv % p.Hkv;
  SPA_DBG_CHECK(b, p.B);
  const int u = 4 * w + wave;
  const bool uvalid = u < upkv;
  const int qb = uvalid ? u / G : 0;
  const int h = hk * G + (uvalid ? u % G : 0);
  // key steps (32 keys) of this wave and of the block (the block's last valid unit is its largest)
  auto unit_steps = [&](int uu) {
    const int qbb = uu / G;
    return CAUSAL ? cdiv(min(p.Tk, qbb * 64 + 64 + p.causal_off), 32) : cdiv(p.Tk, 32);
  };
  const int nsteps_w = uvalid ? unit_steps(u) : 0;
  const int nsteps = unit_steps(min(4 * w + 3, upkv - 1));

  // K tile DMA: wave `wave` fills rows 8*wave .. +7 (two 1 KiB pieces of 4 rows); lane -> row
  // r = 8*wave + 4j + lane/16, image chunk lane%16 holding source chunk (lane%16) ^ swz(r)
  const bf16* kbase = p.k + b * p.skb + hk * p.skh;
  unsigned kvo[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int r = 8 * wave + 4 * j + (lane >> 4);
    kvo[j] = (unsigned)(((long)r * p.skt + 8 * ((lane & 15) ^ swz<HD>(r))) * 2);
  }
  const bf16* dskv = p.dsbuf + ((long)b * p.Hkv + hk) * p.ds_kvstride;
  const int g = h - hk * G;
  auto live = [&](int qt, int kt) { return uvalid && qt < p.ds_nqt && (!CAUSAL || kt <= qt); };
  auto issue = [&](int j, int slot) {
    bf16* sl = smem + slot * SLOT;
    const int key0 = 32 * j;
    const long kbytes = key0 < p.Tk ? ((long)(p.Tk - key0 - 1) * p.skt + HD) * 2 : 0;
    const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(kbase + (long)key0 * p.skt), 0, (int)min(kbytes, 0x7fffffffL), 0x00020000);
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) dma16_asm(rk, kvo[jj], lds_addr(sl + (8 * wave + 4 * jj) * HD));
    // this wave's two blocks of the step (t = 0, 1) are one contiguous 4 KiB piece; a step past the
    // unit's range, or a missing unit, reads zeros (same DMA count in every wave and step)
    const bool lv = live(2 * qb + 1, j) || live(2 * qb, j);
    if (lv) SPA_DBG_CHECK(ds_index(2 * qb, j, g, G, p.ds_nkt, CAUSAL), p.ds_kvstride / 1024);
    const bf16* src = lv ? dskv + ds_index(2 * qb, j, g, G, p.ds_nkt, CAUSAL) * 1024 : p.dsbuf;
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, lv ? 4096 : 0, 0x00020000);
    bf16* dst = sl + KIMG + wave * WSLOT;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) dma16_asm<NT>(rd, (unsigned)(lane * 16 + jj * 1024), lds_addr(dst + jj * 512));
  };
  LdsOff<HD> off;
  off.init(lane);
  // dS^T operand reads (per 16-key k-step s): lane 4q+p of 16-lane group g addresses key
  // 16s + 4hh + q (+8 for the second read), queries 16(g&1) + 4p .. +3 = half p>>1 of the chunk
  // (s_p = g&1, h_p = p&1, key)
  int dso[2];
  {
    const int g = (lane >> 4) & 1, i = lane & 15, q = i >> 2, pp = i & 3;
#pragma unroll
    for (int ab = 0; ab < 2; ++ab) {
      const int key = 4 * hh + q + 8 * ab;
      dso[ab] = 8 * ds_slot(g, pp & 1, key) + 4 * (pp >> 1);   // elements; +512 per 16-key step
    }
  }
  f32x16 acc[2][DT];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int i = 0; i < DT; ++i) acc[t][i] = splat16(0.f);

  auto compute = [&](int j, const bf16* sl) {
    if (j >= nsteps_w) return;
    const bf16* Ks = sl;
    const bf16* Dw = sl + KIMG + wave * WSLOT;
    const bool l0 = live(2 * qb, j), l1 = live(2 * qb + 1, j);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 kt[DT];
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) kt[dt] = ld_tr(Ks + 16 * s * HD, off.tra[dt], off.trb[dt]);
      const bf16x8 d0 = ld_tr(Dw + 512 * s, dso[0], dso[1]);          // keys 16s.. = slots 64s..
      const bf16x8 d1 = ld_tr(Dw + 1024 + 512 * s, dso[0], dso[1]);
      if (l0) {
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) acc[0][dt] = mfma32(kt[dt], d0, acc[0][dt]);
      }
      if (l1) {
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) acc[1][dt] = mfma32(kt[dt], d1, acc[1][dt]);
      }
    }
  };
  if (nsteps > 0) issue(0, 0);
  if (nsteps > 1) issue(1, 1);
  for (int j = 0; j < nsteps; j += 3) {
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int jj = j + r;
      if (jj < nsteps) {
        if (jj + 1 < nsteps) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");   // step jj landed, jj+1 in flight
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // step jj-1's LDS reads done before its slot is restaged
        __builtin_amdgcn_s_barrier();
        // slot (jj+2)%3 was last read in step jj-1, which every wave finished before this barrier
        if (jj + 2 < nsteps) issue(jj + 2, (r + 2) % 3);
        compute(jj, smem + r * SLOT);
      }
    }
  }
  if (!uvalid) return;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int q = qb * 64 + 32 * t + (lane & 31);
    if (q >= p.Tq || !SPA_DBG_BRH(b, q, p.Tq, h, p.H)) continue;
    bf16* op = p.dq + b * p.sdqb + (long)q * p.sdqt + h * p.sdqh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 wv;
#pragma unroll
        for (int i = 0; i < 4; ++i) wv[i] = (bf16)(acc[t][dt][4 * g + i] * p.scale);
        *reinterpret_cast<bf16x4*>(op + 32 * dt + 8 * g + 4 * hh) = wv;
      }
  }
}

// Head dim 256 / 192 form of the above (after attn_bwd_dkdv_kernel<HDK, .., DSOUT>: Gemma's 256 and
// MLA's q/k 192 with v 128): a unit is one (q-head, 32-query tile), so a wave's dQ^T accumulator is
// 32 queries x HDK dims (128 / 96 registers, two waves per SIMD); per 32-key step each wave DMAs its
// one 2 KiB dS block and an eighth of the 16 KiB K tile (4 + 2 pieces: the same vmcnt(6) discipline),
// 3 slots of 24 KiB.
template <int HDK, bool CAUSAL, bool NT>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_ds256_kernel(AttnParams p) {
  // HDK 256 (Gemma) or 192 (MLA q/k): the K image rows are 256 wide either way (img_w<192> = 256;
  // the DMA moves whole 512-B rows, whose columns past HDK are never read by the MFMAs)
  static_assert(HDK == 256 || HDK == 192, "dq_ds256: q/k head dim 192 or 256");
  constexpr int HD = 256, DT = HDK / 32, KIMG = 32 * HD, WSLOT = 1024, SLOT = KIMG + 4 * WSLOT, NSLOT = 3;
  __shared__ __attribute__((aligned(16))) bf16 smem[NSLOT * SLOT];   // [slot][K | 4 waves x 1 dS block]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5;
  const int G = p.H / p.Hkv;
  const int nqt = cdiv(p.Tq, 32);
  const int upkv = nqt * G;
  const int wgpkv = cdiv(upkv, 4);
  const int nbkv = p.B * p.Hkv;
  const int bkv = blockIdx.x % nbkv;
  const int w = CAUSAL ? wgpkv - 1 - (int)(blockIdx.x / nbkv) : (int)(blockIdx.x / nbkv);  // heaviest first
  const int b = bkv / p.Hkv, hk = bkv % p.Hkv;
  SPA_DBG_CHECK(b, p.B);
  const int u = 4 * w + wave;
  const bool uvalid = u < upkv;
  const int qt = uvalid ? u / G : 0;
  const int h = hk * G + (uvalid ? u % G : 0);
  auto unit_steps = [&](int uu) {
    const int qtt = uu / G;
    return CAUSAL ? cdiv(min(p.Tk, qtt * 32 + 32 + p.causal_off), 32) : cdiv(p.Tk, 32);
  };
  const int nsteps_w = uvalid ? unit_steps(u) : 0;
  const int nsteps = unit_steps(min(4 * w + 3, upkv - 1));

  // K tile DMA: wave `wave` fills rows 8*wave .. +7 (four 1 KiB pieces of 2 rows); lane -> row
  // r = 8*wave + 2j + lane/32, image chunk lane%32 holding source chunk (lane%32) ^ swz(r)
  const bf16* kbase = p.k + b * p.skb + hk * p.skh;
  unsigned kvo[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = 8 * wave + 2 * j + (lane >> 5);
    kvo[j] = (unsigned)(((long)r * p.skt + 8 * ((lane & 31) ^ swz<HD>(r))) * 2);
  }
  const bf16* dskv = p.dsbuf + ((long)b * p.Hkv + hk) * p.ds_kvstride;
  const int g = h - hk * G;
  auto live = [&](int kt) { return uvalid && qt < p.ds_nqt && (!CAUSAL || kt <= qt); };
  auto issue = [&](int j, int slot) {
    bf16* sl = smem + slot * SLOT;
    const int key0 = 32 * j;
    const long kbytes = key0 < p.Tk ? ((long)(p.Tk - key0 - 1) * p.skt + HDK) * 2 : 0;
    const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(kbase + (long)key0 * p.skt), 0, (int)min(kbytes, 0x7fffffffL), 0x00020000);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) dma16_asm(rk, kvo[jj], lds_addr(sl + (8 * wave + 2 * jj) * HD));
    const bool lv = live(j);
    if (lv) SPA_DBG_CHECK(ds_index(qt, j, g, G, p.ds_nkt, CAUSAL), p.ds_kvstride / 1024);
    const bf16* src = lv ? dskv + ds_index(qt, j, g, G, p.ds_nkt, CAUSAL) * 1024 : p.dsbuf;
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, lv ? 2048 : 0, 0x00020000);
    bf16* dst = sl + KIMG + wave * WSLOT;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) dma16_asm<NT>(rd, (unsigned)(lane * 16 + jj * 1024), lds_addr(dst + jj * 512));
  };
  LdsOff<HD> off;
  off.init(lane);
  int dso[2];
  {
    const int gg = (lane >> 4) & 1, i = lane & 15, q = i >> 2, pp = i & 3;
#pragma unroll
    for (int ab = 0; ab < 2; ++ab) {
      const int key = 4 * hh + q + 8 * ab;
      dso[ab] = 8 * ds_slot(gg, pp & 1, key) + 4 * (pp >> 1);   // elements; +512 per 16-key step
    }
  }
  f32x16 acc[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) acc[i] = splat16(0.f);

  auto compute = [&](int j, const bf16* sl) {
    if (j >= nsteps_w || !live(j)) return;
    const bf16* Ks = sl;
    const bf16* Dw = sl + KIMG + wave * WSLOT;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 d0 = ld_tr(Dw + 512 * s, dso[0], dso[1]);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) acc[dt] = mfma32(ld_tr(Ks + 16 * s * HD, off.tra[dt], off.trb[dt]), d0, acc[dt]);
      chain_sched<DT, 1, 2, 1>();
    }
  };
  if (nsteps > 0) issue(0, 0);
  if (nsteps > 1) issue(1, 1);
  for (int j = 0; j < nsteps; j += 3) {
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int jj = j + r;
      if (jj < nsteps) {
        if (jj + 1 < nsteps) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");   // step jj landed, jj+1 in flight
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (jj + 2 < nsteps) issue(jj + 2, (r + 2) % 3);
        compute(jj, smem + r * SLOT);
      }
    }
  }
  if (!uvalid) return;
  const int q = qt * 32 + (lane & 31);
  if (q >= p.Tq || !SPA_DBG_BRH(b, q, p.Tq, h, p.H)) return;
  bf16* op = p.dq + b * p.sdqb + (long)q * p.sdqt + h * p.sdqh;
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      bf16x4 wv;
#pragma unroll
      for (int i = 0; i < 4; ++i) wv[i] = (bf16)(acc[dt][4 * gq + i] * p.scale);
      *reinterpret_cast<bf16x4*>(op + 32 * dt + 8 * gq + 4 * hh) = wv;
    }
}

// Backward dK from the materialised dS at head dim 256 (after attn_bwd_dkdv3_kernel<256, 256, .., DSOUT,
// DVS>, whose two roles keep only dV^T):  dK^T[d][key] = sum_q Q^T[d][q] dS[q][key].
// Key-parallel like the dK/dV kernels: block = 4 waves x 32 keys (128 keys), the same (q-head, 32-query
// tile) iteration space and q-head split (hsplit shares, fp32 partials summed by attn_kv_reduce_kernel),
// so dK sums its products in the single-wave kernel's order. Per step the block DMAs the step's 32 x 256
// Q tile (16 KiB, a quarter per wave: four 1 KiB pieces) and each wave its own 2 KiB dS block straight
// into LDS -- 6 DMAs per wave per step, the vmcnt(6) discipline of the dQ pass, 3
// slots of 24 KiB, two blocks per CU. dS comes out of the ds_slot image as the MFMA's B operand with a
// plain 16-B read (the slot of (half s, lane half hh, key) IS the dK/dV kernel's packed accumulator),
// Q^T with the transposed reads of the swizzled Q image.
template <bool CAUSAL, bool NT>
__global__ __launch_bounds__(256, 2) void attn_bwd_dk_ds256_kernel(AttnParams p) {
  constexpr int HD = 256, DT = HD / 32, BNK = 128, QIMG = 32 * HD, WSLOT = 1024, SLOT = QIMG + 4 * WSLOT, NSLOT = 3;
  __shared__ __attribute__((aligned(16))) bf16 smem[NSLOT * SLOT];   // [slot][Q | 4 waves x 1 dS block]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5, lk = lane & 31;
  const int nbh = p.Hkv * p.B;
  const int bh = blockIdx.x % nbh;
  const int rest = blockIdx.x / nbh;   // causal: low key blocks are heaviest, launched first
  const int split = rest % p.hsplit, kb = rest / p.hsplit;
  const int hk = bh % p.Hkv, b = bh / p.Hkv;
  SPA_DBG_CHECK(b, p.B);
  SPA_DBG_CHECK(split, p.hsplit);
  const int G = p.H / p.Hkv;
  const int h0 = hk * G;
  const int kt = kb * (BNK / 32) + wave;   // this wave's 32-key tile
  const int key = kt * 32 + lk;
  const int qstart = CAUSAL ? max(0, kb * BNK - p.causal_off) : 0;
  const int t0 = qstart / 32;
  const int ntq = p.Tq > 0 ? cdiv(p.Tq, 32) : 0;
  const int nper = ntq - t0 > 0 ? ntq - t0 : 0;
  const int tot_all = nper * G;
  const int iper = cdiv(tot_all, p.hsplit);
  const int ib = min(tot_all, split * iper);
  const int nsteps = min(tot_all, ib + iper) - ib;

  // Q tile DMA: wave `wave` fills rows 8*wave .. +7 (four 1 KiB pieces of 2 rows); lane -> row
  // r = 8*wave + 2j + lane/32, image chunk lane%32 holding source chunk (lane%32) ^ swz(r)
  unsigned qvo[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = 8 * wave + 2 * j + (lane >> 5);
    qvo[j] = (unsigned)(((long)r * p.sqt + 8 * ((lane & 31) ^ swz<HD>(r))) * 2);
  }
  const bf16* dskv = p.dsbuf + ((long)b * p.Hkv + hk) * p.ds_kvstride;
  auto live = [&](int tq) { return kt < p.ds_nkt && tq < p.ds_nqt && (!CAUSAL || kt <= tq); };
  auto issue = [&](int j, int slot) {
    bf16* sl = smem + slot * SLOT;
    const int it = ib + j, g = it / nper, tq = t0 + it % nper;
    const int q0 = 32 * tq;
    const long qbytes = q0 < p.Tq ? ((long)(p.Tq - q0 - 1) * p.sqt + HD) * 2 : 0;
    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.q + b * p.sqb + (h0 + g) * p.sqh + (long)q0 * p.sqt), 0, (int)min(qbytes, 0x7fffffffL), 0x00020000);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) dma16_asm(rq, qvo[jj], lds_addr(sl + (8 * wave + 2 * jj) * HD));
    const bool lv = live(tq);
    if (lv) SPA_DBG_CHECK(ds_index(tq, kt, g, G, p.ds_nkt, CAUSAL), p.ds_kvstride / 1024);
    const bf16* src = lv ? dskv + ds_index(tq, kt, g, G, p.ds_nkt, CAUSAL) * 1024 : p.dsbuf;
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, lv ? 2048 : 0, 0x00020000);
    bf16* dst = sl + QIMG + wave * WSLOT;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) dma16_asm<NT>(rd, (unsigned)(lane * 16 + jj * 1024), lds_addr(dst + jj * 512));
  };
  LdsOff<HD> off;
  off.init(lane);
  const int dso0 = 8 * ds_slot(0, hh, lk);   // elements; half s = 1 is 8 slots on (+64 elements)
  f32x16 acc[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) acc[i] = splat16(0.f);

  auto compute = [&](int j, const bf16* sl) {
    const int it = ib + j;
    if (!live(t0 + it % nper)) return;
    const bf16* Qs = sl;
    const bf16* Dw = sl + QIMG + wave * WSLOT;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 d0 = ld_row(Dw, dso0 + 64 * s);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) acc[dt] = mfma32(ld_tr(Qs + 16 * s * HD, off.tra[dt], off.trb[dt]), d0, acc[dt]);
      chain_sched<DT, 2, 2, 1>();
    }
  };
  if (nsteps > 0) issue(0, 0);
  if (nsteps > 1) issue(1, 1);
  for (int j = 0; j < nsteps; j += 3) {
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int jj = j + r;
      if (jj < nsteps) {
        if (jj + 1 < nsteps) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");   // step jj landed, jj+1 in flight
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // step jj-1's LDS reads done before its slot is restaged
        __builtin_amdgcn_s_barrier();
        if (jj + 2 < nsteps) issue(jj + 2, (r + 2) % 3);
        compute(jj, smem + r * SLOT);
      }
    }
  }
  store_kv_grad<HD>(p, acc, true, b, hk, key, split, hh);
}

// sum the q-head-split fp32 partials of ONE tensor (dK with HD = HDK, or dV with HD = HDV)
// -> bf16 dK (scaled) / dV
template <int HD>
__global__ __launch_bounds__(256) void attn_kv_reduce_kernel(AttnParams p, int is_k) {
  constexpr int TPR = HD / 8;
  const long rows = (long)p.B * p.Tk * p.Hkv;
  const long n = rows * TPR;
  const long slab = rows * HD;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int t = i % TPR;
    const long row = i / TPR;  // (b, key, hk)
    const long hk = row % p.Hkv, key = (row / p.Hkv) % p.Tk, b = row / ((long)p.Hkv * p.Tk);
    const float* src = (is_k ? p.dkacc : p.dvacc) + row * HD + 8 * t;
    float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int s = 0; s < p.hsplit; ++s) {
      float x[8];
      load8(src + s * slab, x);
#pragma unroll
      for (int k = 0; k < 8; ++k) a[k] += x[k];
    }
    const float sc = is_k ? p.scale : 1.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] *= sc;
    bf16* dst = is_k ? p.dk + b * p.sdkb + key * p.sdkt + hk * p.sdkh + 8 * t
                     : p.dv + b * p.sdvb + key * p.sdvt + hk * p.sdvh + 8 * t;
    store8(dst, a);
  }
}

// delta[b,h,q] = sum_d dO*O (fp32); TPR = HD/8 threads per row
template <int HD>
__global__ __launch_bounds__(256) void attn_delta_kernel(AttnParams p) {
  constexpr int TPR = HD / 8, RPB = 256 / TPR;
  const long row = (long)blockIdx.x * RPB + threadIdx.x / TPR;
  const int t = threadIdx.x % TPR;
  const long nrows = (long)p.B * p.Tq * p.H;
  float acc = 0.f;
  long b = 0, q = 0, h = 0;
  if (row < nrows) {
    h = row % p.H;
    q = (row / p.H) % p.Tq;
    b = row / ((long)p.H * p.Tq);
    float a[8], c[8];
    load8(p.dout + b * p.sdob + q * p.sdot + h * p.sdoh + 8 * t, a);
    load8(p.o + b * p.sob + q * p.sot + h * p.soh + 8 * t, c);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += a[i] * c[i];
  }
#pragma unroll
  for (int o = TPR / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, TPR);
  if (row < nrows && t == 0 && SPA_DBG_BRH(b, q, p.Tq, h, p.H)) p.delta[(b * p.H + h) * p.Tq + q] = acc;
}
// dq (strided bf16) = scale * dqacc
template <int HD>
__global__ __launch_bounds__(256) void attn_dq_store_kernel(AttnParams p) {
  constexpr int TPR = HD / 8;
  const long n = (long)p.B * p.Tq * p.H * TPR;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int t = i % TPR;
    const long row = i / TPR;
    const long h = row % p.H, q = (row / p.H) % p.Tq, b = row / ((long)p.H * p.Tq);
    float a[8];
    load8(p.dqacc + row * HD + 8 * t, a);
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] *= p.scale;
    if (SPA_DBG_BRH(b, q, p.Tq, h, p.H)) store8(p.dq + b * p.sdqb + q * p.sdqt + h * p.sdqh + 8 * t, a);
  }
}

// (the short-sequence fused backward, ViT T = 197: attention_short.hip)

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static void check_qkv(const at::Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16, n, " must be a bf16 HIP tensor");
  TORCH_CHECK(t.dim() == 4, n, " must be [B, T, H, hd]");
  TORCH_CHECK(t.stride(3) == 1, n, " must be contiguous in hd");
  TORCH_CHECK(((uintptr_t)t.data_ptr() % 16) == 0 && t.stride(1) % 8 == 0 && t.stride(2) % 8 == 0 &&
                  t.stride(0) % 8 == 0,
              n, ": rows must be 16-byte aligned");
}

// forward uses 8 waves (2 per SIMD) for head dims <= 192, 4 waves for 256; dq keeps q, dO and
// the dQ accumulator in registers and needs one wave per SIMD (the AGPR half of the register
// file) beyond square 128
template <int HDK, int HDV> constexpr int fwd_waves() {
  return (HDK <= 192 && HDV <= 192) || (HDK == 256 && HDV == 128) ? 8 : 4;
}
template <int HDK, int HDV> constexpr int dq_waves() { return (HDK <= 128 && HDV <= 128) ? 8 : 4; }

// (q/k head dim, v head dim) instantiations: the square 64/128/256 and MLA's 192/128
#define HDKV_SWITCH(HK, HV, ...)                                                                   \
  if (HK == 64 && HV == 64) { constexpr int HDK_ = 64, HDV_ = 64; __VA_ARGS__; }                  \
  else if (HK == 128 && HV == 128) { constexpr int HDK_ = 128, HDV_ = 128; __VA_ARGS__; }         \
  else if (HK == 256 && HV == 256) { constexpr int HDK_ = 256, HDV_ = 256; __VA_ARGS__; }         \
  else if (HK == 192 && HV == 128) { constexpr int HDK_ = 192, HDV_ = 128; __VA_ARGS__; }         \
  else TORCH_CHECK(false, "flash attention: (qk, v) head dims must be (64,64), (128,128), (256,256) or (192,128)");

static void fill_strides(AttnParams& p, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v) {
  p.sqb = q.stride(0); p.sqt = q.stride(1); p.sqh = q.stride(2);
  p.skb = k.stride(0); p.skt = k.stride(1); p.skh = k.stride(2);
  p.svb = v.stride(0); p.svt = v.stride(1); p.svh = v.stride(2);
}

// XCD-aware block order for the query-parallel kernels (q_block_map) when B * Hkv % 8 == 0;
// SPA_ATTN_XCD=0 (read per call) keeps the q-block-major order
static int xcd_order(int B, int Hkv) {
  const char* e = getenv("SPA_ATTN_XCD");
  if (e && atoi(e) == 0) return 0;
  return ((long)B * Hkv) % 8 == 0 ? 1 : 0;
}

static void fill_dropout(AttnParams& p, double dropout_p, int64_t seed, const c10::optional<at::Tensor>& seed_t) {
  if (seed_t) {
    TORCH_CHECK(seed_t->is_cuda() && seed_t->scalar_type() == at::kLong && seed_t->numel() >= 1,
                "attention seed_t: int64 device tensor");
    p.seed_ptr = seed_t->data_ptr<int64_t>();
  }
  TORCH_CHECK(dropout_p >= 0.0 && dropout_p < 1.0, "attention dropout p must be in [0, 1)");
  p.seed_lo = (unsigned)(seed & 0xffffffffu);
  p.seed_hi = (unsigned)(((uint64_t)seed >> 32) & 0xffffffffu);
  p.drop_thr = (unsigned)std::llround(dropout_p * 16777216.0);  // 24-bit uniform
  p.drop_scale = (float)(1.0 / (1.0 - dropout_p));
}

// Key split of the query-parallel kernels: with few (b, head) pairs (TP-sharded MQA: 2 q-heads
// per rank) the grid is a fraction of the chip -- T 8192 at head dim 256 is 128 blocks of 8 waves
// for 256 CUs, and the longest causal block runs all 256 key tiles alone. Split each query block's
// key tiles into ksplit shares (fp32 partials + a merge pass) until there are >= 512 blocks,
// keeping >= 4 key tiles per share. SPA_ATTN_KSPLIT (read per call): 0/1 off, N forces N.
static int attn_ksplit(long blocks, int ntk) {
  const char* e = getenv("SPA_ATTN_KSPLIT");
  if (e) return std::max(1, std::min(atoi(e), std::max(1, ntk)));
  int ks = 1;
  while (blocks * ks < 512 && ks < 8 && ntk / (2 * ks) >= 4) ks *= 2;
  return ks;
}

// q [B,Tq,H,dk], k [B,Tk,Hkv,dk], v [B,Tk,Hkv,dv] (strided views allowed).
// Returns (out [B,Tq,H,dv], lse [B,H,Tq]). dropout_p > 0: fused dropout on P (seeded hash).
std::vector<at::Tensor> attn_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, double scale,
                                 bool causal, double dropout_p, int64_t seed,
                                 const c10::optional<at::Tensor>& seed_t) {
  check_qkv(q, "q"); check_qkv(k, "k"); check_qkv(v, "v");
  const int B = q.size(0), Tq = q.size(1), H = q.size(2), HDK = q.size(3), HDV = v.size(3);
  const int Tk = k.size(1), Hkv = k.size(2);
  TORCH_CHECK(k.size(0) == B && v.size(0) == B && v.size(1) == Tk && v.size(2) == Hkv && k.size(3) == HDK,
              "attn: shape mismatch");
  TORCH_CHECK(H % Hkv == 0, "attn: H must be a multiple of Hkv");
  const bool drop = dropout_p > 0.0;
  TORCH_CHECK(!drop || HDK == HDV, "attn: dropout needs equal q/k and v head dims");
  DeviceGuard g(q.device());
  auto out = at::empty({B, Tq, H, HDV}, q.options());
  auto lse = at::empty({B, H, Tq}, q.options().dtype(at::kFloat));
  AttnParams p{};
  p.q = (const bf16*)q.data_ptr(); p.k = (const bf16*)k.data_ptr(); p.v = (const bf16*)v.data_ptr();
  p.out = (bf16*)out.data_ptr(); p.lse = lse.data_ptr<float>();
  p.B = B; p.H = H; p.Hkv = Hkv; p.Tq = Tq; p.Tk = Tk;
  fill_strides(p, q, k, v);
  fill_dropout(p, dropout_p, seed, seed_t);
  p.sob = out.stride(0); p.sot = out.stride(1); p.soh = out.stride(2);
  p.scale = (float)scale; p.scale_log2 = (float)(scale * 1.4426950408889634);
  p.causal_off = Tk - Tq;
  p.hsplit = 1;
  p.ksplit = 1;
  p.xcd = xcd_order(B, Hkv);
  if (B * Tq * H == 0) return {out, lse};
  auto st = stream();
  // head dim 256 (Gemma MQA) as the (256, 128) kernel over two column halves (blockIdx.y), each
  // producing half of the output columns: the 128-wide O accumulator lets 8 waves (2 per SIMD)
  // share a CU, where the full 256-wide one holds a wave per SIMD, at the price of computing S
  // twice (1.5x the MFMA work). SPA_ATTN_SPLITV=0 (read per call) keeps the single 4-wave kernel.
  // Default at 256: the S-sharing wave-pair kernel (attn_fwd256p_kernel, 128 queries per block);
  // SPA_ATTN_FWD256=0 (read per call) falls back to the split-V launch.
  const char* f2e = getenv("SPA_ATTN_FWD256");
  const bool pshare = !(f2e && atoi(f2e) == 0) && HDK == 256 && HDV == 256 && !drop;
  const char* sve = getenv("SPA_ATTN_SPLITV");
  const bool splitv = !pshare && !(sve && atoi(sve) == 0) && HDK == 256 && HDV == 256 && !drop;
  const int nw = splitv || pshare ? 8 : (HDK <= 192 && HDV <= 192) || (HDK == 256 && HDV == 128) ? 8 : 4;
  const int blocks = cdiv(Tq, pshare ? 128 : 32 * nw) * H * B * (splitv ? 2 : 1);
  const int ntk = cdiv(Tk, (HDK >= 256 || HDV >= 256) ? 32 : 64);
  p.ksplit = attn_ksplit(blocks, ntk);
  at::Tensor part;
  if (p.ksplit > 1) {
    const long rows = (long)B * H * Tq;
    part = at::empty({(long)p.ksplit * rows * (HDV + 2)}, q.options().dtype(at::kFloat));
    p.part = part.data_ptr<float>();
    p.part_ld = HDV;
    p.mlpart = p.part + (long)p.ksplit * rows * HDV;
  }
  const int gx = blocks / (splitv ? 2 : 1) * p.ksplit;
  if (pshare) {
    if (causal) attn_fwd256p_kernel<true><<<gx, 512, 0, st>>>(p);
    else attn_fwd256p_kernel<false><<<gx, 512, 0, st>>>(p);
  } else if (splitv) {
    p.vhalf = 128;
    if (causal) attn_fwd_kernel<256, 128, 8, true, false><<<dim3(gx, 2), 512, 0, st>>>(p);
    else attn_fwd_kernel<256, 128, 8, false, false><<<dim3(gx, 2), 512, 0, st>>>(p);
  } else {
    HDKV_SWITCH(HDK, HDV, {
      constexpr int NW = fwd_waves<HDK_, HDV_>();
      constexpr bool SQ = HDK_ == HDV_;
      if (drop) {
        if constexpr (SQ) {
          if (causal) attn_fwd_kernel<HDK_, HDV_, NW, true, true><<<gx, NW * 64, 0, st>>>(p);
          else attn_fwd_kernel<HDK_, HDV_, NW, false, true><<<gx, NW * 64, 0, st>>>(p);
        }
      } else {
        if (causal) attn_fwd_kernel<HDK_, HDV_, NW, true, false><<<gx, NW * 64, 0, st>>>(p);
        else attn_fwd_kernel<HDK_, HDV_, NW, false, false><<<gx, NW * 64, 0, st>>>(p);
      }
    });
  }
  if (p.ksplit > 1) {
    const long n = (long)B * H * Tq * (HDV / 8);
    HDKV_SWITCH(HDK, HDV, { attn_fwd_merge_kernel<HDV_><<<(int)cdiv(n, 256L), 256, 0, st>>>(p); });
  }
  SPA_LAUNCH_CHECK();
  return {out, lse};
}

template <int HDK, int HDV, bool DROP>
static void launch_bwd(AttnParams& p, bool causal, bool fused, int dkdv_mode, int nkv, hipStream_t st,
                       const at::TensorOptions& bf16_opts) {
  constexpr int NW = dq_waves<HDK, HDV>();
  constexpr int MT = (HDK <= 128 && HDV <= 128) ? 2 : 1;
  // paired-wave dK/dV keeps half the state per wave at 2 waves/SIMD: spill-free for square
  // head dims <= 128 without dropout (the hash keys of the dropout variant tip the 128 one
  // over; at 256 one role needs > 256 registers, which 2 waves/SIMD cannot hold)
  constexpr bool PAIRED_OK = HDK == HDV && HDK <= 128 && !DROP;
  const int g2 = nkv * p.hsplit;
  if constexpr (HDK == HDV && HDK <= 128 && !DROP) {
    if (fused) {   // hd 256: the fused body exceeds the register file (spills)
      const long rows = (long)p.B * p.Tq * p.H;
      attn_delta_kernel<HDK><<<(int)cdiv(rows, 256 / (HDK / 8)), 256, 0, st>>>(p);
      if (causal) attn_bwd_dkdv_kernel<HDK, HDV, true, MT, true, false><<<g2, 256, 0, st>>>(p);
      else attn_bwd_dkdv_kernel<HDK, HDV, false, MT, true, false><<<g2, 256, 0, st>>>(p);
      const long n = rows * (HDK / 8);
      attn_dq_store_kernel<HDK><<<(int)std::min<long>((n + 255) / 256, 65536), 256, 0, st>>>(p);
      return;
    }
  }
  if constexpr (HDK == 128 && HDV == 128 && !DROP) {
    // dS-materialising backward (default for head dim 128 without a q-head split): delta pass,
    // dK/dV kernel that also stores dS, then dQ = dS K in one streaming product. SPA_ATTN_DQ_DS=0
    // (read per call) keeps the dq kernel that recomputes S and dP.
    const char* de = getenv("SPA_ATTN_DQ_DS");
    const bool want = !(de && atoi(de) == 0);
    // (the per-(b, kv-head) dS region is addressed by a buffer descriptor: < 2 GiB, T <= ~22K causal)
    const long kv_bytes = 2 * ds_kv_elems(cdiv(p.Tq, 64), cdiv(p.Tk, 32), p.H / p.Hkv, causal);
    if (want && p.hsplit == 1 && p.Tk > 0 && dkdv_mode == 0 && (!causal || p.causal_off == 0) &&
        kv_bytes < 0x7fffffffL) {
      const long rows = (long)p.B * p.Tq * p.H;
      const char* v5e = getenv("SPA_ATTN_DKDV5");
      const bool v5 = !(v5e && atoi(v5e) == 0);
      if (!v5) attn_delta_kernel<HDK><<<(int)cdiv(rows, 256 / (HDK / 8)), 256, 0, st>>>(p);
      p.ds_nqt = cdiv(p.Tq, 32);
      p.ds_nkt = cdiv(p.Tk, 32);
      p.ds_kvstride = ds_kv_elems(cdiv(p.Tq, 64), p.ds_nkt, p.H / p.Hkv, causal);
      at::Tensor dsb = at::empty({(long)p.B * p.Hkv * p.ds_kvstride}, bf16_opts);   // freed (stream-ordered) on return
      p.dsbuf = (bf16*)dsb.data_ptr();
      // default: the LDS-DMA-staged dK/dV kernel with incremental bookkeeping (attention_dkdv5.hip,
      // its row-constant pass replaces the delta pass); SPA_ATTN_DKDV5=0 (read per call) keeps dkdv3
      at::Tensor rowk;
      if (v5) {
        p.rowk_ld = cdiv(p.Tq, 64) * 64;
        rowk = at::empty({(long)p.B * p.H * 2 * p.rowk_ld}, bf16_opts.dtype(at::kFloat));
        p.rowk = rowk.data_ptr<float>();
        launch_dkdv5(p, causal, st);
      } else if (causal) attn_bwd_dkdv3_kernel<HDK, HDV, true, true><<<nkv, 512, 0, st>>>(p);
      else attn_bwd_dkdv3_kernel<HDK, HDV, false, true><<<nkv, 512, 0, st>>>(p);
      const int G = p.H / p.Hkv;
      const int wg = cdiv(cdiv(p.Tq, 64) * G, 4) * p.B * p.Hkv;
      // SPA_ATTN_DS_NT (read per call, default 1): dS streamed with non-temporal loads, so the
      // once-read 2 KiB blocks do not evict the K tiles every block of the XCD re-reads
      const char* ne = getenv("SPA_ATTN_DS_NT");
      const bool nt = !(ne && atoi(ne) == 0);
      if (nt) {
        if (causal) attn_bwd_dq_ds_kernel<HDK, true, true><<<wg, 256, 0, st>>>(p);
        else attn_bwd_dq_ds_kernel<HDK, false, true><<<wg, 256, 0, st>>>(p);
      } else {
        if (causal) attn_bwd_dq_ds_kernel<HDK, true, false><<<wg, 256, 0, st>>>(p);
        else attn_bwd_dq_ds_kernel<HDK, false, false><<<wg, 256, 0, st>>>(p);
      }
      return;
    }
  }
  if constexpr (((HDK == 256 && HDV == 256) || (HDK == 192 && HDV == 128)) && !DROP) {
    // dS-materialising backward at head dims 256 (Gemma) and (192, 128) (MLA): the single-wave
    // dK/dV kernel also stores dS, then dQ = dS K streams it (attn_bwd_dq_ds256_kernel) -- instead
    // of the dq kernel's three products (S and dP recomputed over 192 / 256-deep contractions).
    // SPA_ATTN_DQ_DS (per call): 0 keeps the dq kernel, 2 takes this path at any grid size.
    const char* de = getenv("SPA_ATTN_DQ_DS");
    const int dsm = de ? atoi(de) : 1;     // 0 off, 1 by grid size, 2 always
    const bool want = dsm != 0;
    const int G = p.H / p.Hkv;
    const long kv_bytes = 2 * ds_kv_elems(cdiv(p.Tq, 64), cdiv(p.Tk, 32), G, causal);
    // the dQ pass has one block per 4 (q-head, 32-query) units: with few of them (TP-sharded MQA,
    // 2 q-heads: 128 blocks at T 8192) the key-split dq kernel fills the chip better (measured
    // 0.364 vs 0.391 ms there; 1.70 vs 2.21 ms for the 16-head layout)
    const int wg = cdiv(cdiv(p.Tq, 32) * G, 4) * p.B * p.Hkv;
    if (want && (wg >= 512 || dsm == 2) && p.Tk > 0 && dkdv_mode == 0 && (!causal || p.causal_off == 0) &&
        kv_bytes < 0x7fffffffL) {
      const long rows = (long)p.B * p.Tq * p.H;
      attn_delta_kernel<HDV><<<(int)cdiv(rows, 256 / (HDV / 8)), 256, 0, st>>>(p);   // rowsum(dO O): v dims
      p.ds_nqt = cdiv(p.Tq, 32);
      p.ds_nkt = cdiv(p.Tk, 32);
      p.ds_kvstride = ds_kv_elems(cdiv(p.Tq, 64), p.ds_nkt, G, causal);
      at::Tensor dsb = at::empty({(long)p.B * p.Hkv * p.ds_kvstride}, bf16_opts);   // freed (stream-ordered) on return
      p.dsbuf = (bf16*)dsb.data_ptr();
      const int g2 = nkv * p.hsplit;
      // MLA without a head split: the paired, pipelined dK/dV kernel (role A: K fragments + dV^T,
      // role B: V fragments + dK^T, 2 waves per SIMD); SPA_ATTN_DKDV_MLA=1 (per call) keeps the
      // single-wave kernel (both accumulator sets in one wave, 1 wave per SIMD)
      bool paired_mla = false, dvs = false;
      AttnParams pk = p;   // dvs: the dK pass with its own q-head split
      at::Tensor dkpart;
      if constexpr (HDK == 256 && HDV == 256) {
        // Gemma: the paired dK/dV kernel with the dV^T accumulator split over its roles (2 waves per
        // SIMD), then dK = dS^T Q streamed from the stored dS beside the dQ pass; needs whole q-heads
        // per split. SPA_ATTN_DKDV256=0 (per call) keeps the single-wave kernel (dK + dV, 1 wave/SIMD)
        const char* ve = getenv("SPA_ATTN_DKDV256");
        dvs = !(ve && atoi(ve) == 0) && G % p.hsplit == 0;
        if (dvs) {
          if (causal) attn_bwd_dkdv3_kernel<HDK, HDV, true, true, true><<<g2, 512, 0, st>>>(p);
          else attn_bwd_dkdv3_kernel<HDK, HDV, false, true, true><<<g2, 512, 0, st>>>(p);
          // the dK pass runs two blocks per CU, all of one round at Gemma's 512 blocks: the causal
          // key blocks' unequal work (key block 0 sees every query tile, the last one 4) then set its
          // time (0.427 ms, 645 TF). Finer q-head shares (>= 1024 blocks, heaviest launched first)
          // let the light blocks fill in behind the heavy ones
          int hs2 = p.hsplit;
          while (nkv * hs2 < 1024 && hs2 < G) {
            int d = hs2 + 1;
            while (G % d) ++d;
            hs2 = d;
          }
          pk.hsplit = hs2;
          if (hs2 > 1) {
            dkpart = at::empty({(long)hs2 * p.B * p.Tk * p.Hkv * HDK}, bf16_opts.dtype(at::kFloat));
            pk.dkacc = dkpart.data_ptr<float>();
          }
          if (causal) attn_bwd_dk_ds256_kernel<true, true><<<nkv * hs2, 256, 0, st>>>(pk);
          else attn_bwd_dk_ds256_kernel<false, true><<<nkv * hs2, 256, 0, st>>>(pk);
        }
      }
      if constexpr (HDK == 192 && HDV == 128) {
        const char* me = getenv("SPA_ATTN_DKDV_MLA");
        paired_mla = p.hsplit == 1 && !(me && atoi(me) == 1);
        if (paired_mla) {
          if (causal) attn_bwd_dkdv3_kernel<HDK, HDV, true, true><<<g2, 512, 0, st>>>(p);
          else attn_bwd_dkdv3_kernel<HDK, HDV, false, true><<<g2, 512, 0, st>>>(p);
        }
      }
      if (!paired_mla && !dvs) {
        if (causal) attn_bwd_dkdv_kernel<HDK, HDV, true, 1, false, false, true><<<g2, 256, 0, st>>>(p);
        else attn_bwd_dkdv_kernel<HDK, HDV, false, 1, false, false, true><<<g2, 256, 0, st>>>(p);
      }
      const char* ne = getenv("SPA_ATTN_DS_NT");
      const bool nt = !(ne && atoi(ne) == 0);
      if (nt) {
        if (causal) attn_bwd_dq_ds256_kernel<HDK, true, true><<<wg, 256, 0, st>>>(p);
        else attn_bwd_dq_ds256_kernel<HDK, false, true><<<wg, 256, 0, st>>>(p);
      } else {
        if (causal) attn_bwd_dq_ds256_kernel<HDK, true, false><<<wg, 256, 0, st>>>(p);
        else attn_bwd_dq_ds256_kernel<HDK, false, false><<<wg, 256, 0, st>>>(p);
      }
      const long kr = (long)p.B * p.Tk * p.Hkv;
      if ((dvs ? pk : p).hsplit > 1)
        attn_kv_reduce_kernel<HDK><<<(int)std::min<long>((kr * (HDK / 8) + 255) / 256, 65536), 256, 0, st>>>(dvs ? pk : p, 1);
      if (p.hsplit > 1)
        attn_kv_reduce_kernel<HDV><<<(int)std::min<long>((kr * (HDV / 8) + 255) / 256, 65536), 256, 0, st>>>(p, 0);
      return;
    }
  }
  const int grid = cdiv(p.Tq, 32 * NW) * p.H * p.B;
  p.ksplit = p.Tk > 0 ? attn_ksplit(grid, cdiv(p.Tk, attn_bn<HDK, HDV>())) : 1;
  at::Tensor dqpart;
  if (p.ksplit > 1) {
    dqpart = at::empty({(long)p.ksplit * p.B * p.Tq * p.H * HDK}, bf16_opts.dtype(at::kFloat));
    p.part = dqpart.data_ptr<float>();
    p.part_ld = HDK;
  }
  if (causal) attn_bwd_dq_kernel<HDK, HDV, NW, true, DROP><<<grid * p.ksplit, NW * 64, 0, st>>>(p);
  else attn_bwd_dq_kernel<HDK, HDV, NW, false, DROP><<<grid * p.ksplit, NW * 64, 0, st>>>(p);
  if (p.ksplit > 1) {
    const long n = (long)p.B * p.Tq * p.H * (HDK / 8);
    attn_dq_reduce_kernel<HDK><<<(int)cdiv(n, 256L), 256, 0, st>>>(p);
  }
  if (p.Tk == 0) return;
  const bool piped = PAIRED_OK && (dkdv_mode == 3 || (dkdv_mode == 0 && HDV == 128));
  if (piped) {
    if constexpr (PAIRED_OK) {
      if (causal) attn_bwd_dkdv3_kernel<HDK, HDV, true><<<g2, 512, 0, st>>>(p);
      else attn_bwd_dkdv3_kernel<HDK, HDV, false><<<g2, 512, 0, st>>>(p);
    }
  } else {
    if (causal) attn_bwd_dkdv_kernel<HDK, HDV, true, MT, false, DROP><<<g2, 256, 0, st>>>(p);
    else attn_bwd_dkdv_kernel<HDK, HDV, false, MT, false, DROP><<<g2, 256, 0, st>>>(p);
  }
  if (p.hsplit > 1) {
    const long rows = (long)p.B * p.Tk * p.Hkv;
    attn_kv_reduce_kernel<HDK><<<(int)std::min<long>((rows * (HDK / 8) + 255) / 256, 65536), 256, 0, st>>>(p, 1);
    attn_kv_reduce_kernel<HDV><<<(int)std::min<long>((rows * (HDV / 8) + 255) / 256, 65536), 256, 0, st>>>(p, 0);
  }
}

static at::Tensor& last_stamps() {
  static at::Tensor t;
  return t;
}
// profiling: the segment sums of the last SPA_ATTN_STAMP backward ([blocks * 8 waves, 8] int64,
// columns as listed at SPA_DKDV3_STAMP)
at::Tensor attn_bwd_stamps() { return last_stamps().defined() ? last_stamps().view({-1, 8}).clone() : at::Tensor(); }

// Gradients written into dq/dk/dv (strided views allowed, e.g. slices of one dqkv buffer).
void attn_bwd(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
              const at::Tensor& out, const at::Tensor& lse, const at::Tensor& dq, const at::Tensor& dk,
              const at::Tensor& dv, double scale, bool causal, double dropout_p, int64_t seed,
              const c10::optional<at::Tensor>& seed_t) {
  check_qkv(dout, "dout"); check_qkv(q, "q"); check_qkv(k, "k"); check_qkv(v, "v"); check_qkv(out, "out");
  check_qkv(dq, "dq"); check_qkv(dk, "dk"); check_qkv(dv, "dv");
  const int B = q.size(0), Tq = q.size(1), H = q.size(2), HDK = q.size(3), HDV = v.size(3);
  const int Tk = k.size(1), Hkv = k.size(2);
  TORCH_CHECK(lse.is_contiguous() && lse.numel() == (int64_t)B * H * Tq);
  TORCH_CHECK(dq.sizes() == q.sizes() && dk.sizes() == k.sizes() && dv.sizes() == v.sizes());
  TORCH_CHECK(dout.sizes() == out.sizes() && out.size(3) == HDV && out.size(2) == H && out.size(1) == Tq);
  const bool drop = dropout_p > 0.0;
  TORCH_CHECK(!drop || HDK == HDV, "attn: dropout needs equal q/k and v head dims");
  DeviceGuard g(q.device());
  auto delta = at::empty({B, H, Tq}, q.options().dtype(at::kFloat));
  AttnParams p{};
  p.q = (const bf16*)q.data_ptr(); p.k = (const bf16*)k.data_ptr(); p.v = (const bf16*)v.data_ptr();
  p.o = (const bf16*)out.data_ptr(); p.dout = (const bf16*)dout.data_ptr();
  p.dq = (bf16*)dq.data_ptr(); p.dk = (bf16*)dk.data_ptr(); p.dv = (bf16*)dv.data_ptr();
  p.lse_in = lse.data_ptr<float>(); p.delta = delta.data_ptr<float>();
  p.B = B; p.H = H; p.Hkv = Hkv; p.Tq = Tq; p.Tk = Tk;
  fill_strides(p, q, k, v);
  fill_dropout(p, dropout_p, seed, seed_t);
  p.sob = out.stride(0); p.sot = out.stride(1); p.soh = out.stride(2);
  p.sdob = dout.stride(0); p.sdot = dout.stride(1); p.sdoh = dout.stride(2);
  p.sdqb = dq.stride(0); p.sdqt = dq.stride(1); p.sdqh = dq.stride(2);
  p.sdkb = dk.stride(0); p.sdkt = dk.stride(1); p.sdkh = dk.stride(2);
  p.sdvb = dv.stride(0); p.sdvt = dv.stride(1); p.sdvh = dv.stride(2);
  p.scale = (float)scale; p.scale_log2 = (float)(scale * 1.4426950408889634);
  p.causal_off = Tk - Tq;
  p.xcd = xcd_order(B, Hkv);
  p.ksplit = 1;
  if (B * H == 0) return;
  auto st = stream();
  if (Tq == 0) { dk.zero_(); dv.zero_(); return; }
  // default: the deterministic two-kernel path (dq kernel + dkdv kernel, no atomics).
  // SPA_ATTN_BWD_FUSED=1: one pass computing dQ too (5 MFMA products per tile instead of 7)
  // with fp32 dQ atomics. Measured on MI355X at LLaMA3-8B shape (B1 T8192 H32/8 hd128):
  // fused 3.87 ms vs split 2.74 ms -- with 128-key blocks each dQ row receives T/128 atomic
  // adds (~4 GB of adds per call), past the chip-wide atomic rate; kept as an option.
  static const bool want_fused = getenv("SPA_ATTN_BWD_FUSED") && atoi(getenv("SPA_ATTN_BWD_FUSED")) != 0;
  const bool fused = want_fused && Tk > 0 && HDK <= 128 && HDK == HDV && !drop;
  // short sequences (ViT, T = 197): one fused launch per (b, h) with the whole sequence in LDS.
  // SPA_ATTN_SHORT=0 (read per call) keeps the split kernels.
  const char* sse = getenv("SPA_ATTN_SHORT");
  const bool want_short = !(sse && atoi(sse) == 0);
  if (want_short && !fused && !drop && HDK == 64 && HDV == 64 && H == Hkv && Tq <= 256 && Tk <= 256) {
    launch_bwd_short(p, causal, st);
    SPA_LAUNCH_CHECK();
    return;
  }
  at::Tensor dqacc;
  if (fused) {
    dqacc = at::zeros({B, Tq, H, HDK}, q.options().dtype(at::kFloat));
    p.dqacc = dqacc.data_ptr<float>();
  }
  // dK/dV grid: key blocks x kv-heads x batch, times a q-head split when that grid cannot
  // fill the chip (MQA: Hkv = 1 launched 32 blocks at T = 4096); partials are summed by
  // attn_kv_reduce_kernel. dK/dV kernel: software-pipelined paired-wave (3) for v head dim
  // 128, single-wave (1) else.
  // SPA_ATTN_DKDV overrides (1 single-wave, 3 pipelined; read per call, so one process can
  // A/B them). Measured on MI355X (rocprofv3, LLaMA3-8B shape B1 T8192 H32/8 hd128 causal):
  // dK/dV kernel 1.31 ms pipelined vs 1.46 ms for the removed two-phase paired kernel (whole
  // bwd 2.22 ms two-phase vs 2.45 ms single-wave); ViT-B hd 64 (T 197, B 64) whole bwd 0.113
  // pipelined / 0.097-0.103 single-wave.
  const int dkdv_mode = getenv("SPA_ATTN_DKDV") ? atoi(getenv("SPA_ATTN_DKDV")) : 0;
  const int G = H / Hkv;
  const int nkv = cdiv(Tk, 128) * Hkv * B;
  int hsplit = 1;
  // SPA_ATTN_KVBLOCKS (read per call, default 512): the dK/dV grid the q-head split aims for
  const char* kbe = getenv("SPA_ATTN_KVBLOCKS");
  const int kvblocks = kbe ? std::max(1, atoi(kbe)) : 512;
  if (!fused)
    while (nkv * hsplit < kvblocks && hsplit < G) {
      int d = hsplit + 1;
      while (G % d) ++d;
      hsplit = d;
    }
  // the single-wave dK/dV kernel splits the (q-head, q-tile) iterations of a kv-head in any
  // number of shares: past the q-heads (TP-sharded MQA: G = 2), split the q-tiles too
  const bool pairedk = HDK == HDV && HDK <= 128 && !drop && (dkdv_mode == 3 || (dkdv_mode == 0 && HDV == 128));
  if (!fused && !pairedk)
    while (nkv * hsplit < kvblocks && hsplit < 16 && cdiv(Tq, 32) / (2 * hsplit) >= 4) hsplit *= 2;
  p.hsplit = hsplit;
  // SPA_ATTN_STAMP=1: per-wave s_memtime segment sums of the pipelined dK/dV loop (in a build
  // with -DSPA_DKDV3_STAMP=1, tools/build_variant.sh), kept in a process-global buffer the
  // profiling tool reads back (attn_bwd_stamps)
  static at::Tensor stamps;
  const char* se = getenv("SPA_ATTN_STAMP");
  if (se && atoi(se) != 0) {
    const long need = (long)nkv * hsplit * 8 * 8;
    if (!stamps.defined() || stamps.numel() < need || stamps.device() != q.device())
      stamps = at::zeros({need}, q.options().dtype(at::kLong));
    p.stamp = (long long*)stamps.data_ptr<int64_t>();
    last_stamps() = stamps.narrow(0, 0, need);
  }
  at::Tensor kvacc;
  if (hsplit > 1) {
    kvacc = at::empty({(long)hsplit * B * Tk * Hkv * (HDK + HDV)}, q.options().dtype(at::kFloat));
    p.dkacc = kvacc.data_ptr<float>();
    p.dvacc = p.dkacc + (long)hsplit * B * Tk * Hkv * HDK;
  }
  HDKV_SWITCH(HDK, HDV, {
    if (drop) {
      if constexpr (HDK_ == HDV_) launch_bwd<HDK_, HDV_, true>(p, causal, false, dkdv_mode, nkv, st, q.options());
    } else {
      launch_bwd<HDK_, HDV_, false>(p, causal, fused, dkdv_mode, nkv, st, q.options());
    }
  });
  SPA_LAUNCH_CHECK();
}

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.def("attn_fwd(Tensor q, Tensor k, Tensor v, float scale, bool causal, float dropout_p=0.0, int seed=0, "
        "Tensor? seed_t=None) -> Tensor[]");
  m.def("attn_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor out, Tensor lse, Tensor(a!) dq, Tensor(b!) dk, "
        "Tensor(c!) dv, float scale, bool causal, float dropout_p=0.0, int seed=0, Tensor? seed_t=None) -> ()");
  m.def("attn_bwd_stamps() -> Tensor", &spa::attn_bwd_stamps);   // no tensor args: catch-all impl
}
TORCH_LIBRARY_IMPL(spa, CUDA, m) {
  m.impl("attn_fwd", &spa::attn_fwd);
  m.impl("attn_bwd", &spa::attn_bwd);
}
