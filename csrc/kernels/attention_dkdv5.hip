// Backward dK/dV at head dim 128, version 5: the paired-wave, software-pipelined kernel of
// attention.hip (attn_bwd_dkdv3_kernel, DSOUT form) with its Q / dO staging moved to LDS-DMA and
// its per-interval scalar bookkeeping made incremental.
//
// Same algorithm, layout and numerics as dkdv3 (block = 8 waves = 4 pairs x 32 keys; role A (waves
// 0-3) holds K and dV^T, role B (waves 4-7) V and dK^T; one barrier per 64-query interval:
//   interval k, role A:  dV^T += dO(k-1)^T P(k-1)   |  S(k) = Q(k) K^T -> P(k) -> LDS
//   interval k, role B:  dP(k-1) = dO(k-1) V^T - delta;  dS = P(k-1) dP(k-1) -> HBM;  dK^T += Q(k-1)^T dS
// with P through a 2-deep LDS ring and Q / dO tiles in a 3-deep ring). What changed, and why:
//  * Staging is LDS-DMA (buffer_load ... lds, inline asm; attn_common.h dma16_asm): each wave moves
//    rows 4w..4w+3 and 4w+32..4w+35 of the next Q and dO tiles (one 1 KiB piece each; the image's XOR
//    swizzle is applied to the SOURCE address so the LDS side stays lane-linear), and waves 0 / 1
//    the tile's 64 row constants (-lse*log2e | -delta, written by attn_rowk_kernel) with one
//    4-byte-per-lane piece. dkdv3 staged through 16 loader VGPRs, a ds_write pass and plain loads
//    (every wave's commit waited vmcnt at the interval's head); here a wave waits for its own DMA
//    once, before the interval's barrier.
//  * The interval's tile indices, head offsets and descriptor bases advance incrementally (no integer
//    division, no 64-bit multiplies in the loop). dkdv3 spent ~230 SALU instructions per wave per
//    interval on them, x 8 waves through the CU's one scalar unit.
// profiles/r5_attn_dkdv5.txt: stamps, A/Bs against dkdv3. Selected by SPA_ATTN_DKDV5 (attention.hip).
#include "attn_common.h"
#include "attn_params.h"

SPA_DEBUG_TU("attention_dkdv5.hip")

namespace spa {

// 4 B per lane of a buffer straight into LDS (lane i -> lds + 4 i); as dma16_asm (attn_common.h)
__device__ __forceinline__ void dma4_asm(__amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dword %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(rs), "s"(lds) : "memory");
}

// rowk [B*H][2][Tqp]: -lse*log2(e) | -delta (delta = rowsum(dO * O)), zeros for Tq <= q < Tqp
// (the DMA'd row constants of attn_bwd_dkdv5_kernel; a zero row constant on a zero-padded query
// row leaves every product of that row zero, as the masked constants of dkdv3 did)
template <int HD>
__global__ __launch_bounds__(256) void attn_rowk_kernel(AttnParams p) {
  constexpr int TPR = HD / 8, RPB = 256 / TPR;
  const int Tqp = p.rowk_ld;
  const long row = (long)blockIdx.x * RPB + threadIdx.x / TPR;   // (b, q, h), h fastest
  const int t = threadIdx.x % TPR;
  const long nrows = (long)p.B * Tqp * p.H;
  float acc = 0.f;
  long b = 0, q = 0, h = 0;
  if (row < nrows) {
    h = row % p.H;
    q = (row / p.H) % Tqp;
    b = row / ((long)p.H * Tqp);
    if (q < p.Tq) {
      float a[8], c[8];
      load8(p.dout + b * p.sdob + q * p.sdot + h * p.sdoh + 8 * t, a);
      load8(p.o + b * p.sob + q * p.sot + h * p.soh + 8 * t, c);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc += a[i] * c[i];
    }
  }
#pragma unroll
  for (int o = TPR / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, TPR);
  if (row < nrows && t == 0 && SPA_DBG_OK(((b * p.H + h) * 2 + 1) * (long)Tqp + q, (long)p.B * p.H * 2 * Tqp)) {
    float* dst = p.rowk + ((b * p.H + h) * 2) * (long)Tqp + q;
    const bool v = q < p.Tq;
    dst[0] = v ? -p.lse_in[(b * p.H + h) * p.Tq + q] * 1.4426950408889634f : 0.f;
    dst[Tqp] = v ? -acc : 0.f;
  }
}

// SPA_DKDV5_STAMP=1 (profiling build, tools/build_variant.sh): per-wave s_memtime segment sums into
// p.stamp (SPA_ATTN_STAMP=1), [blocks * 8 waves, 8] int64: head (bookkeeping + DMA issue), compute,
// DMA wait (vmcnt), barrier wait, epilogue, intervals, whole wave, 0
#ifndef SPA_DKDV5_STAMP
#define SPA_DKDV5_STAMP 0
#endif
#if SPA_DKDV5_STAMP
#define D5_TICK(i)                                                    \
  do {                                                                \
    const long long tn_ = (long long)__builtin_amdgcn_s_memtime();    \
    seg[i] += tn_ - ts_;                                              \
    ts_ = tn_;                                                        \
  } while (0)
#else
#define D5_TICK(i) \
  do {             \
  } while (0)
#endif

// Wave-uniform position of one tile in the block's sweep (tile = (q-head g, 64-query tile qi),
// qi fastest) with the element offsets of its Q / dO rows and its rowk constants
struct D5Tile {
  int g, qi;
  long qoff, doff, roff;
};

// Measured and removed (profiles/r5_attn_dkdv5.txt): static priority for role B (+2.4 % time), role A
// alone issuing the whole tile (+5 %), each wave's four pieces issued one at a time behind its four
// MFMA chains (+7 %), and role A's S -> P exponentials interleaved into its next MFMA chain with
// sched_group_barrier (+2-3 %; role B's version needs ~32 VGPRs more than 256 and spilled).
template <bool CAUSAL>
__global__ __launch_bounds__(512) void attn_bwd_dkdv5_kernel(AttnParams p) {
  constexpr int HD = 128, MT = 2, BMQ = 64, BNK = 128, KS = HD / 16, DT = HD / 32;
  constexpr int TQ = BMQ * HD, TB = 2 * TQ, PSLOT = 4 * MT * 2 * 64 * 8, RSF = 2 * BMQ;
  // ONE __shared__ array (a second object can make hipcc wait vmcnt(0) ahead of the ds_reads):
  // [ring 3][Q | dO] images | P ring [2][pair][t][half][lane][8] | row constants [ring 3][-lse2 | -delta]
  __shared__ __attribute__((aligned(16))) bf16 smem[3 * TB + 2 * PSLOT + 3 * RSF * 2];
  bf16* const pimg = smem + 3 * TB;
  float* const rowc = reinterpret_cast<float*>(pimg + 2 * PSLOT);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pair = wave & 3, role = wave >> 2;
  const int hh = lane >> 5;
  const int nbh = p.Hkv * p.B;
  const int bh = blockIdx.x % nbh;
  const int kb = blockIdx.x / nbh;                    // causal: low key blocks (heaviest) first
  const int hk = bh % p.Hkv, b = bh / p.Hkv;
  SPA_DBG_CHECK(b, p.B);
  const int G = p.H / p.Hkv;
  const int h0 = hk * G;
  const int kw0 = __builtin_amdgcn_readfirstlane(kb * BNK + pair * 32);
  const int key = kw0 + (lane & 31);
  const bool kvalid = key < p.Tk;
  const float c = p.scale_log2;
#if SPA_DKDV5_STAMP
  long long seg[5] = {0, 0, 0, 0, 0};
  const long long t_start = (long long)__builtin_amdgcn_s_memtime();
  long long ts_ = t_start;
#endif

  bf16x8 xf[KS];  // A: K fragments, B: V fragments of this lane's key
  {
    const bf16* xp = role == 0 ? p.k + b * p.skb + (long)key * p.skt + hk * p.skh + 8 * hh
                               : p.v + b * p.svb + (long)key * p.svt + hk * p.svh + 8 * hh;
#pragma unroll
    for (int s = 0; s < KS; ++s) xf[s] = kvalid ? *reinterpret_cast<const bf16x8*>(xp + 16 * s) : zero8();
  }
  f32x16 acc[DT];  // A: dV^T, B: dK^T
#pragma unroll
  for (int i = 0; i < DT; ++i) acc[i] = splat16(0.f);

  int qstart = 0, wave_qstart = 0;
  if (CAUSAL) {
    qstart = max(0, kb * BNK - p.causal_off);
    wave_qstart = max(0, kw0 - p.causal_off);
  }
  const int t0 = qstart / BMQ;
  const int ntq = p.Tq > 0 ? cdiv(p.Tq, BMQ) : 0;
  const int nper = ntq - t0 > 0 ? ntq - t0 : 0;
  const int total = nper * G;
  const int Tqp = p.rowk_ld;

  // ---- tile sweep bookkeeping (scalar, incremental)
  const bf16* const qbase = p.q + b * p.sqb + (long)h0 * p.sqh;
  const bf16* const dbase = p.dout + b * p.sdob + (long)h0 * p.sdoh;
  const float* const rbase = p.rowk + (long)(b * p.H + h0) * 2 * Tqp;
  const long qstep = (long)BMQ * p.sqt, dstep = (long)BMQ * p.sdot;
  // next q-head: back to tile t0 of the next head
  const long qwrap = p.sqh - (long)(nper - 1) * qstep, dwrap = p.sdoh - (long)(nper - 1) * dstep;
  const long rwrap = 2L * Tqp - (long)(nper - 1) * BMQ;
  // descriptor ranges: a full tile, and the sweep's last (possibly ragged) tile row count
  const int lastrows = p.Tq - (t0 + nper - 1) * BMQ;
  const int qrec_full = (int)(((long)(BMQ - 1) * p.sqt + HD) * 2), drec_full = (int)(((long)(BMQ - 1) * p.sdot + HD) * 2);
  const int qrec_last = lastrows > 0 ? (int)(((long)(lastrows - 1) * p.sqt + HD) * 2) : 0;
  const int drec_last = lastrows > 0 ? (int)(((long)(lastrows - 1) * p.sdot + HD) * 2) : 0;
  auto advance = [&](D5Tile& t) {
    if (t.qi + 1 < nper) {
      ++t.qi;
      t.qoff += qstep;
      t.doff += dstep;
      t.roff += BMQ;
    } else {
      t.qi = 0;
      ++t.g;
      t.qoff += qwrap;
      t.doff += dwrap;
      t.roff += rwrap;
    }
  };
  // DMA source offsets: rows rl and rl + 32 of a tile (rl = 4 wave + lane / 16); image chunk lane % 16
  // of row r holds source chunk (lane % 16) ^ swz(r), and swz(rl + 32) == swz(rl)
  const int rl = 4 * wave + (lane >> 4);
  const int chs = 8 * ((lane & 15) ^ swz<HD>(rl));
  const unsigned qvo = (unsigned)(((long)rl * p.sqt + chs) * 2), qvo2 = qvo + (unsigned)(32 * p.sqt * 2);
  const unsigned dvo = (unsigned)(((long)rl * p.sdot + chs) * 2), dvo2 = dvo + (unsigned)(32 * p.sdot * 2);
  // piece j of tile t into ring slot SL: 0 / 1 Q rows 4w.. / 4w+32.., 2 / 3 the same dO rows
  auto piece = [&](const D5Tile& t, int j, auto slotc) {
    constexpr int SL = decltype(slotc)::value;
    const bool last = t.qi == nper - 1;
    bf16* sl = smem + SL * TB;
    if (j < 2) {
      const __amdgpu_buffer_rsrc_t rq =
          __builtin_amdgcn_make_buffer_rsrc((void*)(qbase + t.qoff), 0, last ? qrec_last : qrec_full, 0x00020000);
      dma16_asm(rq, j == 0 ? qvo : qvo2, lds_addr(sl + (4 * wave + 32 * j) * HD));
    } else {
      const __amdgpu_buffer_rsrc_t rd =
          __builtin_amdgcn_make_buffer_rsrc((void*)(dbase + t.doff), 0, last ? drec_last : drec_full, 0x00020000);
      dma16_asm(rd, j == 2 ? dvo : dvo2, lds_addr(sl + TQ + (4 * wave + 32 * (j - 2)) * HD));
    }
  };
  auto rowk_piece = [&](const D5Tile& t, auto slotc) {
    constexpr int SL = decltype(slotc)::value;
    if (wave < 2) {   // wave 0: -lse2 of the tile's 64 rows, wave 1: -delta
      const __amdgpu_buffer_rsrc_t rr =
          __builtin_amdgcn_make_buffer_rsrc((void*)(rbase + t.roff + wave * Tqp), 0, 4 * BMQ, 0x00020000);
      dma4_asm(rr, (unsigned)(lane * 4), lds_addr(rowc + SL * RSF + wave * BMQ));
    }
  };
  auto issue = [&](const D5Tile& t, auto slotc) {
    // debug build: the incremental bookkeeping still names a tile of this block's sweep, and its
    // row constants lie inside rowk
    SPA_DBG_CHECK(t.g, G);
    SPA_DBG_CHECK(t.qi, nper);
    SPA_DBG_CHECK((long)(b * p.H + h0) * 2 * Tqp + t.roff + Tqp + BMQ - 1, (long)p.B * p.H * 2 * Tqp);
    piece(t, 0, slotc);
    piece(t, 1, slotc);
    piece(t, 2, slotc);
    piece(t, 3, slotc);
    rowk_piece(t, slotc);
  };
  auto tile_active = [&](const D5Tile& t) {
    return kw0 < p.Tk && !(CAUSAL && (t0 + t.qi) * BMQ + BMQ - 1 < wave_qstart);
  };
  // dS stores: one buffer descriptor per (b, kv-head), scalar block offsets (ds_index, 32-bit: the
  // host keeps a (b, kv-head) region under 2 GiB)
  const __amdgpu_buffer_rsrc_t dsr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(p.dsbuf + ((long)b * p.Hkv + hk) * p.ds_kvstride), 0, (int)(p.ds_kvstride * 2), 0x00020000);
  const int dsvo = 16 * ds_slot(0, hh, lane & 31);
  const int kt = kw0 >> 5;
  auto store_ds = [&](const bf16x8& sa, const bf16x8& sb, int qt, int g) {
    const int qb = qt >> 1, t = qt & 1;
    const int step = CAUSAL ? qb * (qb + 1) + kt : qb * p.ds_nkt + kt;
    const int bo = ((step * G + g) * 2 + t) * 2048;
    SPA_DBG_CHECK(bo / 2048, p.ds_kvstride / 1024);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, sa), dsr, dsvo, bo, 0);        // s = 0
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, sb), dsr, dsvo + 128, bo, 0);  // s = 1
  };

  // fragment loads retired here, before any DMA is in flight (hipcc cannot count the asm DMA)
#pragma unroll
  for (int s = 0; s < KS; ++s) asm volatile("" ::"v"(xf[s]));
  D5Tile tC{0, 0, (long)t0 * qstep, (long)t0 * dstep, (long)t0 * BMQ};   // tile k (interval k's S)
  D5Tile tP = tC;                                                       // tile k - 1
  D5Tile tN = tC;                                                       // tile k + 1 (DMA)
  if (total > 0) issue(tC, IC<0>{});
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  LdsOff<HD> off;   // Q and dO images share the width, so one set of offsets serves both
  off.init(lane);
  bf16* pme = pimg + pair * (MT * 2 * 64 * 8) + lane * 8;   // + slot * PSLOT + (t * 2 + half) * 512
  bool prev_act = false;

  // interval k (slot SC = k % 3): tiles k-1 (slot SP) and k (slot SC) resident, tile k+1 DMA'd into SN
  auto interval = [&](const int k, auto slotc, auto rolec) {
    constexpr int SC = decltype(slotc)::value, SP = (SC + 2) % 3, SN = (SC + 1) % 3;
    constexpr int ROLE = decltype(rolec)::value;
    // tile k+1 (past the end: a re-fetch of the last tile into a slot no longer read)
    tN = tC;
    if (k + 1 < total) advance(tN);
    issue(tN, IC<SN>{});
    D5_TICK(0);
    const bool cur = k < total && tile_active(tC);
    const bf16* Qc = smem + SC * TB;
    const bf16* Qp = smem + SP * TB;
    const bf16* Dp = Qp + TQ;
    const float* rcC = rowc + SC * RSF;             // tile k:   -lse2
    const float* rcP = rowc + SP * RSF + BMQ;       // tile k-1: -delta
    const bf16* pr = pme + ((k + 1) & 1) * PSLOT;   // P(k-1)
    bf16* pw = pme + (k & 1) * PSLOT;               // P(k)
    if constexpr (ROLE == 0) {
      if (prev_act) {                                // dV^T += dO(k-1)^T P(k-1)
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          const bf16x8 pa = *reinterpret_cast<const bf16x8*>(pr + (t * 2 + 0) * 512);
          const bf16x8 pb = *reinterpret_cast<const bf16x8*>(pr + (t * 2 + 1) * 512);
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            acc[dt] = mfma32(ld_tr(Dp + 32 * t * HD, off.tra[dt], off.trb[dt]), pa, acc[dt]);
            acc[dt] = mfma32(ld_tr(Dp + (32 * t + 16) * HD, off.tra[dt], off.trb[dt]), pb, acc[dt]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if (cur) {                                     // S(k) -> P(k) -> LDS slot k & 1
        const int qq0 = (t0 + tC.qi) * BMQ;
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          f32x16 s = mfma32(ld_row(Qc + 32 * t * HD, off.row[0]), xf[0], splat16(0.f));
#pragma unroll
          for (int ks = 1; ks < KS; ++ks) s = mfma32(ld_row(Qc + 32 * t * HD, off.row[ks]), xf[ks], s);
          const int qt0 = qq0 + 32 * t;
          if (CAUSAL && qt0 + p.causal_off < kw0 + 31) {
            const int d = key - qt0 - 4 * hh - p.causal_off;   // row offsets below d are masked
#pragma unroll
            for (int r = 0; r < 16; ++r)
              if ((r & 3) + 8 * (r >> 2) < d) s[r] = -INFINITY;
          }
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4 lv = *reinterpret_cast<const f32x4*>(rcC + 32 * t + 8 * g + 4 * hh);
#pragma unroll
            for (int i = 0; i < 4; ++i) s[4 * g + i] = fexp2(fmaf(s[4 * g + i], c, lv[i]));
          }
          *reinterpret_cast<bf16x8*>(pw + (t * 2 + 0) * 512) = pack_acc(s, 0);
          *reinterpret_cast<bf16x8*>(pw + (t * 2 + 1) * 512) = pack_acc(s, 1);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    } else if (!prev_act) {
    } else {                                         // tile k-1: dP, dS (-> HBM), dK^T
      const int qtp = (t0 + tP.qi) * (BMQ / 32);
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        f32x16 dp;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(rcP + 32 * t + 8 * g + 4 * hh);
#pragma unroll
          for (int i = 0; i < 4; ++i) dp[4 * g + i] = v[i];
        }
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) dp = mfma32(ld_row(Dp + 32 * t * HD, off.row[ks]), xf[ks], dp);
        const bf16x8 pa = *reinterpret_cast<const bf16x8*>(pr + (t * 2 + 0) * 512);
        const bf16x8 pb = *reinterpret_cast<const bf16x8*>(pr + (t * 2 + 1) * 512);
        f32x16 ds;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          ds[r] = (float)pa[r] * dp[r];
          ds[8 + r] = (float)pb[r] * dp[8 + r];
        }
        const bf16x8 sa = pack_acc(ds, 0), sb = pack_acc(ds, 1);
        const int qt = qtp + t;
        if ((!CAUSAL || kt <= qt) && qt < p.ds_nqt && kt < p.ds_nkt) store_ds(sa, sb, qt, tP.g);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          acc[dt] = mfma32(ld_tr(Qp + 32 * t * HD, off.tra[dt], off.trb[dt]), sa, acc[dt]);
          acc[dt] = mfma32(ld_tr(Qp + (32 * t + 16) * HD, off.tra[dt], off.trb[dt]), sb, acc[dt]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    prev_act = cur;
    tP = tC;
    tC = tN;
    // this wave's DMA of tile k+1 landed (and its dS stores left: the in-order counter); the barrier
    // publishes tile k+1 and P(k) for interval k+1 and retires every read of tile k-1's slot
    D5_TICK(1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    D5_TICK(2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's LDS reads / P stores done
    __builtin_amdgcn_s_barrier();
    D5_TICK(3);
  };
  // three intervals per trip, unconditionally (past k = total an interval only re-fetches the last
  // tile and meets the barrier; every wave of the block runs the same count): conditional intervals
  // left join points where hipcc re-homed all 64 accumulator registers (32 v_mov_b64) per trip
  if (total == 0) {
  } else if (role == 0) {
    for (int k = 0; k <= total; k += 3) {
      interval(k, IC<0>{}, IC<0>{});
      interval(k + 1, IC<1>{}, IC<0>{});
      interval(k + 2, IC<2>{}, IC<0>{});
    }
  } else {
    for (int k = 0; k <= total; k += 3) {
      interval(k, IC<0>{}, IC<1>{});
      interval(k + 1, IC<1>{}, IC<1>{});
      interval(k + 2, IC<2>{}, IC<1>{});
    }
  }
  store_kv_grad<HD>(p, acc, role == 1, b, hk, key, 0, hh);
#if SPA_DKDV5_STAMP
  D5_TICK(4);
  if (p.stamp != nullptr && lane < 8) {   // one value per lane: vector stores
    long long v = 0;
#pragma unroll
    for (int i = 0; i < 5; ++i) v = lane == i ? seg[i] : v;
    v = lane == 5 ? (long long)(total + 1) : lane == 6 ? ts_ - t_start : v;
    p.stamp[((long)blockIdx.x * 8 + wave) * 8 + lane] = v;
  }
#endif
}

// host side (called from attn_bwd, attention.hip): row constants, then the dK/dV kernel with
// the dS stores; p.dsbuf / ds_* and p.rowk (B*H*2*rowk_ld floats) are set by the caller
void launch_dkdv5(AttnParams& p, bool causal, hipStream_t st) {
  const long rows = (long)p.B * p.rowk_ld * p.H;
  attn_rowk_kernel<128><<<(int)cdiv(rows, 256 / 16), 256, 0, st>>>(p);
  const int nkv = cdiv(p.Tk, 128) * p.Hkv * p.B;
  if (causal) attn_bwd_dkdv5_kernel<true><<<nkv, 512, 0, st>>>(p);
  else attn_bwd_dkdv5_kernel<false><<<nkv, 512, 0, st>>>(p);
}

}  // namespace spa
