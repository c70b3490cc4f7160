// Wide-head flash attention: head dims D = 256 * NCH > 256 (Gemma-ref's 768-wide query heads
// over one shared 768-wide K/V head, gemma/gemma.ipynb:238-249 -- two "query heads" each as wide
// as the model, scale 1/sqrt(768)). The flash kernels of attention.hip hold a head's q/k and
// accumulator fragments in registers, which stops at 256; here the head dim is split in 256-wide
// CHUNKS:
//  * reductions over the head dim (S = Q K^T, dP = dO V^T) run over all NCH chunks, one operand
//    from a chunked LDS image ([NCH][rows][256], the swizzled 256-wide image of attention.hip per
//    chunk) and the other from registers or streamed from L1/L2 per k-step;
//  * every OUTPUT over the head dim (O, dQ, dK, dV) is produced one 256-wide chunk per workgroup
//    (grid.y = chunk), recomputing S (and dP) for each chunk: 2x the QK^T work of one pass, in
//    exchange for 128 accumulator registers instead of NCH x 128.
// Forward: S^T = K Q^T (query on the lane, Q fragments in registers), online softmax over 32-key
// tiles, O^T chunk = V^T P^T. Backward: delta = rowsum(dO * O); dQ (query-parallel, S and dP
// recomputed, dO streamed); dV and dK (key-parallel, key on the lane, K fragments in registers,
// the GQA group's q-heads summed in registers, V streamed for dP). One wave per SIMD (4-wave
// workgroups): the AGPR half of the register file holds the accumulators.
#include "attn_common.h"

namespace spa {

struct WideParams {
  const bf16* q; const bf16* k; const bf16* v; const bf16* o; const bf16* dout;
  bf16* out; bf16* dq; bf16* dk; bf16* dv;
  float* lse; const float* lse_in; float* delta;
  int B, H, Hkv, Tq, Tk;
  long sqb, sqt, sqh, skb, skt, skh, svb, svt, svh, sob, sot, soh;
  long sdob, sdot, sdoh, sdqb, sdqt, sdqh, sdkb, sdkt, sdkh, sdvb, sdvt, sdvh;
  float scale, scale_log2;
  int causal_off;
};

constexpr int kWideBN = 32;  // keys (fwd / dq) or queries (dk / dv) per LDS tile

// [NCH][ROWS][256] chunked image of a ROWS x D tile (rows >= nrows are zeros)
template <int NCH, int ROWS>
__device__ __forceinline__ void load_chunked(bf16* img, const bf16* base, long stride, int row0, int nrows,
                                             int tid) {
  TileLoader<256, ROWS, 256> ld;
  ld.init(stride, tid);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    ld.load(base + 256 * c, stride, row0, nrows);
    ld.store(img + c * ROWS * 256);
  }
}
template <int ROWS>
__device__ __forceinline__ void load_chunk1(bf16* img, const bf16* base, long stride, int row0, int nrows,
                                            int tid) {
  TileLoader<256, ROWS, 256> ld;
  ld.init(stride, tid);
  ld.load(base, stride, row0, nrows);
  ld.store(img);
}

// ----------------------------------------------------------------------------- forward
template <int NCH, bool CAUSAL>
__global__ __launch_bounds__(256) void wide_fwd_kernel(WideParams p) {
  constexpr int D = 256 * NCH, KS = D / 16, BN = kWideBN, BM = 128, DT = 8;
  __shared__ __attribute__((aligned(16))) bf16 smem[NCH * BN * 256 + BN * 256];  // K (all chunks) | V chunk z
  bf16* kimg = smem;
  bf16* vimg = smem + NCH * BN * 256;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lq = lane & 31, hh = lane >> 5;
  const int z = blockIdx.y;  // output chunk
  const int nqb = cdiv(p.Tq, BM), nbh = p.H * p.B;
  int qb = blockIdx.x / nbh;
  const int bh = blockIdx.x % nbh;
  if (CAUSAL) qb = nqb - 1 - qb;
  const int h = bh % p.H, b = bh / p.H, hk = h / (p.H / p.Hkv);
  const int q0 = __builtin_amdgcn_readfirstlane(qb * BM + wave * 32);
  const int q = q0 + lq;
  const float c = p.scale_log2;
  // Q fragments: in registers for NCH = 2; streamed from L1/L2 per k-step for NCH = 3 (the
  // 192 registers of a 768-wide query row would not fit beside the accumulators)
  constexpr bool QREG = NCH <= 2;
  const bool qvalid = q < p.Tq;
  const bf16* qp = p.q + b * p.sqb + (long)(qvalid ? q : 0) * p.sqt + h * p.sqh + 8 * hh;
  bf16x8 qf[QREG ? KS : 1];
  if constexpr (QREG) {
#pragma unroll
    for (int s = 0; s < KS; ++s) qf[s] = qvalid ? *reinterpret_cast<const bf16x8*>(qp + 16 * s) : zero8();
  }
  f32x16 o[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) o[i] = splat16(0.f);
  float m = -1e30f, l = 0.f;
  const int kend = CAUSAL ? min(p.Tk, qb * BM + BM + p.causal_off) : p.Tk;
  const int wave_kend = CAUSAL ? min(p.Tk, q0 + 32 + p.causal_off) : p.Tk;
  const int ntiles = kend > 0 ? cdiv(kend, BN) : 0;
  const bf16* kbase = p.k + b * p.skb + hk * p.skh;
  const bf16* vbase = p.v + b * p.svb + hk * p.svh + 256 * z;
  LdsOff<256> off;
  off.init(lane);
  for (int j = 0; j < ntiles; ++j) {
    const int k0 = j * BN;
    __syncthreads();  // previous tile consumed
    load_chunked<NCH, BN>(kimg, kbase, p.skt, k0, p.Tk, tid);
    load_chunk1<BN>(vimg, vbase, p.svt, k0, p.Tk, tid);
    __syncthreads();
    if (k0 >= wave_kend) continue;
    f32x16 s = splat16(0.f);
    if constexpr (QREG) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) s = mfma32(ld_row(kimg + (ks >> 4) * BN * 256, off.row[ks & 15]), qf[ks], s);
    } else {
#pragma unroll
      for (int cc = 0; cc < NCH; ++cc) {
        bf16x8 qs[16];
#pragma unroll
        for (int s2 = 0; s2 < 16; ++s2)
          qs[s2] = qvalid ? *reinterpret_cast<const bf16x8*>(qp + 256 * cc + 16 * s2) : zero8();
#pragma unroll
        for (int s2 = 0; s2 < 16; ++s2) s = mfma32(ld_row(kimg + cc * BN * 256, off.row[s2]), qs[s2], s);
      }
    }
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
    if (mxs > m) {  // exact online softmax (no deferral: these kernels are not VALU-bound)
      const float alpha = fexp2(m - mxs);
      l *= alpha;
#pragma unroll
      for (int i = 0; i < DT; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[i][r] *= alpha;
      m = mxs;
    }
    float ls = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s[r] = fexp2(fmaf(s[r], c, -m));
      ls += s[r];
    }
    l += ls;
    const bf16x8 pa = pack_acc(s, 0), pb = pack_acc(s, 1);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      o[dt] = mfma32(ld_tr(vimg, off.tra[dt], off.trb[dt]), pa, o[dt]);
      o[dt] = mfma32(ld_tr(vimg + 16 * 256, off.tra[dt], off.trb[dt]), pb, o[dt]);
    }
  }
  l = halfsum(l);
  const float inv = l > 0.f ? 1.f / l : 0.f;
  if (q < p.Tq) {
    bf16* op = p.out + b * p.sob + (long)q * p.sot + h * p.soh + 256 * z;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 w;
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = (bf16)(o[dt][4 * g + i] * inv);
        *reinterpret_cast<bf16x4*>(op + 32 * dt + 8 * g + 4 * hh) = w;
      }
    if (z == 0 && hh == 0)
      p.lse[((long)b * p.H + h) * p.Tq + q] = (l > 0.f) ? (m + __log2f(l)) * 0.69314718055994531f : INFINITY;
  }
}

// ------------------------------------------------------------------- delta = rowsum(dO*O)
template <int NCH>
__global__ __launch_bounds__(256) void wide_delta_kernel(WideParams p) {
  constexpr int D = 256 * NCH;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);  // one wave per (b, q, h) row
  const int lane = threadIdx.x & 63;
  const long nrows = (long)p.B * p.Tq * p.H;
  if (row >= nrows) return;
  const long h = row % p.H, q = (row / p.H) % p.Tq, b = row / ((long)p.H * p.Tq);
  float acc = 0.f;
  for (int d = 8 * lane; d < D; d += 512) {
    float a[8], o8[8];
    load8(p.dout + b * p.sdob + q * p.sdot + h * p.sdoh + d, a);
    load8(p.o + b * p.sob + q * p.sot + h * p.soh + d, o8);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += a[i] * o8[i];
  }
  acc = wave_sum(acc);
  if (lane == 0) p.delta[(b * p.H + h) * p.Tq + q] = acc;
}

// ----------------------------------------------------------------------------- dQ
// S^T = K Q^T (Q in regs), dP^T = V dO^T - delta (dO fragments streamed), dQ^T chunk += K^T dS^T
template <int NCH, bool CAUSAL>
__global__ __launch_bounds__(256) void wide_dq_kernel(WideParams p) {
  constexpr int BN = kWideBN, BM = 128, DT = 8;
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * NCH * BN * 256];  // K | V (all chunks)
  bf16* kimg = smem;
  bf16* vimg = smem + NCH * BN * 256;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lq = lane & 31, hh = lane >> 5;
  const int z = blockIdx.y;
  const int nqb = cdiv(p.Tq, BM), nbh = p.H * p.B;
  int qb = blockIdx.x / nbh;
  const int bh = blockIdx.x % nbh;
  if (CAUSAL) qb = nqb - 1 - qb;
  const int h = bh % p.H, b = bh / p.H, hk = h / (p.H / p.Hkv);
  const int q0 = __builtin_amdgcn_readfirstlane(qb * BM + wave * 32);
  const int q = q0 + lq;
  const bool qvalid = q < p.Tq;
  const float c = p.scale_log2;
  // q and dO fragments are streamed from L1/L2 per k-step (a 768-wide row of each would take
  // 384 registers); only the 256-wide dQ chunk accumulator stays resident
  const bf16* qp = p.q + b * p.sqb + (long)(qvalid ? q : 0) * p.sqt + h * p.sqh + 8 * hh;
  const bf16* dop = p.dout + b * p.sdob + (long)(qvalid ? q : 0) * p.sdot + h * p.sdoh + 8 * hh;
  const long srow = ((long)b * p.H + h) * p.Tq + q;
  const float dlt = qvalid ? p.delta[srow] : 0.f;
  const float nlse2 = qvalid ? -p.lse_in[srow] * 1.4426950408889634f : -INFINITY;
  f32x16 acc[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) acc[i] = splat16(0.f);
  const int kend = CAUSAL ? min(p.Tk, qb * BM + BM + p.causal_off) : p.Tk;
  const int wave_kend = CAUSAL ? min(p.Tk, q0 + 32 + p.causal_off) : p.Tk;
  const int ntiles = kend > 0 ? cdiv(kend, BN) : 0;
  const bf16* kbase = p.k + b * p.skb + hk * p.skh;
  const bf16* vbase = p.v + b * p.svb + hk * p.svh;
  LdsOff<256> off;
  off.init(lane);
  for (int j = 0; j < ntiles; ++j) {
    const int k0 = j * BN;
    __syncthreads();
    load_chunked<NCH, BN>(kimg, kbase, p.skt, k0, p.Tk, tid);
    load_chunked<NCH, BN>(vimg, vbase, p.svt, k0, p.Tk, tid);
    __syncthreads();
    if (k0 >= wave_kend) continue;
    f32x16 s = splat16(0.f), dp = splat16(-dlt);
#pragma unroll
    for (int cc = 0; cc < NCH; ++cc) {
      bf16x8 qs[16];
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2)
        qs[s2] = qvalid ? *reinterpret_cast<const bf16x8*>(qp + 256 * cc + 16 * s2) : zero8();
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) s = mfma32(ld_row(kimg + cc * BN * 256, off.row[s2]), qs[s2], s);
    }
#pragma unroll
    for (int cc = 0; cc < NCH; ++cc) {
      bf16x8 df[16];
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2)
        df[s2] = qvalid ? *reinterpret_cast<const bf16x8*>(dop + 256 * cc + 16 * s2) : zero8();
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) dp = mfma32(ld_row(vimg + cc * BN * 256, off.row[s2]), df[s2], dp);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = k0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
      const bool dead = key >= p.Tk || (CAUSAL && key > q + p.causal_off);
      s[r] = dead ? 0.f : fexp2(fmaf(s[r], c, nlse2)) * dp[r];
    }
    const bf16x8 sa = pack_acc(s, 0), sb = pack_acc(s, 1);
    const bf16* kz = kimg + z * BN * 256;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      acc[dt] = mfma32(ld_tr(kz, off.tra[dt], off.trb[dt]), sa, acc[dt]);
      acc[dt] = mfma32(ld_tr(kz + 16 * 256, off.tra[dt], off.trb[dt]), sb, acc[dt]);
    }
  }
  if (qvalid) {
    bf16* op = p.dq + b * p.sdqb + (long)q * p.sdqt + h * p.sdqh + 256 * z;
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

// ----------------------------------------------------------------------------- dK / dV
// key-parallel: 4 waves x 32 keys, key on the lane, K fragments of the lane's key in registers.
// S = Q K^T (Q image), P = exp2(S c - lse2).
//   IS_K = false: dV^T chunk += dO^T P          (dO chunk image, transposed reads)
//   IS_K = true:  dP = dO V^T - delta (dO image, V fragments streamed), dS = P dP,
//                 dK^T chunk += Q^T dS            (Q image chunk z, transposed reads)
template <int NCH, bool CAUSAL, bool IS_K>
__global__ __launch_bounds__(256) void wide_dkdv_kernel(WideParams p) {
  constexpr int D = 256 * NCH, KS = D / 16, BQ = kWideBN, BNK = 128, DT = 8;
  constexpr int DOIMG = IS_K ? NCH * BQ * 256 : BQ * 256;
  __shared__ __attribute__((aligned(16))) bf16 smem[NCH * BQ * 256 + DOIMG];  // Q (all chunks) | dO
  __shared__ float rowc[2 * BQ];                                                 // -lse2 | -delta
  bf16* qimg = smem;
  bf16* dimg = smem + NCH * BQ * 256;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lk = lane & 31, hh = lane >> 5;
  const int z = blockIdx.y;
  const int nbh = p.Hkv * p.B;
  const int bh = blockIdx.x % nbh, kb = blockIdx.x / nbh;
  const int hk = bh % p.Hkv, b = bh / p.Hkv;
  const int G = p.H / p.Hkv;
  const int kw0 = __builtin_amdgcn_readfirstlane(kb * BNK + wave * 32);
  const int key = kw0 + lk;
  const bool kvalid = key < p.Tk;
  const float c = p.scale_log2;
  bf16x8 kf[KS];
  {
    const bf16* kp = p.k + b * p.skb + (long)key * p.skt + hk * p.skh + 8 * hh;
#pragma unroll
    for (int s = 0; s < KS; ++s) kf[s] = kvalid ? *reinterpret_cast<const bf16x8*>(kp + 16 * s) : zero8();
  }
  const bf16* vp = p.v + b * p.svb + (long)(kvalid ? key : 0) * p.svt + hk * p.svh + 8 * hh;
  f32x16 acc[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) acc[i] = splat16(0.f);
  const int qstart = CAUSAL ? max(0, kb * BNK - p.causal_off) : 0;
  const int wave_qstart = CAUSAL ? max(0, kw0 - p.causal_off) : 0;
  const int t0 = qstart / BQ;
  const int ntq = cdiv(p.Tq, BQ);
  LdsOff<256> off;
  off.init(lane);
  for (int hg = 0; hg < G; ++hg) {
    const int h = hk * G + hg;
    const long rbase = ((long)b * p.H + h) * p.Tq;
    for (int tq = t0; tq < ntq; ++tq) {
      const int qq0 = tq * BQ;
      __syncthreads();
      load_chunked<NCH, BQ>(qimg, p.q + b * p.sqb + h * p.sqh, p.sqt, qq0, p.Tq, tid);
      if constexpr (IS_K) load_chunked<NCH, BQ>(dimg, p.dout + b * p.sdob + h * p.sdoh, p.sdot, qq0, p.Tq, tid);
      else load_chunk1<BQ>(dimg, p.dout + b * p.sdob + h * p.sdoh + 256 * z, p.sdot, qq0, p.Tq, tid);
      if (tid < BQ) {
        const int qq = qq0 + tid;
        rowc[tid] = qq < p.Tq ? -p.lse_in[rbase + qq] * 1.4426950408889634f : -INFINITY;
        rowc[BQ + tid] = qq < p.Tq ? -p.delta[rbase + qq] : 0.f;
      }
      __syncthreads();
      if (!kvalid && kw0 >= p.Tk) continue;
      if (CAUSAL && qq0 + BQ - 1 < wave_qstart) continue;
      // rows of s: queries qq0 + 8g + 4hh + i (r = 4g + i); lane: key
      f32x16 s = splat16(0.f);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) s = mfma32(ld_row(qimg + (ks >> 4) * BQ * 256, off.row[ks & 15]), kf[ks], s);
      f32x16 dp;
      if constexpr (IS_K) {
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int i = 0; i < 4; ++i) dp[4 * g + i] = rowc[BQ + 8 * g + 4 * hh + i];
#pragma unroll
        for (int cc = 0; cc < NCH; ++cc) {
          bf16x8 vf[16];
#pragma unroll
          for (int s2 = 0; s2 < 16; ++s2)
            vf[s2] = kvalid ? *reinterpret_cast<const bf16x8*>(vp + 256 * cc + 16 * s2) : zero8();
#pragma unroll
          for (int s2 = 0; s2 < 16; ++s2) dp = mfma32(ld_row(dimg + cc * BQ * 256, off.row[s2]), vf[s2], dp);
        }
      }
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * g + i, qq = qq0 + 8 * g + 4 * hh + i;
          const bool dead = CAUSAL && key > qq + p.causal_off;
          const float pr = dead ? 0.f : fexp2(fmaf(s[r], c, rowc[8 * g + 4 * hh + i]));
          s[r] = IS_K ? pr * dp[r] : pr;
        }
      const bf16x8 pa = pack_acc(s, 0), pb = pack_acc(s, 1);
      const bf16* img = IS_K ? qimg + z * BQ * 256 : dimg;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        acc[dt] = mfma32(ld_tr(img, off.tra[dt], off.trb[dt]), pa, acc[dt]);
        acc[dt] = mfma32(ld_tr(img + 16 * 256, off.tra[dt], off.trb[dt]), pb, acc[dt]);
      }
    }
  }
  if (kvalid) {
    bf16* dst = IS_K ? p.dk + b * p.sdkb + (long)key * p.sdkt + hk * p.sdkh + 256 * z
                     : p.dv + b * p.sdvb + (long)key * p.sdvt + hk * p.sdvh + 256 * z;
    const float sc = IS_K ? p.scale : 1.f;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 w;
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = (bf16)(acc[dt][4 * g + i] * sc);
        *reinterpret_cast<bf16x4*>(dst + 32 * dt + 8 * g + 4 * hh) = w;
      }
  }
}

// ----------------------------------------------------------------------------- host
static void wide_check(const at::Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.dim() == 4 && t.stride(3) == 1, n,
              " must be a bf16 HIP [B, T, H, D] tensor, contiguous in D");
  TORCH_CHECK(((uintptr_t)t.data_ptr() % 16) == 0 && t.stride(0) % 8 == 0 && t.stride(1) % 8 == 0 &&
                  t.stride(2) % 8 == 0, n, ": rows must be 16-byte aligned");
}

#define WIDE_SWITCH(D, ...)                                                    \
  if (D == 512) { constexpr int NCH_ = 2; __VA_ARGS__; }                       \
  else if (D == 768) { constexpr int NCH_ = 3; __VA_ARGS__; }                  \
  else TORCH_CHECK(false, "wide attention: head dim must be 512 or 768");

static WideParams wide_params(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, double scale) {
  WideParams p{};
  p.q = (const bf16*)q.data_ptr(); p.k = (const bf16*)k.data_ptr(); p.v = (const bf16*)v.data_ptr();
  p.B = q.size(0); p.Tq = q.size(1); p.H = q.size(2); p.Tk = k.size(1); p.Hkv = k.size(2);
  p.sqb = q.stride(0); p.sqt = q.stride(1); p.sqh = q.stride(2);
  p.skb = k.stride(0); p.skt = k.stride(1); p.skh = k.stride(2);
  p.svb = v.stride(0); p.svt = v.stride(1); p.svh = v.stride(2);
  p.scale = (float)scale; p.scale_log2 = (float)(scale * 1.4426950408889634);
  p.causal_off = p.Tk - p.Tq;
  return p;
}

std::vector<at::Tensor> attn_wide_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, double scale,
                                      bool causal) {
  wide_check(q, "q"); wide_check(k, "k"); wide_check(v, "v");
  const int D = q.size(3);
  TORCH_CHECK(k.size(3) == D && v.size(3) == D && k.size(0) == q.size(0) && v.size(1) == k.size(1) &&
              v.size(2) == k.size(2) && q.size(2) % k.size(2) == 0, "wide attention: shape mismatch");
  DeviceGuard g(q.device());
  auto out = at::empty({q.size(0), q.size(1), q.size(2), D}, q.options());
  auto lse = at::empty({q.size(0), q.size(2), q.size(1)}, q.options().dtype(at::kFloat));
  WideParams p = wide_params(q, k, v, scale);
  p.out = (bf16*)out.data_ptr(); p.lse = lse.data_ptr<float>();
  p.sob = out.stride(0); p.sot = out.stride(1); p.soh = out.stride(2);
  if ((long)p.B * p.Tq * p.H == 0) return {out, lse};
  auto st = stream();
  WIDE_SWITCH(D, {
    dim3 grid(cdiv(p.Tq, 128) * p.H * p.B, NCH_);
    if (causal) wide_fwd_kernel<NCH_, true><<<grid, 256, 0, st>>>(p);
    else wide_fwd_kernel<NCH_, false><<<grid, 256, 0, st>>>(p);
  });
  SPA_LAUNCH_CHECK();
  return {out, lse};
}

void attn_wide_bwd(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                   const at::Tensor& out, const at::Tensor& lse, const at::Tensor& dq, const at::Tensor& dk,
                   const at::Tensor& dv, double scale, bool causal) {
  for (auto* t : {&dout, &q, &k, &v, &out, &dq, &dk, &dv}) wide_check(*t, "wide attention bwd tensor");
  TORCH_CHECK(dq.sizes() == q.sizes() && dk.sizes() == k.sizes() && dv.sizes() == v.sizes() &&
              dout.sizes() == q.sizes() && out.sizes() == q.sizes() && lse.is_contiguous());
  DeviceGuard g(q.device());
  WideParams p = wide_params(q, k, v, scale);
  auto delta = at::empty({p.B, p.H, p.Tq}, q.options().dtype(at::kFloat));
  p.o = (const bf16*)out.data_ptr(); p.dout = (const bf16*)dout.data_ptr();
  p.dq = (bf16*)dq.data_ptr(); p.dk = (bf16*)dk.data_ptr(); p.dv = (bf16*)dv.data_ptr();
  p.lse_in = lse.data_ptr<float>(); p.delta = delta.data_ptr<float>();
  p.sob = out.stride(0); p.sot = out.stride(1); p.soh = out.stride(2);
  p.sdob = dout.stride(0); p.sdot = dout.stride(1); p.sdoh = dout.stride(2);
  p.sdqb = dq.stride(0); p.sdqt = dq.stride(1); p.sdqh = dq.stride(2);
  p.sdkb = dk.stride(0); p.sdkt = dk.stride(1); p.sdkh = dk.stride(2);
  p.sdvb = dv.stride(0); p.sdvt = dv.stride(1); p.sdvh = dv.stride(2);
  if (p.B * p.H == 0) return;
  if (p.Tq == 0) { dk.zero_(); dv.zero_(); return; }
  auto st = stream();
  const int D = q.size(3);
  WIDE_SWITCH(D, {
    const long rows = (long)p.B * p.Tq * p.H;
    wide_delta_kernel<NCH_><<<(int)cdiv(rows, 4), 256, 0, st>>>(p);
    dim3 gq(cdiv(p.Tq, 128) * p.H * p.B, NCH_);
    if (causal) wide_dq_kernel<NCH_, true><<<gq, 256, 0, st>>>(p);
    else wide_dq_kernel<NCH_, false><<<gq, 256, 0, st>>>(p);
    if (p.Tk > 0) {
      dim3 gk(cdiv(p.Tk, 128) * p.Hkv * p.B, NCH_);
      if (causal) {
        wide_dkdv_kernel<NCH_, true, false><<<gk, 256, 0, st>>>(p);
        wide_dkdv_kernel<NCH_, true, true><<<gk, 256, 0, st>>>(p);
      } else {
        wide_dkdv_kernel<NCH_, false, false><<<gk, 256, 0, st>>>(p);
        wide_dkdv_kernel<NCH_, false, true><<<gk, 256, 0, st>>>(p);
      }
    }
  });
  SPA_LAUNCH_CHECK();
}

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.def("attn_wide_fwd(Tensor q, Tensor k, Tensor v, float scale, bool causal) -> Tensor[]");
  m.def("attn_wide_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor out, Tensor lse, Tensor(a!) dq, "
        "Tensor(b!) dk, Tensor(c!) dv, float scale, bool causal) -> ()");
}
TORCH_LIBRARY_IMPL(spa, CUDA, m) {
  m.impl("attn_wide_fwd", &spa::attn_wide_fwd);
  m.impl("attn_wide_bwd", &spa::attn_wide_bwd);
}
