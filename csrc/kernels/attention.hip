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
// q/k/v/o and grads are addressed with (batch, seq, head) strides so the kernels
// read/write a fused [B, T, H + 2*Hkv, hd] qkv buffer in place.
#include "spa_common.h"
#include <type_traits>

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
};

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

// deferred-rescale threshold in log2 units (T13): P = 2^(s*c - m) <= 2^8
constexpr float kRescaleThr = 8.f;

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }
// max of x over lanes l and l^32 (one v_permlane32_swap, no LDS)
__device__ __forceinline__ float halfmax(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float halfsum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z[i] = (bf16)0.f;
  return z;
}
__device__ __forceinline__ f32x16 splat16(float v) {
  f32x16 a;
#pragma unroll
  for (int r = 0; r < 16; ++r) a[r] = v;
  return a;
}
// accumulator registers 8s..8s+7 -> bf16 operand fragment (permuted k order)
__device__ __forceinline__ bf16x8 pack_acc(const f32x16& a, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (bf16)a[8 * s + j];
  return r;
}

// ---- swizzled row-major [rows][HD] bf16 LDS images -------------------------
template <int HD>
__device__ __forceinline__ int swz(int r) {
  if constexpr (HD >= 128) return ((r & 3) << 2) | ((r >> 2) & 3);
  else return (((r >> 1) & 1) << 2) | ((r >> 2) & 3);
}
template <int HD>
__device__ __forceinline__ int img_off(int r, int ch) {  // element offset of 16B chunk ch of row r
  return r * HD + 8 * (ch ^ swz<HD>(r));
}
// A/B operand "X^T" for one 16-deep k-step, where X is the row-major image with
// rows = k index, columns = output index. Lane l gets X[r0 + 16s + perm(j)][c0 + (l&31)].
template <int HD>
__device__ __forceinline__ bf16x8 rd_tr(const bf16* img, int rbase, int c0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3, hh = lane >> 5;
  const int c = c0 + 16 * (g & 1) + 4 * pp;  // column (element) this lane addresses
  const int ch = c >> 3, within = c & 7;
  const int ra = rbase + 4 * hh + q, rb = ra + 8;
  typedef __attribute__((address_space(3))) s16x4 lds_s4;
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s4*)(img + ra * HD + 8 * (ch ^ swz<HD>(ra)) + within));
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s4*)(img + rb * HD + 8 * (ch ^ swz<HD>(rb)) + within));
  // whole-vector bit casts: element-wise short->bf16 inserts miscompile (duplicated dwords)
  const bf16x4 av = __builtin_bit_cast(bf16x4, a), bv = __builtin_bit_cast(bf16x4, b);
  return __builtin_shufflevector(av, bv, 0, 1, 2, 3, 4, 5, 6, 7);
}

// Per-lane LDS element offsets, computed once per kernel (the swizzle term is
// invariant under the +32-row / +16-row steps of the loops, which become
// immediate offsets): row reads (row = lane&31, chunk = 2ks + half) and the
// two halves of each transposed read (k-step rows 0..15, d-tile dt).
template <int HD>
struct LdsOff {
  int row[HD / 16];
  int tra[HD / 32], trb[HD / 32];
  __device__ __forceinline__ void init(int lane) {
    const int l32 = lane & 31, hh = lane >> 5, g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
#pragma unroll
    for (int ks = 0; ks < HD / 16; ++ks) row[ks] = l32 * HD + 8 * ((2 * ks + hh) ^ swz<HD>(l32));
    const int ra = 4 * hh + q, rb = ra + 8;
#pragma unroll
    for (int dt = 0; dt < HD / 32; ++dt) {
      const int c = 32 * dt + 16 * (g & 1) + 4 * pp;
      const int ch = c >> 3, within = c & 7;
      tra[dt] = ra * HD + 8 * (ch ^ swz<HD>(ra)) + within;
      trb[dt] = rb * HD + 8 * (ch ^ swz<HD>(rb)) + within;
    }
  }
};
__device__ __forceinline__ bf16x8 ld_row(const bf16* img, int off) {
  return *reinterpret_cast<const bf16x8*>(img + off);
}
__device__ __forceinline__ bf16x8 ld_tr(const bf16* img, int offa, int offb) {
  typedef __attribute__((address_space(3))) s16x4 lds_s4;
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + offa));
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + offb));
  const bf16x4 av = __builtin_bit_cast(bf16x4, a), bv = __builtin_bit_cast(bf16x4, b);
  return __builtin_shufflevector(av, bv, 0, 1, 2, 3, 4, 5, 6, 7);
}
template <int V> using IC = std::integral_constant<int, V>;

// Register-staged tile loader: ROWS x HD bf16 tile of a strided tensor -> regs -> LDS image.
// Global side: one buffer descriptor per tile (scalar work), its range ending at the
// tensor's last valid row, so rows >= nrows load as zeros without a branch. The per-lane
// byte offsets and LDS offsets are loop invariant (computed once).
// Thread -> chunk map: W = min(HD/8, 16) lanes share a row, a lane takes the chunk
// columns ch, ch+16, ... of its row (HD = 256: two) and rows rr, rr+R, ... (R = NT/W,
// a multiple of 16). The XOR swizzle only touches the low 4 chunk bits and repeats
// every 16 rows, so all of a lane's LDS offsets are one register + immediates; on the
// global side each row pass gets its own scalar descriptor and the column step is the
// instruction offset.
template <int HD, int ROWS, int NT>
struct TileLoader {
  static constexpr int CPR = HD / 8;                   // 16B chunks per row
  static constexpr int W = CPR < 16 ? CPR : 16;        // lanes per row
  static constexpr int NC = CPR / W;                   // column chunks per lane (16 apart)
  static constexpr int R = NT / W;                     // rows between a lane's row passes
  static constexpr int NP = ROWS / R;                  // row passes
  static constexpr int CH = NP * NC;
  static_assert(R % 16 == 0 && ROWS % R == 0 && NP >= 1, "tile/threads mismatch");
  bf16x8 r[CH];
  int voff;  // byte offset of this lane's first chunk within its row pass
  int loff;  // element offset of this lane's first chunk in the LDS image
  __device__ __forceinline__ void init(long stride, int tid) {
    const int rr = tid / W, ch = tid % W;
    voff = (int)(((long)rr * stride + ch * 8) * 2);
    loff = img_off<HD>(rr, ch);
  }
  __device__ __forceinline__ void load(const bf16* base, long stride, int row0, int nrows) {
#pragma unroll
    for (int ps = 0; ps < NP; ++ps) {
      const int r0 = row0 + ps * R;
      const int left = nrows - r0;
      const int bytes = left > 0 ? (int)(((long)(left - 1) * stride + HD) * 2) : 0;
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc((void*)(base + (long)r0 * stride), 0, bytes, 0x00020000);
#pragma unroll
      for (int j = 0; j < NC; ++j)
        r[ps * NC + j] =
            __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, voff + 256 * j, 0, 0));
    }
  }
  __device__ __forceinline__ void store(bf16* img) const {
#pragma unroll
    for (int ps = 0; ps < NP; ++ps)
#pragma unroll
      for (int j = 0; j < NC; ++j)
        *reinterpret_cast<bf16x8*>(img + loff + ps * R * HD + 128 * j) = r[ps * NC + j];
  }
};

// ---------------------------------------------------------------------------
// Forward: block = NW waves x 32 query rows; K/V tiles of 64 keys.
// ---------------------------------------------------------------------------
template <int HD, int NW, bool CAUSAL>
__global__ __launch_bounds__(NW * 64) void attn_fwd_kernel(AttnParams p) {
  constexpr int BN = HD >= 256 ? 32 : 64, NSUB = BN / 32, BM = 32 * NW, KS = HD / 16, DT = HD / 32, NT = NW * 64;
  constexpr int TILE = BN * HD;
  __shared__ __attribute__((aligned(16))) bf16 smem[4 * TILE];  // [buf][K|V]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lq = lane & 31, hh = lane >> 5;
  const int nqb = cdiv(p.Tq, BM);
  const int nbh = p.H * p.B;
  int qb = blockIdx.x / nbh;
  const int bh = blockIdx.x % nbh;
  if (CAUSAL) qb = nqb - 1 - qb;  // heaviest q-blocks first
  const int h = bh % p.H, b = bh / p.H;
  const int hk = h / (p.H / p.Hkv);
  const int q0 = __builtin_amdgcn_readfirstlane(qb * BM + wave * 32);
  const int q = q0 + lq;
  const float c = p.scale_log2;

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
  const int wave_kend = CAUSAL ? min(p.Tk, q0 + 32 + p.causal_off) : p.Tk;
  const int ntiles = kend > 0 ? cdiv(kend, BN) : 0;

  const bf16* kbase = p.k + b * p.skb + hk * p.skh;
  const bf16* vbase = p.v + b * p.svb + hk * p.svh;
  TileLoader<HD, BN, NT> lk, lv;
  lk.init(p.skt, tid);
  lv.init(p.svt, tid);
  if (ntiles > 0) {
    lk.load(kbase, p.skt, 0, p.Tk);
    lv.load(vbase, p.svt, 0, p.Tk);
    lk.store(smem);
    lv.store(smem + TILE);
    if (ntiles > 1) { lk.load(kbase, p.skt, BN, p.Tk); lv.load(vbase, p.svt, BN, p.Tk); }
  }
  __syncthreads();
  LdsOff<HD> off;
  off.init(lane);
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
  // body(j, buffer) with the buffer a compile-time constant (loop unrolled x2) so
  // every LDS address is a precomputed lane offset + an immediate
  auto body = [&](const int j, auto bufc) {
    constexpr int BUF = decltype(bufc)::value;
    const int k0 = j * BN;
    const bf16* Ks = smem + BUF * 2 * TILE;
    const bf16* Vs = Ks + TILE;
    if (j + 1 < ntiles) {
      bf16* Kn = smem + (1 - BUF) * 2 * TILE;
      lk.store(Kn);
      lv.store(Kn + TILE);
      if (j + 2 < ntiles) { lk.load(kbase, p.skt, k0 + 2 * BN, p.Tk); lv.load(vbase, p.svt, k0 + 2 * BN, p.Tk); }
    }
#pragma unroll
    for (int t = 0; t < NSUB; ++t) {
      const int ks0 = k0 + 32 * t;
      if (ks0 < wave_kend) {
        f32x16 s = mfma32(ld_row(Ks + 32 * t * HD, off.row[0]), qf[0], splat16(0.f));
#pragma unroll
        for (int ks = 1; ks < KS; ++ks) s = mfma32(ld_row(Ks + 32 * t * HD, off.row[ks]), qf[ks], s);
        const bool need_mask = (ks0 + 32 > p.Tk) || (CAUSAL && ks0 + 31 > q0 + p.causal_off);
        if (need_mask) mask(s, ks0);
        softmax(s);
        const bf16x8 pa = pack_acc(s, 0), pb = pack_acc(s, 1);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          o[dt] = mfma32(ld_tr(Vs + 32 * t * HD, off.tra[dt], off.trb[dt]), pa, o[dt]);
          o[dt] = mfma32(ld_tr(Vs + (32 * t + 16) * HD, off.tra[dt], off.trb[dt]), pb, o[dt]);
        }
      }
    }
    __syncthreads();
  };
  for (int j = 0; j < ntiles; j += 2) {
    body(j, IC<0>{});
    if (j + 1 < ntiles) body(j + 1, IC<1>{});
  }
  l = halfsum(l);
  const float inv = l > 0.f ? 1.f / l : 0.f;
  if (q < p.Tq) {
    bf16* op = p.out + b * p.sob + (long)q * p.sot + h * p.soh;
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
// Backward dQ (query-parallel; also writes delta = rowsum(dO*O)).
//   S^T = K Q^T ; P^T = exp2(S^T*c - lse2) ; dP^T = V dO^T - delta ; dS^T = P^T dP^T
//   dQ^T += K^T dS^T   (K^T via tr reads of the K image)
// ---------------------------------------------------------------------------
template <int HD, int NW, bool CAUSAL>
__global__ __launch_bounds__(NW * 64) void attn_bwd_dq_kernel(AttnParams p) {
  constexpr int BN = HD >= 256 ? 32 : 64, NSUB = BN / 32, BM = 32 * NW, KS = HD / 16, DT = HD / 32, NT = NW * 64;
  constexpr int TILE = BN * HD;
  __shared__ __attribute__((aligned(16))) bf16 smem[4 * TILE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lq = lane & 31, hh = lane >> 5;
  const int nqb = cdiv(p.Tq, BM);
  const int nbh = p.H * p.B;
  int qb = blockIdx.x / nbh;
  const int bh = blockIdx.x % nbh;
  if (CAUSAL) qb = nqb - 1 - qb;
  const int h = bh % p.H, b = bh / p.H;
  const int hk = h / (p.H / p.Hkv);
  const int q0 = __builtin_amdgcn_readfirstlane(qb * BM + wave * 32);
  const int q = q0 + lq;
  const bool qvalid = q < p.Tq;
  const float c = p.scale_log2;

  bf16x8 qf[KS], df[KS];
  float dlt = 0.f;
  {
    const bf16* qp = p.q + b * p.sqb + (long)q * p.sqt + h * p.sqh + 8 * hh;
    const bf16* dp = p.dout + b * p.sdob + (long)q * p.sdot + h * p.sdoh + 8 * hh;
    const bf16* op = p.o + b * p.sob + (long)q * p.sot + h * p.soh + 8 * hh;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      qf[s] = qvalid ? *reinterpret_cast<const bf16x8*>(qp + 16 * s) : zero8();
      df[s] = qvalid ? *reinterpret_cast<const bf16x8*>(dp + 16 * s) : zero8();
      const bf16x8 ov = qvalid ? *reinterpret_cast<const bf16x8*>(op + 16 * s) : zero8();
#pragma unroll
      for (int j = 0; j < 8; ++j) dlt += (float)ov[j] * (float)df[s][j];
    }
    dlt = halfsum(dlt);
  }
  const long srow = ((long)b * p.H + h) * p.Tq + q;
  if (qvalid && hh == 0) p.delta[srow] = dlt;
  const float nlse2 = qvalid ? -p.lse_in[srow] * 1.4426950408889634f : -INFINITY;
  f32x16 acc[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) acc[i] = splat16(0.f);

  int kend = p.Tk;
  if (CAUSAL) kend = min(p.Tk, qb * BM + BM + p.causal_off);
  const int wave_kend = CAUSAL ? min(p.Tk, q0 + 32 + p.causal_off) : p.Tk;
  const int ntiles = kend > 0 ? cdiv(kend, BN) : 0;
  const bf16* kbase = p.k + b * p.skb + hk * p.skh;
  const bf16* vbase = p.v + b * p.svb + hk * p.svh;
  TileLoader<HD, BN, NT> lk, lv;
  lk.init(p.skt, tid);
  lv.init(p.svt, tid);
  if (ntiles > 0) {
    lk.load(kbase, p.skt, 0, p.Tk);
    lv.load(vbase, p.svt, 0, p.Tk);
    lk.store(smem);
    lv.store(smem + TILE);
    if (ntiles > 1) { lk.load(kbase, p.skt, BN, p.Tk); lv.load(vbase, p.svt, BN, p.Tk); }
  }
  __syncthreads();
  LdsOff<HD> off;
  off.init(lane);
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
    const int k0 = j * BN;
    const bf16* Ks = smem + BUF * 2 * TILE;
    const bf16* Vs = Ks + TILE;
    if (j + 1 < ntiles) {
      bf16* Kn = smem + (1 - BUF) * 2 * TILE;
      lk.store(Kn);
      lv.store(Kn + TILE);
      if (j + 2 < ntiles) { lk.load(kbase, p.skt, k0 + 2 * BN, p.Tk); lv.load(vbase, p.svt, k0 + 2 * BN, p.Tk); }
    }
#pragma unroll
    for (int t = 0; t < NSUB; ++t) {
      const int ks0 = k0 + 32 * t;
      if (ks0 < wave_kend) {
        f32x16 s = mfma32(ld_row(Ks + 32 * t * HD, off.row[0]), qf[0], splat16(0.f));
        f32x16 dp = mfma32(ld_row(Vs + 32 * t * HD, off.row[0]), df[0], splat16(-dlt));
#pragma unroll
        for (int ks = 1; ks < KS; ++ks) {
          s = mfma32(ld_row(Ks + 32 * t * HD, off.row[ks]), qf[ks], s);
          dp = mfma32(ld_row(Vs + 32 * t * HD, off.row[ks]), df[ks], dp);
        }
        const bool need_mask = (ks0 + 32 > p.Tk) || (CAUSAL && ks0 + 31 > q0 + p.causal_off);
        if (need_mask) mask(s, ks0);
        dsoft(s, dp);
        const bf16x8 sa = pack_acc(s, 0), sb = pack_acc(s, 1);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          acc[dt] = mfma32(ld_tr(Ks + 32 * t * HD, off.tra[dt], off.trb[dt]), sa, acc[dt]);
          acc[dt] = mfma32(ld_tr(Ks + (32 * t + 16) * HD, off.tra[dt], off.trb[dt]), sb, acc[dt]);
        }
      }
    }
    __syncthreads();
  };
  for (int j = 0; j < ntiles; j += 2) {
    body(j, IC<0>{});
    if (j + 1 < ntiles) body(j + 1, IC<1>{});
  }
  if (qvalid) {
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

// ---------------------------------------------------------------------------
// Backward dK/dV: key-block parallel (4 waves x 32 keys), key on the lane.
//   S = Q K^T, dP = dO V^T - delta   (A = Q / dO row reads, B = K / V fragments in regs;
//                                     the dP accumulator starts at -delta of its row)
//   dV^T += dO^T P, dK^T += Q^T dS   (A = tr reads of the Q / dO images, B = accumulators)
// Loops over the q-heads sharing this kv-head (GQA) so the group sum stays in regs.
// ---------------------------------------------------------------------------
template <int HD, bool CAUSAL, int MT, bool FUSEDQ>
__global__ __launch_bounds__(256) void attn_bwd_dkdv_kernel(AttnParams p) {
  // MT 32-row q sub-tiles per iteration (more MFMA work per barrier / LDS fill)
  constexpr int BMQ = 32 * MT, BNK = 128, KS = HD / 16, DT = HD / 32, NT = 256;
  constexpr int TILE = BMQ * HD;
  // FUSEDQ: dQ computed here too (dQ += dS K over this block's 128 keys, fp32 atomics into
  // p.dqacc) -> 5 MFMA products per tile instead of 7 for the split dq + dkdv kernels.
  // dS crosses LDS once ([key][q] image, transposed reads), K sits in a [key][d] image.
  constexpr int KIMG = FUSEDQ ? BNK * HD : 8, DSIMG = FUSEDQ ? BNK * 64 : 8;
  __shared__ __attribute__((aligned(16))) bf16 smem[4 * TILE + KIMG + DSIMG];  // [buf][Q|dO] | K | dS
  bf16* kimg = smem + 4 * TILE;
  bf16* dsimg = kimg + KIMG;
  __shared__ __attribute__((aligned(16))) float rowc[2][2 * BMQ];  // [buf][-lse2 | -delta]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lk = lane & 31, hh = lane >> 5;
  const int nbh = p.Hkv * p.B;
  const int bh = blockIdx.x % nbh;
  const int rest = blockIdx.x / nbh;  // causal: low key blocks are heaviest, launched first
  const int split = rest % p.hsplit, kb = rest / p.hsplit;
  const int hk = bh % p.Hkv, b = bh / p.Hkv;
  const int G = p.H / p.Hkv / p.hsplit;  // q-heads handled by this block
  const int h0 = hk * (p.H / p.Hkv) + split * G;
  const int kw0 = __builtin_amdgcn_readfirstlane(kb * BNK + wave * 32);
  const int key = kw0 + lk;
  const bool kvalid = key < p.Tk;
  const float c = p.scale_log2;

  bf16x8 kf[KS], vf[KS];
  {
    const bf16* kp = p.k + b * p.skb + (long)key * p.skt + hk * p.skh + 8 * hh;
    const bf16* vp = p.v + b * p.svb + (long)key * p.svt + hk * p.svh + 8 * hh;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      kf[s] = kvalid ? *reinterpret_cast<const bf16x8*>(kp + 16 * s) : zero8();
      vf[s] = kvalid ? *reinterpret_cast<const bf16x8*>(vp + 16 * s) : zero8();
      if constexpr (FUSEDQ)   // row = this lane's key; chunk 2s+hh holds d = 16s + 8hh .. +8
        *reinterpret_cast<bf16x8*>(kimg + img_off<HD>(wave * 32 + lk, 2 * s + hh)) = kf[s];
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
  const int nper = ntq - t0 > 0 ? ntq - t0 : 0;  // q-tiles per head
  const int total = nper * G;                      // (head, q-tile) iterations
  TileLoader<HD, BMQ, NT> lq_, ld_;
  lq_.init(p.sqt, tid);
  ld_.init(p.sdot, tid);
  float rl = 0.f, rd = 0.f;  // per-thread row constants for the prefetched tile (tid < BMQ)
  auto fetch = [&](int it) {
    const int hg = it / nper, tq = t0 + it % nper;
    const int h = h0 + hg;
    const int qq0 = tq * BMQ;
    lq_.load(p.q + b * p.sqb + h * p.sqh, p.sqt, qq0, p.Tq);
    ld_.load(p.dout + b * p.sdob + h * p.sdoh, p.sdot, qq0, p.Tq);
    if (tid < BMQ) {
      const int qq = qq0 + tid;
      const long rbase = ((long)b * p.H + h) * p.Tq;
      rl = qq < p.Tq ? -p.lse_in[rbase + qq] * 1.4426950408889634f : -INFINITY;
      rd = qq < p.Tq ? -p.delta[rbase + qq] : 0.f;
    }
  };
  auto commit_tile = [&](int buf) {
    lq_.store(smem + buf * 2 * TILE);
    ld_.store(smem + buf * 2 * TILE + TILE);
    if (tid < BMQ) { rowc[buf][tid] = rl; rowc[buf][BMQ + tid] = rd; }
  };
  if (total > 0) {
    fetch(0);
    commit_tile(0);
    if (total > 1) fetch(1);
  }
  __syncthreads();
  LdsOff<HD> off;
  off.init(lane);
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
    const int tq = t0 + it % nper;
    const int qq0 = tq * BMQ;
    const bf16* Qs = smem + BUF * 2 * TILE;
    const bf16* Ds = Qs + TILE;
    const float* rc = rowc[BUF];
    if (it + 1 < total) {
      commit_tile(1 - BUF);
      if (it + 2 < total) fetch(it + 2);
    }
    const bool active = kw0 < p.Tk && !(CAUSAL && qq0 + BMQ - 1 < wave_qstart);
    if (active) {
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        // dP accumulator starts at -delta of each row (register r <-> query row 8g+4hh+i)
        f32x16 dp;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 dv = *reinterpret_cast<const f32x4*>(rc + BMQ + 32 * t + 8 * g + 4 * hh);
#pragma unroll
          for (int i = 0; i < 4; ++i) dp[4 * g + i] = dv[i];
        }
        f32x16 s = mfma32(ld_row(Qs + 32 * t * HD, off.row[0]), kf[0], splat16(0.f));
        dp = mfma32(ld_row(Ds + 32 * t * HD, off.row[0]), vf[0], dp);
#pragma unroll
        for (int ks = 1; ks < KS; ++ks) {
          s = mfma32(ld_row(Qs + 32 * t * HD, off.row[ks]), kf[ks], s);
          dp = mfma32(ld_row(Ds + 32 * t * HD, off.row[ks]), vf[ks], dp);
        }
        const int qt0 = qq0 + 32 * t;
        const bool need_mask = CAUSAL && qt0 + p.causal_off < kw0 + 31;
        if (need_mask) mask(s, qt0);
        dsoft(s, dp, rc + 32 * t);
        const bf16x8 pa = pack_acc(s, 0), pb = pack_acc(s, 1), sa = pack_acc(dp, 0), sb = pack_acc(dp, 1);
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
        for (int dt = 0; dt < DT; ++dt) {
          dvt[dt] = mfma32(ld_tr(Ds + 32 * t * HD, off.tra[dt], off.trb[dt]), pa, dvt[dt]);
          dkt[dt] = mfma32(ld_tr(Qs + 32 * t * HD, off.tra[dt], off.trb[dt]), sa, dkt[dt]);
          dvt[dt] = mfma32(ld_tr(Ds + (32 * t + 16) * HD, off.tra[dt], off.trb[dt]), pb, dvt[dt]);
          dkt[dt] = mfma32(ld_tr(Qs + (32 * t + 16) * HD, off.tra[dt], off.trb[dt]), sb, dkt[dt]);
        }
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
      const int h = h0 + it / nper;
#pragma unroll
      for (int tile = wave; tile < MT * DT; tile += 4) {
        const int tq = tile / DT, td = tile % DT;
        const int q0 = qq0 + 32 * tq;
        if (CAUSAL && q0 + 31 + p.causal_off < kb * BNK) continue;   // every key of the block is masked
        if (q0 >= p.Tq) continue;
        f32x16 acc = splat16(0.f);
#pragma unroll
        for (int kk = 0; kk < BNK / 16; ++kk)
          acc = mfma32(rd_tr<64>(dsimg, 16 * kk, 32 * tq, lane), rd_tr<HD>(kimg, 16 * kk, 32 * td, lane), acc);
        float* dst = p.dqacc + ((long)b * p.Tq * p.H + h) * HD + 32 * td + lk;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int qq = q0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if (qq < p.Tq) atomicAdd(dst + (long)qq * p.H * HD, acc[r]);
        }
      }
    }
    __syncthreads();
  };
  for (int it = 0; it < total; it += 2) {
    body(it, IC<0>{});
    if (it + 1 < total) body(it + 1, IC<1>{});
  }
  store_kv_grad<HD>(p, dkt, true, b, hk, key, split, hh);
  store_kv_grad<HD>(p, dvt, false, b, hk, key, split, hh);
}

// ---------------------------------------------------------------------------
// Backward dK/dV with paired waves (HD <= 128): 8 waves = 4 pairs x 32 keys (128 keys per
// block); key on the lane. Splitting the four products of a key column over two waves
// halves each wave's live registers (one of K/V fragments, one of dK^T/dV^T), which puts
// two waves on every SIMD (one wave per SIMD in the single-wave kernel above), and the
// two roles' matrix and vector work interleave on the SIMD:
//   role A (waves 0-3):  S = Q K^T -> P = exp2(S c - lse2) -> P to LDS (fp32);  | dV^T += dO^T P
//   role B (waves 4-7):  dP = dO V^T - delta (kept in registers)                | dS = P dP; dK^T += Q^T dS
// '|' is a block barrier: phase 1 = the left column, phase 2 = the right column, so the
// pair's P crosses LDS once per 32x32 sub-tile ([pair][t][j][lane][4] fp32 image,
// conflict-free 16-byte rows). Q / dO tiles of 64 rows are double-buffered as before.
// ---------------------------------------------------------------------------
template <int HD, bool CAUSAL>
__global__ __launch_bounds__(512) void attn_bwd_dkdv2_kernel(AttnParams p) {
  constexpr int MT = 2, BMQ = 32 * MT, BNK = 128, KS = HD / 16, DT = HD / 32, NT = 512;
  constexpr int TILE = BMQ * HD;
  __shared__ __attribute__((aligned(16))) bf16 smem[4 * TILE];               // [buf][Q|dO]
  __shared__ __attribute__((aligned(16))) float pimg[4 * MT * 4 * 64 * 4];  // [pair][t][j][lane][4]
  __shared__ __attribute__((aligned(16))) float rowc[2][2 * BMQ];           // [buf][-lse2 | -delta]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pair = wave & 3, role = wave >> 2;
  const int lk = lane & 31, hh = lane >> 5;
  const int nbh = p.Hkv * p.B;
  const int bh = blockIdx.x % nbh;
  const int rest = blockIdx.x / nbh;             // causal: low key blocks are heaviest, launched first
  const int split = rest % p.hsplit, kb = rest / p.hsplit;
  const int hk = bh % p.Hkv, b = bh / p.Hkv;
  const int Gs = p.H / p.Hkv / p.hsplit;         // q-heads handled by this block
  const int h0 = hk * (p.H / p.Hkv) + split * Gs;
  const int kw0 = __builtin_amdgcn_readfirstlane(kb * BNK + pair * 32);
  const int key = kw0 + lk;
  const bool kvalid = key < p.Tk;
  const float c = p.scale_log2;

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
  const int total = nper * Gs;
  TileLoader<HD, BMQ, NT> lq_, ld_;
  lq_.init(p.sqt, tid);
  ld_.init(p.sdot, tid);
  float rl = 0.f, rd = 0.f;
  auto fetch = [&](int it) {
    const int h = h0 + it / nper;
    const int qq0 = (t0 + it % nper) * BMQ;
    lq_.load(p.q + b * p.sqb + h * p.sqh, p.sqt, qq0, p.Tq);
    ld_.load(p.dout + b * p.sdob + h * p.sdoh, p.sdot, qq0, p.Tq);
    if (tid < BMQ) {
      const int qq = qq0 + tid;
      const long rbase = ((long)b * p.H + h) * p.Tq;
      rl = qq < p.Tq ? -p.lse_in[rbase + qq] * 1.4426950408889634f : -INFINITY;
      rd = qq < p.Tq ? -p.delta[rbase + qq] : 0.f;
    }
  };
  auto commit_tile = [&](int buf) {
    lq_.store(smem + buf * 2 * TILE);
    ld_.store(smem + buf * 2 * TILE + TILE);
    if (tid < BMQ) { rowc[buf][tid] = rl; rowc[buf][BMQ + tid] = rd; }
  };
  if (total > 0) {
    fetch(0);
    commit_tile(0);
    if (total > 1) fetch(1);
  }
  __syncthreads();
  LdsOff<HD> off;
  off.init(lane);
  float* pme = pimg + pair * (MT * 4 * 64 * 4) + lane * 4;  // + (t*4 + j) * 256
  auto body = [&](const int it, auto bufc) {
    constexpr int BUF = decltype(bufc)::value;
    const int qq0 = (t0 + it % nper) * BMQ;
    const bf16* Qs = smem + BUF * 2 * TILE;
    const bf16* Ds = Qs + TILE;
    const float* rc = rowc[BUF];
    if (it + 1 < total) {
      commit_tile(1 - BUF);
      if (it + 2 < total) fetch(it + 2);
    }
    const bool active = kw0 < p.Tk && !(CAUSAL && qq0 + BMQ - 1 < wave_qstart);
    bf16x8 pk[2 * MT];  // A: packed P of both sub-tiles (kept over the barrier)
    f32x16 dp[MT];      // B: dP - delta of both sub-tiles (kept over the barrier)
    // ---- phase 1
    if (active) {
      if (role == 0) {
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          f32x16 s = mfma32(ld_row(Qs + 32 * t * HD, off.row[0]), xf[0], splat16(0.f));
#pragma unroll
          for (int ks = 1; ks < KS; ++ks) s = mfma32(ld_row(Qs + 32 * t * HD, off.row[ks]), xf[ks], s);
          const int qt0 = qq0 + 32 * t;
          if (CAUSAL && qt0 + p.causal_off < kw0 + 31) {
#pragma unroll
            for (int r = 0; r < 16; ++r)
              if (key > qt0 + 8 * (r >> 2) + 4 * hh + (r & 3) + p.causal_off) s[r] = -INFINITY;
          }
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4 lv = *reinterpret_cast<const f32x4*>(rc + 32 * t + 8 * g + 4 * hh);
            f32x4 pv;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              pv[i] = fexp2(fmaf(s[4 * g + i], c, lv[i]));  // rows >= Tq: -lse2 = -inf -> 0
              s[4 * g + i] = pv[i];
            }
            *reinterpret_cast<f32x4*>(pme + (t * 4 + g) * 256) = pv;
          }
          pk[2 * t] = pack_acc(s, 0);
          pk[2 * t + 1] = pack_acc(s, 1);
        }
      } else {
#pragma unroll
        for (int t = 0; t < MT; ++t) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4 dv = *reinterpret_cast<const f32x4*>(rc + BMQ + 32 * t + 8 * g + 4 * hh);
#pragma unroll
            for (int i = 0; i < 4; ++i) dp[t][4 * g + i] = dv[i];
          }
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) dp[t] = mfma32(ld_row(Ds + 32 * t * HD, off.row[ks]), xf[ks], dp[t]);
        }
      }
    }
    __syncthreads();  // P images complete
    // ---- phase 2
    if (active) {
      if (role == 0) {
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            acc[dt] = mfma32(ld_tr(Ds + 32 * t * HD, off.tra[dt], off.trb[dt]), pk[2 * t], acc[dt]);
            acc[dt] = mfma32(ld_tr(Ds + (32 * t + 16) * HD, off.tra[dt], off.trb[dt]), pk[2 * t + 1], acc[dt]);
          }
      } else {
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          f32x16 ds;
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4 pv = *reinterpret_cast<const f32x4*>(pme + (t * 4 + g) * 256);
#pragma unroll
            for (int i = 0; i < 4; ++i) ds[4 * g + i] = pv[i] * dp[t][4 * g + i];
          }
          const bf16x8 sa = pack_acc(ds, 0), sb = pack_acc(ds, 1);
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            acc[dt] = mfma32(ld_tr(Qs + 32 * t * HD, off.tra[dt], off.trb[dt]), sa, acc[dt]);
            acc[dt] = mfma32(ld_tr(Qs + (32 * t + 16) * HD, off.tra[dt], off.trb[dt]), sb, acc[dt]);
          }
        }
      }
    }
    __syncthreads();
  };
  for (int it = 0; it < total; it += 2) {
    body(it, IC<0>{});
    if (it + 1 < total) body(it + 1, IC<1>{});
  }
  store_kv_grad<HD>(p, acc, role == 1, b, hk, key, split, hh);
}

// sum the q-head-split fp32 partials -> bf16 dK (scaled) / dV
template <int HD>
__global__ __launch_bounds__(256) void attn_kv_reduce_kernel(AttnParams p) {
  constexpr int TPR = HD / 8;
  const long rows = (long)p.B * p.Tk * p.Hkv;
  const long n = rows * TPR * 2;
  const long slab = rows * HD;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const bool is_k = i < rows * TPR;
    const long j = is_k ? i : i - rows * TPR;
    const int t = j % TPR;
    const long row = j / TPR;  // (b, key, hk)
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
  if (row < nrows && t == 0) p.delta[(b * p.H + h) * p.Tq + q] = acc;
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
    store8(p.dq + b * p.sdqb + q * p.sdqt + h * p.sdqh + 8 * t, a);
  }
}

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

// forward / dq use 8 waves (2 per SIMD) for hd <= 128, 4 waves for hd = 256
template <int HD> constexpr int fwd_waves() { return HD <= 128 ? 8 : 4; }

#define HD_SWITCH(HDV, ...)                                                        \
  if (HDV == 64) { constexpr int HD_ = 64; __VA_ARGS__; }                          \
  else if (HDV == 128) { constexpr int HD_ = 128; __VA_ARGS__; }                   \
  else if (HDV == 256) { constexpr int HD_ = 256; __VA_ARGS__; }                   \
  else TORCH_CHECK(false, "flash attention: head dim must be 64, 128 or 256");

static void fill_strides(AttnParams& p, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v) {
  p.sqb = q.stride(0); p.sqt = q.stride(1); p.sqh = q.stride(2);
  p.skb = k.stride(0); p.skt = k.stride(1); p.skh = k.stride(2);
  p.svb = v.stride(0); p.svt = v.stride(1); p.svh = v.stride(2);
}

// q [B,Tq,H,hd], k/v [B,Tk,Hkv,hd] (strided views allowed). Returns (out [B,Tq,H,hd], lse [B,H,Tq]).
std::vector<at::Tensor> attn_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, double scale,
                                 bool causal) {
  check_qkv(q, "q"); check_qkv(k, "k"); check_qkv(v, "v");
  const int B = q.size(0), Tq = q.size(1), H = q.size(2), HD = q.size(3);
  const int Tk = k.size(1), Hkv = k.size(2);
  TORCH_CHECK(k.size(0) == B && v.size(0) == B && v.size(1) == Tk && v.size(2) == Hkv && k.size(3) == HD &&
              v.size(3) == HD, "attn: shape mismatch");
  TORCH_CHECK(H % Hkv == 0, "attn: H must be a multiple of Hkv");
  DeviceGuard g(q.device());
  auto out = at::empty({B, Tq, H, HD}, q.options());
  auto lse = at::empty({B, H, Tq}, q.options().dtype(at::kFloat));
  AttnParams p{};
  p.q = (const bf16*)q.data_ptr(); p.k = (const bf16*)k.data_ptr(); p.v = (const bf16*)v.data_ptr();
  p.out = (bf16*)out.data_ptr(); p.lse = lse.data_ptr<float>();
  p.B = B; p.H = H; p.Hkv = Hkv; p.Tq = Tq; p.Tk = Tk;
  fill_strides(p, q, k, v);
  p.sob = out.stride(0); p.sot = out.stride(1); p.soh = out.stride(2);
  p.scale = (float)scale; p.scale_log2 = (float)(scale * 1.4426950408889634);
  p.causal_off = Tk - Tq;
  p.hsplit = 1;
  if (B * Tq * H == 0) return {out, lse};
  auto st = stream();
  HD_SWITCH(HD, {
    constexpr int NW = fwd_waves<HD_>();
    const int grid = cdiv(Tq, 32 * NW) * H * B;
    if (causal) attn_fwd_kernel<HD_, NW, true><<<grid, NW * 64, 0, st>>>(p);
    else attn_fwd_kernel<HD_, NW, false><<<grid, NW * 64, 0, st>>>(p);
  });
  SPA_LAUNCH_CHECK();
  return {out, lse};
}

// Gradients written into dq/dk/dv (strided views allowed, e.g. slices of one dqkv buffer).
void attn_bwd(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
              const at::Tensor& out, const at::Tensor& lse, const at::Tensor& dq, const at::Tensor& dk,
              const at::Tensor& dv, double scale, bool causal) {
  check_qkv(dout, "dout"); check_qkv(q, "q"); check_qkv(k, "k"); check_qkv(v, "v"); check_qkv(out, "out");
  check_qkv(dq, "dq"); check_qkv(dk, "dk"); check_qkv(dv, "dv");
  const int B = q.size(0), Tq = q.size(1), H = q.size(2), HD = q.size(3);
  const int Tk = k.size(1), Hkv = k.size(2);
  TORCH_CHECK(lse.is_contiguous() && lse.numel() == (int64_t)B * H * Tq);
  TORCH_CHECK(dq.sizes() == q.sizes() && dk.sizes() == k.sizes() && dv.sizes() == v.sizes());
  TORCH_CHECK(dout.sizes() == q.sizes() && out.sizes() == q.sizes());
  DeviceGuard g(q.device());
  auto delta = at::empty({B, H, Tq}, q.options().dtype(at::kFloat));
  AttnParams p{};
  p.q = (const bf16*)q.data_ptr(); p.k = (const bf16*)k.data_ptr(); p.v = (const bf16*)v.data_ptr();
  p.o = (const bf16*)out.data_ptr(); p.dout = (const bf16*)dout.data_ptr();
  p.dq = (bf16*)dq.data_ptr(); p.dk = (bf16*)dk.data_ptr(); p.dv = (bf16*)dv.data_ptr();
  p.lse_in = lse.data_ptr<float>(); p.delta = delta.data_ptr<float>();
  p.B = B; p.H = H; p.Hkv = Hkv; p.Tq = Tq; p.Tk = Tk;
  fill_strides(p, q, k, v);
  p.sob = out.stride(0); p.sot = out.stride(1); p.soh = out.stride(2);
  p.sdob = dout.stride(0); p.sdot = dout.stride(1); p.sdoh = dout.stride(2);
  p.sdqb = dq.stride(0); p.sdqt = dq.stride(1); p.sdqh = dq.stride(2);
  p.sdkb = dk.stride(0); p.sdkt = dk.stride(1); p.sdkh = dk.stride(2);
  p.sdvb = dv.stride(0); p.sdvt = dv.stride(1); p.sdvh = dv.stride(2);
  p.scale = (float)scale; p.scale_log2 = (float)(scale * 1.4426950408889634);
  p.causal_off = Tk - Tq;
  if (B * H == 0) return;
  auto st = stream();
  if (Tq == 0) { dk.zero_(); dv.zero_(); return; }
  // default: the deterministic two-kernel path (dq kernel + dkdv kernel, no atomics).
  // SPA_ATTN_BWD_FUSED=1: one pass computing dQ too (5 MFMA products per tile instead of 7)
  // with fp32 dQ atomics. Measured on MI355X at LLaMA3-8B shape (B1 T8192 H32/8 hd128):
  // fused 3.87 ms vs split 2.74 ms -- with 128-key blocks each dQ row receives T/128 atomic
  // adds (~4 GB of adds per call), past the chip-wide atomic rate; kept as an option.
  static const bool want_fused = getenv("SPA_ATTN_BWD_FUSED") && atoi(getenv("SPA_ATTN_BWD_FUSED")) != 0;
  const bool fused = want_fused && Tk > 0 && HD <= 128;
  at::Tensor dqacc;
  if (fused) {
    dqacc = at::zeros({B, Tq, H, HD}, q.options().dtype(at::kFloat));
    p.dqacc = dqacc.data_ptr<float>();
  }
  // dK/dV grid: key blocks x kv-heads x batch, times a q-head split when that grid cannot
  // fill the chip (MQA: Hkv = 1 launched 32 blocks at T = 4096); partials are summed by
  // attn_kv_reduce_kernel. dK/dV kernel: paired-wave (2) for hd 128, single-wave (1) else;
  // SPA_ATTN_DKDV overrides (read per call, so one process can A/B them). Measured in one
  // process on MI355X: LLaMA3-8B shape bwd 2.22 ms paired vs 2.45 ms single-wave; ViT-B
  // hd 64 (T 197, B 64) 0.121 ms paired vs 0.097 ms single-wave.
  const int dkdv_mode = getenv("SPA_ATTN_DKDV") ? atoi(getenv("SPA_ATTN_DKDV")) : (HD == 128 ? 2 : 1);
  const int G = H / Hkv;
  const int nkv = cdiv(Tk, 128) * Hkv * B;
  int hsplit = 1;
  if (!fused)
    while (nkv * hsplit < 512 && hsplit < G) {
      int d = hsplit + 1;
      while (G % d) ++d;
      hsplit = d;
    }
  p.hsplit = hsplit;
  at::Tensor kvacc;
  if (hsplit > 1) {
    kvacc = at::empty({2, hsplit, B, Tk, Hkv, HD}, q.options().dtype(at::kFloat));
    p.dkacc = kvacc.data_ptr<float>();
    p.dvacc = p.dkacc + (long)hsplit * B * Tk * Hkv * HD;
  }
  HD_SWITCH(HD, {
    constexpr int NW = fwd_waves<HD_>();
    constexpr int MT = HD_ == 128 ? 2 : 1;
    const int g2 = nkv * hsplit;
    if (fused && HD_ <= 128) {   // hd 256: the fused body exceeds the register file (spills)
      const long rows = (long)B * Tq * H;
      attn_delta_kernel<HD_><<<(int)cdiv(rows, 256 / (HD_ / 8)), 256, 0, st>>>(p);
      if (causal) attn_bwd_dkdv_kernel<HD_, true, MT, true><<<g2, 256, 0, st>>>(p);
      else attn_bwd_dkdv_kernel<HD_, false, MT, true><<<g2, 256, 0, st>>>(p);
      const long n = rows * (HD_ / 8);
      attn_dq_store_kernel<HD_><<<(int)std::min<long>((n + 255) / 256, 65536), 256, 0, st>>>(p);
    } else {
      const int grid = cdiv(Tq, 32 * NW) * H * B;
      if (causal) attn_bwd_dq_kernel<HD_, NW, true><<<grid, NW * 64, 0, st>>>(p);
      else attn_bwd_dq_kernel<HD_, NW, false><<<grid, NW * 64, 0, st>>>(p);
      if (Tk > 0) {
        if (HD_ <= 128 && dkdv_mode != 1) {
          if (causal) attn_bwd_dkdv2_kernel<(HD_ <= 128 ? HD_ : 128), true><<<g2, 512, 0, st>>>(p);
          else attn_bwd_dkdv2_kernel<(HD_ <= 128 ? HD_ : 128), false><<<g2, 512, 0, st>>>(p);
        } else {
          if (causal) attn_bwd_dkdv_kernel<HD_, true, MT, false><<<g2, 256, 0, st>>>(p);
          else attn_bwd_dkdv_kernel<HD_, false, MT, false><<<g2, 256, 0, st>>>(p);
        }
        if (hsplit > 1) {
          const long n = (long)B * Tk * Hkv * (HD_ / 8) * 2;
          attn_kv_reduce_kernel<HD_><<<(int)std::min<long>((n + 255) / 256, 65536), 256, 0, st>>>(p);
        }
      }
    }
  });
  SPA_LAUNCH_CHECK();
}

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.def("attn_fwd(Tensor q, Tensor k, Tensor v, float scale, bool causal) -> Tensor[]");
  m.def("attn_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor out, Tensor lse, Tensor(a!) dq, Tensor(b!) dk, "
        "Tensor(c!) dv, float scale, bool causal) -> ()");
}
TORCH_LIBRARY_IMPL(spa, CUDA, m) {
  m.impl("attn_fwd", &spa::attn_fwd);
  m.impl("attn_bwd", &spa::attn_bwd);
}
