// fp32 flash attention on the fp32 matrix cores (v_mfma_f32_16x16x4_f32): the reference's own
// training precision -- gpt/gpt-jax.ipynb:344-353 and llama3/LLaMA-jax.ipynb:809-829 train in fp32 --
// so the same-config parity runs (BASELINE B1 / B5 at --dtype fp32) attend on a hand-written kernel
// instead of a GEMM + softmax fallback. Causal / full, GQA / MQA by head mapping, the bf16 kernels'
// counter-hash dropout, (b, t, h) strides (packed qkv), head dims 16 / 32 / 64 / 128 / 256.
//
// Layout (one wave per block; 16 query rows -- forward, dQ -- or 16 keys -- dK/dV -- per block):
//  * 16x16x4 MFMA, lane l = (group g = l / 16, column c = l % 16): A[i = c][k = g], B[k = g][j = c],
//    D[i = 4g + r][j = c], r = 0..3. The product S^T = K Q^T puts the QUERY on the lane column
//    (c) and four keys 4g + r in the accumulator registers, so the online softmax is lane-local
//    up to one 4-group reduction (two xor shuffles), and P feeds O^T = V^T P^T straight from the
//    accumulator: step r of a 16-key tile takes key 4g + r from lane group g (B = p[r]).
//  * The reduction over the head dim is permuted: lane group g covers d in [g HD/4, (g+1) HD/4) in
//    step order, so every operand a lane streams along d is contiguous (float4 global / LDS reads)
//    and the register fragments are HD/4 floats.
//  * K / V (forward, dQ) and Q / dO (dK/dV) tiles of 16 rows are staged through LDS with rows padded
//    to HD + 4 floats: the row-fragment reads (16 rows at one column) and the column reads (16
//    consecutive columns of 4 rows) both spread over the banks.
//  * Backward = dQ (query-parallel, also writes delta = rowsum(dO * O)) then dK/dV (key-parallel,
//    looping the GQA group's q-heads so dK / dV of a kv-head are summed in registers); no atomics.
#include "spa_common.h"

SPA_DEBUG_TU("attention_f32.hip")

namespace spa {

struct F32AttnParams {
  const float *q, *k, *v, *o, *dout;
  float *out, *dq, *dk, *dv, *lse, *delta;
  const float* lse_in;
  int B, H, Hkv, Tq, Tk;
  long sqb, sqt, sqh, skb, skt, skh, svb, svt, svh, sob, sot, soh, sdob, sdot, sdoh;
  long sdqb, sdqt, sdqh, sdkb, sdkt, sdkh, sdvb, sdvt, sdvh;
  float scale, scale_log2;
  int causal_off;
  unsigned seed_lo, seed_hi, drop_thr;
  float drop_scale;
  const int64_t* seed_ptr;
};

namespace f32a {

constexpr int TILE = 16;

__device__ __forceinline__ f32x4 mfma(float a, float b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// same counter hash as attention.hip (drop_base / drop_keep), so masks agree across dtypes
__device__ __forceinline__ unsigned mix32(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ unsigned drop_base(const F32AttnParams& p, int b, int h) {
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
// max / sum over the 4 lane groups holding one column (lanes c, c+16, c+32, c+48)
__device__ __forceinline__ float gmax(float x) {
  x = fmaxf(x, __shfl_xor(x, 16, 64));
  return fmaxf(x, __shfl_xor(x, 32, 64));
}
__device__ __forceinline__ float gsum(float x) {
  x += __shfl_xor(x, 16, 64);
  return x + __shfl_xor(x, 32, 64);
}

// 16 rows x HD of a strided tensor (rows row0.., stride rs, zeros past nrows) -> LDS rows of HD + 4
template <int HD>
__device__ __forceinline__ void stage(float* lds, const float* base, long rs, int row0, int nrows, int lane) {
  constexpr int C4 = HD / 4, LD = HD + 4;
#pragma unroll
  for (int j = 0; j < TILE * C4 / 64; ++j) {
    const int i = lane + 64 * j, r = i / C4, c4 = i % C4;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (row0 + r < nrows) v = *reinterpret_cast<const f32x4*>(base + (long)(row0 + r) * rs + 4 * c4);
    SPA_DBG_LDS(r * LD + 4 * c4 + 3, TILE * LD);
    *reinterpret_cast<f32x4*>(lds + r * LD + 4 * c4) = v;
  }
}
// this lane's HD/4-float fragment of a row in global memory (group g's d range), zeros if !valid
template <int HD>
__device__ __forceinline__ void frag(float (&f)[HD / 4], const float* row, int g, bool valid) {
#pragma unroll
  for (int j = 0; j < HD / 16; ++j) {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (valid) v = *reinterpret_cast<const f32x4*>(row + g * (HD / 4) + 4 * j);
#pragma unroll
    for (int i = 0; i < 4; ++i) f[4 * j + i] = v[i];
  }
}
// sum_d A[row c][d] B[d] over this lane group's d range: A from an LDS tile (row c), B a fragment
template <int HD>
__device__ __forceinline__ f32x4 dot_tile(const float* lds, int c, int g, const float (&f)[HD / 4], f32x4 acc) {
  const float* r = lds + c * (HD + 4) + g * (HD / 4);
#pragma unroll
  for (int j = 0; j < HD / 16; ++j) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(r + 4 * j);
#pragma unroll
    for (int i = 0; i < 4; ++i) acc = mfma(a[i], f[4 * j + i], acc);
  }
  return acc;
}
// the same with both operands read from LDS tiles (row c of each)
template <int HD>
__device__ __forceinline__ f32x4 dot_tiles(const float* la, const float* lb, int c, int g, f32x4 acc) {
  const float* ra = la + c * (HD + 4) + g * (HD / 4);
  const float* rb = lb + c * (HD + 4) + g * (HD / 4);
#pragma unroll
  for (int j = 0; j < HD / 16; ++j) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(ra + 4 * j);
    const f32x4 b = *reinterpret_cast<const f32x4*>(rb + 4 * j);
#pragma unroll
    for (int i = 0; i < 4; ++i) acc = mfma(a[i], b[i], acc);
  }
  return acc;
}
// acc[dt] += T^T[dt*16 + c][rows 4g + r] x w[r]: the column product over a 16-row LDS tile whose
// row 4g + r pairs with this lane's accumulator register r (P -> O, dS -> dQ / dK, P -> dV)
template <int HD>
__device__ __forceinline__ void col_accum(f32x4 (&acc)[HD / 16], const float* lds, int c, int g, const f32x4& w) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float* row = lds + (4 * g + r) * (HD + 4) + c;
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) acc[dt] = mfma(row[16 * dt], w[r], acc[dt]);
  }
}
// accumulator tile dt (rows d = dt*16 + 4g + i, column = this lane's row) -> global row
template <int HD>
__device__ __forceinline__ void store_rows(float* row, const f32x4 (&acc)[HD / 16], int g, float sc) {
#pragma unroll
  for (int dt = 0; dt < HD / 16; ++dt) {
    f32x4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = acc[dt][i] * sc;
    *reinterpret_cast<f32x4*>(row + 16 * dt + 4 * g) = v;
  }
}

}  // namespace f32a

// ---------------------------------------------------------------------------------------------
// forward: block = 1 wave, 16 queries of one (b, h); K / V tiles of 16 keys through LDS
template <int HD, bool CAUSAL, bool DROP>
__global__ __launch_bounds__(64) void attn_f32_fwd_kernel(F32AttnParams p) {
  using namespace f32a;
  constexpr int LD = HD + 4, DT = HD / 16;
  __shared__ __attribute__((aligned(16))) float ks[TILE * LD], vs[TILE * LD];
  const int lane = threadIdx.x, g = lane >> 4, c = lane & 15;
  const int nqt = cdiv(p.Tq, TILE);
  const int bh = blockIdx.x % (p.B * p.H), qt = blockIdx.x / (p.B * p.H);
  const int b = bh / p.H, h = bh % p.H, hk = h / (p.H / p.Hkv);
  SPA_DBG_CHECK(qt, nqt);
  const int q = qt * TILE + c;
  const bool qv = q < p.Tq;
  float qf[HD / 4];
  frag<HD>(qf, p.q + b * p.sqb + (long)q * p.sqt + h * p.sqh, g, qv);
  f32x4 o[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  const unsigned dbase = DROP ? drop_base(p, b, h) : 0u;
  const float cs = p.scale_log2;
  const int kend = CAUSAL ? min(p.Tk, qt * TILE + TILE + p.causal_off) : p.Tk;
  const float* kb = p.k + b * p.skb + hk * p.skh;
  const float* vb = p.v + b * p.svb + hk * p.svh;
  for (int k0 = 0; k0 < kend; k0 += TILE) {
    stage<HD>(ks, kb, p.skt, k0, p.Tk, lane);
    stage<HD>(vs, vb, p.svt, k0, p.Tk, lane);
    __syncthreads();
    f32x4 s = dot_tile<HD>(ks, c, g, qf, f32x4{0.f, 0.f, 0.f, 0.f});   // S^T[key 4g+r][query c]
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = k0 + 4 * g + r;
      s[r] = (key >= p.Tk || (CAUSAL && key > q + p.causal_off)) ? -INFINITY : s[r] * cs;
      mx = fmaxf(mx, s[r]);
    }
    mx = gmax(mx);
    const float mn = fmaxf(m, mx);
    if (mn > m) {                                    // exact online rescale (fp32 path)
      const float alpha = mn == -INFINITY ? 1.f : exp2f(m - mn);
      l *= alpha;
#pragma unroll
      for (int i = 0; i < DT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[i][r] *= alpha;
      m = mn;
    }
    f32x4 pr;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float e = m == -INFINITY ? 0.f : exp2f(s[r] - m);
      l += e;
      pr[r] = e;
      if (DROP) pr[r] = drop_keep(dbase, q, k0 + 4 * g + r, p.drop_thr) ? e * p.drop_scale : 0.f;
    }
    col_accum<HD>(o, vs, c, g, pr);
    __syncthreads();
  }
  l = gsum(l);
  if (!qv || !(SPA_DBG_OK(b, p.B) & SPA_DBG_OK(h, p.H))) return;
  store_rows<HD>(p.out + b * p.sob + (long)q * p.sot + h * p.soh, o, g, l > 0.f ? 1.f / l : 0.f);
  if (g == 0 && p.lse)
    p.lse[((long)b * p.H + h) * p.Tq + q] = l > 0.f ? (m + log2f(l)) * 0.69314718055994531f : INFINITY;
}

// ---------------------------------------------------------------------------------------------
// dQ (query-parallel) + delta: S^T and dP^T = V dO^T recomputed per 16-key tile, dS = P (dP - delta),
// dQ^T += K^T dS^T
template <int HD, bool CAUSAL, bool DROP>
__global__ __launch_bounds__(64) void attn_f32_dq_kernel(F32AttnParams p) {
  using namespace f32a;
  constexpr int LD = HD + 4, DT = HD / 16;
  __shared__ __attribute__((aligned(16))) float ks[TILE * LD], vs[TILE * LD];
  const int lane = threadIdx.x, g = lane >> 4, c = lane & 15;
  const int bh = blockIdx.x % (p.B * p.H), qt = blockIdx.x / (p.B * p.H);
  const int b = bh / p.H, h = bh % p.H, hk = h / (p.H / p.Hkv);
  const int q = qt * TILE + c;
  const bool qv = q < p.Tq;
  float qf[HD / 4], df[HD / 4];
  frag<HD>(qf, p.q + b * p.sqb + (long)q * p.sqt + h * p.sqh, g, qv);
  frag<HD>(df, p.dout + b * p.sdob + (long)q * p.sdot + h * p.sdoh, g, qv);
  float dlt = 0.f;
  {
    float of[HD / 4];
    frag<HD>(of, p.o + b * p.sob + (long)q * p.sot + h * p.soh, g, qv);
#pragma unroll
    for (int i = 0; i < HD / 4; ++i) dlt += of[i] * df[i];
    dlt = gsum(dlt);
  }
  const long srow = ((long)b * p.H + h) * p.Tq + q;
  if (qv && g == 0 && SPA_DBG_OK(srow, (long)p.B * p.H * p.Tq)) p.delta[srow] = dlt;
  const float nl2 = qv ? -p.lse_in[srow] * 1.4426950408889634f : -INFINITY;
  f32x4 acc[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const unsigned dbase = DROP ? drop_base(p, b, h) : 0u;
  const float cs = p.scale_log2;
  const int kend = CAUSAL ? min(p.Tk, qt * TILE + TILE + p.causal_off) : p.Tk;
  const float* kb = p.k + b * p.skb + hk * p.skh;
  const float* vb = p.v + b * p.svb + hk * p.svh;
  for (int k0 = 0; k0 < kend; k0 += TILE) {
    stage<HD>(ks, kb, p.skt, k0, p.Tk, lane);
    stage<HD>(vs, vb, p.svt, k0, p.Tk, lane);
    __syncthreads();
    const f32x4 s = dot_tile<HD>(ks, c, g, qf, f32x4{0.f, 0.f, 0.f, 0.f});
    const f32x4 dp = dot_tile<HD>(vs, c, g, df, f32x4{0.f, 0.f, 0.f, 0.f});
    f32x4 ds;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = k0 + 4 * g + r;
      const bool live = qv && key < p.Tk && !(CAUSAL && key > q + p.causal_off);
      const float pr = live ? exp2f(fmaf(s[r], cs, nl2)) : 0.f;
      float d = dp[r];
      if (DROP) d = drop_keep(dbase, q, key, p.drop_thr) ? d * p.drop_scale : 0.f;
      ds[r] = pr * (d - dlt);
    }
    col_accum<HD>(acc, ks, c, g, ds);
    __syncthreads();
  }
  if (!qv || !(SPA_DBG_OK(b, p.B) & SPA_DBG_OK(h, p.H))) return;
  store_rows<HD>(p.dq + b * p.sdqb + (long)q * p.sdqt + h * p.sdqh, acc, g, p.scale);
}

// ---------------------------------------------------------------------------------------------
// dK / dV (key-parallel): 16 keys per block (K / V rows in LDS), the GQA group's q-heads x 16-query
// tiles streamed through LDS; S = Q K^T and dP = dO V^T with the key on the lane column
template <int HD, bool CAUSAL, bool DROP>
__global__ __launch_bounds__(64) void attn_f32_dkdv_kernel(F32AttnParams p) {
  using namespace f32a;
  constexpr int LD = HD + 4, DT = HD / 16;
  __shared__ __attribute__((aligned(16))) float kk[TILE * LD], vv[TILE * LD], qs[TILE * LD], ds_[TILE * LD];
  __shared__ float rl[TILE], rd[TILE];
  const int lane = threadIdx.x, g = lane >> 4, c = lane & 15;
  const int bk = blockIdx.x % (p.B * p.Hkv), kt = blockIdx.x / (p.B * p.Hkv);
  const int b = bk / p.Hkv, hk = bk % p.Hkv, G = p.H / p.Hkv;
  const int k0 = kt * TILE, key = k0 + c;
  SPA_DBG_CHECK(k0, p.Tk);
  stage<HD>(kk, p.k + b * p.skb + hk * p.skh, p.skt, k0, p.Tk, lane);
  stage<HD>(vv, p.v + b * p.svb + hk * p.svh, p.svt, k0, p.Tk, lane);
  f32x4 dk[DT], dv[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) dk[i] = dv[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float cs = p.scale_log2;
  // causal: queries below k0 - causal_off see none of these keys
  const int qbeg = CAUSAL ? max(0, k0 - p.causal_off) / TILE * TILE : 0;
  for (int hg = 0; hg < G; ++hg) {
    const int h = hk * G + hg;
    const unsigned dbase = DROP ? drop_base(p, b, h) : 0u;
    for (int q0 = qbeg; q0 < p.Tq; q0 += TILE) {
      __syncthreads();   // the previous tile's readers are done
      stage<HD>(qs, p.q + b * p.sqb + h * p.sqh, p.sqt, q0, p.Tq, lane);
      stage<HD>(ds_, p.dout + b * p.sdob + h * p.sdoh, p.sdot, q0, p.Tq, lane);
      if (lane < TILE) {
        const int qq = q0 + lane;
        const long r = ((long)b * p.H + h) * p.Tq + min(qq, p.Tq - 1);
        rl[lane] = qq < p.Tq ? -p.lse_in[r] * 1.4426950408889634f : -INFINITY;
        rd[lane] = qq < p.Tq ? p.delta[r] : 0.f;
      }
      __syncthreads();
      // lane holds S[q = q0 + 4g + r][key = k0 + c] and dP likewise
      const f32x4 s = dot_tiles<HD>(qs, kk, c, g, f32x4{0.f, 0.f, 0.f, 0.f});
      const f32x4 dp = dot_tiles<HD>(ds_, vv, c, g, f32x4{0.f, 0.f, 0.f, 0.f});
      f32x4 pr, pd, dsv;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qq = q0 + 4 * g + r;
        const bool live = key < p.Tk && qq < p.Tq && !(CAUSAL && key > qq + p.causal_off);
        const float e = live ? exp2f(fmaf(s[r], cs, rl[4 * g + r])) : 0.f;
        float d = dp[r];
        bool kp = true;
        if (DROP) {
          kp = drop_keep(dbase, qq, key, p.drop_thr);
          d = kp ? d * p.drop_scale : 0.f;
        }
        pr[r] = e;
        pd[r] = DROP ? (kp ? e * p.drop_scale : 0.f) : e;
        dsv[r] = e * (d - rd[4 * g + r]);
      }
      col_accum<HD>(dv, ds_, c, g, pd);   // dV^T += dO^T P (dropped P)
      col_accum<HD>(dk, qs, c, g, dsv);   // dK^T += Q^T dS
    }
  }
  if (key >= p.Tk || !(SPA_DBG_OK(b, p.B) & SPA_DBG_OK(hk, p.Hkv))) return;
  store_rows<HD>(p.dk + b * p.sdkb + (long)key * p.sdkt + hk * p.sdkh, dk, g, p.scale);
  store_rows<HD>(p.dv + b * p.sdvb + (long)key * p.sdvt + hk * p.sdvh, dv, g, 1.f);
}

// ---------------------------------------------------------------------------------------------
// host
static void check_f32(const at::Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.dim() == 4, n, ": fp32 HIP tensor [B, T, H, hd]");
  TORCH_CHECK(t.stride(3) == 1 && t.stride(0) % 4 == 0 && t.stride(1) % 4 == 0 && t.stride(2) % 4 == 0 &&
                  ((uintptr_t)t.data_ptr() % 16) == 0,
              n, ": rows must be 16-byte aligned and contiguous in hd");
}

#define F32_HD_SWITCH(HDV, ...)                                   \
  switch (HDV) {                                                  \
    case 16: { constexpr int HD_ = 16; __VA_ARGS__; } break;      \
    case 32: { constexpr int HD_ = 32; __VA_ARGS__; } break;      \
    case 64: { constexpr int HD_ = 64; __VA_ARGS__; } break;      \
    case 128: { constexpr int HD_ = 128; __VA_ARGS__; } break;    \
    case 256: { constexpr int HD_ = 256; __VA_ARGS__; } break;    \
    default: TORCH_CHECK(false, "fp32 attention: head dim must be 16, 32, 64, 128 or 256"); \
  }

static void f32_common(F32AttnParams& p, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                       double scale, double dropout_p, int64_t seed, const c10::optional<at::Tensor>& seed_t) {
  p.B = q.size(0); p.Tq = q.size(1); p.H = q.size(2); p.Tk = k.size(1); p.Hkv = k.size(2);
  TORCH_CHECK(k.size(0) == p.B && v.size(0) == p.B && v.size(1) == p.Tk && v.size(2) == p.Hkv &&
                  k.size(3) == q.size(3) && v.size(3) == q.size(3) && p.H % p.Hkv == 0,
              "fp32 attention: shape mismatch (equal head dims, H % Hkv == 0)");
  p.q = q.data_ptr<float>(); p.k = k.data_ptr<float>(); p.v = v.data_ptr<float>();
  p.sqb = q.stride(0); p.sqt = q.stride(1); p.sqh = q.stride(2);
  p.skb = k.stride(0); p.skt = k.stride(1); p.skh = k.stride(2);
  p.svb = v.stride(0); p.svt = v.stride(1); p.svh = v.stride(2);
  p.scale = (float)scale; p.scale_log2 = (float)(scale * 1.4426950408889634);
  p.causal_off = p.Tk - p.Tq;
  TORCH_CHECK(dropout_p >= 0.0 && dropout_p < 1.0, "fp32 attention: dropout p in [0, 1)");
  if (seed_t) {
    TORCH_CHECK(seed_t->is_cuda() && seed_t->scalar_type() == at::kLong, "fp32 attention: int64 device seed");
    p.seed_ptr = seed_t->data_ptr<int64_t>();
  }
  p.seed_lo = (unsigned)(seed & 0xffffffffu);
  p.seed_hi = (unsigned)(((uint64_t)seed >> 32) & 0xffffffffu);
  p.drop_thr = (unsigned)std::llround(dropout_p * 16777216.0);
  p.drop_scale = (float)(1.0 / (1.0 - dropout_p));
}

std::vector<at::Tensor> attn_f32_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, double scale,
                                     bool causal, double dropout_p, int64_t seed,
                                     const c10::optional<at::Tensor>& seed_t) {
  check_f32(q, "q"); check_f32(k, "k"); check_f32(v, "v");
  DeviceGuard dg(q.device());
  F32AttnParams p{};
  f32_common(p, q, k, v, scale, dropout_p, seed, seed_t);
  auto out = at::empty({p.B, p.Tq, p.H, q.size(3)}, q.options());
  auto lse = at::empty({p.B, p.H, p.Tq}, q.options());
  p.out = out.data_ptr<float>(); p.lse = lse.data_ptr<float>();
  p.sob = out.stride(0); p.sot = out.stride(1); p.soh = out.stride(2);
  const int grid = cdiv(p.Tq, 16) * p.B * p.H;
  if (grid == 0) return {out, lse};
  const bool drop = dropout_p > 0.0;
  F32_HD_SWITCH(q.size(3),
    if (causal) { if (drop) attn_f32_fwd_kernel<HD_, true, true><<<grid, 64, 0, stream()>>>(p);
                  else attn_f32_fwd_kernel<HD_, true, false><<<grid, 64, 0, stream()>>>(p); }
    else { if (drop) attn_f32_fwd_kernel<HD_, false, true><<<grid, 64, 0, stream()>>>(p);
           else attn_f32_fwd_kernel<HD_, false, false><<<grid, 64, 0, stream()>>>(p); })
  SPA_LAUNCH_CHECK();
  return {out, lse};
}

// dq / dk / dv: outputs (strided views allowed, e.g. slices of one packed dqkv)
void attn_f32_bwd(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                  const at::Tensor& o, const at::Tensor& lse, at::Tensor& dq, at::Tensor& dk, at::Tensor& dv, double scale,
                  bool causal, double dropout_p, int64_t seed, const c10::optional<at::Tensor>& seed_t) {
  check_f32(q, "q"); check_f32(k, "k"); check_f32(v, "v"); check_f32(o, "o"); check_f32(dout, "dout");
  check_f32(dq, "dq"); check_f32(dk, "dk"); check_f32(dv, "dv");
  DeviceGuard dg(q.device());
  F32AttnParams p{};
  f32_common(p, q, k, v, scale, dropout_p, seed, seed_t);
  TORCH_CHECK(lse.is_contiguous() && lse.numel() == (long)p.B * p.H * p.Tq, "fp32 attention: lse [B, H, Tq]");
  auto delta = at::empty({p.B, p.H, p.Tq}, q.options());
  p.o = o.data_ptr<float>(); p.dout = dout.data_ptr<float>(); p.lse_in = lse.data_ptr<float>();
  p.delta = delta.data_ptr<float>();
  p.dq = dq.data_ptr<float>(); p.dk = dk.data_ptr<float>(); p.dv = dv.data_ptr<float>();
  p.sob = o.stride(0); p.sot = o.stride(1); p.soh = o.stride(2);
  p.sdob = dout.stride(0); p.sdot = dout.stride(1); p.sdoh = dout.stride(2);
  p.sdqb = dq.stride(0); p.sdqt = dq.stride(1); p.sdqh = dq.stride(2);
  p.sdkb = dk.stride(0); p.sdkt = dk.stride(1); p.sdkh = dk.stride(2);
  p.sdvb = dv.stride(0); p.sdvt = dv.stride(1); p.sdvh = dv.stride(2);
  const int gq = cdiv(p.Tq, 16) * p.B * p.H, gk = cdiv(p.Tk, 16) * p.B * p.Hkv;
  if (gq == 0 || gk == 0) return;
  const bool drop = dropout_p > 0.0;
  auto st = stream();
#define F32_BWD(C, D)                                                  \
  attn_f32_dq_kernel<HD_, C, D><<<gq, 64, 0, st>>>(p);                 \
  attn_f32_dkdv_kernel<HD_, C, D><<<gk, 64, 0, st>>>(p)
  F32_HD_SWITCH(q.size(3),
    if (causal) { if (drop) { F32_BWD(true, true); } else { F32_BWD(true, false); } }
    else { if (drop) { F32_BWD(false, true); } else { F32_BWD(false, false); } })
#undef F32_BWD
  SPA_LAUNCH_CHECK();
}

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.def("attn_f32_fwd(Tensor q, Tensor k, Tensor v, float scale, bool causal, float dropout_p=0.0, int seed=0, "
        "Tensor? seed_t=None) -> Tensor[]");
  m.def("attn_f32_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, Tensor(a!) dq, Tensor(b!) dk, "
        "Tensor(c!) dv, float scale, bool causal, float dropout_p=0.0, int seed=0, Tensor? seed_t=None) -> ()");
}
TORCH_LIBRARY_IMPL(spa, CUDA, m) {
  m.impl("attn_f32_fwd", &spa::attn_f32_fwd);
  m.impl("attn_f32_bwd", &spa::attn_f32_bwd);
}
