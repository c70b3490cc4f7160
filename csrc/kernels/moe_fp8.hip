// FP8 (OCP e4m3) MoE expert GEMMs on CDNA4's block-scaled MFMA
// v_mfma_scale_f32_32x32x64_f8f6f4 (2x the bf16 MFMA rate).
//
// BASELINE.json config #5 ("DeepSeek-V3-style MLA + MoE grouped GEMM, fp8 CDNA4 MFMA").
// The reference runs its experts in fp16 autocast (deepseekv3/deepseekv3.ipynb:2411) in a
// Python loop; here the routed-expert projections of the forward and the activation
// gradient run in fp8 with per-row scales, the weight gradient stays bf16:
//   quant_rows_fp8:  x [R, K] bf16 -> q [R, K] e4m3 + s [R] fp32  (s = amax / 448)
//   grouped_gemm_fp8: Y_e = (Xq_e Wq_e^T) * sx[m] * sw[e, n]  -> bf16
// The dX product uses the same NT kernel on a per-expert transposed, re-quantized weight
// (dX = dYq (Wt_q)^T with Wt = W^T), so no fp8 transposed LDS reads are needed.
//
// Tile 256 x 256 x 128 (fp8 bytes), 8 waves as 2 (m) x 4 (n), wave tile 128 x 64 computed
// as C^T (MFMA A operand = weight rows, B = token rows). MFMA operand map (probed on
// MI355X, tools/probe_fp8.hip): lane (row l&31, half h) holds 32 bytes of k; any k order
// shared by A and B is valid, so each lane reads its row's bytes [64s + 32h, +32) with
// two ds_read_b128. K-contiguous LDS images [rows][128 B] with a 16-byte-chunk XOR
// swizzle c ^ ((r >> 1) & 7): 16 consecutive rows of one chunk hit 16 distinct 16-B
// slots -> conflict-free b128 reads. Register-staged, double-buffered, one barrier per
// k-step. Per-expert row offsets on the device (block-scan tile -> expert map, as in
// moe.hip), XCD-remapped tile order.
#include "spa_common.h"

SPA_DEBUG_TU("moe_fp8.hip")

namespace spa {

typedef int i32x8 __attribute__((ext_vector_type(8)));

// --------------------------------------------------------------------------- quantize
__global__ __launch_bounds__(256) void quant_rows_fp8_kernel(const bf16* __restrict__ x, uint8_t* __restrict__ q,
                                                             float* __restrict__ scale, int R, int K) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= R) return;
  const bf16* xr = x + (long)row * K;
  float amax = 0.f;
  for (int c = lane * 8; c < K; c += 512) {
    float v[8];
    load8(xr + c, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) amax = fmaxf(amax, fabsf(v[i]));
  }
  amax = wave_max(amax);
  const float s = amax > 0.f ? amax / 448.f : 1.f;
  const float inv = 1.f / s;
  if (lane == 0) scale[row] = s;
  uint8_t* qr = q + (long)row * K;
  for (int c = lane * 8; c < K; c += 512) {
    float v[8];
    load8(xr + c, v);
    int lo = 0, hi = 0;
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[0] * inv, v[1] * inv, lo, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[2] * inv, v[3] * inv, lo, true);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[4] * inv, v[5] * inv, hi, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[6] * inv, v[7] * inv, hi, true);
    *reinterpret_cast<int2*>(qr + c) = make_int2(lo, hi);
  }
}

// --------------------------------------------------------------------------- block-scaled quantize
// DeepSeek-V3 fp8 recipe (arXiv 2412.19437 sec. 3.3) on CDNA4's MX scale operands: activations in
// 1 x 128 tiles, weights in 128 x 128 blocks, each with a power-of-two (E8M0) scale 2^e chosen as
// the smallest with amax / 2^e <= 448. The GEMM hands the E8M0 bytes straight to
// v_mfma_scale_f32_32x32x64_f8f6f4, so the accumulation over differently scaled k-blocks happens
// inside the MFMA in fp32 -- no per-block promotion pass.
__device__ __forceinline__ int e8m0_exp(float amax) {       // e with amax / 2^e <= 448, minimal
  if (!(amax > 0.f)) return 0;
  const unsigned b = __float_as_uint(amax * (1.f / 448.f));
  int e = (int)((b >> 23) & 0xff) - 127;
  if (b & 0x7fffff) ++e;                                     // round the power up
  return max(-126, min(127, e));
}
__device__ __forceinline__ float e8m0_inv(int e) { return __uint_as_float((unsigned)(127 - e) << 23); }
__device__ __forceinline__ int2 q8(const float (&v)[8], float inv) {
  float w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = fminf(fmaxf(v[i] * inv, -448.f), 448.f);
  int lo = 0, hi = 0;
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(w[0], w[1], lo, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(w[2], w[3], lo, true);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(w[4], w[5], hi, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(w[6], w[7], hi, true);
  return make_int2(lo, hi);
}

// x [R, K] bf16 -> q [R, K] e4m3, s [R, K/128] E8M0; 16 lanes per 128-wide tile, one read of x
__global__ __launch_bounds__(256) void quant_act_blk_kernel(const bf16* __restrict__ x, uint8_t* __restrict__ q,
                                                            uint8_t* __restrict__ s, long units, int KB) {
  const long u = ((long)blockIdx.x * 256 + threadIdx.x) >> 4;
  const int l = threadIdx.x & 15;
  if (u >= units) return;                                    // whole 16-lane groups exit together
  const long off = u * 128 + l * 8;                          // [R][K] with K = 128 KB: tile u is contiguous
  float v[8];
  load8(x + off, v);
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) amax = fmaxf(amax, fabsf(v[i]));
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 16));
  const int e = e8m0_exp(amax);
  *reinterpret_cast<int2*>(q + off) = q8(v, e8m0_inv(e));
  if (l == 0) s[u] = (uint8_t)(e + 127);
}

// W [E, N, K] bf16 -> wq [E, N, K] e4m3, wtq [E, K, N] e4m3 (the same bytes transposed: a 128 x 128
// block scale is transpose-invariant), s [E, N/128, K/128], st [E, K/128, N/128] E8M0.
// One workgroup per block: one read of W, two writes of the fp8 bytes.
__global__ __launch_bounds__(256) void quant_weight_blk_kernel(const bf16* __restrict__ w, uint8_t* __restrict__ wq,
                                                               uint8_t* __restrict__ wtq, uint8_t* __restrict__ s,
                                                               uint8_t* __restrict__ st, int N, int K) {
  __shared__ __attribute__((aligned(16))) uint8_t tile[128 * 132];
  __shared__ float red[4];
  const int NB = N / 128, KB = K / 128;
  const int kb = blockIdx.x % KB, nb = (blockIdx.x / KB) % NB, e = blockIdx.x / (KB * NB);
  const int tid = threadIdx.x, c8 = (tid & 15) * 8, r0 = tid >> 4;
  const bf16* wb = w + ((long)e * N + nb * 128) * K + kb * 128;
  float v[8][8], amax = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    load8(wb + (long)(r0 + 16 * i) * K + c8, v[i]);
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v[i][j]));
  }
  amax = block_max<256>(amax, red);
  const int ex = e8m0_exp(amax);
  const float inv = e8m0_inv(ex);
  uint8_t* qb = wq + ((long)e * N + nb * 128) * K + kb * 128;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int2 p = q8(v[i], inv);
    *reinterpret_cast<int2*>(qb + (long)(r0 + 16 * i) * K + c8) = p;
    *reinterpret_cast<int2*>(tile + (r0 + 16 * i) * 132 + c8) = p;
  }
  if (tid == 0) {
    s[((long)e * NB + nb) * KB + kb] = (uint8_t)(ex + 127);
    st[((long)e * KB + kb) * NB + nb] = (uint8_t)(ex + 127);
  }
  __syncthreads();
  // transposed write: 4 x 4 byte blocks, lanes along n for coalesced 4-byte stores
  const int bn = tid & 31;
  uint8_t* tb = wtq + ((long)e * K + kb * 128) * N + nb * 128;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int bk = (tid >> 5) + 8 * i;
    unsigned r[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = *reinterpret_cast<const unsigned*>(tile + (4 * bn + j) * 132 + 4 * bk);
    // r[j] byte c = (n = 4bn + j, k = 4bk + c); output row c gathers byte c of r[0..3]
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const unsigned o = ((r[0] >> (8 * c)) & 0xff) | (((r[1] >> (8 * c)) & 0xff) << 8) |
                         (((r[2] >> (8 * c)) & 0xff) << 16) | (((r[3] >> (8 * c)) & 0xff) << 24);
      *reinterpret_cast<unsigned*>(tb + (long)(4 * bk + c) * N + 4 * bn) = o;
    }
  }
}

// q [R, K] e4m3 + s [R, ldS] E8M0 (first K/128 used) -> bf16 [R, K]; 8 elements per lane
__global__ __launch_bounds__(256) void dequant_act_blk_kernel(const uint8_t* __restrict__ q,
                                                              const uint8_t* __restrict__ s, bf16* __restrict__ y,
                                                              long n8, int K, int ldS) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    const long off = i * 8;
    const long row = off / K;
    const int col = off % K;
    const float sc = __uint_as_float((unsigned)s[row * ldS + col / 128] << 23);
    const int2 p = *reinterpret_cast<const int2*>(q + off);
    float f[8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int w = h ? p.y : p.x;
      const f32x2 a = __builtin_amdgcn_cvt_pk_f32_fp8(w, false), b = __builtin_amdgcn_cvt_pk_f32_fp8(w, true);
      f[4 * h + 0] = a[0] * sc; f[4 * h + 1] = a[1] * sc; f[4 * h + 2] = b[0] * sc; f[4 * h + 3] = b[1] * sc;
    }
    store8(y + off, f);
  }
}

// Weight-gradient operands (dW_e = dY_e^T X_e, reduction over the expert's tokens): x [T, C] bf16
// with rows grouped by expert (offsets [E+1]) -> qt [C, ldq] e4m3 TRANSPOSED (token-contiguous)
// with each expert's segment starting at the 128-aligned padded offset poff[e] and zero-filled to
// it, and st [C, ldq/128] E8M0: one scale per (channel, 128-token block) -- the 128 x 1 tiles of
// the DeepSeek-V3 recipe for the Wgrad operands. Optionally ALSO the row-major 1 x 128 image the
// forward / dX GEMMs consume (qr [T, C], sr [T, C/128], as quant_act_blk_kernel), from the same
// read of x. Block (tb, cb): padded tokens [128 tb, +128) x channels [128 cb, +128), 256 threads;
// thread t holds channels 8 (t & 15) .. +8 of rows (t >> 4) + 16 i: row amax over the 16 lanes of
// a row group, column amax over the 32 threads of a channel group (shuffles + LDS), values staged
// once in a padded bf16 LDS tile for the transposed 32-token stores.
__global__ __launch_bounds__(256) void quant_t_fp8_seg_kernel(const bf16* __restrict__ x, const int* __restrict__ offsets,
                                                              const int* __restrict__ poff, int E, int C,
                                                              uint8_t* __restrict__ qt, uint8_t* __restrict__ st, long ldq,
                                                              uint8_t* __restrict__ qr, uint8_t* __restrict__ sr) {
  constexpr int TS = 128 + 8;                           // bf16 row stride of the LDS tile
  __shared__ __attribute__((aligned(16))) bf16 tile[128 * TS];
  __shared__ float cm[4][128];
  __shared__ float cinv[128];
  const int tb = blockIdx.x, cb = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int p0 = tb * 128;
  if (p0 >= poff[E]) return;
  int lo = 0, hi = E;                                   // expert e: poff[e] <= p0 < poff[e + 1]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (poff[mid] <= p0) lo = mid; else hi = mid;
  }
  const long src0 = offsets[lo] + (p0 - poff[lo]), send = offsets[lo + 1];
  // debug build: the padded segment of expert lo covers this block and starts at a real token
  SPA_DBG_ASSERT(poff[lo] <= p0 && p0 < poff[lo + 1] && offsets[lo] <= offsets[lo + 1], p0, poff[lo + 1]);
  SPA_DBG_ASSERT(poff[lo + 1] - poff[lo] >= offsets[lo + 1] - offsets[lo], poff[lo + 1] - poff[lo], offsets[lo + 1] - offsets[lo]);
  const int c8 = (tid & 15) * 8, rg = tid >> 4;
  const int KB = C / 128;
  float v[8][8];
  float cmax[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = rg + 16 * i;
    const bool ok = src0 + r < send;
    if (ok) load8(x + (src0 + r) * C + cb * 128 + c8, v[i]);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
    }
    bf16x8 w;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      w[j] = (bf16)v[i][j];
      cmax[j] = fmaxf(cmax[j], fabsf(v[i][j]));
    }
    *reinterpret_cast<bf16x8*>(tile + r * TS + c8) = w;
    if (qr != nullptr && ok) {                          // 1 x 128 row tile = this block's 128 channels
      float am = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) am = fmaxf(am, fabsf(v[i][j]));
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) am = fmaxf(am, __shfl_xor(am, o, 16));
      const int ex = e8m0_exp(am);
      *reinterpret_cast<int2*>(qr + (src0 + r) * C + cb * 128 + c8) = q8(v[i], e8m0_inv(ex));
      if ((tid & 15) == 0) sr[(src0 + r) * KB + cb] = (uint8_t)(ex + 127);
    }
  }
  // column amax: lanes l, l^16, l^32 (same channel group, other row groups) then the 4 waves
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    cmax[j] = fmaxf(cmax[j], __shfl_xor(cmax[j], 16, 64));
    cmax[j] = fmaxf(cmax[j], __shfl_xor(cmax[j], 32, 64));
  }
  if (lane < 16) {
#pragma unroll
    for (int j = 0; j < 8; ++j) cm[wave][c8 + j] = cmax[j];
  }
  __syncthreads();
  if (tid < 128) {
    const float am = fmaxf(fmaxf(cm[0][tid], cm[1][tid]), fmaxf(cm[2][tid], cm[3][tid]));
    const int ex = e8m0_exp(am);
    cinv[tid] = e8m0_inv(ex);
    st[(long)(cb * 128 + tid) * (ldq / 128) + tb] = (uint8_t)(ex + 127);
  }
  __syncthreads();
  // transposed stores: thread -> channel pair cp (2cp, 2cp+1), tokens [32 qq, +32)
  const int cp = tid & 63, qq = tid >> 6;
  const float i0 = cinv[2 * cp], i1 = cinv[2 * cp + 1];
  float a[32], b2[32];
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const bf16x2 w = *reinterpret_cast<const bf16x2*>(tile + (32 * qq + j) * TS + 2 * cp);
    a[j] = (float)w[0];
    b2[j] = (float)w[1];
  }
  uint8_t* o0 = qt + (long)(cb * 128 + 2 * cp) * ldq + p0 + 32 * qq;
  uint8_t* o1 = o0 + ldq;
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    float t0[8], t1[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { t0[j] = a[8 * h + j]; t1[j] = b2[8 * h + j]; }
    *reinterpret_cast<int2*>(o0 + 8 * h) = q8(t0, i0);
    *reinterpret_cast<int2*>(o1 + 8 * h) = q8(t1, i1);
  }
}

// --------------------------------------------------------------------------- GEMM
__device__ __forceinline__ int f8_off(int r, int c) { return r * 128 + 16 * (c ^ ((r >> 1) & 7)); }

// BLK = false: per-row fp32 scales sa [M], sb [E, N] applied in the epilogue (unit MFMA scales).
// BLK = true: E8M0 block scales sa [M, K/128] (1 x 128 activation tiles), sb [E, N/128, K/128]
// (128 x 128 weight blocks) fed to the MFMA scale operands per k-step; no epilogue scaling.
// WG (weight gradient, with BLK): C_e [M, N] (+)= A[:, seg_e] B[:, seg_e]^T over expert e's
// padded token segment [poff[e], poff[e+1]) (offsets = poff) of the transposed images of
// quant_t_fp8_seg (row stride ld, per-row E8M0 scales [rows, ld/128] for BOTH operands);
// grid = E x M-tiles x N-tiles; fp32 or bf16 output straight from the fragments.
template <int BM, int BN, int WGM, int WGN, bool BLK, bool WG = false>
__global__ __launch_bounds__(64 * WGM * WGN) void grouped_gemm_fp8_kernel(
    const uint8_t* __restrict__ A, const void* __restrict__ sa_, const uint8_t* __restrict__ B,
    const void* __restrict__ sb_, bf16* __restrict__ C, const int* __restrict__ offsets, int E, int N, int K,
    long strideB, int Mw, long ld, int accumulate, int out_f32) {
  const float* sa = static_cast<const float*>(sa_);
  const float* sb = static_cast<const float*>(sb_);
  const uint8_t* sa8 = static_cast<const uint8_t*>(sa_);
  const uint8_t* sb8 = static_cast<const uint8_t*>(sb_);
  constexpr int BK = 128;                                  // bytes (= fp8 elements) per k-step
  constexpr int NT = 64 * WGM * WGN;
  constexpr int TM = BM / WGM, TN = BN / WGN, IM = TM / 32, IN = TN / 32;
  constexpr int AB = BM * BK, BB = BN * BK;                // bytes per stage
  constexpr int CA = AB / 16 / NT, CB = BB / 16 / NT;
  static_assert(CA * 16 * NT == AB && CB * 16 * NT == BB, "tile/threads mismatch");
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * (AB + BB)];
  __shared__ uint8_t scl[2][BM + BN];                      // BLK: E8M0 scales of the staged k-tile
  __shared__ int s_e, s_mt;
  __shared__ int wsum[NT / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int nnt = (N + BN - 1) / BN;
  int lid = xcd_remap(blockIdx.x, gridDim.x);
  int nt = lid % nnt;
  int mt = lid / nnt;
  if (WG) {
    const int mtn = (Mw + BM - 1) / BM;
    if (tid == 0) { s_e = mt / mtn; s_mt = mt % mtn; }
    __syncthreads();
  } else {  // tile -> expert (block scan of per-expert tile counts; thread e owns expert e)
    const int cnt = tid < E ? offsets[tid + 1] - offsets[tid] : 0;
    const int tiles = (cnt + BM - 1) / BM;
    int inc = tiles;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(inc, o, 64);
      if (lane >= o) inc += v;
    }
    if (lane == 63) wsum[wave] = inc;
    if (tid == 0) s_e = -1;
    __syncthreads();
    int pre = inc - tiles, rows = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
      const int v = wsum[w];
      pre += w < wave ? v : 0;
      rows += v;
    }
    // real tiles on the lowest block ids, XCD remap over them only (see gemm8.hip)
    const int R = rows * nnt;
    if ((int)blockIdx.x >= R) return;
    lid = xcd_remap(blockIdx.x, R);
    nt = lid % nnt;
    mt = lid / nnt;
    if (tid < E && tiles > 0 && mt >= pre && mt < pre + tiles) { s_e = tid; s_mt = mt - pre; }
    __syncthreads();
  }
  const int e = s_e;
  if (e < 0 || e >= E) return;
  mt = s_mt;
  // WG: rows m of A run over [0, Mw); the k (token) range is the expert's padded segment
  const int m0 = WG ? mt * BM : offsets[e] + mt * BM, mend = WG ? Mw : offsets[e + 1];
  const int n0 = nt * BN;
  const long kbeg = WG ? offsets[e] : 0, kstop = WG ? offsets[e + 1] : K;
  SPA_DBG_ASSERT(m0 < mend && kbeg <= kstop, m0, mend);   // debug build: a live tile of expert e
  const long lda = WG ? ld : K;
  const uint8_t* Bp = WG ? B : B + e * strideB;
  uint4 ra[CA], rb[CB];
  int rs = 127;                                             // BLK: this thread's staged scale byte
  const int KB = WG ? (int)(ld / 128) : K / 128, NB = (N + 127) / 128;
  auto load_tiles = [&](long kk) {
    if (BLK) {
      const int kb = (int)(kk / 128);
      if (tid < BM) rs = (m0 + tid < mend) ? sa8[(long)(m0 + tid) * KB + kb] : 127;
      else if (WG) {
        const int gn = n0 + (tid - BM);
        rs = (tid < BM + BN && gn < N) ? sb8[(long)gn * KB + kb] : 127;
      } else if (tid < BM + BN / 128) {
        const int nb = n0 / 128 + (tid - BM);
        rs = nb < NB ? sb8[((long)e * NB + nb) * KB + kb] : 127;
      }
    }
#pragma unroll
    for (int c = 0; c < CA; ++c) {
      const int idx = tid + c * NT, r = idx >> 3, ch = idx & 7;
      const long gm = m0 + r, gk = kk + 16 * ch;
      ra[c] = (gm < mend && gk < kstop) ? *reinterpret_cast<const uint4*>(A + gm * lda + gk) : uint4{0, 0, 0, 0};
    }
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      const int idx = tid + c * NT, r = idx >> 3, ch = idx & 7;
      const long gn = n0 + r, gk = kk + 16 * ch;
      rb[c] = (gn < N && gk < kstop) ? *reinterpret_cast<const uint4*>(Bp + gn * (WG ? ld : (long)K) + gk)
                                     : uint4{0, 0, 0, 0};
    }
  };
  auto store_tiles = [&](int buf) {
    if (BLK && tid < BM + (WG ? BN : BN / 128)) scl[buf][tid] = (uint8_t)rs;
    uint8_t* At = smem + buf * (AB + BB);
    uint8_t* Bt = At + AB;
#pragma unroll
    for (int c = 0; c < CA; ++c) {
      const int idx = tid + c * NT;
      *reinterpret_cast<uint4*>(At + f8_off(idx >> 3, idx & 7)) = ra[c];
    }
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      const int idx = tid + c * NT;
      *reinterpret_cast<uint4*>(Bt + f8_off(idx >> 3, idx & 7)) = rb[c];
    }
  };
  auto frag = [&](const uint8_t* t, int row, int s, int hh) {
    const uint4 a = *reinterpret_cast<const uint4*>(t + f8_off(row, 4 * s + 2 * hh));
    const uint4 b = *reinterpret_cast<const uint4*>(t + f8_off(row, 4 * s + 2 * hh + 1));
    i32x8 v;
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    return v;
  };
  f32x16 acc[IN][IM];
#pragma unroll
  for (int i = 0; i < IN; ++i)
#pragma unroll
    for (int j = 0; j < IM; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int kt = (int)((kstop - kbeg + BK - 1) / BK);
  const int l32 = lane & 31, hh = lane >> 5;
  if (kt > 0) {
    load_tiles(kbeg);
    store_tiles(0);
    if (kt > 1) load_tiles(kbeg + BK);
  }
  __syncthreads();
  for (int t = 0; t < kt; ++t) {
    const int buf = t & 1;
    if (t + 1 < kt) {
      store_tiles(buf ^ 1);
      if (t + 2 < kt) load_tiles(kbeg + (long)(t + 2) * BK);
    }
    const uint8_t* At = smem + buf * (AB + BB);
    const uint8_t* Bt = At + AB;
#pragma unroll
    for (int s = 0; s < BK / 64; ++s) {
      i32x8 af[IM], bfr[IN];
#pragma unroll
      for (int j = 0; j < IM; ++j) af[j] = frag(At, wm * TM + j * 32 + l32, s, hh);
#pragma unroll
      for (int i = 0; i < IN; ++i) bfr[i] = frag(Bt, wn * TN + i * 32 + l32, s, hh);
      int sca[IM], scb[IN];
#pragma unroll
      for (int j = 0; j < IM; ++j) sca[j] = BLK ? (int)scl[buf][wm * TM + j * 32 + l32] : 127;
#pragma unroll
      for (int i = 0; i < IN; ++i)
        scb[i] = !BLK ? 127 : WG ? (int)scl[buf][BM + wn * TN + i * 32 + l32] : (int)scl[buf][BM + (wn * TN) / 128];
#pragma unroll
      for (int i = 0; i < IN; ++i)
#pragma unroll
        for (int j = 0; j < IM; ++j)   // e4m3 x e4m3; MX scales: weight block (A), token tile (B)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(bfr[i], af[j], acc[i][j], 0, 0, 0, scb[i], 0,
                                                                      sca[j]);
    }
    __syncthreads();
  }
  if constexpr (WG) {
    // C_e [Mw, N]: lane holds rows m = wm*TM + 32j + l32, columns n = wn*TN + 32i + 8g + 4hh + q
    const long cbase = (long)e * Mw * N;
#pragma unroll
    for (int j = 0; j < IM; ++j) {
      const long gm = m0 + wm * TM + j * 32 + l32;
      if (gm >= mend) continue;
#pragma unroll
      for (int i = 0; i < IN; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int gn = n0 + wn * TN + i * 32 + 8 * g + 4 * hh;
          if (gn >= N) continue;
          f32x4 v{acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
          if (out_f32) {
            float* cp = reinterpret_cast<float*>(C) + cbase + gm * N + gn;
            if (accumulate) v += *reinterpret_cast<const f32x4*>(cp);
            *reinterpret_cast<f32x4*>(cp) = v;
          } else {
            bf16* cp = C + cbase + gm * N + gn;
            bf16x4 w4;
            if (accumulate) {
              const bf16x4 o = *reinterpret_cast<const bf16x4*>(cp);
#pragma unroll
              for (int q = 0; q < 4; ++q) v[q] += (float)o[q];
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) w4[q] = (bf16)v[q];
            *reinterpret_cast<bf16x4*>(cp) = w4;
          }
        }
    }
    return;
  }
  // epilogue through LDS, one 128-token half (= the waves with wm == half) at a time: C^T
  // fragments (lane = token m, rows n = 8g + 4hh + {0..3}) -> padded [m][n] bf16 image ->
  // whole-row 16-byte global stores
  static_assert(BM == 256 && BN == 256 && WGM == 2, "fp8 epilogue: 256 x 256 tile, 2 wave rows");
  constexpr int RS = BN * 2 + 16;
  __syncthreads();
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    if (wm == half) {
#pragma unroll
      for (int j = 0; j < IM; ++j) {
        const int rm = j * 32 + l32;
        const int gm = m0 + wm * TM + rm;
        const float sm = (BLK || gm >= mend) ? 1.f : sa[gm];
#pragma unroll
        for (int i = 0; i < IN; ++i)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int cn = wn * TN + i * 32 + 8 * g + 4 * hh;
            const int gn = n0 + cn;
            const f32x4 sw = (BLK || gn >= N) ? f32x4{1.f, 1.f, 1.f, 1.f}
                                               : *reinterpret_cast<const f32x4*>(sb + (long)e * N + gn);
            bf16x4 w4;
#pragma unroll
            for (int q = 0; q < 4; ++q) w4[q] = (bf16)(acc[i][j][4 * g + q] * sm * sw[q]);
            *reinterpret_cast<bf16x4*>(smem + rm * RS + cn * 2) = w4;
          }
      }
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 128 * (BN / 8) / NT; ++c) {
      const int idx = tid + c * NT, r = idx / (BN / 8), ch = idx % (BN / 8);
      const int gm = m0 + half * 128 + r, gn = n0 + ch * 8;
      if (gm < mend && gn < N)
        *reinterpret_cast<uint4*>(C + (long)gm * N + gn) = *reinterpret_cast<const uint4*>(smem + r * RS + ch * 16);
    }
    __syncthreads();
  }
}

// --------------------------------------------------------------------------- host
std::vector<at::Tensor> quant_rows_fp8(const at::Tensor& x_) {
  SPA_CHECK_CUDA(x_);
  auto x = x_.contiguous();
  TORCH_CHECK(x.scalar_type() == at::kBFloat16, "quant_rows_fp8: bf16 input");
  const int K = x.size(-1);
  const int R = x.numel() / std::max(K, 1);
  TORCH_CHECK(K % 8 == 0, "quant_rows_fp8: K % 8 == 0");
  DeviceGuard g(x.device());
  auto q = at::empty(x.sizes(), x.options().dtype(at::kFloat8_e4m3fn));
  auto s = at::empty({R}, x.options().dtype(at::kFloat));
  if (R == 0) return {q, s};
  quant_rows_fp8_kernel<<<cdiv(R, 4), 256, 0, stream()>>>((const bf16*)x.data_ptr(), (uint8_t*)q.data_ptr(),
                                                         s.data_ptr<float>(), R, K);
  SPA_LAUNCH_CHECK();
  return {q, s};
}

// xq [M, K] e4m3 (rows grouped by offsets), sx [M]; wq [E, N, K] e4m3, sw [E, N] -> y [M, N] bf16
at::Tensor grouped_gemm_fp8(const at::Tensor& xq, const at::Tensor& sx, const at::Tensor& wq, const at::Tensor& sw,
                            const at::Tensor& offsets) {
  TORCH_CHECK(xq.scalar_type() == at::kFloat8_e4m3fn && wq.scalar_type() == at::kFloat8_e4m3fn, "e4m3 operands");
  TORCH_CHECK(xq.is_contiguous() && wq.is_contiguous() && sx.is_contiguous() && sw.is_contiguous());
  TORCH_CHECK(offsets.scalar_type() == at::kInt);
  const int E = offsets.numel() - 1;
  TORCH_CHECK(E >= 1 && E <= 256 && wq.dim() == 3 && wq.size(0) == E);
  const int M = xq.size(0), K = xq.size(1), N = wq.size(1);
  TORCH_CHECK(wq.size(2) == K && K % 16 == 0 && N % 8 == 0, "grouped_gemm_fp8: K % 16, N % 8");
  TORCH_CHECK(sx.numel() == M && sw.numel() == (long)E * N);
  DeviceGuard g(xq.device());
  auto out = at::empty({M, N}, xq.options().dtype(at::kBFloat16));
  if (M == 0) return out;
  constexpr int BM = 256, BN = 256;
  const int grid = (cdiv(M, BM) + E) * cdiv(N, BN);
  grouped_gemm_fp8_kernel<BM, BN, 2, 4, false><<<grid, 512, 0, stream()>>>(
      (const uint8_t*)xq.data_ptr(), sx.data_ptr<float>(), (const uint8_t*)wq.data_ptr(), sw.data_ptr<float>(),
      (bf16*)out.data_ptr(), offsets.data_ptr<int>(), E, N, K, (long)N * K, 0, 0, 0, 0);
  SPA_LAUNCH_CHECK();
  return out;
}

// block-scaled: xq [M, K] e4m3 + sx [M, K/128] E8M0 (uint8); wq [E, N, K] e4m3 + sw [E, N/128, K/128]
std::vector<at::Tensor> quant_act_fp8_blk(const at::Tensor& x_) {
  SPA_CHECK_CUDA(x_);
  auto x = x_.contiguous();
  TORCH_CHECK(x.scalar_type() == at::kBFloat16, "quant_act_fp8_blk: bf16 input");
  const int K = x.size(-1);
  TORCH_CHECK(K % 128 == 0, "quant_act_fp8_blk: K % 128 == 0");
  const long R = x.numel() / K;
  DeviceGuard g(x.device());
  auto q = at::empty(x.sizes(), x.options().dtype(at::kFloat8_e4m3fn));
  auto s = at::empty({R, K / 128}, x.options().dtype(at::kByte));
  const long units = R * (K / 128);
  if (units == 0) return {q, s};
  quant_act_blk_kernel<<<(int)((units * 16 + 255) / 256), 256, 0, stream()>>>(
      (const bf16*)x.data_ptr(), (uint8_t*)q.data_ptr(), s.data_ptr<uint8_t>(), units, K / 128);
  SPA_LAUNCH_CHECK();
  return {q, s};
}

// returns (wq [E,N,K], wtq [E,K,N], s [E,N/128,K/128], st [E,K/128,N/128])
std::vector<at::Tensor> quant_weight_fp8_blk(const at::Tensor& w_) {
  SPA_CHECK_CUDA(w_);
  auto w = w_.contiguous();
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.dim() == 3, "quant_weight_fp8_blk: bf16 [E, N, K]");
  const int E = w.size(0), N = w.size(1), K = w.size(2);
  TORCH_CHECK(N % 128 == 0 && K % 128 == 0, "quant_weight_fp8_blk: N, K % 128 == 0");
  DeviceGuard g(w.device());
  auto o8 = w.options().dtype(at::kFloat8_e4m3fn);
  auto wq = at::empty({E, N, K}, o8), wtq = at::empty({E, K, N}, o8);
  auto s = at::empty({E, N / 128, K / 128}, w.options().dtype(at::kByte));
  auto st = at::empty({E, K / 128, N / 128}, w.options().dtype(at::kByte));
  const long blocks = (long)E * (N / 128) * (K / 128);
  if (blocks == 0) return {wq, wtq, s, st};
  quant_weight_blk_kernel<<<(int)blocks, 256, 0, stream()>>>((const bf16*)w.data_ptr(), (uint8_t*)wq.data_ptr(),
                                                             (uint8_t*)wtq.data_ptr(), s.data_ptr<uint8_t>(),
                                                             st.data_ptr<uint8_t>(), N, K);
  SPA_LAUNCH_CHECK();
  return {wq, wtq, s, st};
}

// (q [R, K] e4m3, s [R, >= K/128] E8M0 rows) -> bf16 [R, K]
at::Tensor dequant_act_fp8_blk(const at::Tensor& q, const at::Tensor& s) {
  SPA_CHECK_CUDA(q);
  TORCH_CHECK(q.is_contiguous() && s.is_contiguous() && s.scalar_type() == at::kByte && q.dim() == 2 && s.dim() == 2);
  const long R = q.size(0);
  const int K = q.size(1), ldS = s.size(1);
  TORCH_CHECK(K % 128 == 0 && s.size(0) == R && ldS >= K / 128, "dequant_act_fp8_blk: shapes");
  DeviceGuard g(q.device());
  auto y = at::empty({R, K}, q.options().dtype(at::kBFloat16));
  const long n8 = R * K / 8;
  if (n8 == 0) return y;
  dequant_act_blk_kernel<<<(int)std::min<long>((n8 + 255) / 256, 16384), 256, 0, stream()>>>(
      (const uint8_t*)q.data_ptr(), s.data_ptr<uint8_t>(), (bf16*)y.data_ptr(), n8, K, ldS);
  SPA_LAUNCH_CHECK();
  return y;
}

at::Tensor grouped_gemm_fp8_blk(const at::Tensor& xq, const at::Tensor& sx, const at::Tensor& wq, const at::Tensor& sw,
                                const at::Tensor& offsets) {
  TORCH_CHECK(xq.scalar_type() == at::kFloat8_e4m3fn && wq.scalar_type() == at::kFloat8_e4m3fn, "e4m3 operands");
  TORCH_CHECK(sx.scalar_type() == at::kByte && sw.scalar_type() == at::kByte, "E8M0 (uint8) scales");
  TORCH_CHECK(xq.is_contiguous() && wq.is_contiguous() && sx.is_contiguous() && sw.is_contiguous());
  TORCH_CHECK(offsets.scalar_type() == at::kInt);
  const int E = offsets.numel() - 1;
  TORCH_CHECK(E >= 1 && E <= 256 && wq.dim() == 3 && wq.size(0) == E);
  const int M = xq.size(0), K = xq.size(1), N = wq.size(1);
  TORCH_CHECK(wq.size(2) == K && K % 128 == 0 && N % 8 == 0, "grouped_gemm_fp8_blk: K % 128, N % 8");
  TORCH_CHECK(sx.numel() == (long)M * (K / 128) && sw.numel() == (long)E * ((N + 127) / 128) * (K / 128),
              "grouped_gemm_fp8_blk: scale shapes");
  DeviceGuard g(xq.device());
  auto out = at::empty({M, N}, xq.options().dtype(at::kBFloat16));
  if (M == 0) return out;
  constexpr int BM = 256, BN = 256;
  const int grid = (cdiv(M, BM) + E) * cdiv(N, BN);
  grouped_gemm_fp8_kernel<BM, BN, 2, 4, true><<<grid, 512, 0, stream()>>>(
      (const uint8_t*)xq.data_ptr(), sx.data_ptr<uint8_t>(), (const uint8_t*)wq.data_ptr(), sw.data_ptr<uint8_t>(),
      (bf16*)out.data_ptr(), offsets.data_ptr<int>(), E, N, K, (long)N * K, 0, 0, 0, 0);
  SPA_LAUNCH_CHECK();
  return out;
}

// x [T, C] bf16 (rows grouped by offsets [E+1]), poff [E+1] (128-aligned padded segment starts,
// poff[E] <= ldq) -> (qt [C, ldq] e4m3, st [C, ldq/128] E8M0): transposed Wgrad operand; with
// ``rows``, also (qr [T, C] e4m3, sr [T, C/128]) = quant_act_fp8_blk(x) from the same read
std::vector<at::Tensor> quant_t_fp8_seg(const at::Tensor& x_, const at::Tensor& offsets, const at::Tensor& poff,
                                        int64_t ldq, bool rows) {
  SPA_CHECK_CUDA(x_);
  auto x = x_.contiguous();
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() == 2, "quant_t_fp8_seg: bf16 [T, C]");
  TORCH_CHECK(offsets.scalar_type() == at::kInt && poff.scalar_type() == at::kInt && offsets.numel() == poff.numel(),
              "quant_t_fp8_seg: int32 offsets / padded offsets [E+1]");
  const long T = x.size(0);
  const int C = x.size(1), E = offsets.numel() - 1;
  TORCH_CHECK(C % 128 == 0 && ldq % 128 == 0 && ldq >= T, "quant_t_fp8_seg: C % 128, ldq % 128");
  DeviceGuard g(x.device());
  auto o8 = x.options().dtype(at::kFloat8_e4m3fn);
  auto q = at::empty({C, ldq}, o8);
  auto s = at::empty({C, ldq / 128}, x.options().dtype(at::kByte));
  at::Tensor qr, sr;
  if (rows) {
    qr = at::empty({T, C}, o8);
    sr = at::empty({T, C / 128}, x.options().dtype(at::kByte));
  }
  if (ldq > 0 && C > 0) {
    quant_t_fp8_seg_kernel<<<dim3((unsigned)(ldq / 128), C / 128), 256, 0, stream()>>>(
        (const bf16*)x.data_ptr(), offsets.data_ptr<int>(), poff.data_ptr<int>(), E, C, (uint8_t*)q.data_ptr(),
        s.data_ptr<uint8_t>(), ldq, rows ? (uint8_t*)qr.data_ptr() : nullptr, rows ? sr.data_ptr<uint8_t>() : nullptr);
    SPA_LAUNCH_CHECK();
  }
  if (rows) return {q, s, qr, sr};
  return {q, s};
}

// dW_e [M, N] (+)= aq[:, seg_e] bq[:, seg_e]^T for the quant_t_fp8_seg images aq [M, ld], bq [N, ld]
// (scales [rows, ld/128]); out [E, M, N] bf16 or fp32 (a main_grad view), new bf16 if absent
at::Tensor wgrad_fp8_blk(const at::Tensor& aq, const at::Tensor& sa, const at::Tensor& bq, const at::Tensor& sb,
                         const at::Tensor& poff, const c10::optional<at::Tensor>& out_, bool accumulate) {
  TORCH_CHECK(aq.scalar_type() == at::kFloat8_e4m3fn && bq.scalar_type() == at::kFloat8_e4m3fn, "e4m3 operands");
  TORCH_CHECK(sa.scalar_type() == at::kByte && sb.scalar_type() == at::kByte, "E8M0 (uint8) scales");
  TORCH_CHECK(aq.is_contiguous() && bq.is_contiguous() && sa.is_contiguous() && sb.is_contiguous());
  TORCH_CHECK(poff.scalar_type() == at::kInt, "wgrad_fp8_blk: int32 padded offsets");
  const int E = poff.numel() - 1;
  const int M = aq.size(0), N = bq.size(0);
  const long ld = aq.size(1);
  TORCH_CHECK(bq.size(1) == ld && ld % 128 == 0 && N % 8 == 0, "wgrad_fp8_blk: shapes");
  TORCH_CHECK(sa.size(0) == M && sb.size(0) == N && sa.size(1) == ld / 128 && sb.size(1) == ld / 128,
              "wgrad_fp8_blk: scale shapes");
  DeviceGuard g(aq.device());
  auto out = out_ ? *out_ : at::empty({E, M, N}, aq.options().dtype(at::kBFloat16));
  TORCH_CHECK(out.is_contiguous() && out.numel() == (long)E * M * N &&
                  (out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat),
              "wgrad_fp8_blk: out [E, M, N] bf16/fp32 contiguous");
  if (E == 0 || M == 0 || N == 0) return out;
  constexpr int BM = 256, BN = 256;
  const int grid = E * cdiv(M, BM) * cdiv(N, BN);
  grouped_gemm_fp8_kernel<BM, BN, 2, 4, true, true><<<grid, 512, 0, stream()>>>(
      (const uint8_t*)aq.data_ptr(), sa.data_ptr<uint8_t>(), (const uint8_t*)bq.data_ptr(), sb.data_ptr<uint8_t>(),
      (bf16*)out.data_ptr(), poff.data_ptr<int>(), E, N, 0, 0, M, ld, accumulate ? 1 : 0,
      out.scalar_type() == at::kFloat ? 1 : 0);
  SPA_LAUNCH_CHECK();
  return out;
}

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.def("quant_rows_fp8(Tensor x) -> Tensor[]");
  m.def("grouped_gemm_fp8(Tensor xq, Tensor sx, Tensor wq, Tensor sw, Tensor offsets) -> Tensor");
  m.def("quant_act_fp8_blk(Tensor x) -> Tensor[]");
  m.def("dequant_act_fp8_blk(Tensor q, Tensor s) -> Tensor");
  m.def("quant_weight_fp8_blk(Tensor w) -> Tensor[]");
  m.def("grouped_gemm_fp8_blk(Tensor xq, Tensor sx, Tensor wq, Tensor sw, Tensor offsets) -> Tensor");
  m.def("quant_t_fp8_seg(Tensor x, Tensor offsets, Tensor poff, int ldq, bool rows) -> Tensor[]");
  m.def("wgrad_fp8_blk(Tensor aq, Tensor sa, Tensor bq, Tensor sb, Tensor poff, Tensor(a!)? out, bool accumulate) -> Tensor");
}
TORCH_LIBRARY_IMPL(spa, CUDA, m) {
  m.impl("quant_rows_fp8", &spa::quant_rows_fp8);
  m.impl("grouped_gemm_fp8", &spa::grouped_gemm_fp8);
  m.impl("quant_act_fp8_blk", &spa::quant_act_fp8_blk);
  m.impl("dequant_act_fp8_blk", &spa::dequant_act_fp8_blk);
  m.impl("quant_weight_fp8_blk", &spa::quant_weight_fp8_blk);
  m.impl("grouped_gemm_fp8_blk", &spa::grouped_gemm_fp8_blk);
  m.impl("quant_t_fp8_seg", &spa::quant_t_fp8_seg);
  m.impl("wgrad_fp8_blk", &spa::wgrad_fp8_blk);
}
