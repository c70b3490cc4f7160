// Mixture-of-Experts kernels for gfx950: router top-k, deterministic token permute,
// row gather / weighted combine, and an MFMA grouped GEMM (fwd, dX, dW) whose
// per-expert row counts live on the device (no host sync, no per-expert launches).
//
// Reference: deepseekv3/deepseekv3.ipynb:1014-1088 (MoeLayer): gate GEMM -> +routing_bias
// -> topk(2) -> softmax over the masked (top-k only) logits -> shared expert + Python
// loop over 8 experts with boolean gathers, a host sync per expert (`mask.any()`) and
// masked_scatter_; aux-free bias update sign(mean - load). Here the loop becomes:
//   moe_route      one wave per token: top-k (register insertion sort) + renormalised
//                  softmax over the selected logits (+ optional bias in the weights);
//   moe_permute    per-expert stable counting sort -> perm / inverse / offsets [E+1];
//   gather_rows    x_perm[i] = x[perm[i] / k]  (16-byte vectors);
//   grouped_gemm   Y_e = X_e W_e^T  and its two backward products, one launch each;
//   combine        y[n] = sum_j w[n,j] * y_perm[inv[n,j]]  (gather form: deterministic).
#include "spa_common.h"
#include "gemm_common.h"

SPA_DEBUG_TU("moe.hip")

namespace spa {

// --------------------------------------------------------------------------- router
// logits [N, E] fp32; bias [E] (may be null). Outputs idx [N, k] int32 (descending score),
// w [N, k] fp32 = softmax over the k selected values of (logits + bias if bias_in_w else logits).
template <int MAXK>
__global__ __launch_bounds__(256) void moe_route_kernel(const float* __restrict__ logits, const float* __restrict__ bias,
                                                        int* __restrict__ idx, float* __restrict__ w, int N, int E,
                                                        int k, int bias_in_w) {
  const int tok = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (tok >= N) return;
  const float* lg = logits + (long)tok * E;
  // each lane keeps its best candidates; merge k times with wave argmax
  float sel_v[MAXK];
  int sel_i[MAXK];
  float prev = INFINITY;
  int prev_i = -1;
  for (int j = 0; j < k; ++j) {
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int e = lane; e < E; e += 64) {
      const float v = lg[e] + (bias ? bias[e] : 0.f);
      // strictly below the previous pick (ties broken by lower index first)
      const bool ok = (v < prev) || (v == prev && e > prev_i);
      if (ok && (v > best || (v == best && e < bi))) { best = v; bi = e; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
    }
    sel_v[j] = best;
    sel_i[j] = bi;
    prev = best;
    prev_i = bi;
  }
  if (lane == 0) {
    float m = -INFINITY;
    for (int j = 0; j < k; ++j) {
      const float v = bias_in_w ? sel_v[j] : lg[sel_i[j]];
      sel_v[j] = v;
      m = fmaxf(m, v);
    }
    float z = 0.f;
    for (int j = 0; j < k; ++j) z += __expf(sel_v[j] - m);
    for (int j = 0; j < k; ++j) {
      idx[(long)tok * k + j] = sel_i[j];
      w[(long)tok * k + j] = __expf(sel_v[j] - m) / z;
    }
  }
}

// --------------------------------------------------------------------------- permute
// Block per expert: stable order of assignments a = n*k + j with idx[a] == e.
// perm[off_e + r] = a ; inv[a] = off_e + r. counts computed by a first pass kernel.
__global__ __launch_bounds__(256) void moe_count_kernel(const int* __restrict__ idx, int A, int E,
                                                        int* __restrict__ counts) {
  const int e = blockIdx.x;
  __shared__ int red[4];
  int c = 0;
  for (int a = threadIdx.x; a < A; a += 256) c += idx[a] == e;
  c = (int)block_sum<256>((float)c, (float*)red);
  if (threadIdx.x == 0) counts[e] = c;
}
__global__ void moe_offsets_kernel(const int* __restrict__ counts, int E, int* __restrict__ offsets) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    int s = 0;
    for (int e = 0; e < E; ++e) { offsets[e] = s; s += counts[e]; }
    offsets[E] = s;
  }
}
__global__ __launch_bounds__(256) void moe_scatter_kernel(const int* __restrict__ idx, int A,
                                                          const int* __restrict__ offsets, int* __restrict__ perm,
                                                          int* __restrict__ inv) {
  const int e = blockIdx.x;
  __shared__ int wcount[4];
  int base = offsets[e];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int a0 = 0; a0 < A; a0 += 256) {
    const int a = a0 + threadIdx.x;
    const bool hit = a < A && idx[a] == e;
    const unsigned long long bal = __ballot(hit);
    const int before = __popcll(bal & ((1ULL << lane) - 1ULL));
    if (lane == 0) wcount[wv] = __popcll(bal);
    __syncthreads();
    int woff = 0;
    for (int i = 0; i < wv; ++i) woff += wcount[i];
    const int tot = wcount[0] + wcount[1] + wcount[2] + wcount[3];
    if (hit) {
      const int pos = base + woff + before;
      perm[pos] = a;
      inv[a] = pos;
    }
    base += tot;
    __syncthreads();
  }
}

// --------------------------------------------------------------------------- gather / combine
// rows are moved as 16-byte units (bf16 or fp32 rows alike): nv = row_bytes / 16
__global__ __launch_bounds__(256) void gather_rows_kernel(const uint4* __restrict__ x, const int* __restrict__ perm,
                                                          uint4* __restrict__ out, int rows, int nv, int div,
                                                          long x_rows) {
  const long total = (long)rows * nv;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long r = i / nv;
    const int c = i % nv;
    const int src = perm[r];
    if (src < 0) {            // no source row (EP capacity maps: an empty block slot): zeros
      out[r * nv + c] = make_uint4(0u, 0u, 0u, 0u);
      continue;
    }
    if (!SPA_DBG_OK(src / div, x_rows)) continue;   // debug build: a routed row of x
    out[r * nv + c] = x[(long)(src / div) * nv + c];
  }
}
// y[n] = sum_j w[n, j] * yp[inv[n*k + j]]; also usable for the dX of the gather (w = 1)
template <typename T>
__global__ __launch_bounds__(256) void combine_kernel(const T* __restrict__ yp, const int* __restrict__ inv,
                                                      const float* __restrict__ w, T* __restrict__ y, int N, int D,
                                                      int k, long yrows) {
  const int dv = D / 8;
  const long total = (long)N * dv;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long n = i / dv;
    const int c = (i % dv) * 8;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < k; ++j) {
      const float wj = w ? w[n * k + j] : 1.f;
      if (!SPA_DBG_OK(inv[n * k + j], yrows)) continue;   // debug build: a row of yp
      float v[8];
      load8(yp + (long)inv[n * k + j] * D + c, v);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += wj * v[q];
    }
    store8(y + n * D + c, acc);
  }
}
// dw[n, j] = <dy[n], yp[inv[n*k+j]]>  (gradient of the combine weights), one wave per (n, j)
template <typename T>
__global__ __launch_bounds__(256) void combine_dw_kernel(const T* __restrict__ dy, const T* __restrict__ yp,
                                                         const int* __restrict__ inv, float* __restrict__ dw, int N,
                                                         int D, int k) {
  const int a = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (a >= N * k) return;
  const long n = a / k;
  if (!SPA_DBG_OK(inv[a], N * k)) return;   // debug build: inv is a permutation of the assignments
  const T* yr = yp + (long)inv[a] * D;
  const T* dr = dy + n * D;
  float acc = 0.f;
  for (int c = lane * 8; c < D; c += 512) {
    float u[8], v[8];
    load8(dr + c, u);
    load8(yr + c, v);
#pragma unroll
    for (int q = 0; q < 8; ++q) acc += u[q] * v[q];
  }
  acc = wave_sum(acc);
  if (lane == 0) dw[a] = acc;
}
// rows of yp scaled by per-assignment weight: out[i] = w[perm[i]] * g[perm[i]/k] (dY_perm of the combine)
template <typename T>
__global__ __launch_bounds__(256) void scatter_grad_kernel(const T* __restrict__ g, const int* __restrict__ perm,
                                                           const float* __restrict__ w, T* __restrict__ out, int rows,
                                                           int D, int k) {
  const int dv = D / 8;
  const long total = (long)rows * dv;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long r = i / dv;
    const int c = (i % dv) * 8;
    const int a = perm[r];
    if (!SPA_DBG_OK(a, rows)) continue;   // debug build: perm is a permutation of the assignments
    const float wa = w[a];
    float v[8];
    load8(g + (long)(a / k) * D + c, v);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] *= wa;
    store8(out + r * D + c, v);
  }
}

// --------------------------------------------------------------------------- grouped GEMM
// C (M x N, row-major, ldc) = A (M x K) * B (K x N), grouped by expert. Operand storage:
//   A_KC: A stored [M][K] (lda) else [K][M];  B_KC: B stored [N][K] (ldb) else [K][N].
// GROUP_K = false: groups split M (rows of A and C): expert e owns rows [off_e, off_e+1),
//                  B_e = B + e * strideB.   (fwd:  X_e W_e^T ; dX: dY_e W_e)
// GROUP_K = true : groups split K (the token dim): C_e = C + e * strideC, reduction over
//                  rows [off_e, off_e+1) of the token-major A and B. (dW_e = dY_e^T X_e)
// Block tile BM x BN x BK, WGM x WGN waves (wave tile TM x TN of 32x32 MFMA sub-tiles,
// v_mfma_f32_32x32x16_bf16); each wave computes C^T so the epilogue writes 4 consecutive
// columns (8 bytes) per lane. Register-staged double-buffered LDS, one barrier per k-step.
// LDS images: K-contiguous tiles [rows][BK] with an 8-byte-unit XOR swizzle
// (u ^ (r / P) where P rows span the 64 banks); K-strided tiles [BK][cols] read with
// ds_read_b64_tr_b16 through the attention image swizzle. Zero bank conflicts by design.
// Tile -> expert: per-block scan of the per-expert tile counts (E <= threads), so launch
// count and grid are independent of the routing (no host sync); logical tile ids are
// XCD-remapped so tiles sharing an A panel run on one XCD's L2.
template <int BM, int BN, int BK, int WGM, int WGN, bool A_KC, bool B_KC, bool GROUP_K>
__global__ __launch_bounds__(64 * WGM * WGN, (BM * BN / (WGM * WGN) <= 8192 && WGM * WGN == 4) ? 2 : 1)
void grouped_gemm_kernel(
    const bf16* __restrict__ A, const bf16* __restrict__ B, bf16* __restrict__ C, const int* __restrict__ offsets,
    int E, int M, int N, int K, long lda, long ldb, long ldc, long strideB, long strideC, int accumulate) {
  constexpr int NT = 64 * WGM * WGN;
  constexpr int TM = BM / WGM, TN = BN / WGN;         // wave tile (m, n)
  constexpr int IM = TM / 32, IN = TN / 32;
  constexpr int AEL = BM * BK, BEL = BN * BK;          // elements per stage
  constexpr int CA = AEL / 8 / NT, CB = BEL / 8 / NT;  // 16B chunks per thread
  static_assert(CA * 8 * NT == AEL && CB * 8 * NT == BEL, "tile/threads mismatch");
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * (AEL + BEL)];
  __shared__ int s_e, s_mt;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int nnt = (N + BN - 1) / BN;
  int lid = xcd_remap(blockIdx.x, gridDim.x);
  int nt = lid % nnt;
  int mt = lid / nnt;
  int e = 0, m0 = 0, mend = M, k0 = 0, kend = K;
  const bf16* Bp = B;
  bf16* Cp = C;
  if (!GROUP_K) {
    // block-wide exclusive scan of per-expert tile counts; thread e owns expert e
    __shared__ int wsum[NT / 64];
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
    e = s_e;
    if (e < 0) return;                                  // beyond the last tile
    mt = s_mt;
    m0 = offsets[e] + mt * BM;
    mend = offsets[e + 1];
    SPA_DBG_CHECK(e, E);
    SPA_DBG_ASSERT(m0 < mend && mend <= M, m0, mend);   // debug build: a live tile of expert e
    Bp = B + e * strideB;
  } else {
    const int nmt = (M + BM - 1) / BM;
    e = mt / nmt;
    mt = mt % nmt;
    if (e >= E) return;
    m0 = mt * BM;
    k0 = offsets[e];
    kend = offsets[e + 1];
    Cp = C + e * strideC;
  }
  const int n0 = nt * BN;
  bf16x8 ra[CA], rb[CB];
  auto load_tiles = [&](int kk) {
#pragma unroll
    for (int c = 0; c < CA; ++c) {
      const int idx = tid + c * NT;
      if (A_KC) {  // [BM rows][BK k]
        const int r = idx / (BK / 8), kc = (idx % (BK / 8)) * 8;
        const int gm = m0 + r, gk = kk + kc;
        ra[c] = (gm < mend && gk < kend) ? *reinterpret_cast<const bf16x8*>(A + (long)gm * lda + gk) : bf16x8{};
      } else {     // [BK k][BM m]
        const int r = idx / (BM / 8), mc = (idx % (BM / 8)) * 8;
        const int gk = kk + r, gm = m0 + mc;
        ra[c] = (gk < kend && gm < mend) ? *reinterpret_cast<const bf16x8*>(A + (long)gk * lda + gm) : bf16x8{};
      }
    }
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      const int idx = tid + c * NT;
      if (B_KC) {  // [BN n][BK k]
        const int r = idx / (BK / 8), kc = (idx % (BK / 8)) * 8;
        const int gn = n0 + r, gk = kk + kc;
        rb[c] = (gn < N && gk < kend) ? *reinterpret_cast<const bf16x8*>(Bp + (long)gn * ldb + gk) : bf16x8{};
      } else {     // [BK k][BN n]
        const int r = idx / (BN / 8), nc = (idx % (BN / 8)) * 8;
        const int gk = kk + r, gn = n0 + nc;
        rb[c] = (gk < kend && gn < N) ? *reinterpret_cast<const bf16x8*>(Bp + (long)gk * ldb + gn) : bf16x8{};
      }
    }
  };
  auto store_tiles = [&](int buf) {
    bf16* At = smem + buf * (AEL + BEL);
    bf16* Bt = At + AEL;
#pragma unroll
    for (int c = 0; c < CA; ++c) {
      const int idx = tid + c * NT;
      if (A_KC) {
        const int r = idx / (BK / 8), u = (idx % (BK / 8)) * 2;
        *reinterpret_cast<bf16x4*>(At + kc_off<BK>(r, u)) = __builtin_shufflevector(ra[c], ra[c], 0, 1, 2, 3);
        *reinterpret_cast<bf16x4*>(At + kc_off<BK>(r, u + 1)) = __builtin_shufflevector(ra[c], ra[c], 4, 5, 6, 7);
      } else {
        const int r = idx / (BM / 8), ch = idx % (BM / 8);
        *reinterpret_cast<bf16x8*>(At + ks_off<BM>(r, ch)) = ra[c];
      }
    }
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      const int idx = tid + c * NT;
      if (B_KC) {
        const int r = idx / (BK / 8), u = (idx % (BK / 8)) * 2;
        *reinterpret_cast<bf16x4*>(Bt + kc_off<BK>(r, u)) = __builtin_shufflevector(rb[c], rb[c], 0, 1, 2, 3);
        *reinterpret_cast<bf16x4*>(Bt + kc_off<BK>(r, u + 1)) = __builtin_shufflevector(rb[c], rb[c], 4, 5, 6, 7);
      } else {
        const int r = idx / (BN / 8), ch = idx % (BN / 8);
        *reinterpret_cast<bf16x8*>(Bt + ks_off<BN>(r, ch)) = rb[c];
      }
    }
  };
  f32x16 acc[IN][IM];  // [n sub-tile][m sub-tile]: C^T tiles (rows = n, cols = m)
#pragma unroll
  for (int i = 0; i < IN; ++i)
#pragma unroll
    for (int j = 0; j < IM; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int kt = (kend - k0 + BK - 1) / BK;
  const int l32 = lane & 31, hh = lane >> 5;
  if (kt > 0) {
    load_tiles(k0);
    store_tiles(0);
    if (kt > 1) load_tiles(k0 + BK);
  }
  __syncthreads();
  for (int t = 0; t < kt; ++t) {
    const int buf = t & 1;
    if (t + 1 < kt) {
      store_tiles(buf ^ 1);
      if (t + 2 < kt) load_tiles(k0 + (t + 2) * BK);
    }
    const bf16* At = smem + buf * (AEL + BEL);
    const bf16* Bt = At + AEL;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      bf16x8 af[IM], bfr[IN];
#pragma unroll
      for (int j = 0; j < IM; ++j) {
        const int mrow = wm * TM + j * 32;
        af[j] = A_KC ? ld_kc<BK>(At, mrow + l32, s, hh) : ld_ks<BM>(At, mrow, s, lane);
      }
#pragma unroll
      for (int i = 0; i < IN; ++i) {
        const int ncol = wn * TN + i * 32;
        bfr[i] = B_KC ? ld_kc<BK>(Bt, ncol + l32, s, hh) : ld_ks<BN>(Bt, ncol, s, lane);
      }
#pragma unroll
      for (int i = 0; i < IN; ++i)
#pragma unroll
        for (int j = 0; j < IM; ++j)  // C^T[n][m] += B^T-frag (rows n) x A-frag^T (cols m)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[i], af[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  // ---- epilogue: lane holds column m = l32 of each C^T tile, rows n = 8g + 4hh + {0..3}
#pragma unroll
  for (int i = 0; i < IN; ++i)
#pragma unroll
    for (int j = 0; j < IM; ++j) {
      const int gm = m0 + wm * TM + j * 32 + l32;
      if (GROUP_K ? gm >= M : gm >= mend) continue;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int gn = n0 + wn * TN + i * 32 + 8 * g + 4 * hh;
        if (gn >= N) continue;
        bf16* cp = Cp + (long)gm * ldc + gn;
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = acc[i][j][4 * g + q];
        if (accumulate) {
          const bf16x4 o = *reinterpret_cast<const bf16x4*>(cp);
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] += (float)o[q];
        }
        bf16x4 w4;
#pragma unroll
        for (int q = 0; q < 4; ++q) w4[q] = (bf16)v[q];
        *reinterpret_cast<bf16x4*>(cp) = w4;
      }
    }
}

// tile configurations: id -> (BM, BN, BK, WGM, WGN)
template <int CFG> struct GG;
template <> struct GG<0> { static constexpr int BM = 128, BN = 128, BK = 32, WGM = 2, WGN = 2; };
template <> struct GG<1> { static constexpr int BM = 128, BN = 256, BK = 32, WGM = 2, WGN = 2; };
template <> struct GG<2> { static constexpr int BM = 256, BN = 256, BK = 32, WGM = 2, WGN = 4; };
template <> struct GG<3> { static constexpr int BM = 256, BN = 256, BK = 64, WGM = 2, WGN = 2; };
template <> struct GG<4> { static constexpr int BM = 128, BN = 256, BK = 64, WGM = 2, WGN = 2; };
template <> struct GG<5> { static constexpr int BM = 256, BN = 128, BK = 32, WGM = 2, WGN = 2; };

template <int CFG, bool A_KC, bool B_KC, bool GROUP_K>
void launch_gg(int grid_m, const bf16* A, const bf16* B, bf16* C, const int* off, int E, int M, int N, int K, long lda,
               long ldb, long ldc, long sB, long sC, int acc, hipStream_t st) {
  using G = GG<CFG>;
  const int nnt = cdiv(N, G::BN);
  grouped_gemm_kernel<G::BM, G::BN, G::BK, G::WGM, G::WGN, A_KC, B_KC, GROUP_K>
      <<<grid_m * nnt, 64 * G::WGM * G::WGN, 0, st>>>(A, B, C, off, E, M, N, K, lda, ldb, ldc, sB, sC, acc);
}

template <bool A_KC, bool B_KC, bool GROUP_K>
void dispatch_gg(int cfg, int Mtot, int E, const bf16* A, const bf16* B, bf16* C, const int* off, int M, int N, int K,
                 long lda, long ldb, long ldc, long sB, long sC, int acc, hipStream_t st) {
  auto gm = [&](int BM) { return GROUP_K ? E * cdiv(M, BM) : cdiv(Mtot, BM) + E; };
  switch (cfg) {
#define GG_CASE(I) \
  case I: launch_gg<I, A_KC, B_KC, GROUP_K>(gm(GG<I>::BM), A, B, C, off, E, M, N, K, lda, ldb, ldc, sB, sC, acc, st); break;
    GG_CASE(0) GG_CASE(1) GG_CASE(2) GG_CASE(3) GG_CASE(4) GG_CASE(5)
#undef GG_CASE
    default: TORCH_CHECK(false, "grouped_gemm: unknown tile config ", cfg);
  }
}

// measured on MI355X at DeepSeek-style shapes (tools/bench_moe.py: 49152 assignments, E64,
// D2048, F1408): 256x256 / 8 waves wins every mode (551-717 TF vs 436-627 for 128x128)
static int default_cfg(int mode) {
  const char* e = getenv("SPA_GG_CFG");
  if (e) return atoi(e);
  return 2;
}

// --------------------------------------------------------------------------- host
std::vector<at::Tensor> moe_route(const at::Tensor& logits_, const c10::optional<at::Tensor>& bias, int64_t k,
                                  bool bias_in_w) {
  auto logits = logits_.contiguous().to(at::kFloat);
  const int N = logits.size(0), E = logits.size(1);
  TORCH_CHECK(k >= 1 && k <= 8 && k <= E, "moe_route: 1 <= k <= 8");
  DeviceGuard g(logits.device());
  auto idx = at::empty({N, k}, logits.options().dtype(at::kInt));
  auto w = at::empty({N, k}, logits.options());
  if (N == 0) return {idx, w};
  at::Tensor b = bias ? bias->contiguous().to(at::kFloat) : at::Tensor();
  moe_route_kernel<8><<<cdiv(N, 4), 256, 0, stream()>>>(logits.data_ptr<float>(), bias ? b.data_ptr<float>() : nullptr,
                                                       idx.data_ptr<int>(), w.data_ptr<float>(), N, E, k,
                                                       bias_in_w ? 1 : 0);
  SPA_LAUNCH_CHECK();
  return {idx, w};
}

// returns (perm [A], inv [A], offsets [E+1], counts [E]) for assignments idx [N, k]
std::vector<at::Tensor> moe_permute(const at::Tensor& idx_, int64_t E) {
  auto idx = idx_.contiguous();
  TORCH_CHECK(idx.scalar_type() == at::kInt);
  const int A = idx.numel();
  DeviceGuard g(idx.device());
  auto opts = idx.options();
  auto perm = at::empty({A}, opts), inv = at::empty({A}, opts);
  auto counts = at::empty({E}, opts), offsets = at::empty({E + 1}, opts);
  auto st = stream();
  moe_count_kernel<<<E, 256, 0, st>>>(idx.data_ptr<int>(), A, E, counts.data_ptr<int>());
  moe_offsets_kernel<<<1, 64, 0, st>>>(counts.data_ptr<int>(), E, offsets.data_ptr<int>());
  moe_scatter_kernel<<<E, 256, 0, st>>>(idx.data_ptr<int>(), A, offsets.data_ptr<int>(), perm.data_ptr<int>(),
                                        inv.data_ptr<int>());
  SPA_LAUNCH_CHECK();
  return {perm, inv, offsets, counts};
}

// out[r] = x[perm[r] / div], or a zero row where perm[r] < 0; rows of any dtype whose byte width
// is a multiple of 16 (bf16 / fp32 activations, the uint8 fp8 dispatch payload)
at::Tensor moe_gather(const at::Tensor& x_, const at::Tensor& perm, int64_t div) {
  auto x = x_.contiguous();
  const int D = x.size(-1);
  TORCH_CHECK(x.dim() == 2 && (long)D * x.element_size() % 16 == 0, "moe_gather: [rows, D] with 16-byte rows");
  TORCH_CHECK(perm.scalar_type() == at::kInt && perm.is_contiguous(), "moe_gather: int32 map");
  const int rows = perm.numel();
  DeviceGuard g(x.device());
  auto out = at::empty({rows, D}, x.options());
  if (rows == 0) return out;
  const int nv = D * (int)x.element_size() / 16;
  const int grid = (int)std::min<long>(((long)rows * nv + 255) / 256, 16384);
  gather_rows_kernel<<<grid, 256, 0, stream()>>>((const uint4*)x.data_ptr(), perm.data_ptr<int>(),
                                                 (uint4*)out.data_ptr(), rows, nv, div, (long)x.size(0));
  SPA_LAUNCH_CHECK();
  return out;
}

at::Tensor moe_combine(const at::Tensor& yp_, const at::Tensor& inv, const c10::optional<at::Tensor>& w,
                       int64_t N, int64_t k) {
  auto yp = yp_.contiguous();
  const int D = yp.size(-1);
  DeviceGuard g(yp.device());
  auto y = at::empty({N, D}, yp.options());
  if (N == 0) return y;
  const int grid = (int)std::min<long>((N * D / 8 + 255) / 256, 16384);
  const float* wp = w ? w->data_ptr<float>() : nullptr;
  if (yp.scalar_type() == at::kBFloat16)
    combine_kernel<bf16><<<grid, 256, 0, stream()>>>((const bf16*)yp.data_ptr(), inv.data_ptr<int>(), wp,
                                                     (bf16*)y.data_ptr(), N, D, k, (long)yp.size(0));
  else
    combine_kernel<float><<<grid, 256, 0, stream()>>>(yp.data_ptr<float>(), inv.data_ptr<int>(), wp,
                                                      y.data_ptr<float>(), N, D, k, (long)yp.size(0));
  SPA_LAUNCH_CHECK();
  return y;
}

// backward of combine: (dyp [A, D] = w * dy rows in permuted order, dw [N, k])
std::vector<at::Tensor> moe_combine_bwd(const at::Tensor& dy_, const at::Tensor& yp_, const at::Tensor& perm,
                                        const at::Tensor& inv, const at::Tensor& w, int64_t k) {
  auto dy = dy_.contiguous(), yp = yp_.contiguous();
  const int N = dy.size(0), D = dy.size(1);
  const int A = perm.numel();
  DeviceGuard g(dy.device());
  auto dyp = at::empty({A, D}, dy.options());
  auto dw = at::empty({N, k}, dy.options().dtype(at::kFloat));
  if (A == 0) return {dyp, dw};
  auto st = stream();
  const int grid = (int)std::min<long>(((long)A * D / 8 + 255) / 256, 16384);
  if (dy.scalar_type() == at::kBFloat16) {
    scatter_grad_kernel<bf16><<<grid, 256, 0, st>>>((const bf16*)dy.data_ptr(), perm.data_ptr<int>(),
                                                    w.data_ptr<float>(), (bf16*)dyp.data_ptr(), A, D, k);
    combine_dw_kernel<bf16><<<cdiv(A, 4), 256, 0, st>>>((const bf16*)dy.data_ptr(), (const bf16*)yp.data_ptr(),
                                                        inv.data_ptr<int>(), dw.data_ptr<float>(), N, D, k);
  } else {
    scatter_grad_kernel<float><<<grid, 256, 0, st>>>(dy.data_ptr<float>(), perm.data_ptr<int>(), w.data_ptr<float>(),
                                                     dyp.data_ptr<float>(), A, D, k);
    combine_dw_kernel<float><<<cdiv(A, 4), 256, 0, st>>>(dy.data_ptr<float>(), yp.data_ptr<float>(),
                                                         inv.data_ptr<int>(), dw.data_ptr<float>(), N, D, k);
  }
  SPA_LAUNCH_CHECK();
  return {dyp, dw};
}

// mode 0: Y[M,N] = X[M,K] W_e[N,K]^T   (rows grouped by offsets; W [E, N, K])
// mode 1: dX[M,K] = dY[M,N] W_e[N,K]   (rows grouped; W [E, N, K])
// mode 2: dW_e[N,K] = dY_e[.,N]^T X_e[.,K]  (token dim grouped; out [E, N, K]); accumulate -> +=
at::Tensor grouped_gemm(const at::Tensor& a, const at::Tensor& w, const at::Tensor& offsets, int64_t mode,
                        const c10::optional<at::Tensor>& out_, bool accumulate, int64_t cfg) {
  TORCH_CHECK(a.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16, "grouped_gemm: bf16");
  TORCH_CHECK(a.is_contiguous() && w.is_contiguous() && offsets.scalar_type() == at::kInt);
  const int E = offsets.numel() - 1;
  TORCH_CHECK(E >= 1 && E <= 256, "grouped_gemm: 1..256 experts");
  DeviceGuard g(a.device());
  auto st = stream();
  if (cfg < 0) cfg = default_cfg((int)mode);
  if (mode == 0 || mode == 1) {
    TORCH_CHECK(w.dim() == 3 && w.size(0) == E);
    const int M = a.size(0);
    const int Nw = w.size(1), Kw = w.size(2);
    const int N = mode == 0 ? Nw : Kw;   // output cols
    const int K = mode == 0 ? Kw : Nw;   // reduction
    TORCH_CHECK(a.size(1) == K, "grouped_gemm: A/W shape mismatch");
    TORCH_CHECK(N % 8 == 0 && K % 8 == 0, "grouped_gemm: dims must be multiples of 8");
    auto out = out_ ? *out_ : at::empty({M, N}, a.options());
    if (M == 0) return out;
    const bf16* A = (const bf16*)a.data_ptr();
    const bf16* W = (const bf16*)w.data_ptr();
    bf16* C = (bf16*)out.data_ptr();
    if (mode == 0)
      dispatch_gg<true, true, false>(cfg, M, E, A, W, C, offsets.data_ptr<int>(), M, N, K, K, Kw, N,
                                     (long)Nw * Kw, 0, accumulate ? 1 : 0, st);
    else
      dispatch_gg<true, false, false>(cfg, M, E, A, W, C, offsets.data_ptr<int>(), M, N, K, K, Kw, N,
                                      (long)Nw * Kw, 0, accumulate ? 1 : 0, st);
    SPA_LAUNCH_CHECK();
    return out;
  }
  TORCH_CHECK(mode == 2, "grouped_gemm: mode 0/1/2");
  // a = dY [T, N], w = X [T, K]  -> out [E, N, K]
  const int N = a.size(1), K = w.size(1);
  TORCH_CHECK(a.size(0) == w.size(0) && N % 8 == 0 && K % 8 == 0);
  auto out = out_ ? *out_ : at::empty({E, N, K}, a.options());
  TORCH_CHECK(out.is_contiguous() && out.numel() == (long)E * N * K);
  // C_e (M=N rows, N=K cols) = A (dY^T, stored [k=token][m]) * B (X, stored [k=token][n])
  dispatch_gg<false, false, true>(cfg, 0, E, (const bf16*)a.data_ptr(), (const bf16*)w.data_ptr(), (bf16*)out.data_ptr(),
                                  offsets.data_ptr<int>(), N, K, 0, N, K, K, 0, (long)N * K, accumulate ? 1 : 0, st);
  SPA_LAUNCH_CHECK();
  return out;
}

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.def("moe_route(Tensor logits, Tensor? bias, int k, bool bias_in_w) -> Tensor[]");
  m.def("moe_permute(Tensor idx, int E) -> Tensor[]");
  m.def("moe_gather(Tensor x, Tensor perm, int div) -> Tensor");
  m.def("moe_combine(Tensor yp, Tensor inv, Tensor? w, int N, int k) -> Tensor");
  m.def("moe_combine_bwd(Tensor dy, Tensor yp, Tensor perm, Tensor inv, Tensor w, int k) -> Tensor[]");
  m.def("grouped_gemm(Tensor a, Tensor w, Tensor offsets, int mode, Tensor(a!)? out, bool accumulate, int cfg=-1) -> Tensor");
}
TORCH_LIBRARY_IMPL(spa, CUDA, m) {
  m.impl("moe_route", &spa::moe_route);
  m.impl("moe_permute", &spa::moe_permute);
  m.impl("moe_gather", &spa::moe_gather);
  m.impl("moe_combine", &spa::moe_combine);
  m.impl("moe_combine_bwd", &spa::moe_combine_bwd);
  m.impl("grouped_gemm", &spa::grouped_gemm);
}
