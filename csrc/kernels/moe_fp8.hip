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

// --------------------------------------------------------------------------- GEMM
__device__ __forceinline__ int f8_off(int r, int c) { return r * 128 + 16 * (c ^ ((r >> 1) & 7)); }

template <int BM, int BN, int WGM, int WGN>
__global__ __launch_bounds__(64 * WGM * WGN) void grouped_gemm_fp8_kernel(
    const uint8_t* __restrict__ A, const float* __restrict__ sa, const uint8_t* __restrict__ B,
    const float* __restrict__ sb, bf16* __restrict__ C, const int* __restrict__ offsets, int E, int N, int K,
    long strideB) {
  constexpr int BK = 128;                                  // bytes (= fp8 elements) per k-step
  constexpr int NT = 64 * WGM * WGN;
  constexpr int TM = BM / WGM, TN = BN / WGN, IM = TM / 32, IN = TN / 32;
  constexpr int AB = BM * BK, BB = BN * BK;                // bytes per stage
  constexpr int CA = AB / 16 / NT, CB = BB / 16 / NT;
  static_assert(CA * 16 * NT == AB && CB * 16 * NT == BB, "tile/threads mismatch");
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * (AB + BB)];
  __shared__ int s_e, s_mt;
  __shared__ int wsum[NT / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int nnt = (N + BN - 1) / BN;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int nt = lid % nnt;
  int mt = lid / nnt;
  {  // tile -> expert (block scan of per-expert tile counts; thread e owns expert e)
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
    int pre = inc - tiles;
    for (int w = 0; w < wave; ++w) pre += wsum[w];
    if (tid < E && tiles > 0 && mt >= pre && mt < pre + tiles) { s_e = tid; s_mt = mt - pre; }
    __syncthreads();
  }
  const int e = s_e;
  if (e < 0) return;
  mt = s_mt;
  const int m0 = offsets[e] + mt * BM, mend = offsets[e + 1];
  const int n0 = nt * BN;
  const uint8_t* Bp = B + e * strideB;
  uint4 ra[CA], rb[CB];
  auto load_tiles = [&](int kk) {
#pragma unroll
    for (int c = 0; c < CA; ++c) {
      const int idx = tid + c * NT, r = idx >> 3, ch = idx & 7;
      const int gm = m0 + r, gk = kk + 16 * ch;
      ra[c] = (gm < mend && gk < K) ? *reinterpret_cast<const uint4*>(A + (long)gm * K + gk) : uint4{0, 0, 0, 0};
    }
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      const int idx = tid + c * NT, r = idx >> 3, ch = idx & 7;
      const int gn = n0 + r, gk = kk + 16 * ch;
      rb[c] = (gn < N && gk < K) ? *reinterpret_cast<const uint4*>(Bp + (long)gn * K + gk) : uint4{0, 0, 0, 0};
    }
  };
  auto store_tiles = [&](int buf) {
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
  const int kt = (K + BK - 1) / BK;
  const int l32 = lane & 31, hh = lane >> 5;
  load_tiles(0);
  store_tiles(0);
  if (kt > 1) load_tiles(BK);
  __syncthreads();
  for (int t = 0; t < kt; ++t) {
    const int buf = t & 1;
    if (t + 1 < kt) {
      store_tiles(buf ^ 1);
      if (t + 2 < kt) load_tiles((t + 2) * BK);
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
#pragma unroll
      for (int i = 0; i < IN; ++i)
#pragma unroll
        for (int j = 0; j < IM; ++j)   // fp8 e4m3 x fp8 e4m3, unit block scales (E8M0 127 = 1.0)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(bfr[i], af[j], acc[i][j], 0, 0, 0, 127, 0, 127);
    }
    __syncthreads();
  }
  // epilogue: C^T tiles, lane = token column m, rows n = 8g + 4hh + {0..3}
#pragma unroll
  for (int j = 0; j < IM; ++j) {
    const int gm = m0 + wm * TM + j * 32 + l32;
    if (gm >= mend) continue;
    const float sm = sa[gm];
#pragma unroll
    for (int i = 0; i < IN; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int gn = n0 + wn * TN + i * 32 + 8 * g + 4 * hh;
        if (gn >= N) continue;
        const f32x4 sw = *reinterpret_cast<const f32x4*>(sb + (long)e * N + gn);
        bf16x4 w4;
#pragma unroll
        for (int q = 0; q < 4; ++q) w4[q] = (bf16)(acc[i][j][4 * g + q] * sm * sw[q]);
        *reinterpret_cast<bf16x4*>(C + (long)gm * N + gn) = w4;
      }
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
  grouped_gemm_fp8_kernel<BM, BN, 2, 4><<<grid, 512, 0, stream()>>>(
      (const uint8_t*)xq.data_ptr(), sx.data_ptr<float>(), (const uint8_t*)wq.data_ptr(), sw.data_ptr<float>(),
      (bf16*)out.data_ptr(), offsets.data_ptr<int>(), E, N, K, (long)N * K);
  SPA_LAUNCH_CHECK();
  return out;
}

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.def("quant_rows_fp8(Tensor x) -> Tensor[]");
  m.def("grouped_gemm_fp8(Tensor xq, Tensor sx, Tensor wq, Tensor sw, Tensor offsets) -> Tensor");
}
TORCH_LIBRARY_IMPL(spa, CUDA, m) {
  m.impl("quant_rows_fp8", &spa::quant_rows_fp8);
  m.impl("grouped_gemm_fp8", &spa::grouped_gemm_fp8);
}
