// Weight-streaming GEMV for decode: y[M, N] = x[M, K] @ W[N, K]^T, bf16 in / out, fp32
// accumulation, M <= 4 (the decode batch).
//
// A decode step multiplies a handful of token rows by every projection matrix: pure weight
// streaming (LLaMA3-8B: 16 GB per token), so the kernel is built for HBM, not for MFMA:
//  * each wave owns RW consecutive rows of W; its lanes split K in 16-byte chunks (lane l
//    reads k = 8l + 512i), so one wave-instruction reads 1 KB contiguous of a row;
//  * U chunks x RW rows of weight loads are issued before any is consumed (U * RW * 16 B in
//    flight per lane), non-temporal (read once, kept out of L2): latency is hidden by
//    memory-level parallelism, no LDS round trip (cdna_hip_programming.md, 'GEMV / M <= 16');
//  * RW = 2 for narrow outputs (N < 8192: o-proj, down-proj) so the grid still holds >= 2
//    waves per SIMD; RW = 4 otherwise;
//  * x (M x K, a few KB) is re-read per chunk from L1/L2, where it stays;
//  * products with v_dot2_f32_bf16 (2 bf16 MACs per instruction), one 64-lane xor
//    reduction per output at the end.
// torch.mm at M = 1 goes to hipBLASLt 16x16 macro tiles at 2.5-5 TB/s on streamed weights
// (decode profile: wo 2.5, wqkv 3.3, w13 3.9, w2 5.0 TB/s); this is the op the decode path uses.
#include "spa_common.h"

namespace spa {

__device__ __forceinline__ float dot8(const bf16x8& a, const bf16x8& b, float c) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bf16x2 a2 = {a[2 * j], a[2 * j + 1]};
    const bf16x2 b2 = {b[2 * j], b[2 * j + 1]};
    c = __builtin_amdgcn_fdot2_f32_bf16(a2, b2, c, false);
  }
  return c;
}

__device__ __forceinline__ bf16x8 ld_stream(const bf16* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(p));
}

template <int M, int RW, int U>
__global__ __launch_bounds__(256) void gemv_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                   bf16* __restrict__ y, int N, int K, long ldx, long ldw,
                                                   long ldy) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const int row0 = wave * RW;
  if (row0 >= N) return;  // wave-uniform
  float acc[M][RW];
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int r = 0; r < RW; ++r) acc[m][r] = 0.f;
  const bf16* wr[RW];
#pragma unroll
  for (int r = 0; r < RW; ++r) wr[r] = w + (long)min(row0 + r, N - 1) * ldw;  // tail rows: duplicate, not stored
  auto consume = [&](const int k, const bf16x8* wv) {
    bf16x8 xv[M];
#pragma unroll
    for (int m = 0; m < M; ++m) xv[m] = *reinterpret_cast<const bf16x8*>(x + m * ldx + k);
#pragma unroll
    for (int m = 0; m < M; ++m)
#pragma unroll
      for (int r = 0; r < RW; ++r) acc[m][r] = dot8(xv[m], wv[r], acc[m][r]);
  };
  int k = 8 * lane;
  for (; k + (U - 1) * 512 < K; k += U * 512) {
    bf16x8 wv[U][RW];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < RW; ++r) wv[u][r] = ld_stream(wr[r] + k + u * 512);
#pragma unroll
    for (int u = 0; u < U; ++u) consume(k + u * 512, wv[u]);
  }
  for (; k < K; k += 512) {
    bf16x8 wv[RW];
#pragma unroll
    for (int r = 0; r < RW; ++r) wv[r] = ld_stream(wr[r] + k);
    consume(k, wv);
  }
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const float v = wave_sum(acc[m][r]);
      if (lane == m * RW + r && row0 + r < N) y[m * ldy + row0 + r] = (bf16)v;
    }
}

template <int M>
static void launch_gemv(const bf16* x, const bf16* w, bf16* y, int N, int K, long ldx, long ldw, hipStream_t st) {
  if (N >= 8192) gemv_kernel<M, 4, 4><<<cdiv(cdiv(N, 4), 4), 256, 0, st>>>(x, w, y, N, K, ldx, ldw, N);
  else gemv_kernel<M, 2, 4><<<cdiv(cdiv(N, 2), 4), 256, 0, st>>>(x, w, y, N, K, ldx, ldw, N);
}

// x [M, K] (row stride ldx), w [N, K] row-major -> y [M, N]; M <= 4, K % 8 == 0.
at::Tensor gemv(const at::Tensor& x, const at::Tensor& w) {
  TORCH_CHECK(x.is_cuda() && w.is_cuda() && x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16,
              "gemv: bf16 HIP tensors");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1), "gemv: x [M, K], w [N, K]");
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(M >= 1 && M <= 4, "gemv: M must be 1..4");
  TORCH_CHECK(K % 8 == 0 && x.stride(1) == 1 && w.stride(1) == 1 && x.stride(0) % 8 == 0 && w.stride(0) % 8 == 0 &&
                  ((uintptr_t)x.data_ptr() % 16) == 0 && ((uintptr_t)w.data_ptr() % 16) == 0,
              "gemv: rows must be 16-byte aligned with K % 8 == 0");
  DeviceGuard g(x.device());
  auto y = at::empty({M, N}, x.options());
  if (N == 0) return y;
  auto st = stream();
  const bf16* xp = (const bf16*)x.data_ptr();
  const bf16* wp = (const bf16*)w.data_ptr();
  bf16* yp = (bf16*)y.data_ptr();
  switch (M) {
    case 1: launch_gemv<1>(xp, wp, yp, N, K, x.stride(0), w.stride(0), st); break;
    case 2: launch_gemv<2>(xp, wp, yp, N, K, x.stride(0), w.stride(0), st); break;
    case 3: launch_gemv<3>(xp, wp, yp, N, K, x.stride(0), w.stride(0), st); break;
    default: launch_gemv<4>(xp, wp, yp, N, K, x.stride(0), w.stride(0), st); break;
  }
  SPA_LAUNCH_CHECK();
  return y;
}


// ---------------------------------------------------------------------------------------
// Grouped (MoE) weight-streaming GEMV for decode: y[a, :] = x[a, :] @ W_e^T for the rows
// a in [off[e], off[e+1]) of every expert e (the expert-sorted assignments of a few tokens:
// 6 rows over 64 experts at batch 1). The MFMA grouped GEMM pays a 256-row tile per active
// expert for one or two real rows; this streams each ACTIVE expert's weights once instead.
// Grid: experts x column chunks; a wave owns RW weight rows (output columns) and walks the
// expert's token rows in groups of 4 (re-reading its weight rows from L2 past 4 rows).
// Experts with no rows exit at once (the row counts live on the device: no host sync).
template <int RW, int U>
__global__ __launch_bounds__(256) void grouped_gemv_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                           bf16* __restrict__ y, const int* __restrict__ offsets,
                                                           int N, int K, long strideW) {
  constexpr int MB = 4;
  const int lane = threadIdx.x & 63;
  const int nwb = cdiv(cdiv(N, RW), 4);  // blocks per expert
  const int e = blockIdx.x / nwb;
  const int wave = __builtin_amdgcn_readfirstlane((blockIdx.x % nwb) * 4 + (threadIdx.x >> 6));
  const int r_begin = offsets[e], r_end = offsets[e + 1];
  const int row0 = wave * RW;
  if (r_begin >= r_end || row0 >= N) return;  // wave-uniform
  const bf16* we = w + (long)e * strideW;
  const bf16* wr[RW];
#pragma unroll
  for (int r = 0; r < RW; ++r) wr[r] = we + (long)min(row0 + r, N - 1) * K;
  for (int m0 = r_begin; m0 < r_end; m0 += MB) {
    const int mn = min(MB, r_end - m0);
    float acc[MB][RW];
#pragma unroll
    for (int m = 0; m < MB; ++m)
#pragma unroll
      for (int r = 0; r < RW; ++r) acc[m][r] = 0.f;
    auto consume = [&](const int k, const bf16x8* wv) {
#pragma unroll
      for (int m = 0; m < MB; ++m) {
        if (m < mn) {
          const bf16x8 xv = *reinterpret_cast<const bf16x8*>(x + (long)(m0 + m) * K + k);
#pragma unroll
          for (int r = 0; r < RW; ++r) acc[m][r] = dot8(xv, wv[r], acc[m][r]);
        }
      }
    };
    int k = 8 * lane;
    for (; k + (U - 1) * 512 < K; k += U * 512) {
      bf16x8 wv[U][RW];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < RW; ++r) wv[u][r] = *reinterpret_cast<const bf16x8*>(wr[r] + k + u * 512);
#pragma unroll
      for (int u = 0; u < U; ++u) consume(k + u * 512, wv[u]);
    }
    for (; k < K; k += 512) {
      bf16x8 wv[RW];
#pragma unroll
      for (int r = 0; r < RW; ++r) wv[r] = *reinterpret_cast<const bf16x8*>(wr[r] + k);
      consume(k, wv);
    }
#pragma unroll
    for (int m = 0; m < MB; ++m)
#pragma unroll
      for (int r = 0; r < RW; ++r) {
        const float v = wave_sum(acc[m][r]);
        if (lane == m * RW + r && m < mn && row0 + r < N) y[(long)(m0 + m) * N + row0 + r] = (bf16)v;
      }
  }
}

// x [A, K] expert-sorted rows, w [E, N, K], offsets [E+1] (device) -> y [A, N]
at::Tensor grouped_gemv(const at::Tensor& x, const at::Tensor& w, const at::Tensor& offsets) {
  TORCH_CHECK(x.is_cuda() && w.is_cuda() && x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16,
              "grouped_gemv: bf16 HIP tensors");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 3 && x.size(1) == w.size(2) && x.is_contiguous() && w.is_contiguous(),
              "grouped_gemv: x [A, K], w [E, N, K] contiguous");
  TORCH_CHECK(offsets.scalar_type() == at::kInt && offsets.numel() == w.size(0) + 1, "grouped_gemv: offsets [E+1]");
  const int A = x.size(0), K = x.size(1), E = w.size(0), N = w.size(1);
  TORCH_CHECK(K % 8 == 0 && ((uintptr_t)x.data_ptr() % 16) == 0 && ((uintptr_t)w.data_ptr() % 16) == 0,
              "grouped_gemv: K % 8 == 0, 16-byte aligned");
  DeviceGuard g(x.device());
  auto y = at::empty({A, N}, x.options());
  if (A == 0 || N == 0) return y;
  const int nwb = cdiv(cdiv(N, 2), 4);
  grouped_gemv_kernel<2, 4><<<E * nwb, 256, 0, stream()>>>((const bf16*)x.data_ptr(), (const bf16*)w.data_ptr(),
                                                          (bf16*)y.data_ptr(), offsets.data_ptr<int>(), N, K,
                                                          (long)N * K);
  SPA_LAUNCH_CHECK();
  return y;
}

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.def("gemv(Tensor x, Tensor w) -> Tensor");
  m.def("grouped_gemv(Tensor x, Tensor w, Tensor offsets) -> Tensor");
}
TORCH_LIBRARY_IMPL(spa, CUDA, m) {
  m.impl("gemv", &spa::gemv);
  m.impl("grouped_gemv", &spa::grouped_gemv);
}
