// Layout kernels: bf16/fp32 2-D transpose through a padded LDS tile.
//
// Used to feed the weight-gradient GEMM dW = dY^T X in the layout hipBLASLt runs fastest
// on gfx950: with both operands transposed to K(token)-contiguous rows the product is the
// "NT" form x @ w^T, measured at LLaMA3-8B shapes (T = 8192) at 1.2-1.63 PF vs 0.94-1.13 PF
// for the "TN" form (tools/bench_gemm_layouts.py) -- the transposes cost far less than that.
//
// Tile 64 x 64, 256 threads: 16-byte global loads of rows -> LDS [64][72] (row pad keeps the
// column gathers on distinct banks) -> 8 column elements per thread -> 16-byte global stores.
#include "spa_common.h"

namespace spa {

// build-time A/B knobs (profiles/r5_transpose_variants.txt): tile size, diagonal block order
#ifndef SPA_TRANSPOSE_TS
#define SPA_TRANSPOSE_TS 64
#endif
#ifndef SPA_TRANSPOSE_DIAG
#define SPA_TRANSPOSE_DIAG 0
#endif
template <typename T>
__global__ __launch_bounds__(256) void transpose_kernel(const T* __restrict__ x, T* __restrict__ y, int R, int C,
                                                        long ldx, long ldy, long bsx, long bsy) {
  x += blockIdx.z * bsx;   // batch (e.g. one expert's [N, K] weight per z)
  y += blockIdx.z * bsy;
  constexpr int TS = SPA_TRANSPOSE_TS, PAD = 16 / sizeof(T), LD = TS + PAD, VE = 16 / sizeof(T);  // VE elements per 16 B
  __shared__ __attribute__((aligned(16))) T tile[TS * LD];
#if SPA_TRANSPOSE_DIAG
  // diagonal block order: blocks that run together read one input row band but write output
  // row bands that start at different column offsets (spreads the writes over HBM channels)
  const int bx = (blockIdx.x + blockIdx.y) % gridDim.x;
  const int r0 = blockIdx.y * TS, c0 = bx * TS;
#else
  const int r0 = blockIdx.y * TS, c0 = blockIdx.x * TS;
#endif
  constexpr int CPR = TS / VE;                  // 16-byte chunks per tile row
  constexpr int NCH = TS * CPR;                 // chunks per tile
#pragma unroll
  for (int c = 0; c < NCH / 256; ++c) {
    const int idx = threadIdx.x + 256 * c;
    const int r = idx / CPR, ch = idx % CPR;
    const int gr = r0 + r, gc = c0 + ch * VE;
    uint4 v = {0, 0, 0, 0};
    if (gr < R && gc < C) v = *reinterpret_cast<const uint4*>(x + (long)gr * ldx + gc);
    *reinterpret_cast<uint4*>(tile + r * LD + ch * VE) = v;
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < NCH / 256; ++c) {
    const int idx = threadIdx.x + 256 * c;
    const int j = idx / CPR, ch = idx % CPR;     // output row j (= input column), chunk of input rows
    const int orow = c0 + j, ocol = r0 + ch * VE;
    if (orow < C && ocol < R) {
      T o[VE];
#pragma unroll
      for (int e = 0; e < VE; ++e) o[e] = tile[(ch * VE + e) * LD + j];
      *reinterpret_cast<uint4*>(y + (long)orow * ldy + ocol) = *reinterpret_cast<uint4*>(o);
    }
  }
}

// x [R, C] or [Bt, R, C] (row stride ldx, unit column stride) -> y [C, R] / [Bt, C, R] contiguous
at::Tensor transpose2d(const at::Tensor& x_) {
  SPA_CHECK_CUDA(x_);
  TORCH_CHECK((x_.dim() == 2 || x_.dim() == 3) && x_.stride(-1) == 1, "transpose2d: [(Bt,) R, C], unit column stride");
  const bool batched = x_.dim() == 3;
  const at::Tensor x = batched ? x_.contiguous() : x_;
  const int Bt = batched ? x.size(0) : 1;
  const int R = x.size(-2), C = x.size(-1);
  const int ve = 16 / (int)x.element_size();
  TORCH_CHECK(R % ve == 0 && C % ve == 0 && x.stride(-2) % ve == 0 && (uintptr_t)x.data_ptr() % 16 == 0,
              "transpose2d: rows/cols must be 16-byte multiples");
  DeviceGuard g(x.device());
  auto y = batched ? at::empty({Bt, C, R}, x.options()) : at::empty({C, R}, x.options());
  if (R == 0 || C == 0 || Bt == 0) return y;
  dim3 grid(cdiv(C, SPA_TRANSPOSE_TS), cdiv(R, SPA_TRANSPOSE_TS), Bt);
  const long ld = x.stride(-2), bsx = batched ? x.stride(0) : 0, bsy = (long)R * C;
  if (x.scalar_type() == at::kBFloat16)
    transpose_kernel<bf16><<<grid, 256, 0, stream()>>>((const bf16*)x.data_ptr(), (bf16*)y.data_ptr(), R, C, ld, R,
                                                       bsx, bsy);
  else if (x.scalar_type() == at::kFloat)
    transpose_kernel<float><<<grid, 256, 0, stream()>>>(x.data_ptr<float>(), y.data_ptr<float>(), R, C, ld, R, bsx,
                                                        bsy);
  else
    TORCH_CHECK(false, "transpose2d: bf16/fp32");
  SPA_LAUNCH_CHECK();
  return y;
}

// Collective-footprint proxy (tools/overlap_interference.py): nwg workgroups of 256 threads
// stream src -> dst `reps` times with 16-byte accesses, the way an RCCL ring kernel keeps one
// workgroup per channel busy moving bytes for the whole collective. Lets a 1-GPU box measure
// what a concurrent all-reduce costs the backward's GEMMs (which CUs it takes, for how long)
// without a second GPU.
__global__ __launch_bounds__(256) void stream_copy_wg_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                             long n, int reps) {
  for (int r = 0; r < reps; ++r)
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) dst[i] = src[i];
}

void stream_copy_wg(const at::Tensor& src, at::Tensor& dst, int64_t nwg, int64_t reps) {
  SPA_CHECK_CUDA(src);
  TORCH_CHECK(src.is_contiguous() && dst.is_contiguous() && src.nbytes() == dst.nbytes() && src.nbytes() % 16 == 0,
              "stream_copy_wg: contiguous, equal sizes, 16-byte multiple");
  TORCH_CHECK(nwg > 0 && nwg <= 65536 && reps >= 0, "stream_copy_wg: nwg in [1, 65536], reps >= 0");
  DeviceGuard g(src.device());
  const long n = (long)(src.nbytes() / 16);
  if (n == 0 || reps == 0) return;
  stream_copy_wg_kernel<<<(int)nwg, 256, 0, stream()>>>((const uint4*)src.data_ptr(), (uint4*)dst.data_ptr(), n,
                                                       (int)reps);
  SPA_LAUNCH_CHECK();
}

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.def("transpose2d(Tensor x) -> Tensor");
  m.def("stream_copy_wg(Tensor src, Tensor(a!) dst, int nwg, int reps) -> ()");
}
TORCH_LIBRARY_IMPL(spa, CUDA, m) {
  m.impl("transpose2d", &spa::transpose2d);
  m.impl("stream_copy_wg", &spa::stream_copy_wg);
}
