// Token embedding gather (forward) and scatter-add (backward) for gfx950.
// Reference: every LM's `nn.Embedding` / `params['token_embedding'][inputs]`
// (llama3/LLaMA-jax.ipynb:918, gemma/gemma.ipynb:363, deepseekv3/deepseekv3.ipynb:1507)
// plus the optional additive position table (learned pos_embed gpt/gpt-jax.ipynb:441-472,
// sinusoidal pe deepseekv3/deepseekv3.ipynb:836-842,867-869) fused into the gather.
//
// Forward: one thread per 16-byte vector, rows gathered straight from the table.
// Backward: fp32 scatter-add with atomics shaped as whole 256-byte row segments per
// wave instruction (64 lanes x 4 B on one row), the budget-friendly atomic form on
// MI355X; the fp32 accumulator is then cast to the parameter dtype.
#include "spa_common.h"

namespace spa {

template <typename T, bool POS>
__global__ __launch_bounds__(256) void emb_fwd_kernel(const T* __restrict__ W, const int64_t* __restrict__ idx,
                                                      const T* __restrict__ pos, T* __restrict__ out, long N, int D,
                                                      int T_, float scale) {
  const int dv = D / 8;
  const long total = N * dv;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long n = i / dv;
    const int c = (i % dv) * 8;
    float v[8];
    load8(W + idx[n] * D + c, v);
    if (scale != 1.f)
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] *= scale;
    if constexpr (POS) {
      float p[8];
      load8(pos + (n % T_) * D + c, p);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += p[k];
    }
    store8(out + n * D + c, v);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void emb_bwd_kernel(const T* __restrict__ dout, const int64_t* __restrict__ idx,
                                                      float* __restrict__ dW, long N, int D, float scale) {
  // one wave per (row n, 256-column chunk): lane l adds column chunk*256 + 4l .. +3
  const int lane = threadIdx.x & 63;
  const int nchunk = (D + 255) / 256;
  const long nw = N * nchunk;
  for (long w = blockIdx.x * 4L + (threadIdx.x >> 6); w < nw; w += (long)gridDim.x * 4) {
    const long n = w / nchunk;
    const int c = (w % nchunk) * 256 + lane * 4;
    if (c >= D) continue;
    const int64_t r = idx[n];
    float* dst = dW + r * D + c;
    const T* src = dout + n * D + c;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (c + k < D) atomicAdd(dst + k, (float)src[k] * scale);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void cast_kernel(const float* __restrict__ a, T* __restrict__ b, long n) {
  const long nv = n / 8;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < nv; i += (long)gridDim.x * 256) {
    float v[8];
    load8(a + i * 8, v);
    store8(b + i * 8, v);
  }
  for (long i = nv * 8 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) b[i] = (T)a[i];
}

at::Tensor emb_fwd(const at::Tensor& W, const at::Tensor& idx, const c10::optional<at::Tensor>& pos, double scale) {
  SPA_CHECK_CUDA(W); SPA_CHECK_CONTIG(W);
  TORCH_CHECK(idx.scalar_type() == at::kLong);
  auto ix = idx.contiguous();
  const int D = W.size(1);
  TORCH_CHECK(D % 8 == 0, "embedding: D must be a multiple of 8");
  const long N = ix.numel();
  auto sizes = ix.sizes().vec();
  sizes.push_back(D);
  auto out = at::empty(sizes, W.options());
  if (N == 0) return out;
  DeviceGuard g(W.device());
  auto st = stream();
  const int T_ = (ix.dim() >= 2) ? ix.size(-1) : N;
  if (pos) TORCH_CHECK(pos->scalar_type() == W.scalar_type() && pos->is_contiguous() && pos->size(-1) == D &&
                           pos->numel() >= (long)T_ * D);
  const int grid = (int)std::min<long>((N * D / 8 + 255) / 256, 8192);
#define EL(T, P)                                                                                             \
  emb_fwd_kernel<T, P><<<grid, 256, 0, st>>>((const T*)W.data_ptr(), ix.data_ptr<int64_t>(),                 \
                                             P ? (const T*)pos->data_ptr() : nullptr, (T*)out.data_ptr(), N, D, \
                                             T_, (float)scale)
  if (W.scalar_type() == at::kBFloat16) { if (pos) EL(bf16, true); else EL(bf16, false); }
  else if (W.scalar_type() == at::kFloat) { if (pos) EL(float, true); else EL(float, false); }
  else TORCH_CHECK(false, "embedding: bf16/fp32 only");
#undef EL
  SPA_LAUNCH_CHECK();
  return out;
}

// Returns dW [V, D] in `dtype_like`'s dtype (fp32 accumulation inside).
at::Tensor emb_bwd(const at::Tensor& dout_, const at::Tensor& idx, int64_t V, double scale,
                   const at::Tensor& dtype_like) {
  auto dout = dout_.contiguous();
  auto ix = idx.contiguous();
  const int D = dout.size(-1);
  const long N = ix.numel();
  TORCH_CHECK(dout.numel() == N * D);
  DeviceGuard g(dout.device());
  auto acc = at::zeros({V, D}, dout.options().dtype(at::kFloat));
  auto st = stream();
  if (N > 0) {
    const long nw = N * ((D + 255) / 256);
    const int grid = (int)std::min<long>((nw + 3) / 4, 16384);
    if (dout.scalar_type() == at::kBFloat16)
      emb_bwd_kernel<bf16><<<grid, 256, 0, st>>>((const bf16*)dout.data_ptr(), ix.data_ptr<int64_t>(),
                                                 acc.data_ptr<float>(), N, D, (float)scale);
    else
      emb_bwd_kernel<float><<<grid, 256, 0, st>>>(dout.data_ptr<float>(), ix.data_ptr<int64_t>(),
                                                  acc.data_ptr<float>(), N, D, (float)scale);
    SPA_LAUNCH_CHECK();
  }
  if (dtype_like.scalar_type() == at::kFloat) return acc;
  auto outp = at::empty({V, D}, dout.options().dtype(dtype_like.scalar_type()));
  const long n = (long)V * D;
  cast_kernel<bf16><<<(int)std::min<long>((n / 8 + 255) / 256 + 1, 8192), 256, 0, st>>>(
      acc.data_ptr<float>(), (bf16*)outp.data_ptr(), n);
  SPA_LAUNCH_CHECK();
  return outp;
}

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.def("emb_fwd(Tensor W, Tensor idx, Tensor? pos, float scale) -> Tensor");
  m.def("emb_bwd(Tensor dout, Tensor idx, int V, float scale, Tensor dtype_like) -> Tensor");
}
TORCH_LIBRARY_IMPL(spa, CUDA, m) {
  m.impl("emb_fwd", &spa::emb_fwd);
  m.impl("emb_bwd", &spa::emb_bwd);
}
