// Softmax cross-entropy over a vocabulary row, with the gradient written IN PLACE
// over the logits during the forward pass (the logits are dead after the loss),
// so a [T, V] = 8192 x 128256 LM head never holds a second V-wide buffer.
//
// Reference sites: gpt/gpt-jax.ipynb:503 (optax integer-label CE),
// llama3/LLaMA-jax.ipynb:961-967 (-mean(log_softmax gathered)),
// gemma/gemma.ipynb:534,564 and deepseekv3/deepseekv3.ipynb:2417-2421 (F.cross_entropy).
//
// The vocab-chunked variant (xent_chunk_stats / xent_chunk_grad_) serves the fused LM head
// that never materialises [N, V] and its vocab-parallel (TP) form; see below.
//
// One 256-thread block per row: pass 1 online (max, sum-exp) with 16-byte loads,
// block-combine, loss = lse - x[target]; pass 2 (optional) re-reads the row and
// writes (softmax - onehot) * scale, where scale lives on the device (1/num_valid)
// so there is no host sync. ignore_index rows get loss 0 and zero gradient.
#include "spa_common.h"

SPA_DEBUG_TU("xent.hip")

namespace spa {

// Block-wide (max, sum exp(x - max), sum x) of one row x[0..V), every thread gets the result.
// Vector body over the 16-byte-aligned part with a scalar head/tail (odd V such as GPT-2's
// 50257 leaves every row start misaligned).
template <typename T, bool VEC>
__device__ __forceinline__ void row_stats(const T* __restrict__ x, int V, float& M, float& S, float& SX, int& h0,
                                          int& nv, float* red_m, float* red_s, float* red_x) {
  float m = -INFINITY, s = 0.f, sx = 0.f;
  auto upd = [&](float v) {
    if (v > m) { s = s * __expf(m - v) + 1.f; m = v; }
    else s += __expf(v - m);
    sx += v;
  };
  h0 = 0; nv = 0;
  if constexpr (VEC) {
    h0 = (int)(((16 - ((uintptr_t)x & 15)) & 15) / sizeof(T));
    h0 = min(h0, V);
    nv = (V - h0) / 8;
    for (int i = threadIdx.x; i < nv; i += 256) {
      float v[8];
      load8(x + h0 + i * 8, v);
      float lm = v[0];
#pragma unroll
      for (int k = 1; k < 8; ++k) lm = fmaxf(lm, v[k]);
      const float nm = fmaxf(m, lm);
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) { acc += __expf(v[k] - nm); sx += v[k]; }
      s = s * __expf(m - nm) + acc;
      m = nm;
    }
    for (int i = threadIdx.x; i < h0; i += 256) upd((float)x[i]);
    for (int i = h0 + nv * 8 + threadIdx.x; i < V; i += 256) upd((float)x[i]);
  } else {
    for (int i = threadIdx.x; i < V; i += 256) upd((float)x[i]);
  }
  float wm = wave_max(m);
  float ws = (m == -INFINITY) ? 0.f : s * __expf(m - wm);  // idle threads (V < 8*256) hold m=-inf
  ws = wave_sum(ws);
  float wx = wave_sum(sx);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) { red_m[w] = wm; red_s[w] = ws; red_x[w] = wx; }
  __syncthreads();
  M = fmaxf(fmaxf(red_m[0], red_m[1]), fmaxf(red_m[2], red_m[3]));
  S = 0.f;
  SX = red_x[0] + red_x[1] + red_x[2] + red_x[3];
#pragma unroll
  for (int i = 0; i < 4; ++i) S += (red_m[i] == -INFINITY) ? 0.f : red_s[i] * __expf(red_m[i] - M);
}

// x <- sc * (exp(x - lse) - off - onv * [col == y]) over one row; col = v0 + local index
template <typename T, bool VEC>
__device__ __forceinline__ void row_grad(T* __restrict__ x, int V, int h0, int nv, long y, long v0, float lse,
                                         float sc, float off, float onv) {
  auto g1 = [&](int i) {
    const float v = (float)x[i];
    x[i] = (T)(sc * (__expf(v - lse) - off - (v0 + i == y ? onv : 0.f)));
  };
  if constexpr (VEC) {
    for (int i = threadIdx.x; i < nv; i += 256) {
      float v[8];
      load8(x + h0 + i * 8, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const long c = v0 + h0 + i * 8 + k;
        v[k] = sc * (__expf(v[k] - lse) - off - (c == y ? onv : 0.f));
      }
      store8(x + h0 + i * 8, v);
    }
    for (int i = threadIdx.x; i < h0; i += 256) g1(i);
    for (int i = h0 + nv * 8 + threadIdx.x; i < V; i += 256) g1(i);
  } else {
    for (int i = threadIdx.x; i < V; i += 256) g1(i);
  }
}

template <typename T, bool VEC, bool GRAD>
__global__ __launch_bounds__(256) void xent_kernel(T* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                   float* __restrict__ loss, float* __restrict__ lse_out,
                                                   const float* __restrict__ scale_ptr, int V, long ld,
                                                   int64_t ignore_index, float smoothing) {
  __shared__ float red_m[4], red_s[4], red_x[4];
  const int row = blockIdx.x;
  T* x = logits + (long)row * ld;
  const int64_t y = tgt[row];
  SPA_DBG_ASSERT(y == ignore_index || (y >= 0 && y < V), y, V);   // debug build: a real class or ignored
  float M, S, SX;
  int h0, nv;
  row_stats<T, VEC>(x, V, M, S, SX, h0, nv, red_m, red_s, red_x);
  const float lse = M + __logf(S);
  const bool valid = y != ignore_index;
  if (threadIdx.x == 0) {
    float li = 0.f;
    if (valid) {
      const float xt = (float)x[y];
      li = (1.f - smoothing) * (lse - xt) + smoothing * (lse - SX / V);
    }
    loss[row] = li;
    if (lse_out) lse_out[row] = lse;
  }
  if constexpr (GRAD) {
    __syncthreads();  // thread 0 has read x[y] before anyone overwrites it
    const float sc = valid ? (scale_ptr ? *scale_ptr : 1.f) : 0.f;
    row_grad<T, VEC>(x, V, h0, nv, y, 0, lse, sc, smoothing / V, 1.f - smoothing);
  }
}

// ---------------------------------------------------------------------------------------
// Vocab-chunked LM head + CE (ops/xent.py _ChunkedLinearXent): the [N, V] logits are never
// held; the head GEMM runs per vocab chunk of Vc columns [v0, v0 + Vc) and these kernels
// fold each chunk into per-row running statistics (online logsumexp), then -- in backward,
// on the recomputed chunk -- write d(loss)/d(logits) in place for the dW / dh GEMMs.
// Under tensor parallelism v0 is the GLOBAL column of the chunk's first entry; the running
// statistics are then exchanged as [N] floats only (max, then sum-exp / target logit / sum).
// ---------------------------------------------------------------------------------------
template <typename T, bool VEC>
__global__ __launch_bounds__(256) void xent_chunk_stats_kernel(const T* __restrict__ logits, long ld, int Vc,
                                                               long v0, const int64_t* __restrict__ tgt,
                                                               float* __restrict__ run_m, float* __restrict__ run_s,
                                                               float* __restrict__ run_t, float* __restrict__ run_x) {
  __shared__ float red_m[4], red_s[4], red_x[4];
  const int row = blockIdx.x;
  const T* x = logits + (long)row * ld;
  float M, S, SX;
  int h0, nv;
  row_stats<T, VEC>(x, Vc, M, S, SX, h0, nv, red_m, red_s, red_x);
  if (threadIdx.x == 0) {
    const float m0 = run_m[row], s0 = run_s[row];
    const float nm = fmaxf(m0, M);
    run_s[row] = (m0 == -INFINITY ? 0.f : s0 * __expf(m0 - nm)) + (M == -INFINITY ? 0.f : S * __expf(M - nm));
    run_m[row] = nm;
    run_x[row] += SX;
    const int64_t y = tgt[row];
    if (y >= v0 && y < v0 + Vc) run_t[row] = (float)x[y - v0];
  }
}

template <typename T, bool VEC>
__global__ __launch_bounds__(256) void xent_chunk_grad_kernel(T* __restrict__ logits, long ld, int Vc, long v0,
                                                              const int64_t* __restrict__ tgt,
                                                              const float* __restrict__ lse,
                                                              const float* __restrict__ scale_ptr, int64_t ignore_index,
                                                              float smoothing, long Vtot) {
  const int row = blockIdx.x;
  T* x = logits + (long)row * ld;
  const int64_t y = tgt[row];
  const float sc = (y != ignore_index) ? *scale_ptr : 0.f;
  int h0 = 0, nv = 0;
  if constexpr (VEC) {
    h0 = min((int)(((16 - ((uintptr_t)x & 15)) & 15) / sizeof(T)), Vc);
    nv = (Vc - h0) / 8;
  }
  row_grad<T, VEC>(x, Vc, h0, nv, y, v0, lse[row], sc, smoothing / (float)Vtot, 1.f - smoothing);
}

// logits [N, V] (row stride ld, last dim contiguous). Returns (loss[N], lse[N]).
// If write_grad, logits is overwritten with d(sum_i scale*loss_i)/dlogits.
std::vector<at::Tensor> xent_fwd(const at::Tensor& logits, const at::Tensor& target, int64_t ignore_index,
                                 double smoothing, bool write_grad, const c10::optional<at::Tensor>& scale) {
  SPA_CHECK_CUDA(logits);
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "xent: logits must be [N, V] with contiguous V");
  TORCH_CHECK(target.scalar_type() == at::kLong && target.is_contiguous() && target.numel() == logits.size(0));
  const int N = logits.size(0), V = logits.size(1);
  const long ld = logits.stride(0);
  DeviceGuard g(logits.device());
  auto opts = logits.options().dtype(at::kFloat);
  auto loss = at::empty({N}, opts);
  auto lse = at::empty({N}, opts);
  if (N == 0) return {loss, lse};
  if (scale) TORCH_CHECK(scale->scalar_type() == at::kFloat && scale->numel() == 1);
  // every row start is 2-byte (bf16) / 4-byte (fp32) aligned: the kernel peels a scalar head
  // to reach 16-byte alignment, so the vector path works for any V and row stride
  const bool vec = ((uintptr_t)logits.data_ptr() % logits.element_size() == 0);
  auto st = stream();
  const float* sp = scale ? scale->data_ptr<float>() : nullptr;
#define XL(T, VEC, GR)                                                                                     \
  xent_kernel<T, VEC, GR><<<N, 256, 0, st>>>((T*)logits.data_ptr(), target.data_ptr<int64_t>(),            \
                                             loss.data_ptr<float>(), lse.data_ptr<float>(), sp, V, ld,      \
                                             ignore_index, (float)smoothing)
#define XL2(T)                                 \
  if (vec) { if (write_grad) XL(T, true, true); else XL(T, true, false); } \
  else { if (write_grad) XL(T, false, true); else XL(T, false, false); }
  if (logits.scalar_type() == at::kBFloat16) { XL2(bf16) }
  else if (logits.scalar_type() == at::kFloat) { XL2(float) }
  else TORCH_CHECK(false, "xent: bf16/fp32 only");
#undef XL2
#undef XL
  SPA_LAUNCH_CHECK();
  return {loss, lse};
}


// chunk [N, Vc] (row stride ld) with global first column v0: fold into running (m, s, t, x)
void xent_chunk_stats(const at::Tensor& logits, const at::Tensor& target, int64_t v0, const at::Tensor& run_m,
                      const at::Tensor& run_s, const at::Tensor& run_t, const at::Tensor& run_x) {
  SPA_CHECK_CUDA(logits);
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "xent_chunk_stats: logits [N, Vc], contiguous Vc");
  TORCH_CHECK(target.scalar_type() == at::kLong && target.is_contiguous() && target.numel() == logits.size(0));
  for (auto* t : {&run_m, &run_s, &run_t, &run_x})
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == logits.size(0));
  const int N = logits.size(0), Vc = logits.size(1);
  if (N == 0 || Vc == 0) return;
  DeviceGuard g(logits.device());
  const long ld = logits.stride(0);
  const bool vec = ((uintptr_t)logits.data_ptr() % logits.element_size() == 0);
  auto st = stream();
#define XS(T, VEC)                                                                                          \
  xent_chunk_stats_kernel<T, VEC><<<N, 256, 0, st>>>((const T*)logits.data_ptr(), ld, Vc, v0,               \
                                                     target.data_ptr<int64_t>(), run_m.data_ptr<float>(),   \
                                                     run_s.data_ptr<float>(), run_t.data_ptr<float>(),      \
                                                     run_x.data_ptr<float>())
  if (logits.scalar_type() == at::kBFloat16) { if (vec) XS(bf16, true); else XS(bf16, false); }
  else if (logits.scalar_type() == at::kFloat) { if (vec) XS(float, true); else XS(float, false); }
  else TORCH_CHECK(false, "xent_chunk_stats: bf16/fp32 only");
#undef XS
  SPA_LAUNCH_CHECK();
}

// in place: chunk <- scale * (softmax - smoothing/Vtot - (1-smoothing) onehot), softmax from lse
void xent_chunk_grad_(const at::Tensor& logits, const at::Tensor& target, int64_t v0, const at::Tensor& lse,
                      const at::Tensor& scale, int64_t ignore_index, double smoothing, int64_t Vtot) {
  SPA_CHECK_CUDA(logits);
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "xent_chunk_grad_: logits [N, Vc], contiguous Vc");
  TORCH_CHECK(target.scalar_type() == at::kLong && target.is_contiguous() && target.numel() == logits.size(0));
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == logits.size(0));
  TORCH_CHECK(scale.scalar_type() == at::kFloat && scale.numel() == 1);
  const int N = logits.size(0), Vc = logits.size(1);
  if (N == 0 || Vc == 0) return;
  DeviceGuard g(logits.device());
  const long ld = logits.stride(0);
  const bool vec = ((uintptr_t)logits.data_ptr() % logits.element_size() == 0);
  auto st = stream();
#define XG(T, VEC)                                                                                          \
  xent_chunk_grad_kernel<T, VEC><<<N, 256, 0, st>>>((T*)logits.data_ptr(), ld, Vc, v0,                      \
                                                    target.data_ptr<int64_t>(), lse.data_ptr<float>(),      \
                                                    scale.data_ptr<float>(), ignore_index, (float)smoothing, \
                                                    Vtot)
  if (logits.scalar_type() == at::kBFloat16) { if (vec) XG(bf16, true); else XG(bf16, false); }
  else if (logits.scalar_type() == at::kFloat) { if (vec) XG(float, true); else XG(float, false); }
  else TORCH_CHECK(false, "xent_chunk_grad_: bf16/fp32 only");
#undef XG
  SPA_LAUNCH_CHECK();
}

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.def("xent_fwd(Tensor(a!) logits, Tensor target, int ignore_index, float smoothing, bool write_grad, "
        "Tensor? scale) -> Tensor[]");
  m.def("xent_chunk_stats(Tensor logits, Tensor target, int v0, Tensor(a!) run_m, Tensor(b!) run_s, "
        "Tensor(c!) run_t, Tensor(d!) run_x) -> ()");
  m.def("xent_chunk_grad_(Tensor(a!) logits, Tensor target, int v0, Tensor lse, Tensor scale, int ignore_index, "
        "float smoothing, int Vtot) -> ()");
}
TORCH_LIBRARY_IMPL(spa, CUDA, m) {
  m.impl("xent_fwd", &spa::xent_fwd);
  m.impl("xent_chunk_stats", &spa::xent_chunk_stats);
  m.impl("xent_chunk_grad_", &spa::xent_chunk_grad_);
}
