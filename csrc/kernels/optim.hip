// Fused optimizer kernels over FLAT parameter buffers.
//
// Every trainable tensor of a model is a view into one contiguous buffer per
// param group (see solvingpapers_amd/utils/flat.py), so one launch updates all
// 8B parameters of LLaMA3-8B with no multi-tensor pointer lists; DP gradient
// buckets and ZeRO-1 shards are plain contiguous slices of the same buffers.
//
// Reference optimizers: AdamW (gpt/gpt-jax.ipynb:600 optax.adamw; gemma/gemma.ipynb:517;
// deepseekv3/deepseekv3.ipynb:2350-2356 betas (0.9,0.95), wd 0.1, eps 1e-8), Adam
// (vision transformer/ViT.ipynb:287, autoencoder, knowledge distillation/kd.py:92,109),
// plain SGD (llama3/LLaMA-jax.ipynb:996-1000). Grad-norm clipping
// (deepseekv3/deepseekv3.ipynb:2434-2439) is applied via a device-resident
// coefficient so clipping never syncs the host.
//
// Math matches torch.optim.AdamW: p *= 1 - lr*wd; p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps).
// Moments fp32, or bf16 (MT): the DeepSeek-V3 recipe (arXiv 2412.19437 sec. 3.3.2: AdamW moments
// tracked in BF16, master weights fp32) -- 20 instead of 28 bytes of HBM traffic per parameter.
#include "spa_common.h"

namespace spa {

template <typename PT, typename GT, bool MASTER, typename MT = float>
__global__ __launch_bounds__(256) void adamw_kernel(PT* __restrict__ p, float* __restrict__ master,
                                                    const GT* __restrict__ g, MT* __restrict__ m,
                                                    MT* __restrict__ v, long n, float lr, float b1, float b2,
                                                    float eps, float wd, float inv_bc1, float inv_sqrt_bc2,
                                                    const float* __restrict__ coef_ptr, int adam_l2,
                                                    const float* __restrict__ hyper) {
  const float coef = coef_ptr ? *coef_ptr : 1.f;
  // non-finite global grad norm -> the coefficient is NaN: skip the whole update. The norm is
  // reduced over every group that holds gradients, so all ranks take the same decision
  // without a host sync (train/optim.py FlatOptimizer.clip_coef).
  if (!(coef == coef)) return;
  if (hyper) {  // graph-safe: lr and step read from the device (hyper = [lr, step])
    lr = hyper[0];
    inv_bc1 = 1.f / (1.f - __powf(b1, hyper[1]));
    inv_sqrt_bc2 = rsqrtf(1.f - __powf(b2, hyper[1]));
  }
  const long nv = n / 8;
  const long stride = (long)gridDim.x * 256;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < nv + (n % 8 ? 1 : 0); i += stride) {
    const long base = i * 8;
    float pv[8], gv[8], mv[8], vv[8];
    const bool full = base + 8 <= n;
    if (full) {
      if constexpr (MASTER) load8(master + base, pv); else load8(p + base, pv);
      load8(g + base, gv);
      load8(m + base, mv);
      load8(v + base, vv);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const long j = base + k;
        pv[k] = j < n ? (MASTER ? master[j] : (float)p[j]) : 0.f;
        gv[k] = j < n ? (float)g[j] : 0.f;
        mv[k] = j < n ? (float)m[j] : 0.f;
        vv[k] = j < n ? (float)v[j] : 0.f;
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float gr = gv[k] * coef;
      if (adam_l2) gr += wd * pv[k];  // classic Adam weight decay (L2 in the gradient)
      mv[k] = b1 * mv[k] + (1.f - b1) * gr;
      vv[k] = b2 * vv[k] + (1.f - b2) * gr * gr;
      const float denom = sqrtf(vv[k]) * inv_sqrt_bc2 + eps;
      float pp = pv[k];
      if (!adam_l2) pp *= (1.f - lr * wd);
      pv[k] = pp - lr * inv_bc1 * mv[k] / denom;
    }
    if (full) {
      if constexpr (MASTER) { store8(master + base, pv); store8(p + base, pv); }
      else store8(p + base, pv);
      store8(m + base, mv);
      store8(v + base, vv);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const long j = base + k;
        if (j < n) {
          if constexpr (MASTER) master[j] = pv[k];
          p[j] = (PT)pv[k];
          m[j] = (MT)mv[k];
          v[j] = (MT)vv[k];
        }
      }
    }
  }
}

template <typename PT, typename GT, bool MASTER>
__global__ __launch_bounds__(256) void sgd_kernel(PT* __restrict__ p, float* __restrict__ master,
                                                  const GT* __restrict__ g, float* __restrict__ buf, long n, float lr,
                                                  float momentum, float wd, const float* __restrict__ coef_ptr,
                                                  const float* __restrict__ hyper) {
  const float coef = coef_ptr ? *coef_ptr : 1.f;
  if (!(coef == coef)) return;  // non-finite grad norm: skip (see adamw_kernel)
  if (hyper) lr = hyper[0];
  for (long j = blockIdx.x * 256L + threadIdx.x; j < n; j += (long)gridDim.x * 256) {
    float pv = MASTER ? master[j] : (float)p[j];
    float gr = (float)g[j] * coef + wd * pv;
    if (buf) { gr = momentum * buf[j] + gr; buf[j] = gr; }
    pv -= lr * gr;
    if constexpr (MASTER) master[j] = pv;
    p[j] = (PT)pv;
  }
}

// partial sums of squares; one partial per block
template <typename GT>
__global__ __launch_bounds__(256) void sqsum_kernel(const GT* __restrict__ g, long n, float* __restrict__ part) {
  __shared__ float red[4];
  float acc = 0.f;
  const long nv = n / 8;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < nv; i += (long)gridDim.x * 256) {
    float v[8];
    load8(g + i * 8, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += v[k] * v[k];
  }
  for (long j = nv * 8 + blockIdx.x * 256L + threadIdx.x; j < n; j += (long)gridDim.x * 256) {
    const float x = (float)g[j];
    acc += x * x;
  }
  acc = block_sum<256>(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}
__global__ __launch_bounds__(256) void sum_partials_kernel(const float* __restrict__ part, int np,
                                                           float* __restrict__ out) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int i = threadIdx.x; i < np; i += 256) acc += part[i];
  acc = block_sum<256>(acc, red);
  if (threadIdx.x == 0) out[0] = acc;
}

static int opt_grid(long n) { return (int)std::max<long>(1, std::min<long>((n / 8 + 255) / 256 + 1, 4096)); }
// Grid of AdamW (SPA_ADAMW_GRID overrides the block count for A/Bs): one 8-element vector per thread,
// no grid stride. The overlapped optimizer shares the GPU with the next step's forward, and short
// blocks let the forward's kernels in as they retire: dsv3_style +0.6 % (65.3K vs 64.9K tok/s B N N B),
// headline and Gemma-7B even. In isolation one 4-wave block per CU runs bf16-moment AdamW 20 % faster
// (5.40 vs 4.48 TB/s), but in the step it holds every CU for a whole bucket: dsv3_style 57.1K vs 65.0K
// (profiles/r6_adamw_grid.txt).
static int stream_grid(long n, const char* env) {
  const char* e = getenv(env);
  const long full = std::min<long>((n / 8 + 255) / 256 + 1, 1L << 30);   // one 8-element vector per thread
  return (int)(e ? std::min<long>(std::max(1, atoi(e)), full) : full);
}

void adamw_(const at::Tensor& p, const c10::optional<at::Tensor>& master, const at::Tensor& g, const at::Tensor& m,
            const at::Tensor& v, double lr, double b1, double b2, double eps, double wd, int64_t step,
            const c10::optional<at::Tensor>& coef, bool adam_l2, const c10::optional<at::Tensor>& hyper) {
  SPA_CHECK_CUDA(p);
  for (auto* t : {&p, &g, &m, &v}) TORCH_CHECK(t->is_contiguous(), "adamw: flat contiguous buffers required");
  const long n = p.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n);
  const bool mb = m.scalar_type() == at::kBFloat16;
  TORCH_CHECK(m.scalar_type() == v.scalar_type() && (mb || m.scalar_type() == at::kFloat), "adamw: fp32 or bf16 moments");
  if (master) TORCH_CHECK(master->scalar_type() == at::kFloat && master->numel() == n && master->is_contiguous());
  if (coef) TORCH_CHECK(coef->scalar_type() == at::kFloat && coef->numel() == 1);
  if (n == 0) return;
  DeviceGuard gd(p.device());
  auto st = stream();
  const float inv_bc1 = 1.f / (1.f - std::pow((float)b1, (float)step));
  const float inv_sqrt_bc2 = 1.f / std::sqrt(1.f - std::pow((float)b2, (float)step));
  const float* cp = coef ? coef->data_ptr<float>() : nullptr;
  if (hyper) TORCH_CHECK(hyper->scalar_type() == at::kFloat && hyper->numel() >= 2 && hyper->is_cuda());
  const float* hp = hyper ? hyper->data_ptr<float>() : nullptr;
  const int grid = stream_grid(n, "SPA_ADAMW_GRID");
#define ALM(PT, GT, MS, MT)                                                                                      \
  adamw_kernel<PT, GT, MS, MT><<<grid, 256, 0, st>>>(                                                            \
      (PT*)p.data_ptr(), MS ? master->data_ptr<float>() : nullptr, (const GT*)g.data_ptr(), (MT*)m.data_ptr(),   \
      (MT*)v.data_ptr(), n, (float)lr, (float)b1, (float)b2, (float)eps, (float)wd, inv_bc1, inv_sqrt_bc2, cp,    \
      adam_l2 ? 1 : 0, hp)
#define AL(PT, GT, MS) ALM(PT, GT, MS, float)
  const bool pb = p.scalar_type() == at::kBFloat16, gb = g.scalar_type() == at::kBFloat16;
  if (mb) {
    TORCH_CHECK(master.has_value(), "adamw: bf16 moments need an fp32 master");
    if (pb && gb) ALM(bf16, bf16, true, bf16);
    else if (pb) ALM(bf16, float, true, bf16);
    else if (gb) ALM(float, bf16, true, bf16);
    else ALM(float, float, true, bf16);
  } else if (pb && gb) { TORCH_CHECK(master.has_value(), "bf16 params need an fp32 master"); AL(bf16, bf16, true); }
  else if (pb && !gb) { TORCH_CHECK(master.has_value(), "bf16 params need an fp32 master"); AL(bf16, float, true); }
  else if (!pb && gb) { if (master) AL(float, bf16, true); else AL(float, bf16, false); }
  else { if (master) AL(float, float, true); else AL(float, float, false); }
#undef AL
#undef ALM
  SPA_LAUNCH_CHECK();
}

void sgd_(const at::Tensor& p, const c10::optional<at::Tensor>& master, const at::Tensor& g,
          const c10::optional<at::Tensor>& buf, double lr, double momentum, double wd,
          const c10::optional<at::Tensor>& coef, const c10::optional<at::Tensor>& hyper) {
  const long n = p.numel();
  TORCH_CHECK(p.is_contiguous() && g.is_contiguous() && g.numel() == n);
  if (n == 0) return;
  DeviceGuard gd(p.device());
  auto st = stream();
  const float* cp = coef ? coef->data_ptr<float>() : nullptr;
  float* bp = buf ? buf->data_ptr<float>() : nullptr;
  const int grid = (int)std::min<long>((n + 255) / 256, 8192);
#define SL(PT, GT, MS)                                                                                          \
  sgd_kernel<PT, GT, MS><<<grid, 256, 0, st>>>((PT*)p.data_ptr(), MS ? master->data_ptr<float>() : nullptr,     \
                                               (const GT*)g.data_ptr(), bp, n, (float)lr, (float)momentum,       \
                                               (float)wd, cp, hyper ? hyper->data_ptr<float>() : nullptr)
  const bool pb = p.scalar_type() == at::kBFloat16, gb = g.scalar_type() == at::kBFloat16;
  if (pb) { TORCH_CHECK(master.has_value()); if (gb) SL(bf16, bf16, true); else SL(bf16, float, true); }
  else { if (gb) { if (master) SL(float, bf16, true); else SL(float, bf16, false); }
         else { if (master) SL(float, float, true); else SL(float, float, false); } }
#undef SL
  SPA_LAUNCH_CHECK();
}

// Sum of squares of a flat buffer -> fp32 [1] tensor (deterministic two-stage reduction).
at::Tensor sqsum(const at::Tensor& g) {
  SPA_CHECK_CUDA(g); TORCH_CHECK(g.is_contiguous());
  const long n = g.numel();
  DeviceGuard gd(g.device());
  auto out = at::zeros({1}, g.options().dtype(at::kFloat));
  if (n == 0) return out;
  const char* se = getenv("SPA_SQSUM_GRID");
  const int nb = (int)std::max<long>(1, std::min<long>((n / 8 + 255) / 256, se ? std::max(1, atoi(se)) : 2048));
  auto part = at::empty({nb}, g.options().dtype(at::kFloat));
  auto st = stream();
  if (g.scalar_type() == at::kBFloat16)
    sqsum_kernel<bf16><<<nb, 256, 0, st>>>((const bf16*)g.data_ptr(), n, part.data_ptr<float>());
  else if (g.scalar_type() == at::kFloat)
    sqsum_kernel<float><<<nb, 256, 0, st>>>(g.data_ptr<float>(), n, part.data_ptr<float>());
  else TORCH_CHECK(false, "sqsum: bf16/fp32 only");
  sum_partials_kernel<<<1, 256, 0, st>>>(part.data_ptr<float>(), nb, out.data_ptr<float>());
  SPA_LAUNCH_CHECK();
  return out;
}

// DP reduce-scatter over the xGMI mesh (parallel/data_parallel.py reduce="a2a"): after one
// all-to-all every rank holds the N bf16 copies of its gradient shard, [N, n] rows; this sums them
// in fp32 and rounds ONCE (out = bf16(scale * sum_s in[s])), instead of the N-1 bf16 roundings of
// a ring reduce-scatter's running partial (profiles/r6_dp_reduce_numerics.txt). HBM-bound: reads
// N*n, writes n.
template <typename T>
__global__ __launch_bounds__(256) void shard_sum_kernel(const T* __restrict__ in, T* __restrict__ out, long n,
                                                        int N, float scale) {
  const long nv = n / 8;
  const long stride = (long)gridDim.x * 256;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < nv; i += stride) {
    float acc[8], v[8];
    load8(in + i * 8, acc);
    for (int s = 1; s < N; ++s) {
      load8(in + (long)s * n + i * 8, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += v[k];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] *= scale;
    store8(out + i * 8, acc);
  }
  for (long j = nv * 8 + blockIdx.x * 256L + threadIdx.x; j < n; j += stride) {
    float a = 0.f;
    for (int s = 0; s < N; ++s) a += (float)in[(long)s * n + j];
    out[j] = (T)(a * scale);
  }
}

void shard_sum_(const at::Tensor& out, const at::Tensor& in, int64_t N, double scale) {
  SPA_CHECK_CUDA(in);
  TORCH_CHECK(in.is_contiguous() && out.is_contiguous() && in.scalar_type() == out.scalar_type(),
              "shard_sum: contiguous, same dtype");
  const long n = out.numel();
  TORCH_CHECK(N >= 1 && in.numel() == N * n, "shard_sum: in must hold N x out.numel() values");
  if (n == 0) return;
  DeviceGuard gd(in.device());
  const int grid = opt_grid(n);
  if (in.scalar_type() == at::kBFloat16)
    shard_sum_kernel<bf16><<<grid, 256, 0, stream()>>>((const bf16*)in.data_ptr(), (bf16*)out.data_ptr(), n,
                                                        (int)N, (float)scale);
  else if (in.scalar_type() == at::kFloat)
    shard_sum_kernel<float><<<grid, 256, 0, stream()>>>(in.data_ptr<float>(), out.data_ptr<float>(), n, (int)N,
                                                         (float)scale);
  else TORCH_CHECK(false, "shard_sum: bf16/fp32 only");
  SPA_LAUNCH_CHECK();
}

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.def("adamw_(Tensor(a!) p, Tensor(b!)? master, Tensor g, Tensor(c!) m, Tensor(d!) v, float lr, float b1, "
        "float b2, float eps, float wd, int step, Tensor? coef, bool adam_l2, Tensor? hyper=None) -> ()");
  m.def("sgd_(Tensor(a!) p, Tensor(b!)? master, Tensor g, Tensor(c!)? buf, float lr, float momentum, float wd, "
        "Tensor? coef, Tensor? hyper=None) -> ()");
  m.def("sqsum(Tensor g) -> Tensor");
  m.def("shard_sum_(Tensor(a!) out, Tensor inp, int N, float scale) -> ()");
}
TORCH_LIBRARY_IMPL(spa, CUDA, m) {
  m.impl("adamw_", &spa::adamw_);
  m.impl("sgd_", &spa::sgd_);
  m.impl("sqsum", &spa::sqsum);
  m.impl("shard_sum_", &spa::shard_sum_);
}
