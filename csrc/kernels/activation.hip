// Elementwise activations (fwd + bwd) and gated linear units for gfx950.
//
// Activation suite of the reference: activation functions/GELU.ipynb:54-55 (tanh GELU),
// activation functions/ReLU.ipynb:20-54 (relu, leaky 0.01, prelu(alpha), elu(alpha)),
// exact-erf GELU (gemma/gemma.ipynb:282, vision transformer/ViT.ipynb:212), SiLU
// (deepseekv3/deepseekv3.ipynb:959-960), sigmoid (autoencoder decoders).
// Gated units: SwiGLU silu(g)*u (llama3/LLaMA-jax.ipynb:854-855,
// deepseekv3/deepseekv3.ipynb:963-972) and GeGLU gelu(g)*u (gemma/gemma.ipynb:269-286)
// on the output of ONE fused [gate | up] GEMM (row layout [M, 2F]).
//
// Memory bound: 16-byte vector I/O (8 bf16 or 2x4 fp32 per thread), grid-stride,
// fp32 math; one kernel template per (kind, dtype).
#include "spa_common.h"

namespace spa {

enum ActKind : int { RELU = 0, LEAKY = 1, PRELU = 2, ELU = 3, GELU_TANH = 4, GELU_ERF = 5, SILU = 6,
                     SIGMOID = 7, TANH = 8, IDENT = 9 };

__device__ __forceinline__ float act_f(int kind, float x, float a) {
  switch (kind) {
    case RELU: return x > 0.f ? x : 0.f;
    case LEAKY:
    case PRELU: return x > 0.f ? x : a * x;
    case ELU: return x > 0.f ? x : a * (__expf(x) - 1.f);
    case GELU_TANH: {
      const float k0 = 0.7978845608028654f, k1 = 0.044715f;
      const float u = k0 * (x + k1 * x * x * x);
      return 0.5f * x * (1.f + tanhf(u));
    }
    case GELU_ERF: return 0.5f * x * (1.f + erff(x * 0.7071067811865476f));
    case SILU: return x / (1.f + __expf(-x));
    case SIGMOID: return 1.f / (1.f + __expf(-x));
    case TANH: return tanhf(x);
    default: return x;
  }
}
// derivative d act / dx
__device__ __forceinline__ float act_df(int kind, float x, float a) {
  switch (kind) {
    case RELU: return x > 0.f ? 1.f : 0.f;
    case LEAKY:
    case PRELU: return x > 0.f ? 1.f : a;
    case ELU: return x > 0.f ? 1.f : a * __expf(x);
    case GELU_TANH: {
      const float k0 = 0.7978845608028654f, k1 = 0.044715f;
      const float u = k0 * (x + k1 * x * x * x);
      const float th = tanhf(u);
      return 0.5f * (1.f + th) + 0.5f * x * (1.f - th * th) * k0 * (1.f + 3.f * k1 * x * x);
    }
    case GELU_ERF: {
      const float cdf = 0.5f * (1.f + erff(x * 0.7071067811865476f));
      const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
      return cdf + x * pdf;
    }
    case SILU: {
      const float s = 1.f / (1.f + __expf(-x));
      return s * (1.f + x * (1.f - s));
    }
    case SIGMOID: {
      const float s = 1.f / (1.f + __expf(-x));
      return s * (1.f - s);
    }
    case TANH: {
      const float t = tanhf(x);
      return 1.f - t * t;
    }
    default: return 1.f;
  }
}

template <typename T, int KIND>
__global__ __launch_bounds__(256) void act_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, long n, float a) {
  const long nv = n / 8;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < nv; i += (long)gridDim.x * 256) {
    float v[8];
    load8(x + i * 8, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = act_f(KIND, v[k], a);
    store8(y + i * 8, v);
  }
  for (long i = nv * 8 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    y[i] = (T)act_f(KIND, (float)x[i], a);
}
template <typename T, int KIND>
__global__ __launch_bounds__(256) void act_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                      T* __restrict__ dx, long n, float a) {
  const long nv = n / 8;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < nv; i += (long)gridDim.x * 256) {
    float v[8], g[8];
    load8(x + i * 8, v);
    load8(dy + i * 8, g);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = g[k] * act_df(KIND, v[k], a);
    store8(dx + i * 8, v);
  }
  for (long i = nv * 8 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    dx[i] = (T)((float)dy[i] * act_df(KIND, (float)x[i], a));
}

// gated: y[m, f] = act(gu[m, f]) * gu[m, F + f]
template <typename T, int KIND>
__global__ __launch_bounds__(256) void glu_fwd_kernel(const T* __restrict__ gu, T* __restrict__ y, long M, int F) {
  const int fv = F / 8;
  const long nv = M * fv;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < nv; i += (long)gridDim.x * 256) {
    const long m = i / fv;
    const int f = (i % fv) * 8;
    float g[8], u[8];
    load8(gu + m * 2 * F + f, g);
    load8(gu + m * 2 * F + F + f, u);
#pragma unroll
    for (int k = 0; k < 8; ++k) g[k] = act_f(KIND, g[k], 0.f) * u[k];
    store8(y + m * F + f, g);
  }
}
template <typename T, int KIND>
__global__ __launch_bounds__(256) void glu_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ gu,
                                                      T* __restrict__ dgu, long M, int F) {
  const int fv = F / 8;
  const long nv = M * fv;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < nv; i += (long)gridDim.x * 256) {
    const long m = i / fv;
    const int f = (i % fv) * 8;
    float g[8], u[8], d[8], dg[8], du[8];
    load8(gu + m * 2 * F + f, g);
    load8(gu + m * 2 * F + F + f, u);
    load8(dy + m * F + f, d);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      du[k] = d[k] * act_f(KIND, g[k], 0.f);
      dg[k] = d[k] * u[k] * act_df(KIND, g[k], 0.f);
    }
    store8(dgu + m * 2 * F + f, dg);
    store8(dgu + m * 2 * F + F + f, du);
  }
}

static int ew_grid(long n) { return (int)std::max<long>(1, std::min<long>((n + 255) / 256, 8192)); }

#define ACT_SWITCH(KIND, ...)                                         \
  switch (KIND) {                                                     \
    case RELU: { constexpr int K_ = RELU; __VA_ARGS__; break; }       \
    case LEAKY: { constexpr int K_ = LEAKY; __VA_ARGS__; break; }     \
    case PRELU: { constexpr int K_ = PRELU; __VA_ARGS__; break; }     \
    case ELU: { constexpr int K_ = ELU; __VA_ARGS__; break; }         \
    case GELU_TANH: { constexpr int K_ = GELU_TANH; __VA_ARGS__; break; } \
    case GELU_ERF: { constexpr int K_ = GELU_ERF; __VA_ARGS__; break; }   \
    case SILU: { constexpr int K_ = SILU; __VA_ARGS__; break; }       \
    case SIGMOID: { constexpr int K_ = SIGMOID; __VA_ARGS__; break; } \
    case TANH: { constexpr int K_ = TANH; __VA_ARGS__; break; }       \
    default: TORCH_CHECK(false, "unknown activation kind");          \
  }

#define DTYPE_SWITCH(ST, ...)                                                       \
  if (ST == at::kBFloat16) { using T_ = bf16; __VA_ARGS__; }                        \
  else if (ST == at::kFloat) { using T_ = float; __VA_ARGS__; }                     \
  else TORCH_CHECK(false, "only bf16 / fp32 supported");

at::Tensor act_fwd(const at::Tensor& x_, int64_t kind, double alpha) {
  SPA_CHECK_CUDA(x_);
  auto x = dense(x_);
  auto y = at::empty_like(x);
  const long n = x.numel();
  if (n == 0) return y;
  DeviceGuard g(x.device());
  auto st = stream();
  DTYPE_SWITCH(x.scalar_type(), ACT_SWITCH(kind, act_fwd_kernel<T_, K_><<<ew_grid(n / 8 + 1), 256, 0, st>>>(
                                                    (const T_*)x.data_ptr(), (T_*)y.data_ptr(), n, (float)alpha)));
  SPA_LAUNCH_CHECK();
  return y;
}
at::Tensor act_bwd(const at::Tensor& dy_, const at::Tensor& x_, int64_t kind, double alpha) {
  auto x = dense(x_);
  auto dy = dense_like(dy_, x);
  TORCH_CHECK(dy.scalar_type() == x.scalar_type() && dy.numel() == x.numel());
  auto dx = at::empty_like(x);
  const long n = x.numel();
  if (n == 0) return dx;
  DeviceGuard g(x.device());
  auto st = stream();
  DTYPE_SWITCH(x.scalar_type(),
               ACT_SWITCH(kind, act_bwd_kernel<T_, K_><<<ew_grid(n / 8 + 1), 256, 0, st>>>(
                                    (const T_*)dy.data_ptr(), (const T_*)x.data_ptr(), (T_*)dx.data_ptr(), n,
                                    (float)alpha)));
  SPA_LAUNCH_CHECK();
  return dx;
}
at::Tensor glu_fwd(const at::Tensor& gu_, int64_t kind) {
  SPA_CHECK_CUDA(gu_);
  auto gu = gu_.contiguous();
  const int F2 = gu.size(-1);
  TORCH_CHECK(F2 % 16 == 0, "glu: last dim must be 2F with F % 8 == 0");
  const int F = F2 / 2;
  const long M = gu.numel() / F2;
  auto sizes = gu.sizes().vec();
  sizes.back() = F;
  auto y = at::empty(sizes, gu.options());
  if (M == 0) return y;
  DeviceGuard g(gu.device());
  auto st = stream();
  DTYPE_SWITCH(gu.scalar_type(), ACT_SWITCH(kind, glu_fwd_kernel<T_, K_><<<ew_grid(M * F / 8), 256, 0, st>>>(
                                                     (const T_*)gu.data_ptr(), (T_*)y.data_ptr(), M, F)));
  SPA_LAUNCH_CHECK();
  return y;
}
at::Tensor glu_bwd(const at::Tensor& dy_, const at::Tensor& gu_, int64_t kind) {
  auto gu = gu_.contiguous();
  auto dy = dy_.contiguous();
  const int F2 = gu.size(-1), F = F2 / 2;
  const long M = gu.numel() / F2;
  TORCH_CHECK(dy.numel() == M * F && dy.scalar_type() == gu.scalar_type());
  auto dgu = at::empty_like(gu);
  if (M == 0) return dgu;
  DeviceGuard g(gu.device());
  auto st = stream();
  DTYPE_SWITCH(gu.scalar_type(),
               ACT_SWITCH(kind, glu_bwd_kernel<T_, K_><<<ew_grid(M * F / 8), 256, 0, st>>>(
                                    (const T_*)dy.data_ptr(), (const T_*)gu.data_ptr(), (T_*)dgu.data_ptr(), M, F)));
  SPA_LAUNCH_CHECK();
  return dgu;
}

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.def("act_fwd(Tensor x, int kind, float alpha) -> Tensor");
  m.def("act_bwd(Tensor dy, Tensor x, int kind, float alpha) -> Tensor");
  m.def("glu_fwd(Tensor gu, int kind) -> Tensor");
  m.def("glu_bwd(Tensor dy, Tensor gu, int kind) -> Tensor");
}
TORCH_LIBRARY_IMPL(spa, CUDA, m) {
  m.impl("act_fwd", &spa::act_fwd);
  m.impl("act_bwd", &spa::act_bwd);
  m.impl("glu_fwd", &spa::glu_fwd);
  m.impl("glu_bwd", &spa::glu_bwd);
}
