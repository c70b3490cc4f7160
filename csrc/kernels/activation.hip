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
#include "act_common.h"

namespace spa {

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

// Backward of act(u) fused with the bias gradient of the Linear that produced u: dU = dY * act'(u)
// is written AND summed over rows (the bias gradient is colsum(dU)), so dU is not read a second
// time. Layout of rowsum_part_kernel (norm.hip): block (bx, by) covers 256 columns x rows
// [by*rpb, (by+1)*rpb); 32 lanes x 8 columns span a 512-byte row segment, 8 row groups stride
// the rows two at a time (4 16-byte loads in flight per lane); fp32 partials part[by, :] are
// summed by reduce_col_parts (deterministic).
template <int KIND>
__global__ __launch_bounds__(256) void act_bwd_colsum_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ u,
                                                             bf16* __restrict__ du, float* __restrict__ part,
                                                             long R, int N, long rpb, float a) {
  __shared__ __attribute__((aligned(16))) float red[8][256];
  const int cl = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int c0 = blockIdx.x * 256 + cl * 8;
  const long r0 = (long)blockIdx.y * rpb, r1 = min(R, r0 + rpb);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto one = [&](const float* g, const float* x, long r) {
    float d[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      d[k] = g[k] * act_df(KIND, x[k], a);
    }
    store8(du + r * N + c0, d);
    // sum what was stored (bf16-rounded), as a separate bias-grad pass over dU would
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] += (float)(bf16)d[k];
  };
  if (c0 < N) {
    long r = r0 + rg;
    for (; r + 24 < r1; r += 32) {                 // 8 16-byte loads in flight per lane
      float g[4][8], x[4][8];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        load8(dy + (r + 8 * k) * N + c0, g[k]);
        load8(u + (r + 8 * k) * N + c0, x[k]);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) one(g[k], x[k], r + 8 * k);
    }
    for (; r < r1; r += 8) {
      float g0[8], x0[8];
      load8(dy + r * N + c0, g0);
      load8(u + r * N + c0, x0);
      one(g0, x0, r);
    }
  }
  *reinterpret_cast<float4*>(&red[rg][cl * 8]) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  *reinterpret_cast<float4*>(&red[rg][cl * 8 + 4]) = make_float4(acc[4], acc[5], acc[6], acc[7]);
  __syncthreads();
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c < N) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 8; ++g) t += red[g][threadIdx.x];
    part[(long)blockIdx.y * N + c] = t;
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
// (dU [R, N] bf16, colsum(dU) fp32 [N]) for dy, u [R, N] bf16 contiguous, N % 8 == 0
std::vector<at::Tensor> act_bwd_colsum(const at::Tensor& dy, const at::Tensor& u, int64_t kind, double alpha) {
  SPA_CHECK_CUDA(u);
  TORCH_CHECK(u.dim() == 2 && u.scalar_type() == at::kBFloat16 && u.is_contiguous(), "act_bwd_colsum: [R, N] bf16");
  TORCH_CHECK(dy.sizes() == u.sizes() && dy.scalar_type() == at::kBFloat16 && dy.is_contiguous(),
              "act_bwd_colsum: dy must match u");
  const long R = u.size(0);
  const int N = u.size(1);
  TORCH_CHECK(N % 8 == 0 && (uintptr_t)u.data_ptr() % 16 == 0 && (uintptr_t)dy.data_ptr() % 16 == 0,
              "act_bwd_colsum: 16-byte rows");
  DeviceGuard g(u.device());
  auto du = at::empty_like(u);
  auto opts = u.options().dtype(at::kFloat);
  if (N == 0) return {du, at::empty({0}, opts)};
  if (R == 0) return {du, at::zeros({N}, opts)};
  auto st = stream();
  const int nx = cdiv(N, 256);
  // >= 2048 blocks (8 per CU), each at least 128 rows
  const long want = std::max<long>(1, std::min<long>(cdiv(2048, nx), cdiv(R, 128)));
  const long rpb = (R + want - 1) / want;
  const int P = (int)cdiv(R, rpb);
  auto part = at::empty({P, N}, opts);
  ACT_SWITCH(kind, act_bwd_colsum_kernel<K_><<<dim3(nx, P), 256, 0, st>>>(
                       (const bf16*)dy.data_ptr(), (const bf16*)u.data_ptr(), (bf16*)du.data_ptr(),
                       part.data_ptr<float>(), R, N, rpb, (float)alpha));
  SPA_LAUNCH_CHECK();
  return {du, reduce_col_parts(part)};
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
  m.def("act_bwd_colsum(Tensor dy, Tensor u, int kind, float alpha) -> Tensor[]");
  m.def("glu_fwd(Tensor gu, int kind) -> Tensor");
  m.def("glu_bwd(Tensor dy, Tensor gu, int kind) -> Tensor");
}
TORCH_LIBRARY_IMPL(spa, CUDA, m) {
  m.impl("act_fwd", &spa::act_fwd);
  m.impl("act_bwd", &spa::act_bwd);
  m.impl("act_bwd_colsum", &spa::act_bwd_colsum);
  m.impl("glu_fwd", &spa::glu_fwd);
  m.impl("glu_bwd", &spa::glu_bwd);
}
