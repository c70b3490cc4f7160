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

// token rows per block of the GLU transpose kernels below (64 or 128; tools/bench_glu_t.py, one box:
// glu_bwd_t 0.340 ms at 64 vs 0.320 at 128, glu_fwd_t 0.200 at 64 vs 0.213 at 128)
#ifndef GLU_T_TT_BWD
#define GLU_T_TT_BWD 128
#endif
#ifndef GLU_T_TT_FWD
#define GLU_T_TT_FWD 64
#endif
// glu_bwd that also writes the transposed gradient dgu^T [2F, M] (bf16): the weight gradient of the
// [gate | up] projection is dW = dgu^T X, which hipBLASLt runs fastest with both operands
// token-contiguous ("both" form, profiles/r6_wgrad_glu_t.txt); producing dgu^T here saves the
// separate transpose's read of dgu. Block = 64 tokens x 64 features of F (gate and up halves):
// 16-byte loads of gu / dy, dgu in fp32 -> bf16, stored row-major AND staged in two padded LDS
// tiles whose columns leave as 16-byte runs of 8 tokens of dgu^T rows (f and F + f).
template <int KIND>
__global__ __launch_bounds__(256) void glu_bwd_t_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ gu,
                                                        bf16* __restrict__ dgu, bf16* __restrict__ dgut, int M, int F) {
  // block = 64 tokens x 128 features (256-B row segments per half on the read side, 128-B runs of
  // dgu^T rows on the write side). LDS tiles [gate / up][token][feature], 272-B rows, the 16-B chunk
  // index XOR-swizzled by the token row's 8-row group so the transposed phase's 8-byte reads (4
  // features of one token) spread over the banks
  constexpr int TT = GLU_T_TT_BWD, TF = 128, LD = TF + 8, CT = TT / 8;
  __shared__ __attribute__((aligned(16))) bf16 tile[2][TT * LD];
  const int r0 = blockIdx.y * TT, f0 = blockIdx.x * TF;
  auto soff = [](int r, int c16) { return r * LD + 8 * (c16 ^ ((r >> 3) & 7)); };
#pragma unroll
  for (int c = 0; c < TT / 16; ++c) {        // TT tokens x 16 chunks of 8 features
    const int idx = threadIdx.x + 256 * c, r = idx >> 4, ch = idx & 15;
    const int m = r0 + r, f = f0 + ch * 8;
    float g[8], u[8], d[8], dg[8], du[8];
    const bool ok = m < M && f < F;
    if (ok) {
      load8(gu + (long)m * 2 * F + f, g);
      load8(gu + (long)m * 2 * F + F + f, u);
      load8(dy + (long)m * F + f, d);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      du[k] = ok ? d[k] * act_f(KIND, g[k], 0.f) : 0.f;
      dg[k] = ok ? d[k] * u[k] * act_df(KIND, g[k], 0.f) : 0.f;
    }
    if (ok) {
      store8(dgu + (long)m * 2 * F + f, dg);
      store8(dgu + (long)m * 2 * F + F + f, du);
    }
    bf16x8 a8, b8;
#pragma unroll
    for (int k = 0; k < 8; ++k) { a8[k] = (bf16)dg[k]; b8[k] = (bf16)du[k]; }
    *reinterpret_cast<bf16x8*>(&tile[0][soff(r, ch)]) = a8;
    *reinterpret_cast<bf16x8*>(&tile[1][soff(r, ch)]) = b8;
  }
  __syncthreads();
  // jobs: half h, features 4 jq .. 4 jq + 3 (32 groups), tokens 8 ch .. 8 ch + 7 -> four 16-B runs of
  // dgu^T rows each (8 x ds_read_b64 + 16 v_perm)
#pragma unroll
  for (int c = 0; c < CT / 4; ++c) {
    const int idx = threadIdx.x + 256 * c, h = idx / (32 * CT), jq = (idx / CT) & 31, ch = idx % CT;
    uint2 rw[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int r = ch * 8 + e;
      rw[e] = *reinterpret_cast<const uint2*>(&tile[h][soff(r, jq >> 1) + 4 * (jq & 1)]);
    }
    const int m = r0 + ch * 8;
    if (m < M) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {         // feature 4 jq + q: 16-bit half (q & 1) of word (q >> 1)
        const int f = f0 + 4 * jq + q;
        if (f < F) {
          const unsigned sel = (q & 1) ? 0x07060302u : 0x05040100u;   // high / low halves of (b, a)
          unsigned w[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) w[e] = (q >> 1) ? rw[e].y : rw[e].x;
          uint4 o;
          o.x = __builtin_amdgcn_perm(w[1], w[0], sel);
          o.y = __builtin_amdgcn_perm(w[3], w[2], sel);
          o.z = __builtin_amdgcn_perm(w[5], w[4], sel);
          o.w = __builtin_amdgcn_perm(w[7], w[6], sel);
          *reinterpret_cast<uint4*>(dgut + (long)(h * F + f) * M + m) = o;
        }
      }
    }
  }
}

// glu_fwd that also writes y^T [F, M] (bf16): the down projection's weight gradient dW2 = dY^T y then
// runs in the both-token-contiguous form too (ops/linear.py swiglu_mlp keeps y^T instead of y for the
// backward). Same tiling as glu_bwd_t: 64 tokens x 128 features, swizzled LDS tile, 8-byte reads + v_perm.
template <int KIND>
__global__ __launch_bounds__(256) void glu_fwd_t_kernel(const bf16* __restrict__ gu, bf16* __restrict__ y,
                                                        bf16* __restrict__ yt, int M, int F) {
  constexpr int TT = GLU_T_TT_FWD, TF = 128, LD = TF + 8, CT = TT / 8;
  __shared__ __attribute__((aligned(16))) bf16 tile[TT * LD];
  const int r0 = blockIdx.y * TT, f0 = blockIdx.x * TF;
  auto soff = [](int r, int c16) { return r * LD + 8 * (c16 ^ ((r >> 3) & 7)); };
#pragma unroll
  for (int c = 0; c < TT / 16; ++c) {
    const int idx = threadIdx.x + 256 * c, r = idx >> 4, ch = idx & 15;
    const int m = r0 + r, f = f0 + ch * 8;
    float g[8], u[8];
    const bool ok = m < M && f < F;
    if (ok) {
      load8(gu + (long)m * 2 * F + f, g);
      load8(gu + (long)m * 2 * F + F + f, u);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) g[k] = ok ? act_f(KIND, g[k], 0.f) * u[k] : 0.f;
    if (ok) store8(y + (long)m * F + f, g);
    bf16x8 a8;
#pragma unroll
    for (int k = 0; k < 8; ++k) a8[k] = (bf16)g[k];
    *reinterpret_cast<bf16x8*>(&tile[soff(r, ch)]) = a8;
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < CT / 8; ++c) {        // features 4 jq .., tokens 8 ch ..
  const int idx = threadIdx.x + 256 * c, jq = idx / CT, ch = idx % CT;
  uint2 rw[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) rw[e] = *reinterpret_cast<const uint2*>(&tile[soff(ch * 8 + e, jq >> 1) + 4 * (jq & 1)]);
  const int m = r0 + ch * 8;
  if (m < M) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int f = f0 + 4 * jq + q;
      if (f < F) {
        const unsigned sel = (q & 1) ? 0x07060302u : 0x05040100u;
        unsigned w[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) w[e] = (q >> 1) ? rw[e].y : rw[e].x;
        uint4 o;
        o.x = __builtin_amdgcn_perm(w[1], w[0], sel);
        o.y = __builtin_amdgcn_perm(w[3], w[2], sel);
        o.z = __builtin_amdgcn_perm(w[5], w[4], sel);
        o.w = __builtin_amdgcn_perm(w[7], w[6], sel);
        *reinterpret_cast<uint4*>(yt + (long)f * M + m) = o;
      }
    }
  }
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

// (y [.., F], y^T [F, M]) -- see glu_fwd_t_kernel; bf16, M % 8 == 0 and F % 8 == 0
std::vector<at::Tensor> glu_fwd_t(const at::Tensor& gu_, int64_t kind) {
  auto gu = gu_.contiguous();
  TORCH_CHECK(gu.scalar_type() == at::kBFloat16, "glu_fwd_t: bf16");
  const int F2 = gu.size(-1), F = F2 / 2;
  const long M = gu.numel() / F2;
  TORCH_CHECK(F2 % 16 == 0 && M % 8 == 0 && M < (1L << 31), "glu_fwd_t: M % 8, F % 8");
  auto sizes = gu.sizes().vec();
  sizes.back() = F;
  auto y = at::empty(sizes, gu.options());
  auto yt = at::empty({F, M}, gu.options());
  if (M == 0) return {y, yt};
  DeviceGuard g(gu.device());
  const dim3 grid(cdiv(F, 128), (int)cdiv(M, (long)GLU_T_TT_FWD));
  ACT_SWITCH(kind, glu_fwd_t_kernel<K_><<<grid, 256, 0, stream()>>>((const bf16*)gu.data_ptr(), (bf16*)y.data_ptr(),
                                                                      (bf16*)yt.data_ptr(), (int)M, F));
  SPA_LAUNCH_CHECK();
  return {y, yt};
}

// (dgu [.., 2F], dgu^T [2F, M]) -- see glu_bwd_t_kernel; bf16, M % 8 == 0 and F % 8 == 0
std::vector<at::Tensor> glu_bwd_t(const at::Tensor& dy_, const at::Tensor& gu_, int64_t kind) {
  auto gu = gu_.contiguous();
  auto dy = dy_.contiguous();
  TORCH_CHECK(gu.scalar_type() == at::kBFloat16 && dy.scalar_type() == at::kBFloat16, "glu_bwd_t: bf16");
  const int F2 = gu.size(-1), F = F2 / 2;
  const long M = gu.numel() / F2;
  TORCH_CHECK(dy.numel() == M * F, "glu_bwd_t: dy must be [.., F]");
  TORCH_CHECK(M % 8 == 0 && F % 8 == 0 && M < (1L << 31) && (long)F2 * M < (1L << 40), "glu_bwd_t: M, F % 8");
  auto dgu = at::empty_like(gu);
  auto dgut = at::empty({F2, M}, gu.options());
  if (M == 0) return {dgu, dgut};
  DeviceGuard g(gu.device());
  const dim3 grid(cdiv(F, 128), (int)cdiv(M, (long)GLU_T_TT_BWD));
  ACT_SWITCH(kind, glu_bwd_t_kernel<K_><<<grid, 256, 0, stream()>>>(
                       (const bf16*)dy.data_ptr(), (const bf16*)gu.data_ptr(), (bf16*)dgu.data_ptr(),
                       (bf16*)dgut.data_ptr(), (int)M, F));
  SPA_LAUNCH_CHECK();
  return {dgu, dgut};
}

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.def("glu_bwd_t(Tensor dy, Tensor gu, int kind) -> Tensor[]");
  m.def("glu_fwd_t(Tensor gu, int kind) -> Tensor[]");
  m.def("act_fwd(Tensor x, int kind, float alpha) -> Tensor");
  m.def("act_bwd(Tensor dy, Tensor x, int kind, float alpha) -> Tensor");
  m.def("act_bwd_colsum(Tensor dy, Tensor u, int kind, float alpha) -> Tensor[]");
  m.def("glu_fwd(Tensor gu, int kind) -> Tensor");
  m.def("glu_bwd(Tensor dy, Tensor gu, int kind) -> Tensor");
}
TORCH_LIBRARY_IMPL(spa, CUDA, m) {
  m.impl("glu_bwd_t", &spa::glu_bwd_t);
  m.impl("glu_fwd_t", &spa::glu_fwd_t);
  m.impl("act_fwd", &spa::act_fwd);
  m.impl("act_bwd", &spa::act_bwd);
  m.impl("act_bwd_colsum", &spa::act_bwd_colsum);
  m.impl("glu_fwd", &spa::glu_fwd);
  m.impl("glu_bwd", &spa::glu_bwd);
}
