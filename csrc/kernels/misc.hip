// Smaller paper-specific ops of the catalogue, each fwd + bwd, fp32 math, bf16/fp32 I/O.
//
//  dropout      counter-hash RNG (mask regenerated in bwd, never stored)   K22
//               gpt/gpt-jax.ipynb:351,356,387,467; gemma/gemma.ipynb:235,248,258; alexnet/alexnet.py:31,34
//  kd_loss      alpha*CE(s,y) + (1-alpha)*T^2*KL(softmax(t/T)||log_softmax(s/T)), batchmean   K17
//               knowledge distillation/kd.py:48-68 (gradient written during fwd, one block per row)
//  vae          reparameterise z = mu + eps*exp(logvar/2) (hash-normal eps) and the fused
//               BCE(sum) + KL loss with its gradients          K18   autoencoder/variational autoencoder.ipynb:94-120
//  mse          mean squared error + grad                      K19   autoencoder/autoencoder.ipynb:98
//  lrn          LocalResponseNorm(size, alpha, beta, k) NCHW   K21   alexnet/alexnet.py:13,18
//  maxpool2d    kernel/stride, argmax indices, scatter bwd    K21   alexnet/alexnet.py:14,19,27
//  im2col       NCHW image -> [N*OH*OW, C*KH*KW] rows for the conv-as-GEMM path, col2im
//               bwd (gather form, no atomics); k == stride == patch gives ViT patchify  K20
//  luong        global dot attention: w = softmax_s <st, h_s>, ctx = sum_s w h_s   K05
//               attention/luong.ipynb:22-36
#include "spa_common.h"

namespace spa {

// --------------------------------------------------------------------------- RNG
__device__ __forceinline__ uint32_t mix32(uint64_t k) {
  k ^= k >> 33; k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return (uint32_t)k;
}
__device__ __forceinline__ float u01(uint64_t seed, uint64_t i) {  // (0, 1]
  return ((float)(mix32(seed * 0x9E3779B97F4A7C15ULL + i) >> 8) + 1.f) * (1.f / 16777216.f);
}

// --------------------------------------------------------------------------- dropout
// 8 elements per thread per step (16-byte bf16 / 2 x 16-byte fp32 vectors); the keep bit of
// element i is a 32-bit counter hash of (seed, i) -- ~10 integer ops, so the kernel stays on the
// HBM roof (a 64-bit mix per element made it VALU-bound at 3.2 TB/s).
__device__ __forceinline__ unsigned hash32(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ bool drop_keep_elem(unsigned base, unsigned hi_mix, long i, unsigned thr) {
  return (hash32(base + (unsigned)i * 0x9E3779B1U + hi_mix) >> 8) >= thr;
}
template <typename T>
__global__ __launch_bounds__(256) void dropout_kernel(const T* __restrict__ x, T* __restrict__ y, long n, float p,
                                                      uint64_t seed, const int64_t* __restrict__ seed_ptr, bool vec) {
  if (seed_ptr) seed = (uint64_t)*seed_ptr;   // device seed: fresh mask per HIP-graph replay
  const unsigned base = hash32((unsigned)seed ^ 0x5bd1e995U), shi = (unsigned)(seed >> 32);
  const unsigned thr = (unsigned)(p * 16777216.f);
  const float scale = 1.f / (1.f - p);
  const long nv = vec ? n / 8 : 0;
  for (long v = blockIdx.x * 256L + threadIdx.x; v < nv; v += (long)gridDim.x * 256) {
    const long i0 = v * 8;
    const unsigned hm = hash32(shi + (unsigned)(i0 >> 32) * 0x85EBCA6BU);
    float f[8];
    load8(x + i0, f);
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] = drop_keep_elem(base, hm, i0 + k, thr) ? f[k] * scale : 0.f;
    store8(y + i0, f);
  }
  for (long i = nv * 8 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const unsigned hm = hash32(shi + (unsigned)(i >> 32) * 0x85EBCA6BU);
    y[i] = (T)(drop_keep_elem(base, hm, i, thr) ? (float)x[i] * scale : 0.f);
  }
}
at::Tensor dropout_apply(const at::Tensor& x_, double p, int64_t seed, const c10::optional<at::Tensor>& seed_t) {
  SPA_CHECK_CUDA(x_);
  if (seed_t) TORCH_CHECK(seed_t->scalar_type() == at::kLong && seed_t->is_cuda() && seed_t->numel() >= 1);
  const int64_t* sp = seed_t ? seed_t->data_ptr<int64_t>() : nullptr;
  auto x = dense(x_);
  auto y = at::empty_like(x);
  const long n = x.numel();
  if (n == 0) return y;
  const bool vec = (uintptr_t)x.data_ptr() % 32 == 0;   // y is fresh (allocator-aligned); views may not be
  DeviceGuard g(x.device());
  const int grid = (int)std::max<long>(1, std::min<long>((n / 8 + 255) / 256, 4096));
  if (x.scalar_type() == at::kBFloat16)
    dropout_kernel<bf16><<<grid, 256, 0, stream()>>>((const bf16*)x.data_ptr(), (bf16*)y.data_ptr(), n, (float)p, seed, sp, vec);
  else if (x.scalar_type() == at::kFloat)
    dropout_kernel<float><<<grid, 256, 0, stream()>>>(x.data_ptr<float>(), y.data_ptr<float>(), n, (float)p, seed, sp, vec);
  else TORCH_CHECK(false, "dropout: bf16/fp32 only");
  SPA_LAUNCH_CHECK();
  return y;
}


// --------------------------------------------------------------------------- kd loss
// per row: hard = lse(s) - s[y]; soft = sum_c p_c (log p_c - log q_c), p = softmax(t/T), q = softmax(s/T)
// grad (in place into gs): alpha/B (softmax(s) - onehot) + (1-alpha) T / B (q - p)
// One WAVE per row with the row held in registers (VPL values of s and of t per lane, C <= 64 VPL):
// one HBM read of each input, three online (max, sum-exp) pairs, wave reductions only -- the
// reference shape (C = 10) leaves no 256-thread block idle, and C = 1000 reads each row once.
template <typename T, int VPL>
__global__ __launch_bounds__(256) void kd_wave_kernel(const T* __restrict__ s, const T* __restrict__ t,
                                                      const int64_t* __restrict__ y, float* __restrict__ hard,
                                                      float* __restrict__ soft, T* __restrict__ gs, int B, int C,
                                                      float invT, float alpha, float invB) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= B) return;
  const T* sr = s + (long)row * C;
  const T* tr = t + (long)row * C;
  float a[VPL], b[VPL];
  float m1 = -INFINITY, m2 = -INFINITY, m3 = -INFINITY;
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int c = lane + 64 * v;
    a[v] = c < C ? (float)sr[c] : -INFINITY;
    b[v] = c < C ? (float)tr[c] : -INFINITY;
    m1 = fmaxf(m1, a[v]);
    m3 = fmaxf(m3, b[v]);
  }
  m1 = wave_max(m1);
  m3 = wave_max(m3) * invT;
  m2 = m1 * invT;  // T > 0: max(s/T) = max(s)/T
  float z1 = 0.f, z2 = 0.f, z3 = 0.f;
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    if (lane + 64 * v < C) {
      z1 += __expf(a[v] - m1);
      z2 += __expf(a[v] * invT - m2);
      z3 += __expf(b[v] * invT - m3);
    }
  }
  z1 = wave_sum(z1); z2 = wave_sum(z2); z3 = wave_sum(z3);
  const float l1 = m1 + __logf(z1), l2 = m2 + __logf(z2), l3 = m3 + __logf(z3);
  const int64_t yy = y[row];
  float kl = 0.f, sy = 0.f;
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int c = lane + 64 * v;
    if (c < C) {
      const float lp = b[v] * invT - l3, lq = a[v] * invT - l2;
      const float pc = __expf(lp);
      kl += pc * (lp - lq);
      if (c == yy) sy = a[v];
      if (gs) {
        const float g = alpha * invB * (__expf(a[v] - l1) - (c == yy ? 1.f : 0.f)) +
                        (1.f - alpha) * invB / invT * (__expf(lq) - pc);
        gs[(long)row * C + c] = (T)g;
      }
    }
  }
  kl = wave_sum(kl);
  sy = wave_sum(sy);
  if (lane == 0) {
    hard[row] = l1 - sy;
    soft[row] = kl;
  }
}

// tiny rows (C <= 16, the reference's 10-class heads): one LANE per row, the row in registers,
// no cross-lane reductions at all -- a wave per row would idle 54 of 64 lanes and spend its time
// in shuffles.
template <typename T, int CM>
__global__ __launch_bounds__(256) void kd_lane_kernel(const T* __restrict__ s, const T* __restrict__ t,
                                                      const int64_t* __restrict__ y, float* __restrict__ hard,
                                                      float* __restrict__ soft, T* __restrict__ gs, int B, int C,
                                                      float invT, float alpha, float invB) {
  const int row = blockIdx.x * 256 + threadIdx.x;
  if (row >= B) return;
  const T* sr = s + (long)row * C;
  const T* tr = t + (long)row * C;
  float a[CM], b[CM];
  float m1 = -INFINITY, m3 = -INFINITY;
#pragma unroll
  for (int c = 0; c < CM; ++c) {
    a[c] = c < C ? (float)sr[c] : -INFINITY;
    b[c] = c < C ? (float)tr[c] : -INFINITY;
    m1 = fmaxf(m1, a[c]);
    m3 = fmaxf(m3, b[c]);
  }
  const float m2 = m1 * invT;
  m3 *= invT;
  float z1 = 0.f, z2 = 0.f, z3 = 0.f;
#pragma unroll
  for (int c = 0; c < CM; ++c)
    if (c < C) {
      z1 += __expf(a[c] - m1);
      z2 += __expf(a[c] * invT - m2);
      z3 += __expf(b[c] * invT - m3);
    }
  const float l1 = m1 + __logf(z1), l2 = m2 + __logf(z2), l3 = m3 + __logf(z3);
  const int64_t yy = y[row];
  float kl = 0.f, sy = 0.f;
#pragma unroll
  for (int c = 0; c < CM; ++c)
    if (c < C) {
      const float lp = b[c] * invT - l3, lq = a[c] * invT - l2;
      const float pc = __expf(lp);
      kl += pc * (lp - lq);
      if (c == yy) sy = a[c];
      if (gs)
        gs[(long)row * C + c] = (T)(alpha * invB * (__expf(a[c] - l1) - (c == yy ? 1.f : 0.f)) +
                                    (1.f - alpha) * invB / invT * (__expf(lq) - pc));
    }
  hard[row] = l1 - sy;
  soft[row] = kl;
}

// rows wider than 64 x 32 values: one block per row, three passes (the general fallback)
template <typename T>
__global__ __launch_bounds__(256) void kd_kernel(const T* __restrict__ s, const T* __restrict__ t,
                                                 const int64_t* __restrict__ y, float* __restrict__ hard,
                                                 float* __restrict__ soft, T* __restrict__ gs, int C, float invT,
                                                 float alpha, float invB) {
  __shared__ float red[4];
  const int row = blockIdx.x;
  const T* sr = s + (long)row * C;
  const T* tr = t + (long)row * C;
  float m1 = -INFINITY, m2 = -INFINITY, m3 = -INFINITY;
  for (int c = threadIdx.x; c < C; c += 256) {
    const float a = (float)sr[c], b = (float)tr[c];
    m1 = fmaxf(m1, a); m2 = fmaxf(m2, a * invT); m3 = fmaxf(m3, b * invT);
  }
  m1 = block_max<256>(m1, red); __syncthreads();
  m2 = block_max<256>(m2, red); __syncthreads();
  m3 = block_max<256>(m3, red); __syncthreads();
  float z1 = 0.f, z2 = 0.f, z3 = 0.f;
  for (int c = threadIdx.x; c < C; c += 256) {
    const float a = (float)sr[c], b = (float)tr[c];
    z1 += __expf(a - m1); z2 += __expf(a * invT - m2); z3 += __expf(b * invT - m3);
  }
  z1 = block_sum<256>(z1, red); __syncthreads();
  z2 = block_sum<256>(z2, red); __syncthreads();
  z3 = block_sum<256>(z3, red); __syncthreads();
  const float l1 = m1 + __logf(z1), l2 = m2 + __logf(z2), l3 = m3 + __logf(z3);
  float kl = 0.f;
  for (int c = threadIdx.x; c < C; c += 256) {
    const float a = (float)sr[c], b = (float)tr[c];
    const float lp = b * invT - l3, lq = a * invT - l2;
    const float pc = __expf(lp);
    kl += pc * (lp - lq);
    if (gs) {
      const float sm = __expf(a - l1);
      const float g = alpha * invB * (sm - (c == y[row] ? 1.f : 0.f)) +
                      (1.f - alpha) * invB / invT * (__expf(lq) - pc);
      gs[(long)row * C + c] = (T)g;
    }
  }
  kl = block_sum<256>(kl, red);
  if (threadIdx.x == 0) {
    hard[row] = l1 - (float)sr[y[row]];
    soft[row] = kl;
  }
}
// returns (hard[B], soft[B], grad_s or empty)
std::vector<at::Tensor> kd_loss_fwd(const at::Tensor& s_, const at::Tensor& t_, const at::Tensor& y, double T,
                                    double alpha, bool want_grad) {
  auto s = s_.contiguous(), t = t_.contiguous();
  TORCH_CHECK(s.dim() == 2 && t.sizes() == s.sizes() && s.scalar_type() == t.scalar_type());
  TORCH_CHECK(y.scalar_type() == at::kLong && y.numel() == s.size(0));
  const int B = s.size(0), C = s.size(1);
  DeviceGuard g(s.device());
  auto opts = s.options().dtype(at::kFloat);
  auto hard = at::empty({B}, opts), soft = at::empty({B}, opts);
  auto gs = want_grad ? at::empty_like(s) : at::Tensor();
  if (B == 0) return {hard, soft, gs};
  auto yc = y.contiguous();
  TORCH_CHECK(T > 0, "kd_loss: temperature must be positive");
#define KDW(TT, V)                                                                                            \
  (kd_wave_kernel<TT, V>)<<<cdiv(B, 4), 256, 0, stream()>>>(                                                     \
      (const TT*)s.data_ptr(), (const TT*)t.data_ptr(), yc.data_ptr<int64_t>(), hard.data_ptr<float>(),       \
      soft.data_ptr<float>(), want_grad ? (TT*)gs.data_ptr() : nullptr, B, C, (float)(1.0 / T), (float)alpha, \
      1.f / B)
#define KDL(TT)                                                                                              \
  if (C <= 16) (kd_lane_kernel<TT, 16>)<<<cdiv(B, 256), 256, 0, stream()>>>(                                   \
      (const TT*)s.data_ptr(), (const TT*)t.data_ptr(), yc.data_ptr<int64_t>(), hard.data_ptr<float>(),       \
      soft.data_ptr<float>(), want_grad ? (TT*)gs.data_ptr() : nullptr, B, C, (float)(1.0 / T), (float)alpha, \
      1.f / B);                                                                                               \
  else if (C <= 64) KDW(TT, 1);                                                                                   \
  else if (C <= 256) KDW(TT, 4);                                                                             \
  else if (C <= 1024) KDW(TT, 16);                                                                           \
  else if (C <= 2048) KDW(TT, 32);                                                                           \
  else (kd_kernel<TT>)<<<B, 256, 0, stream()>>>((const TT*)s.data_ptr(), (const TT*)t.data_ptr(),              \
                                              yc.data_ptr<int64_t>(), hard.data_ptr<float>(),                 \
                                              soft.data_ptr<float>(), want_grad ? (TT*)gs.data_ptr() : nullptr, \
                                              C, (float)(1.0 / T), (float)alpha, 1.f / B)
  if (s.scalar_type() == at::kBFloat16) { KDL(bf16); } else { KDL(float); }
#undef KDL
#undef KDW
  SPA_LAUNCH_CHECK();
  return {hard, soft, gs};
}

// --------------------------------------------------------------------------- VAE
__device__ __forceinline__ float randn(uint64_t seed, uint64_t i) {  // Box-Muller on two hashed uniforms
  const float u1 = u01(seed, 2 * i), u2 = u01(seed, 2 * i + 1);
  return sqrtf(-2.f * __logf(u1)) * __cosf(6.283185307179586f * u2);
}
template <typename T>
__global__ __launch_bounds__(256) void reparam_kernel(const T* __restrict__ mu, const T* __restrict__ lv,
                                                      const T* __restrict__ dz, T* __restrict__ out,
                                                      T* __restrict__ dlv, long n, uint64_t seed) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float e = randn(seed, i);
    const float sd = __expf(0.5f * (float)lv[i]);
    if (dz == nullptr) out[i] = (T)((float)mu[i] + e * sd);                  // fwd: z
    else dlv[i] = (T)((float)dz[i] * e * 0.5f * sd);                        // bwd: dlogvar (dmu = dz)
  }
}
at::Tensor vae_reparam(const at::Tensor& mu_, const at::Tensor& lv_, const c10::optional<at::Tensor>& dz_,
                       int64_t seed) {
  auto mu = mu_.contiguous(), lv = lv_.contiguous();
  TORCH_CHECK(mu.sizes() == lv.sizes() && mu.scalar_type() == lv.scalar_type());
  DeviceGuard g(mu.device());
  auto out = at::empty_like(mu);
  const long n = mu.numel();
  if (n == 0) return out;
  at::Tensor dz = dz_ ? dz_->contiguous() : at::Tensor();
  const int grid = (int)std::min<long>((n + 255) / 256, 8192);
#define RPL(TT)                                                                                     \
  reparam_kernel<TT><<<grid, 256, 0, stream()>>>((const TT*)mu.data_ptr(), (const TT*)lv.data_ptr(), \
                                                 dz_ ? (const TT*)dz.data_ptr() : nullptr,           \
                                                 (TT*)out.data_ptr(), (TT*)out.data_ptr(), n, seed)
  if (mu.scalar_type() == at::kBFloat16) RPL(bf16); else RPL(float);
#undef RPL
  SPA_LAUNCH_CHECK();
  return out;
}

// fused VAE loss: sum BCE(r, x) + -0.5 sum(1 + lv - mu^2 - e^lv); grads dr, dmu, dlv (unscaled)
template <typename T>
__global__ __launch_bounds__(256) void vae_loss_kernel(const T* __restrict__ r, const T* __restrict__ x, long n,
                                                       const T* __restrict__ mu, const T* __restrict__ lv, long m,
                                                       float* __restrict__ part, T* __restrict__ dr,
                                                       T* __restrict__ dmu, T* __restrict__ dlv) {
  __shared__ float red[4];
  float bce = 0.f, kl = 0.f;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float rv = (float)r[i], xv = (float)x[i];
    const float lr = fmaxf(__logf(rv), -100.f), l1r = fmaxf(__logf(1.f - rv), -100.f);  // torch clamps log at -100
    bce -= xv * lr + (1.f - xv) * l1r;
    dr[i] = (T)((rv - xv) / fmaxf(rv * (1.f - rv), 1e-12f));
  }
  for (long i = blockIdx.x * 256L + threadIdx.x; i < m; i += (long)gridDim.x * 256) {
    const float a = (float)mu[i], b = (float)lv[i], e = __expf(b);
    kl += -0.5f * (1.f + b - a * a - e);
    dmu[i] = (T)a;
    dlv[i] = (T)(0.5f * (e - 1.f));
  }
  bce = block_sum<256>(bce, red);
  __syncthreads();
  kl = block_sum<256>(kl, red);
  if (threadIdx.x == 0) { part[2 * blockIdx.x] = bce; part[2 * blockIdx.x + 1] = kl; }
}
// returns (bce_sum[1], kl_sum[1], dr, dmu, dlv)
std::vector<at::Tensor> vae_loss_fwd(const at::Tensor& r_, const at::Tensor& x_, const at::Tensor& mu_,
                                     const at::Tensor& lv_) {
  auto r = r_.contiguous(), x = x_.contiguous(), mu = mu_.contiguous(), lv = lv_.contiguous();
  TORCH_CHECK(r.sizes() == x.sizes() && mu.sizes() == lv.sizes());
  TORCH_CHECK(r.scalar_type() == x.scalar_type() && mu.scalar_type() == r.scalar_type());
  DeviceGuard g(r.device());
  const long n = r.numel(), m = mu.numel();
  const int nb = (int)std::max<long>(1, std::min<long>((std::max(n, m) + 255) / 256, 1024));
  auto part = at::zeros({nb, 2}, r.options().dtype(at::kFloat));
  auto dr = at::empty_like(r), dmu = at::empty_like(mu), dlv = at::empty_like(lv);
#define VL(TT)                                                                                              \
  vae_loss_kernel<TT><<<nb, 256, 0, stream()>>>((const TT*)r.data_ptr(), (const TT*)x.data_ptr(), n,         \
                                                (const TT*)mu.data_ptr(), (const TT*)lv.data_ptr(), m,       \
                                                part.data_ptr<float>(), (TT*)dr.data_ptr(), (TT*)dmu.data_ptr(), \
                                                (TT*)dlv.data_ptr())
  if (r.scalar_type() == at::kBFloat16) VL(bf16); else VL(float);
#undef VL
  SPA_LAUNCH_CHECK();
  auto sums = part.sum(0);
  return {sums.narrow(0, 0, 1), sums.narrow(0, 1, 1), dr, dmu, dlv};
}

// --------------------------------------------------------------------------- MSE
template <typename T>
__global__ __launch_bounds__(256) void mse_kernel(const T* __restrict__ a, const T* __restrict__ b, long n,
                                                  float* __restrict__ part, T* __restrict__ ga, float gscale) {
  __shared__ float red[4];
  float acc = 0.f;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float d = (float)a[i] - (float)b[i];
    acc += d * d;
    if (ga) ga[i] = (T)(gscale * d);
  }
  acc = block_sum<256>(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}
// returns (sum_sq[1], grad_a = 2(a-b)/n or empty)
std::vector<at::Tensor> mse_fwd(const at::Tensor& a_, const at::Tensor& b_, bool want_grad) {
  auto a = a_.contiguous(), b = b_.contiguous();
  TORCH_CHECK(a.sizes() == b.sizes() && a.scalar_type() == b.scalar_type());
  DeviceGuard g(a.device());
  const long n = a.numel();
  const int nb = (int)std::max<long>(1, std::min<long>((n + 255) / 256, 1024));
  auto part = at::zeros({nb}, a.options().dtype(at::kFloat));
  auto ga = want_grad ? at::empty_like(a) : at::Tensor();
#define ML(TT)                                                                                            \
  mse_kernel<TT><<<nb, 256, 0, stream()>>>((const TT*)a.data_ptr(), (const TT*)b.data_ptr(), n,            \
                                           part.data_ptr<float>(), want_grad ? (TT*)ga.data_ptr() : nullptr, \
                                           2.f / (float)std::max<long>(n, 1))
  if (a.scalar_type() == at::kBFloat16) ML(bf16); else ML(float);
#undef ML
  SPA_LAUNCH_CHECK();
  return {part.sum().reshape({1}), ga};
}

// --------------------------------------------------------------------------- LRN (NCHW or channels-last)
// b_c = a_c * s_c^-beta, s_c = k + alpha/n * sum_{c' in [c-(n-1)/2, c+n/2]} a_c'^2   (torch convention)
// i walks the storage; cs is the channel stride (H*W for NCHW, 1 for NHWC): c = (i / cs) % C and
// channel j of the same pixel sits at i + (j - c) * cs.
template <typename T>
__global__ __launch_bounds__(256) void lrn_fwd_kernel(const T* __restrict__ a, T* __restrict__ b,
                                                      float* __restrict__ sc, long total, int C, long cs, int size,
                                                      float alpha, float beta, float k) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c = (i / cs) % C;
    const int lo = max(0, c - size / 2), hi = min(C - 1, c + (size - 1) / 2);
    float ss = 0.f;
    for (int j = lo; j <= hi; ++j) { const float v = (float)a[i + (j - c) * cs]; ss += v * v; }
    const float s = k + alpha / size * ss;
    sc[i] = s;
    b[i] = (T)((float)a[i] * __powf(s, -beta));
  }
}
// da_c = dy_c s_c^-beta - 2 alpha beta / n * a_c * sum_{c': c in window(c')} dy_c' a_c' s_c'^(-beta-1)
template <typename T>
__global__ __launch_bounds__(256) void lrn_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ a,
                                                      const float* __restrict__ sc, T* __restrict__ da, long total,
                                                      int C, long cs, int size, float alpha, float beta) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c = (i / cs) % C;
    // c' whose window contains c: c' - size/2 <= c <= c' + (size-1)/2
    const int lo = max(0, c - (size - 1) / 2), hi = min(C - 1, c + size / 2);
    float acc = 0.f;
    for (int j = lo; j <= hi; ++j) {
      const long o = i + (j - c) * cs;
      acc += (float)dy[o] * (float)a[o] * __powf(sc[o], -beta - 1.f);
    }
    da[i] = (T)((float)dy[i] * __powf(sc[i], -beta) - 2.f * alpha * beta / size * (float)a[i] * acc);
  }
}
static bool channels_last(const at::Tensor& t) {
  return t.dim() == 4 && !t.is_contiguous() && t.is_contiguous(at::MemoryFormat::ChannelsLast);
}
std::vector<at::Tensor> lrn_fwd(const at::Tensor& a_, int64_t size, double alpha, double beta, double k) {
  TORCH_CHECK(a_.dim() == 4, "lrn: 4-D input");
  const bool cl = channels_last(a_);
  auto a = cl ? a_ : a_.contiguous();
  DeviceGuard g(a.device());
  auto b = at::empty_like(a);
  auto sc = at::empty_like(a, a.options().dtype(at::kFloat));
  const long total = a.numel();
  if (total == 0) return {b, sc};
  const long cs = cl ? 1 : a.size(2) * a.size(3);
  const int grid = (int)std::min<long>((total + 255) / 256, 8192);
#define LF(TT)                                                                                                \
  lrn_fwd_kernel<TT><<<grid, 256, 0, stream()>>>((const TT*)a.data_ptr(), (TT*)b.data_ptr(), sc.data_ptr<float>(), \
                                                 total, a.size(1), cs, size, alpha, beta, k)
  if (a.scalar_type() == at::kBFloat16) LF(bf16); else LF(float);
#undef LF
  SPA_LAUNCH_CHECK();
  return {b, sc};
}
at::Tensor lrn_bwd(const at::Tensor& dy_, const at::Tensor& a_, const at::Tensor& sc, int64_t size, double alpha,
                   double beta) {
  const bool cl = channels_last(a_);
  const auto fmt = cl ? at::MemoryFormat::ChannelsLast : at::MemoryFormat::Contiguous;
  auto a = a_.contiguous(fmt), dy = dy_.contiguous(fmt);
  TORCH_CHECK(sc.is_contiguous(fmt), "lrn_bwd: scale layout");
  DeviceGuard g(a.device());
  auto da = at::empty_like(a);
  const long total = a.numel();
  if (total == 0) return da;
  const long cs = cl ? 1 : a.size(2) * a.size(3);
  const int grid = (int)std::min<long>((total + 255) / 256, 8192);
#define LB(TT)                                                                                                  \
  lrn_bwd_kernel<TT><<<grid, 256, 0, stream()>>>((const TT*)dy.data_ptr(), (const TT*)a.data_ptr(),              \
                                                 sc.data_ptr<float>(), (TT*)da.data_ptr(), total, a.size(1), cs, \
                                                 size, alpha, beta)
  if (a.scalar_type() == at::kBFloat16) LB(bf16); else LB(float);
#undef LB
  SPA_LAUNCH_CHECK();
  return da;
}

// --------------------------------------------------------------------------- maxpool2d (NCHW or NHWC, no padding)
// i walks the output storage; arg holds h * W + w of the window max (first max, NaN wins)
template <typename T, bool NHWC>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                          int* __restrict__ arg, int N, int C, int H, int W, int OH,
                                                          int OW, int ks, int st) {
  const long total = (long)N * C * OH * OW;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    int c, ow, oh;
    long n;
    if (NHWC) { c = i % C; ow = (i / C) % OW; oh = (i / ((long)C * OW)) % OH; n = i / ((long)C * OW * OH); }
    else { ow = i % OW; oh = (i / OW) % OH; c = (i / ((long)OW * OH)) % C; n = i / ((long)OW * OH * C); }
    // element (h, w) of this (n, c) plane: x[pb + (h * W + w) * ps]
    const long pb = NHWC ? n * H * W * C + c : (n * C + c) * H * W;
    const int ps = NHWC ? C : 1;
    float best = -INFINITY;
    int bi = 0;
    for (int r = 0; r < ks; ++r)
      for (int q = 0; q < ks; ++q) {
        const int hw = (oh * st + r) * W + ow * st + q;
        const float v = (float)x[pb + (long)hw * ps];
        if (v > best || (v != v)) { best = v; bi = hw; }
      }
    y[i] = (T)best;
    arg[i] = bi;
  }
}
// gather-form backward: each input pixel sums the gradients of the windows whose argmax it is
template <typename T, bool NHWC>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const T* __restrict__ dy, const int* __restrict__ arg,
                                                          T* __restrict__ dx, int N, int C, int H, int W, int OH,
                                                          int OW, int ks, int st) {
  const long total = (long)N * C * H * W;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    int c, w, h;
    long n;
    if (NHWC) { c = i % C; w = (i / C) % W; h = (i / ((long)C * W)) % H; n = i / ((long)C * W * H); }
    else { w = i % W; h = (i / W) % H; c = (i / ((long)W * H)) % C; n = i / ((long)W * H * C); }
    const long ob = NHWC ? n * OH * OW * C + c : (n * C + c) * OH * OW;
    const int os = NHWC ? C : 1;
    const int oh0 = max(0, (h - ks + st) / st), oh1 = min(OH - 1, h / st);
    const int ow0 = max(0, (w - ks + st) / st), ow1 = min(OW - 1, w / st);
    float acc = 0.f;
    for (int oh = oh0; oh <= oh1; ++oh)
      for (int ow = ow0; ow <= ow1; ++ow) {
        const long o = ob + (long)(oh * OW + ow) * os;
        if (arg[o] == h * W + w) acc += (float)dy[o];
      }
    dx[i] = (T)acc;
  }
}
std::vector<at::Tensor> maxpool2d_fwd(const at::Tensor& x_, int64_t ks, int64_t st) {
  TORCH_CHECK(x_.dim() == 4, "maxpool2d: 4-D input");
  const bool cl = channels_last(x_);
  const auto fmt = cl ? at::MemoryFormat::ChannelsLast : at::MemoryFormat::Contiguous;
  auto x = x_.contiguous(fmt);
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int OH = (H - ks) / st + 1, OW = (W - ks) / st + 1;
  DeviceGuard g(x.device());
  auto y = at::empty({N, C, OH, OW}, x.options().memory_format(fmt));
  auto arg = at::empty({N, C, OH, OW}, x.options().dtype(at::kInt).memory_format(fmt));
  const long total = (long)N * C * OH * OW;
  if (total == 0) return {y, arg};
  const int grid = (int)std::min<long>((total + 255) / 256, 8192);
#define MP(TT, L)                                                                                   \
  maxpool_fwd_kernel<TT, L><<<grid, 256, 0, stream()>>>((const TT*)x.data_ptr(), (TT*)y.data_ptr(), \
                                                        arg.data_ptr<int>(), N, C, H, W, OH, OW, ks, st)
  if (x.scalar_type() == at::kBFloat16) { if (cl) MP(bf16, true); else MP(bf16, false); }
  else { if (cl) MP(float, true); else MP(float, false); }
#undef MP
  SPA_LAUNCH_CHECK();
  return {y, arg};
}
at::Tensor maxpool2d_bwd(const at::Tensor& dy_, const at::Tensor& arg, int64_t H, int64_t W, int64_t ks,
                         int64_t st) {
  const bool cl = channels_last(arg);
  const auto fmt = cl ? at::MemoryFormat::ChannelsLast : at::MemoryFormat::Contiguous;
  TORCH_CHECK(arg.is_contiguous(fmt), "maxpool2d_bwd: argmax layout");
  auto dy = dy_.contiguous(fmt);
  const int N = dy.size(0), C = dy.size(1), OH = dy.size(2), OW = dy.size(3);
  DeviceGuard g(dy.device());
  auto dx = at::empty({N, C, H, W}, dy.options().memory_format(fmt));
  const long total = (long)N * C * H * W;
  if (total == 0) return dx;
  const int grid = (int)std::min<long>((total + 255) / 256, 8192);
#define MB(TT, L)                                                                                   \
  maxpool_bwd_kernel<TT, L><<<grid, 256, 0, stream()>>>((const TT*)dy.data_ptr(), arg.data_ptr<int>(), \
                                                        (TT*)dx.data_ptr(), N, C, H, W, OH, OW, ks, st)
  if (dy.scalar_type() == at::kBFloat16) { if (cl) MB(bf16, true); else MB(bf16, false); }
  else { if (cl) MB(float, true); else MB(float, false); }
#undef MB
  SPA_LAUNCH_CHECK();
  return dx;
}

// --------------------------------------------------------------------------- im2col / col2im (NCHW)
// cols row r = (n, oh, ow), column q = (c, kh, kw)
template <typename T>
__global__ __launch_bounds__(256) void im2col_kernel(const T* __restrict__ x, T* __restrict__ cols, int N, int C,
                                                     int H, int W, int KH, int KW, int sh, int sw, int ph, int pw,
                                                     int OH, int OW) {
  const long K = (long)C * KH * KW;
  const long total = (long)N * OH * OW * K;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long q = i % K, r = i / K;
    const int kw = q % KW, kh = (q / KW) % KH, c = q / (KW * KH);
    const int ow = r % OW, oh = (r / OW) % OH, n = r / (OW * OH);
    const int h = oh * sh - ph + kh, w = ow * sw - pw + kw;
    cols[i] = (h >= 0 && h < H && w >= 0 && w < W) ? x[(((long)n * C + c) * H + h) * W + w] : (T)0.f;
  }
}
// gather: every input pixel sums the column entries that read it (no atomics, deterministic)
template <typename T>
__global__ __launch_bounds__(256) void col2im_kernel(const T* __restrict__ cols, T* __restrict__ dx, int N, int C,
                                                     int H, int W, int KH, int KW, int sh, int sw, int ph, int pw,
                                                     int OH, int OW) {
  const long K = (long)C * KH * KW;
  const long total = (long)N * C * H * W;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int w = i % W, h = (i / W) % H, c = (i / ((long)W * H)) % C, n = i / ((long)W * H * C);
    float acc = 0.f;
    for (int kh = 0; kh < KH; ++kh) {
      const int t = h + ph - kh;
      if (t < 0 || t % sh) continue;
      const int oh = t / sh;
      if (oh >= OH) continue;
      for (int kw = 0; kw < KW; ++kw) {
        const int u = w + pw - kw;
        if (u < 0 || u % sw) continue;
        const int ow = u / sw;
        if (ow >= OW) continue;
        acc += (float)cols[(((long)n * OH + oh) * OW + ow) * K + ((long)c * KH + kh) * KW + kw];
      }
    }
    dx[i] = (T)acc;
  }
}
at::Tensor im2col(const at::Tensor& x_, int64_t KH, int64_t KW, int64_t sh, int64_t sw, int64_t ph, int64_t pw) {
  auto x = x_.contiguous();
  TORCH_CHECK(x.dim() == 4, "im2col: NCHW input");
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int OH = (H + 2 * ph - KH) / sh + 1, OW = (W + 2 * pw - KW) / sw + 1;
  DeviceGuard g(x.device());
  auto cols = at::empty({(long)N * OH * OW, (long)C * KH * KW}, x.options());
  const long total = cols.numel();
  if (total == 0) return cols;
  const int grid = (int)std::min<long>((total + 255) / 256, 16384);
#define IC_(TT)                                                                                          \
  im2col_kernel<TT><<<grid, 256, 0, stream()>>>((const TT*)x.data_ptr(), (TT*)cols.data_ptr(), N, C, H, W, KH, \
                                                KW, sh, sw, ph, pw, OH, OW)
  if (x.scalar_type() == at::kBFloat16) IC_(bf16); else IC_(float);
#undef IC_
  SPA_LAUNCH_CHECK();
  return cols;
}
at::Tensor col2im(const at::Tensor& cols_, int64_t N, int64_t C, int64_t H, int64_t W, int64_t KH, int64_t KW,
                  int64_t sh, int64_t sw, int64_t ph, int64_t pw) {
  auto cols = cols_.contiguous();
  const int OH = (H + 2 * ph - KH) / sh + 1, OW = (W + 2 * pw - KW) / sw + 1;
  TORCH_CHECK(cols.size(0) == N * OH * OW && cols.size(1) == C * KH * KW, "col2im: shape mismatch");
  DeviceGuard g(cols.device());
  auto dx = at::empty({N, C, H, W}, cols.options());
  const long total = dx.numel();
  if (total == 0) return dx;
  const int grid = (int)std::min<long>((total + 255) / 256, 16384);
#define CI(TT)                                                                                            \
  col2im_kernel<TT><<<grid, 256, 0, stream()>>>((const TT*)cols.data_ptr(), (TT*)dx.data_ptr(), N, C, H, W, KH, \
                                                KW, sh, sw, ph, pw, OH, OW)
  if (cols.scalar_type() == at::kBFloat16) CI(bf16); else CI(float);
#undef CI
  SPA_LAUNCH_CHECK();
  return dx;
}

// --------------------------------------------------------------------------- Luong attention
// st [B, H], hs [B, S, H] -> ctx [B, H], w [B, S]. One block per batch row.
template <typename T>
__global__ __launch_bounds__(256) void luong_fwd_kernel(const T* __restrict__ st, const T* __restrict__ hs,
                                                        T* __restrict__ ctx, float* __restrict__ wout, int S, int H) {
  extern __shared__ float sm[];  // S scores
  __shared__ float red[4];
  const int b = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const T* hb = hs + (long)b * S * H;
  const T* sb = st + (long)b * H;
  for (int s = wv; s < S; s += 4) {  // one wave per key position
    float acc = 0.f;
    for (int h = lane; h < H; h += 64) acc += (float)sb[h] * (float)hb[(long)s * H + h];
    acc = wave_sum(acc);
    if (lane == 0) sm[s] = acc;
  }
  __syncthreads();
  float m = -INFINITY;
  for (int s = threadIdx.x; s < S; s += 256) m = fmaxf(m, sm[s]);
  m = block_max<256>(m, red);
  __syncthreads();
  float z = 0.f;
  for (int s = threadIdx.x; s < S; s += 256) z += __expf(sm[s] - m);
  z = block_sum<256>(z, red);
  __syncthreads();
  for (int s = threadIdx.x; s < S; s += 256) {
    const float w = __expf(sm[s] - m) / z;
    sm[s] = w;
    wout[(long)b * S + s] = w;
  }
  __syncthreads();
  for (int h = threadIdx.x; h < H; h += 256) {
    float acc = 0.f;
    for (int s = 0; s < S; ++s) acc += sm[s] * (float)hb[(long)s * H + h];
    ctx[(long)b * H + h] = (T)acc;
  }
}
// dctx [B,H] -> dw_s = <dctx, h_s>; dscore_s = w_s (dw_s - sum w dw); dst = sum_s dscore_s h_s;
// dh_s = w_s dctx + dscore_s st
template <typename T>
__global__ __launch_bounds__(256) void luong_bwd_kernel(const T* __restrict__ dctx, const T* __restrict__ st,
                                                        const T* __restrict__ hs, const float* __restrict__ w,
                                                        T* __restrict__ dst, T* __restrict__ dhs, int S, int H) {
  extern __shared__ float sm[];  // S dscore
  __shared__ float red[4];
  const int b = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const T* hb = hs + (long)b * S * H;
  const T* db = dctx + (long)b * H;
  const float* wb = w + (long)b * S;
  for (int s = wv; s < S; s += 4) {
    float acc = 0.f;
    for (int h = lane; h < H; h += 64) acc += (float)db[h] * (float)hb[(long)s * H + h];
    acc = wave_sum(acc);
    if (lane == 0) sm[s] = acc;  // dw_s
  }
  __syncthreads();
  float dot = 0.f;
  for (int s = threadIdx.x; s < S; s += 256) dot += wb[s] * sm[s];
  dot = block_sum<256>(dot, red);
  __syncthreads();
  for (int s = threadIdx.x; s < S; s += 256) sm[s] = wb[s] * (sm[s] - dot);
  __syncthreads();
  const T* sb = st + (long)b * H;
  for (int h = threadIdx.x; h < H; h += 256) {
    float acc = 0.f;
    for (int s = 0; s < S; ++s) {
      const float hv = (float)hb[(long)s * H + h];
      acc += sm[s] * hv;
      dhs[((long)b * S + s) * H + h] = (T)(wb[s] * (float)db[h] + sm[s] * (float)sb[h]);
    }
    dst[(long)b * H + h] = (T)acc;
  }
}
std::vector<at::Tensor> luong_fwd(const at::Tensor& st_, const at::Tensor& hs_) {
  auto st = st_.contiguous(), hs = hs_.contiguous();
  TORCH_CHECK(st.dim() == 2 && hs.dim() == 3 && hs.size(0) == st.size(0) && hs.size(2) == st.size(1));
  const int B = hs.size(0), S = hs.size(1), H = hs.size(2);
  TORCH_CHECK(S <= 16384, "luong: S too large for the LDS score buffer");
  DeviceGuard g(st.device());
  auto ctx = at::empty({B, H}, st.options());
  auto w = at::empty({B, S}, st.options().dtype(at::kFloat));
  if (B == 0) return {ctx, w};
#define LUF(TT)                                                                                           \
  luong_fwd_kernel<TT><<<B, 256, S * sizeof(float), stream()>>>((const TT*)st.data_ptr(), (const TT*)hs.data_ptr(), \
                                                                (TT*)ctx.data_ptr(), w.data_ptr<float>(), S, H)
  if (st.scalar_type() == at::kBFloat16) LUF(bf16); else LUF(float);
#undef LUF
  SPA_LAUNCH_CHECK();
  return {ctx, w};
}
std::vector<at::Tensor> luong_bwd(const at::Tensor& dctx_, const at::Tensor& st_, const at::Tensor& hs_,
                                  const at::Tensor& w) {
  auto dctx = dctx_.contiguous(), st = st_.contiguous(), hs = hs_.contiguous();
  const int B = hs.size(0), S = hs.size(1), H = hs.size(2);
  DeviceGuard g(st.device());
  auto dst = at::empty_like(st), dhs = at::empty_like(hs);
  if (B == 0) return {dst, dhs};
#define LUB(TT)                                                                                                 \
  luong_bwd_kernel<TT><<<B, 256, S * sizeof(float), stream()>>>((const TT*)dctx.data_ptr(), (const TT*)st.data_ptr(), \
                                                                (const TT*)hs.data_ptr(), w.data_ptr<float>(),        \
                                                                (TT*)dst.data_ptr(), (TT*)dhs.data_ptr(), S, H)
  if (st.scalar_type() == at::kBFloat16) LUB(bf16); else LUB(float);
#undef LUB
  SPA_LAUNCH_CHECK();
  return {dst, dhs};
}

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.def("dropout_apply(Tensor x, float p, int seed, Tensor? seed_t=None) -> Tensor");
  m.def("kd_loss_fwd(Tensor s, Tensor t, Tensor y, float T, float alpha, bool want_grad) -> Tensor[]");
  m.def("vae_reparam(Tensor mu, Tensor logvar, Tensor? dz, int seed) -> Tensor");
  m.def("vae_loss_fwd(Tensor r, Tensor x, Tensor mu, Tensor logvar) -> Tensor[]");
  m.def("mse_fwd(Tensor a, Tensor b, bool want_grad) -> Tensor[]");
  m.def("lrn_fwd(Tensor a, int size, float alpha, float beta, float k) -> Tensor[]");
  m.def("lrn_bwd(Tensor dy, Tensor a, Tensor scale, int size, float alpha, float beta) -> Tensor");
  m.def("maxpool2d_fwd(Tensor x, int ks, int st) -> Tensor[]");
  m.def("maxpool2d_bwd(Tensor dy, Tensor arg, int H, int W, int ks, int st) -> Tensor");
  m.def("im2col(Tensor x, int KH, int KW, int sh, int sw, int ph, int pw) -> Tensor");
  m.def("col2im(Tensor cols, int N, int C, int H, int W, int KH, int KW, int sh, int sw, int ph, int pw) -> Tensor");
  m.def("luong_fwd(Tensor st, Tensor hs) -> Tensor[]");
  m.def("luong_bwd(Tensor dctx, Tensor st, Tensor hs, Tensor w) -> Tensor[]");
}
TORCH_LIBRARY_IMPL(spa, CUDA, m) {
  m.impl("dropout_apply", &spa::dropout_apply);
  m.impl("kd_loss_fwd", &spa::kd_loss_fwd);
  m.impl("vae_reparam", &spa::vae_reparam);
  m.impl("vae_loss_fwd", &spa::vae_loss_fwd);
  m.impl("mse_fwd", &spa::mse_fwd);
  m.impl("lrn_fwd", &spa::lrn_fwd);
  m.impl("lrn_bwd", &spa::lrn_bwd);
  m.impl("maxpool2d_fwd", &spa::maxpool2d_fwd);
  m.impl("maxpool2d_bwd", &spa::maxpool2d_bwd);
  m.impl("im2col", &spa::im2col);
  m.impl("col2im", &spa::col2im);
  m.impl("luong_fwd", &spa::luong_fwd);
  m.impl("luong_bwd", &spa::luong_bwd);
}
