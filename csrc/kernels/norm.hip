// RMSNorm / LayerNorm forward + backward for gfx950, with an optional fused
// residual add (h = x + r; y = norm(h)) so the pre-norm transformer block reads
// its residual stream exactly once per norm.
//
// Reference semantics: RMSNorm `x*w*rsqrt(mean(x^2)+eps)`
//   llama3/LLaMA-jax.ipynb:536-538, gemma/gemma.ipynb:139-150 (fp32 compute),
//   deepseekv3/deepseekv3.ipynb:911-917;
// LayerNorm (weight+bias) gpt/gpt-jax.ipynb:414-416, vision transformer/ViT.ipynb:205-206.
//
// Mapping: one row per NT-thread group (NT = 256 for D >= 2048, else 64 = one wave
// with 4 rows per 256-thread block). Each thread keeps its 8-element bf16 vectors
// in registers (MAXV of them) so the row is read from HBM once. Stats in fp32.
// Backward dw/db: each block accumulates a per-column partial over a strided set
// of rows in registers, writes one fp32 partial row, a second tiny kernel sums the
// partials (deterministic, no atomics).
#include "spa_common.h"

namespace spa {

template <typename T, int NT, int MAXV, bool LN, bool RES, bool RESOUT>
__global__ __launch_bounds__(256) void norm_fwd_kernel(
    const T* __restrict__ x, const T* __restrict__ r, const T* __restrict__ w,
    const T* __restrict__ b, T* __restrict__ y, T* __restrict__ hout,
    float* __restrict__ rstd_out, float* __restrict__ mean_out, int M, int D, float eps) {
  constexpr int RPB = 256 / NT;  // rows per block
  __shared__ float red[RPB][NT / 64 > 0 ? NT / 64 : 1];
  const int sub = threadIdx.x / NT, t = threadIdx.x % NT;
  const int row = blockIdx.x * RPB + sub;
  if (row >= M) return;  // whole group exits together (NT-aligned)
  const int nv = D / 8;
  float v[MAXV][8];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = t + k * NT;
    if (vi < nv) {
      load8(x + (size_t)row * D + vi * 8, v[k]);
      if constexpr (RES) {
        float rr[8];
        load8(r + (size_t)row * D + vi * 8, rr);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[k][i] += rr[i];
        if constexpr (RESOUT) {
          // round the residual stream to the I/O dtype once, and normalise the rounded value
#pragma unroll
          for (int i = 0; i < 8; ++i) v[k][i] = (float)(T)v[k][i];
          store8(hout + (size_t)row * D + vi * 8, v[k]);
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) s += LN ? v[k][i] : v[k][i] * v[k][i];
    }
  }
  float mean = 0.f;
  if constexpr (LN) {
    float tot = NT == 64 ? wave_sum(s) : block_sum<NT>(s, red[sub]);
    mean = tot / D;
    s = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k)
      if (t + k * NT < nv)
#pragma unroll
        for (int i = 0; i < 8; ++i) { float d = v[k][i] - mean; s += d * d; }
    if (NT != 64) __syncthreads();
  }
  float tot = NT == 64 ? wave_sum(s) : block_sum<NT>(s, red[sub]);
  const float rstd = rsqrtf(tot / D + eps);
  if (t == 0) {
    rstd_out[row] = rstd;
    if constexpr (LN) mean_out[row] = mean;
  }
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int vi = t + k * NT;
    if (vi < nv) {
      float wv[8], o[8];
      load8(w + vi * 8, wv);
      if constexpr (LN) {
        float bv[8];
        load8(b + vi * 8, bv);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = (v[k][i] - mean) * rstd * wv[i] + bv[i];
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = v[k][i] * rstd * wv[i];
      }
      store8(y + (size_t)row * D + vi * 8, o);
    }
  }
}

// Backward. grid.x = number of partial blocks; each block walks rows
// blockIdx.x*RPB + sub, stepping by gridDim.x*RPB.
template <typename T, int NT, int MAXV, bool LN, bool DRES>
__global__ __launch_bounds__(256) void norm_bwd_kernel(
    const T* __restrict__ dy, const T* __restrict__ h, const T* __restrict__ w,
    const float* __restrict__ rstd_in, const float* __restrict__ mean_in,
    const T* __restrict__ dres, T* __restrict__ dx, float* __restrict__ dw_part,
    float* __restrict__ db_part, int M, int D) {
  constexpr int RPB = 256 / NT;
  __shared__ float red[RPB][NT / 64 > 0 ? NT / 64 : 1];
  const int sub = threadIdx.x / NT, t = threadIdx.x % NT;
  const int nv = D / 8;
  float dwacc[MAXV][8], dbacc[MAXV][8];
#pragma unroll
  for (int k = 0; k < MAXV; ++k)
#pragma unroll
    for (int i = 0; i < 8; ++i) { dwacc[k][i] = 0.f; dbacc[k][i] = 0.f; }
  float wv[MAXV][8];
#pragma unroll
  for (int k = 0; k < MAXV; ++k)
    if (t + k * NT < nv) load8(w + (t + k * NT) * 8, wv[k]);

  for (int row0 = blockIdx.x * RPB; row0 < M; row0 += gridDim.x * RPB) {
    const int row = row0 + sub;
    const bool valid = row < M;
    float xh[MAXV][8], g[MAXV][8];
    float s1 = 0.f, s2 = 0.f;
    const float rstd = valid ? rstd_in[row] : 0.f;
    const float mean = (LN && valid) ? mean_in[row] : 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int vi = t + k * NT;
      if (valid && vi < nv) {
        float hv[8], dv[8];
        load8(h + (size_t)row * D + vi * 8, hv);
        load8(dy + (size_t)row * D + vi * 8, dv);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          xh[k][i] = (hv[i] - mean) * rstd;
          g[k][i] = dv[i] * wv[k][i];
          s1 += g[k][i] * xh[k][i];
          if constexpr (LN) s2 += g[k][i];
          dwacc[k][i] += dv[i] * xh[k][i];
          if constexpr (LN) dbacc[k][i] += dv[i];
        }
      }
    }
    float a1, a2 = 0.f;
    if (NT == 64) {
      a1 = wave_sum(s1);
      if constexpr (LN) a2 = wave_sum(s2);
    } else {
      a1 = block_sum<NT>(s1, red[sub]);
      if constexpr (LN) { __syncthreads(); a2 = block_sum<NT>(s2, red[sub]); }
      __syncthreads();
    }
    a1 /= D;
    a2 /= D;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int vi = t + k * NT;
      if (valid && vi < nv) {
        float o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = rstd * (g[k][i] - a2 - xh[k][i] * a1);
        if constexpr (DRES) {
          float rr[8];
          load8(dres + (size_t)row * D + vi * 8, rr);
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] += rr[i];
        }
        store8(dx + (size_t)row * D + vi * 8, o);
      }
    }
  }
  if constexpr (RPB == 1) {
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int vi = t + k * NT;
      if (vi < nv) {
        store8(dw_part + (size_t)blockIdx.x * D + vi * 8, dwacc[k]);
        if constexpr (LN) store8(db_part + (size_t)blockIdx.x * D + vi * 8, dbacc[k]);
      }
    }
  } else {
    // small D (<= 2048): per-sub partial rows, reduced by the column kernel
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int vi = t + k * NT;
      if (vi < nv) {
        const size_t prow = (size_t)blockIdx.x * RPB + sub;
        store8(dw_part + prow * D + vi * 8, dwacc[k]);
        if constexpr (LN) store8(db_part + prow * D + vi * 8, dbacc[k]);
      }
    }
  }
}

// Column sums of a [P, D] fp32 partial matrix -> out[D] (dtype of param).
template <typename OT>
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ part, OT* __restrict__ out,
                                                     int P, int D) {
  // 256 threads = 64 columns x 4 row-slices
  __shared__ float s[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rs = threadIdx.x >> 6;
  float acc = 0.f;
  if (c < D)
    for (int p = rs; p < P; p += 4) acc += part[(size_t)p * D + c];
  s[rs][threadIdx.x & 63] = acc;
  __syncthreads();
  if (rs == 0 && c < D) out[c] = (OT)(s[0][threadIdx.x] + s[1][threadIdx.x] + s[2][threadIdx.x] + s[3][threadIdx.x]);
}
// First level of a two-level deterministic column sum: block (bx, by) reduces rows
// [by*chunk, (by+1)*chunk) of 64 columns -> part2[by, c]. Enough blocks to fill the chip
// (a single-level sum over thousands of partial rows ran on D/64 blocks: latency bound).
__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* __restrict__ part, float* __restrict__ part2,
                                                             int P, int D, int chunk) {
  __shared__ float s[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rs = threadIdx.x >> 6;
  const int p0 = blockIdx.y * chunk, p1 = min(P, p0 + chunk);
  float acc = 0.f;
  if (c < D)
    for (int p = p0 + rs; p < p1; p += 4) acc += part[(size_t)p * D + c];
  s[rs][threadIdx.x & 63] = acc;
  __syncthreads();
  if (rs == 0 && c < D)
    part2[(size_t)blockIdx.y * D + c] = s[0][threadIdx.x] + s[1][threadIdx.x] + s[2][threadIdx.x] + s[3][threadIdx.x];
}

// Bias gradient: fp32 column sums of a bf16 [R, N] matrix (row stride ld). Block (bx, by) sums
// rows [by*rpb, (by+1)*rpb) of 256 columns: 32 lanes x 8 columns cover one 512-byte row segment,
// 8 row groups stride the rows with 4 16-byte loads in flight each; the 8 group partials meet in
// LDS and one fp32 row of part[by, :] is written (summed by colsum_kernel: deterministic).
__global__ __launch_bounds__(256) void rowsum_part_kernel(const bf16* __restrict__ x, float* __restrict__ part,
                                                          long R, int N, long ld, long rpb) {
  __shared__ __attribute__((aligned(16))) float red[8][256];
  const int cl = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int c0 = blockIdx.x * 256 + cl * 8;
  const long r0 = (long)blockIdx.y * rpb, r1 = min(R, r0 + rpb);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto add = [&](const uint4& v) {
    const unsigned* u = reinterpret_cast<const unsigned*>(&v);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      acc[2 * k] += __uint_as_float(u[k] << 16);
      acc[2 * k + 1] += __uint_as_float(u[k] & 0xffff0000u);
    }
  };
  if (c0 < N) {
    const bf16* p = x + c0;
    long r = r0 + rg;
    for (; r + 24 < r1; r += 32) {
      const uint4 a = *reinterpret_cast<const uint4*>(p + r * ld);
      const uint4 b = *reinterpret_cast<const uint4*>(p + (r + 8) * ld);
      const uint4 c = *reinterpret_cast<const uint4*>(p + (r + 16) * ld);
      const uint4 d = *reinterpret_cast<const uint4*>(p + (r + 24) * ld);
      add(a); add(b); add(c); add(d);
    }
    for (; r < r1; r += 8) add(*reinterpret_cast<const uint4*>(p + r * ld));
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

#define NORM_FWD_DISPATCH(NT, MAXV)                                                              \
  do {                                                                                           \
    dim3 grid(cdiv(M, 256 / NT));                                                                \
    if (is_ln) {                                                                                 \
      if (has_res) norm_fwd_kernel<T, NT, MAXV, true, true, true><<<grid, 256, 0, st>>>(ARGS);   \
      else norm_fwd_kernel<T, NT, MAXV, true, false, false><<<grid, 256, 0, st>>>(ARGS);         \
    } else {                                                                                     \
      if (has_res) norm_fwd_kernel<T, NT, MAXV, false, true, true><<<grid, 256, 0, st>>>(ARGS);  \
      else norm_fwd_kernel<T, NT, MAXV, false, false, false><<<grid, 256, 0, st>>>(ARGS);        \
    }                                                                                            \
  } while (0)

// Returns (y, h_or_empty, rstd, mean_or_empty). bf16 or fp32 I/O (weights same dtype).
std::vector<at::Tensor> norm_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& residual,
                                 const at::Tensor& w, const c10::optional<at::Tensor>& b, double eps) {
  SPA_CHECK_CUDA(x); SPA_CHECK_CONTIG(x);
  const auto dt = x.scalar_type();
  TORCH_CHECK(dt == at::kBFloat16 || dt == at::kFloat, "norm: bf16/fp32 only");
  TORCH_CHECK(w.scalar_type() == dt, "norm: weight dtype must match x");
  const bool is_ln = b.has_value();
  const bool has_res = residual.has_value();
  const int D = x.size(-1);
  const int M = x.numel() / D;
  TORCH_CHECK(D % 8 == 0 && D <= 16384, "norm: D must be a multiple of 8 and <= 16384");
  TORCH_CHECK(w.numel() == D && w.is_contiguous());
  DeviceGuard g(x.device());
  auto y = at::empty_like(x);
  at::Tensor h = has_res ? at::empty_like(x) : at::Tensor();
  if (has_res) { TORCH_CHECK(residual->scalar_type() == dt); SPA_CHECK_CONTIG(*residual); TORCH_CHECK(residual->sizes() == x.sizes()); }
  if (is_ln) { TORCH_CHECK(b->scalar_type() == dt); TORCH_CHECK(b->numel() == D && b->is_contiguous()); }
  auto opts = x.options().dtype(at::kFloat);
  auto rstd = at::empty({M}, opts);
  auto mean = is_ln ? at::empty({M}, opts) : at::Tensor();
  auto st = stream();
  if (M == 0) return {y, h, rstd, mean};
  const int nv = D / 8;
  auto run = [&](auto tag) {
    using T = decltype(tag);
#define ARGS                                                                                   \
  (const T*)x.data_ptr(), has_res ? (const T*)residual->data_ptr() : nullptr,                  \
      (const T*)w.data_ptr(), is_ln ? (const T*)b->data_ptr() : nullptr, (T*)y.data_ptr(),     \
      has_res ? (T*)h.data_ptr() : nullptr, rstd.data_ptr<float>(),                            \
      is_ln ? mean.data_ptr<float>() : nullptr, M, D, (float)eps
    if (nv <= 64) NORM_FWD_DISPATCH(64, 1);
    else if (nv <= 128) NORM_FWD_DISPATCH(64, 2);
    else if (nv <= 256) NORM_FWD_DISPATCH(256, 1);
    else if (nv <= 512) NORM_FWD_DISPATCH(256, 2);
    else if (nv <= 1024) NORM_FWD_DISPATCH(256, 4);
    else NORM_FWD_DISPATCH(256, 8);
#undef ARGS
  };
  if (dt == at::kBFloat16) run(bf16{}); else run(float{});
  SPA_LAUNCH_CHECK();
  return {y, h, rstd, mean};
}

#define NORM_BWD_DISPATCH(NT, MAXV)                                                        \
  do {                                                                                     \
    constexpr int RPB = 256 / NT;                                                          \
    nblk = std::min(cdiv(M, RPB), 1024);                                                   \
    nparts = nblk * RPB;                                                                   \
    dw_part = at::empty({nparts, D}, opts);                                                \
    if (is_ln) db_part = at::empty({nparts, D}, opts);                                     \
    if (is_ln) {                                                                           \
      if (has_dres) norm_bwd_kernel<T, NT, MAXV, true, true><<<nblk, 256, 0, st>>>(ARGS);  \
      else norm_bwd_kernel<T, NT, MAXV, true, false><<<nblk, 256, 0, st>>>(ARGS);          \
    } else {                                                                               \
      if (has_dres) norm_bwd_kernel<T, NT, MAXV, false, true><<<nblk, 256, 0, st>>>(ARGS); \
      else norm_bwd_kernel<T, NT, MAXV, false, false><<<nblk, 256, 0, st>>>(ARGS);         \
    }                                                                                      \
  } while (0)

// Returns (dx, dw, db_or_empty). dres (optional) is added into dx (gradient flowing
// along the residual stream past the fused add). dw_out / db_out (optional): write the
// weight gradients straight into these (e.g. main_grad views) instead of new tensors.
std::vector<at::Tensor> norm_bwd(const at::Tensor& dy, const at::Tensor& h, const at::Tensor& w,
                                 const at::Tensor& rstd, const c10::optional<at::Tensor>& mean,
                                 const c10::optional<at::Tensor>& dres, const c10::optional<at::Tensor>& dw_out,
                                 const c10::optional<at::Tensor>& db_out) {
  SPA_CHECK_CONTIG(dy); SPA_CHECK_CONTIG(h);
  const auto dt = h.scalar_type();
  TORCH_CHECK(dy.scalar_type() == dt && w.scalar_type() == dt, "norm_bwd: dtype mismatch");
  const bool is_ln = mean.has_value();
  const bool has_dres = dres.has_value();
  const int D = h.size(-1);
  const int M = h.numel() / D;
  DeviceGuard g(h.device());
  auto dx = at::empty_like(h);
  auto opts = h.options().dtype(at::kFloat);
  auto st = stream();
  at::Tensor dw_part, db_part;
  int nblk = 0, nparts = 0;
  if (has_dres) { TORCH_CHECK(dres->scalar_type() == dt); SPA_CHECK_CONTIG(*dres); }
  auto dw = dw_out ? *dw_out : at::empty({D}, w.options());
  auto db = is_ln ? (db_out ? *db_out : at::empty({D}, w.options())) : at::Tensor();
  TORCH_CHECK(dw.is_contiguous() && dw.numel() == D);
  if (M == 0) { dw.zero_(); if (is_ln) db.zero_(); return {dx, dw, db}; }
  const int nv = D / 8;
  auto run = [&](auto tag) {
    using T = decltype(tag);
#define ARGS                                                                            \
  (const T*)dy.data_ptr(), (const T*)h.data_ptr(), (const T*)w.data_ptr(),              \
      rstd.data_ptr<float>(), is_ln ? mean->data_ptr<float>() : nullptr,                \
      has_dres ? (const T*)dres->data_ptr() : nullptr, (T*)dx.data_ptr(),               \
      dw_part.data_ptr<float>(), is_ln ? db_part.data_ptr<float>() : nullptr, M, D
    if (nv <= 64) NORM_BWD_DISPATCH(64, 1);
    else if (nv <= 128) NORM_BWD_DISPATCH(64, 2);
    else if (nv <= 256) NORM_BWD_DISPATCH(256, 1);
    else if (nv <= 512) NORM_BWD_DISPATCH(256, 2);
    else if (nv <= 1024) NORM_BWD_DISPATCH(256, 4);
    else NORM_BWD_DISPATCH(256, 8);
#undef ARGS
    SPA_LAUNCH_CHECK();
    auto colsum = [&](const at::Tensor& part, const at::Tensor& out) {
      const float* src = part.data_ptr<float>();
      int P = nparts;
      at::Tensor p2;
      if (P > 64) {
        const int Y = std::min(64, cdiv(P, 16));
        const int chunk = cdiv(P, Y);
        p2 = at::empty({Y, D}, opts);
        colsum_partial_kernel<<<dim3(cdiv(D, 64), Y), 256, 0, st>>>(src, p2.data_ptr<float>(), P, D, chunk);
        src = p2.data_ptr<float>();
        P = Y;
      }
      if (out.scalar_type() == at::kFloat)
        colsum_kernel<float><<<cdiv(D, 64), 256, 0, st>>>(src, out.data_ptr<float>(), P, D);
      else
        colsum_kernel<bf16><<<cdiv(D, 64), 256, 0, st>>>(src, (bf16*)out.data_ptr(), P, D);
    };
    colsum(dw_part, dw);
    if (is_ln) colsum(db_part, db);
  };
  if (dt == at::kBFloat16) run(bf16{}); else run(float{});
  SPA_LAUNCH_CHECK();
  return {dx, dw, db};
}

// x [R, N] bf16 (unit column stride, N and the row stride % 8) -> fp32 [N] column sums
at::Tensor rowsum_bf16(const at::Tensor& x) {
  SPA_CHECK_CUDA(x);
  TORCH_CHECK(x.dim() == 2 && x.scalar_type() == at::kBFloat16 && x.stride(1) == 1, "rowsum_bf16: [R, N] bf16");
  const long R = x.size(0);
  const int N = x.size(1);
  const long ld = x.stride(0);
  TORCH_CHECK(N % 8 == 0 && ld % 8 == 0 && (uintptr_t)x.data_ptr() % 16 == 0, "rowsum_bf16: 16-byte rows");
  DeviceGuard g(x.device());
  auto opts = x.options().dtype(at::kFloat);
  auto out = at::empty({N}, opts);
  if (N == 0) return out;
  if (R == 0) return out.zero_();
  auto st = stream();
  // enough row blocks for >= 1024 blocks, each at least 64 rows
  const int nx = cdiv(N, 256);
  const long want = std::max<long>(1, std::min<long>(cdiv(1024, nx), cdiv(R, 64)));
  const long rpb = (R + want - 1) / want;
  const int P = (int)cdiv(R, rpb);
  auto part = at::empty({P, N}, opts);
  rowsum_part_kernel<<<dim3(nx, P), 256, 0, st>>>((const bf16*)x.data_ptr(), part.data_ptr<float>(), R, N, ld, rpb);
  SPA_LAUNCH_CHECK();
  return reduce_col_parts(part, out);
}

// fp32 [P, N] row partials -> fp32 [N] column sums (two levels when P > 64; deterministic)
at::Tensor reduce_col_parts(const at::Tensor& part, c10::optional<at::Tensor> out_) {
  TORCH_CHECK(part.dim() == 2 && part.scalar_type() == at::kFloat && part.is_contiguous());
  const int PP0 = part.size(0), N = part.size(1);
  auto opts = part.options();
  auto out = out_ ? *out_ : at::empty({N}, opts);
  if (N == 0) return out;
  auto st = stream();
  const float* src = part.data_ptr<float>();
  int PP = PP0;
  at::Tensor p2;
  if (PP > 64) {
    const int Y = std::min(64, cdiv(PP, 16));
    const int chunk = cdiv(PP, Y);
    p2 = at::empty({Y, N}, opts);
    colsum_partial_kernel<<<dim3(cdiv(N, 64), Y), 256, 0, st>>>(src, p2.data_ptr<float>(), PP, N, chunk);
    src = p2.data_ptr<float>();
    PP = Y;
  }
  colsum_kernel<float><<<cdiv(N, 64), 256, 0, st>>>(src, out.data_ptr<float>(), PP, N);
  SPA_LAUNCH_CHECK();
  return out;
}

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.def("rowsum_bf16(Tensor x) -> Tensor");
  m.def("norm_fwd(Tensor x, Tensor? residual, Tensor w, Tensor? b, float eps) -> Tensor[]");
  m.def("norm_bwd(Tensor dy, Tensor h, Tensor w, Tensor rstd, Tensor? mean, Tensor? dres, Tensor(a!)? dw_out, "
        "Tensor(b!)? db_out) -> Tensor[]");
}
TORCH_LIBRARY_IMPL(spa, CUDA, m) {
  m.impl("rowsum_bf16", &spa::rowsum_bf16);
  m.impl("norm_fwd", &spa::norm_fwd);
  m.impl("norm_bwd", &spa::norm_bwd);
}
