// Shared helpers for the gfx950 (CDNA4, MI355X) kernels of solvingpapers_amd.
//
// Conventions used by every kernel in csrc/kernels:
//  * wave64 everywhere: lane = threadIdx.x & 63, reductions over 64 lanes;
//  * bf16 is moved as 16-byte vectors (8 x bf16) — hipcc never vectorises
//    scalar bf16 loads on its own;
//  * fp32 accumulation, bf16 (or fp32) I/O;
//  * launches go on torch's current HIP stream so they compose with
//    hipBLASLt GEMMs, RCCL collectives and hipGraph capture.
#pragma once

#include <hip/hip_runtime.h>
#include <torch/library.h>
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <cstdint>

#include "spa_debug.h"  // SPA_DBG_* device bounds guards (empty unless -DSPA_DEBUG_BOUNDS=1)

namespace spa {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

constexpr int kWave = 64;

using DeviceGuard = c10::hip::HIPGuardMasqueradingAsCUDA;
inline hipStream_t stream() { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

__host__ __device__ inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x = NT (multiple of 64). `red` must hold NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (NT == 64) return v;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) s += red[i];
  return s;
}
template <int NT>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (NT == 64) return v;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float s = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) s = fmaxf(s, red[i]);
  return s;
}

__device__ __forceinline__ void load8(const bf16* p, float (&f)[8]) {
  bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = (float)v[i];
}
__device__ __forceinline__ void store8(bf16* p, const float (&f)[8]) {
  bf16x8 v;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (bf16)f[i];
  *reinterpret_cast<bf16x8*>(p) = v;
}
__device__ __forceinline__ void load8(const float* p, float (&f)[8]) {
  f32x4 a = *reinterpret_cast<const f32x4*>(p);
  f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
  for (int i = 0; i < 4; ++i) { f[i] = a[i]; f[i + 4] = b[i]; }
}
__device__ __forceinline__ void store8(float* p, const float (&f)[8]) {
  f32x4 a, b;
#pragma unroll
  for (int i = 0; i < 4; ++i) { a[i] = f[i]; b[i] = f[i + 4]; }
  *reinterpret_cast<f32x4*>(p) = a;
  *reinterpret_cast<f32x4*>(p + 4) = b;
}

// XCD-aware bijective remap of a 1-D block id (8 XCDs, round-robin dispatch):
// consecutive logical tiles land on the same XCD so they share its L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

// Elementwise kernels walk storage order: any dense (non-overlapping, gap-free) tensor -- e.g. a
// channels-last conv activation -- is used as is and its output keeps the same strides.
inline at::Tensor dense(const at::Tensor& t) { return t.is_non_overlapping_and_dense() ? t : t.contiguous(); }
// `t` laid out exactly like `like` (a no-op when the strides already match)
inline at::Tensor dense_like(const at::Tensor& t, const at::Tensor& like) {
  if (t.strides() == like.strides() && t.is_non_overlapping_and_dense()) return t;
  return at::empty_like(like, t.options()).copy_(t);
}

// fp32 [P, N] row partials -> fp32 [N] column sums into out (or a new tensor); norm.hip
at::Tensor reduce_col_parts(const at::Tensor& part, c10::optional<at::Tensor> out = c10::nullopt);

}  // namespace spa

#define SPA_CHECK_CUDA(t) TORCH_CHECK((t).is_cuda(), #t " must be a HIP tensor")
#define SPA_CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define SPA_CHECK_BF16(t) TORCH_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bf16")
#define SPA_LAUNCH_CHECK() C10_HIP_KERNEL_LAUNCH_CHECK()
