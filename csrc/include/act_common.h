// Activation functions shared by the elementwise kernels (activation.hip) and the GEMM
// epilogues (gemm8.hip): value and derivative in fp32.
#pragma once
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

}  // namespace spa
