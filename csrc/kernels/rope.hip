// Rotary position embedding, applied in place on the q/k heads of a fused
// [B, T, NH, hd] projection buffer (NH = H + 2*Hkv for a packed qkv), so no
// split/transpose copy is ever made. Backward = the same kernel with the
// inverse rotation (sin negated) on the incoming gradient.
//
// Reference: llama3/LLaMA-jax.ipynb:563-601 (precompute_freqs_cis / apply_rotary_emb:
// interleaved pairs (x[2i], x[2i+1]) rotated by t*theta^(-2i/hd)). A non-interleaved
// "rotate_half" layout is also provided (pairs (x[i], x[i+hd/2])).
//
// Layout: each thread owns 8 contiguous bf16 of one head row (16-byte load/store);
// cos/sin come from an fp32 table [Tmax, hd/2] (L2/LLC resident).
#include "spa_common.h"
#include <type_traits>

namespace spa {

// MODE 0: interleaved pairs (x[2i], x[2i+1]) rotated (LLaMA-jax);
// MODE 1: rotate_half pairs (x[i], x[i+hd/2]);
// MODE 2: Gemma-ref quirk (gemma/gemma.ipynb:182-200: per-position dense matrix with
//         2x2 blocks [[cos, cos], [-sin, sin]], NOT a rotation) applied elementwise:
//         y_e = c (x_e + x_o), y_o = s (x_o - x_e); "inverse" applies the transpose
//         (the exact backward of the forward map).
template <typename DT, int MODE>
__global__ __launch_bounds__(256) void rope_kernel(DT* __restrict__ x, const float* __restrict__ cosT,
                                                   const float* __restrict__ sinT, const int* __restrict__ pos,
                                                   long sb, long st, long sh, int B, int T, int nrot, int hd,
                                                   int pos_off, float sign) {
  const int vpr = hd / 8;                 // vectors per head row
  const long total = (long)B * T * nrot * vpr;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int v = i % vpr;
    long r = i / vpr;
    const int hh = r % nrot;
    r /= nrot;
    const int t = r % T;
    const int b = r / T;
    const int ps = pos ? pos[b * T + t] : t + pos_off;
    DT* p = x + b * sb + t * st + hh * sh;
    const float* c = cosT + (long)ps * (hd / 2);
    const float* s = sinT + (long)ps * (hd / 2);
    if constexpr (MODE == 0 || MODE == 2) {
      float a[8];
      load8(p + v * 8, a);
      const f32x4 cv = *reinterpret_cast<const f32x4*>(c + v * 4);
      const f32x4 sv = *reinterpret_cast<const f32x4*>(s + v * 4);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float x0 = a[2 * k], x1 = a[2 * k + 1];
        const float cs = cv[k];
        if constexpr (MODE == 0) {
          const float sn = sign * sv[k];
          a[2 * k] = x0 * cs - x1 * sn;
          a[2 * k + 1] = x0 * sn + x1 * cs;
        } else if (sign > 0.f) {   // forward: [[c, c], [-s, s]] x
          a[2 * k] = cs * (x0 + x1);
          a[2 * k + 1] = sv[k] * (x1 - x0);
        } else {                   // transpose: [[c, -s], [c, s]] dy
          a[2 * k] = cs * x0 - sv[k] * x1;
          a[2 * k + 1] = cs * x0 + sv[k] * x1;
        }
      }
      store8(p + v * 8, a);
    } else {
      // rotate_half: thread v < vpr/2 handles elements [8v, 8v+8) and their partners at +hd/2
      if (v >= vpr / 2) continue;
      float a[8], bq[8];
      load8(p + v * 8, a);
      load8(p + hd / 2 + v * 8, bq);
      float cv[8], sv[8];
      load8(c + v * 8, cv);
      load8(s + v * 8, sv);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float x0 = a[k], x1 = bq[k], sn = sign * sv[k];
        a[k] = x0 * cv[k] - x1 * sn;
        bq[k] = x0 * sn + x1 * cv[k];
      }
      store8(p + v * 8, a);
      store8(p + hd / 2 + v * 8, bq);
    }
  }
}

// x: [B, T, NH, hd] view (hd contiguous), rotates heads [0, nrot). In place.
void rope_(const at::Tensor& x, const at::Tensor& cos, const at::Tensor& sin, const c10::optional<at::Tensor>& pos,
           int64_t nrot, int64_t pos_off, int64_t mode, bool inverse) {
  SPA_CHECK_CUDA(x);
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat, "rope: bf16/fp32");
  TORCH_CHECK(x.dim() == 4 && x.stride(3) == 1, "rope: x must be [B,T,NH,hd] with contiguous hd");
  const int B = x.size(0), T = x.size(1), hd = x.size(3);
  TORCH_CHECK(hd % 16 == 0, "rope: hd must be a multiple of 16");
  TORCH_CHECK(nrot <= x.size(2));
  TORCH_CHECK(cos.scalar_type() == at::kFloat && cos.is_contiguous() && sin.is_contiguous() && cos.size(1) == hd / 2);
  TORCH_CHECK(x.stride(1) % 8 == 0 && x.stride(2) % 8 == 0 && x.stride(0) % 8 == 0 && (uintptr_t)x.data_ptr() % 16 == 0);
  if (pos) { TORCH_CHECK(pos->scalar_type() == at::kInt && pos->is_contiguous() && pos->numel() == (int64_t)B * T); }
  else { TORCH_CHECK(pos_off + T <= cos.size(0), "rope: table too short"); }
  DeviceGuard g(x.device());
  const long total = (long)B * T * nrot * (hd / 8);
  if (total == 0) return;
  const int grid = (int)std::min<long>((total + 255) / 256, 4096);
  auto st = stream();
  const float sign = inverse ? -1.f : 1.f;
  auto launch = [&](auto modec) {
    constexpr int M = decltype(modec)::value;
    if (x.scalar_type() == at::kBFloat16)
      rope_kernel<bf16, M><<<grid, 256, 0, st>>>((bf16*)x.data_ptr(), cos.data_ptr<float>(), sin.data_ptr<float>(),
                                                 pos ? pos->data_ptr<int>() : nullptr, x.stride(0), x.stride(1),
                                                 x.stride(2), B, T, (int)nrot, hd, (int)pos_off, sign);
    else
      rope_kernel<float, M><<<grid, 256, 0, st>>>(x.data_ptr<float>(), cos.data_ptr<float>(), sin.data_ptr<float>(),
                                                  pos ? pos->data_ptr<int>() : nullptr, x.stride(0), x.stride(1),
                                                  x.stride(2), B, T, (int)nrot, hd, (int)pos_off, sign);
  };
  if (mode == 0) launch(std::integral_constant<int, 0>{});
  else if (mode == 1) launch(std::integral_constant<int, 1>{});
  else if (mode == 2) launch(std::integral_constant<int, 2>{});
  else TORCH_CHECK(false, "rope: mode must be 0, 1 or 2");
  SPA_LAUNCH_CHECK();
}

// Decode-step prologue in one launch: for a packed qkv buffer [B, T, H + 2 Hkv, hd], rotate
// the q heads in place, rotate the k heads into the KV cache and copy the v heads into it, at
// cache row *index + t. MODE 0: interleaved pairs (LLaMA), MODE 1: rotate_half (Gemma). The
// row and the RoPE positions are read from device memory, so a captured hipGraph replays it
// at every position (replaces rope_ + two index_copy_ launches per layer). Rows past the
// cache end are dropped.
template <int MODE>
__global__ __launch_bounds__(256) void rope_kv_write_kernel(bf16* __restrict__ x, const float* __restrict__ cosT,
                                                            const float* __restrict__ sinT,
                                                            const int* __restrict__ pos,
                                                            const long* __restrict__ index, bf16* __restrict__ kc,
                                                            bf16* __restrict__ vc, long sb, long st, long sh,
                                                            long kcb, long kct, long kch, long vcb, long vct,
                                                            long vch, int B, int T, int H, int Hkv, int hd,
                                                            int Tmax) {
  const int vpr = hd / 8;
  const int NH = H + 2 * Hkv;
  const long total = (long)B * T * NH * vpr;
  const long row0 = *index;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int v = i % vpr;
    long r = i / vpr;
    const int hh = r % NH;
    r /= NH;
    const int t = r % T;
    const int b = r / T;
    const long row = row0 + t;
    if (hh >= H && row >= Tmax) continue;
    const bf16* src = x + b * sb + t * st + hh * sh;
    bf16* dst = hh < H ? x + b * sb + t * st + hh * sh
                       : (hh < H + Hkv ? kc + b * kcb + row * kct + (hh - H) * kch
                                       : vc + b * vcb + row * vct + (hh - H - Hkv) * vch);
    float a[8];
    if (hh >= H + Hkv) {  // v: plain copy into the cache
      load8(src + v * 8, a);
      store8(dst + v * 8, a);
      continue;
    }
    const int ps = pos[b * T + t];
    const float* c = cosT + (long)ps * (hd / 2);
    const float* s = sinT + (long)ps * (hd / 2);
    if constexpr (MODE == 0) {
      load8(src + v * 8, a);
      const f32x4 cv = *reinterpret_cast<const f32x4*>(c + v * 4);
      const f32x4 sv = *reinterpret_cast<const f32x4*>(s + v * 4);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float x0 = a[2 * k], x1 = a[2 * k + 1];
        a[2 * k] = x0 * cv[k] - x1 * sv[k];
        a[2 * k + 1] = x0 * sv[k] + x1 * cv[k];
      }
      store8(dst + v * 8, a);
    } else {  // rotate_half: thread v < vpr/2 owns elements [8v, 8v+8) and their partners at +hd/2
      if (v >= vpr / 2) continue;
      float bq[8], cv[8], sv[8];
      load8(src + v * 8, a);
      load8(src + hd / 2 + v * 8, bq);
      load8(c + v * 8, cv);
      load8(s + v * 8, sv);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float x0 = a[k], x1 = bq[k];
        a[k] = x0 * cv[k] - x1 * sv[k];
        bq[k] = x0 * sv[k] + x1 * cv[k];
      }
      store8(dst + v * 8, a);
      store8(dst + hd / 2 + v * 8, bq);
    }
  }
}

void rope_kv_write_(const at::Tensor& x, const at::Tensor& cos, const at::Tensor& sin, const at::Tensor& pos,
                    const at::Tensor& index, const at::Tensor& kc, const at::Tensor& vc, int64_t H, int64_t Hkv,
                    int64_t mode) {
  for (auto* t : {&x, &kc, &vc}) {
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->dim() == 4 && t->stride(3) == 1,
                "rope_kv_write: bf16 [B, T, heads, hd] tensors with contiguous hd");
    TORCH_CHECK(t->stride(0) % 8 == 0 && t->stride(1) % 8 == 0 && t->stride(2) % 8 == 0 &&
                    (uintptr_t)t->data_ptr() % 16 == 0,
                "rope_kv_write: 16-byte aligned rows");
  }
  const int B = x.size(0), T = x.size(1), hd = x.size(3);
  TORCH_CHECK(x.size(2) == H + 2 * Hkv && hd % 16 == 0, "rope_kv_write: x must be packed [B, T, H + 2 Hkv, hd]");
  TORCH_CHECK(kc.size(0) == B && vc.size(0) == B && kc.size(2) == Hkv && vc.size(2) == Hkv && kc.size(3) == hd &&
                  vc.size(3) == hd && vc.size(1) == kc.size(1),
              "rope_kv_write: cache shape mismatch");
  TORCH_CHECK(cos.scalar_type() == at::kFloat && cos.is_contiguous() && sin.is_contiguous() && cos.size(1) == hd / 2,
              "rope_kv_write: fp32 [Tmax, hd/2] tables");
  TORCH_CHECK(pos.is_cuda() && pos.scalar_type() == at::kInt && pos.is_contiguous() && pos.numel() == (int64_t)B * T,
              "rope_kv_write: pos must be device int32 [B, T]");
  TORCH_CHECK(index.is_cuda() && index.scalar_type() == at::kLong && index.numel() >= 1,
              "rope_kv_write: index must be a device int64 tensor");
  TORCH_CHECK(mode == 0 || mode == 1, "rope_kv_write: mode 0 (interleaved) or 1 (rotate_half)");
  DeviceGuard g(x.device());
  const long total = (long)B * T * (H + 2 * Hkv) * (hd / 8);
  if (total == 0) return;
  const int grid = (int)std::min<long>((total + 255) / 256, 4096);
  auto launch = [&](auto modec) {
    constexpr int M = decltype(modec)::value;
    rope_kv_write_kernel<M><<<grid, 256, 0, stream()>>>(
        (bf16*)x.data_ptr(), cos.data_ptr<float>(), sin.data_ptr<float>(), pos.data_ptr<int>(),
        index.data_ptr<int64_t>(), (bf16*)kc.data_ptr(), (bf16*)vc.data_ptr(), x.stride(0), x.stride(1),
        x.stride(2), kc.stride(0), kc.stride(1), kc.stride(2), vc.stride(0), vc.stride(1), vc.stride(2), B, T,
        (int)H, (int)Hkv, hd, (int)kc.size(1));
  };
  if (mode == 0) launch(std::integral_constant<int, 0>{});
  else launch(std::integral_constant<int, 1>{});
  SPA_LAUNCH_CHECK();
}

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.def("rope_(Tensor(a!) x, Tensor cos, Tensor sin, Tensor? pos, int nrot, int pos_off, int mode, "
        "bool inverse) -> ()");
  m.def("rope_kv_write_(Tensor(a!) x, Tensor cos, Tensor sin, Tensor pos, Tensor index, Tensor(b!) kc, "
        "Tensor(c!) vc, int n_heads, int n_kv_heads, int mode=0) -> ()");
}
TORCH_LIBRARY_IMPL(spa, CUDA, m) {
  m.impl("rope_", &spa::rope_);
  m.impl("rope_kv_write_", &spa::rope_kv_write_);
}
