// DeepSeek MLA attention in latent space for cached decoding (models/deepseekv3.py MLA._decode).
//
// The cache holds, per token and layer, the compressed KV latent c (kv_lora = C values) and the
// shared decoupled-RoPE key r (R values) instead of 2*H*hd up-projected values. With W_uk
// absorbed into the query (q_abs = q_nope W_uk, per head) every head scores
//     s[h, j] = scale * (q_abs[h] . c[j] + q_rope[h] . r[j])
// and reads o_lat[h] = softmax(s[h]) c  (W_uv is applied afterwards by a GEMM). That is
// multi-query attention with ONE (C + R)-wide key head and a C-wide value head shared by all H
// query heads -- 576 / 512 for DeepSeek-V2/V3 widths, past the 256 of the flash kernels.
//
// Kernel: flash-decoding. A workgroup (4 waves) owns 16 query rows (a row = one (token, head)
// pair) of one sequence and a split of the key range; per 64-key tile:
//   1. S = Q K^T with v_mfma_f32_16x16x32_bf16: wave w scores keys 16w..16w+15 over the C + R
//      reduction (Q rows from LDS, key rows from the padded LDS tile: conflict-free b128 reads);
//   2. online softmax over the tile by all 256 threads (row max / row sum over 16 lanes);
//   3. O += P C: wave w owns output columns [C/4 w, C/4 (w+1)); P (bf16) from LDS, the C tile
//      read transposed (ds_read_b64_tr_b16) from the same padded image.
// Splits write unnormalised partials (O, m, l); mla_merge_kernel combines them. The valid
// cache length may come from a device int (HIP-graph decode: one capture serves every position).
#include "spa_common.h"

namespace spa {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4m __attribute__((ext_vector_type(4)));

struct MlaParams {
  const bf16* q; const bf16* qr; const bf16* cc; const bf16* cr;
  bf16* out;
  float* part_o; float* part_ml;    // [nsplit][B][rows][C], [nsplit][B][rows][2]
  const int* kv_len_ptr;            // device valid-length (graph mode) or null
  int kv_len;                       // host valid-length when kv_len_ptr is null
  int B, T, H, rows, nsplit, tiles_per_split;
  long sqb, sqt, sqh, srb, srt, srh, scb, sct, srcb, srct, sob, sot, soh;
  float scale_log2;
};

constexpr int kMlaRB = 16, kMlaKT = 64;

__device__ __forceinline__ f32x4 mfma16(const bf16x8_t& a, const bf16x8_t& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <int C, int R>
__global__ __launch_bounds__(256) void mla_decode_kernel(MlaParams p) {
  constexpr int CR = C + R, QS = CR + 8, CS = C + 8, RS = R + 8, PS = kMlaKT + 8;
  constexpr int NCW = C / 4, NT = NCW / 16;  // output columns per wave, 16-col tiles per wave
  static_assert(C % 64 == 0 && R % 32 == 0 && C % 32 == 0, "MLA decode: C % 64, R % 32");
  __shared__ __attribute__((aligned(16))) bf16 qimg[kMlaRB * QS];
  __shared__ __attribute__((aligned(16))) bf16 cimg[kMlaKT * CS];
  __shared__ __attribute__((aligned(16))) bf16 rimg[kMlaKT * RS];
  __shared__ __attribute__((aligned(16))) bf16 pimg[kMlaRB * PS];
  __shared__ float simg[kMlaRB * kMlaKT];
  __shared__ float mrow[kMlaRB], lrow[kMlaRB], arow[kMlaRB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nrb = cdiv(p.rows, kMlaRB);
  const int b = blockIdx.x / nrb, rb = blockIdx.x % nrb, split = blockIdx.y;
  const int r0 = rb * kMlaRB;
  const int S = p.kv_len_ptr ? *p.kv_len_ptr : p.kv_len;
  const int kbeg = split * p.tiles_per_split * kMlaKT;
  const int kend = min(S, kbeg + p.tiles_per_split * kMlaKT);
  // ---- query rows (token t = row / H, head h = row % H): [q_abs | q_rope] -> padded LDS rows
  for (int i = tid; i < kMlaRB * (CR / 8); i += 256) {
    const int r = i / (CR / 8), ch = i % (CR / 8), row = r0 + r;
    bf16x8_t v = {};
    if (row < p.rows) {
      const int t = row / p.H, h = row % p.H;
      const bf16* src = ch < C / 8 ? p.q + b * p.sqb + t * p.sqt + h * p.sqh + 8 * ch
                                   : p.qr + b * p.srb + t * p.srt + h * p.srh + 8 * (ch - C / 8);
      v = *reinterpret_cast<const bf16x8_t*>(src);
    }
    *reinterpret_cast<bf16x8_t*>(qimg + r * QS + 8 * ch) = v;
  }
  if (tid < kMlaRB) { mrow[tid] = -INFINITY; lrow[tid] = 0.f; }
  f32x4 o[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int l16 = lane & 15, g4 = lane >> 4;
  // softmax-phase thread layout: row = tid / 16, keys 4 (tid % 16) .. +3
  const int srw = tid >> 4, sk = 4 * (tid & 15);
  const int my_row = r0 + srw;
  // causal limit of this thread's row: token t sees keys < S - T + 1 + t
  const int lim = my_row < p.rows ? S - p.T + 1 + my_row / p.H : 0;
  for (int k0 = kbeg; k0 < kend; k0 += kMlaKT) {
    __syncthreads();  // previous tile's LDS reads done
    for (int i = tid; i < kMlaKT * (C / 8); i += 256) {
      const int kk = i / (C / 8), ch = i % (C / 8), key = k0 + kk;
      bf16x8_t v = {};
      if (key < kend) v = *reinterpret_cast<const bf16x8_t*>(p.cc + b * p.scb + (long)key * p.sct + 8 * ch);
      *reinterpret_cast<bf16x8_t*>(cimg + kk * CS + 8 * ch) = v;
    }
    for (int i = tid; i < kMlaKT * (R / 8); i += 256) {
      const int kk = i / (R / 8), ch = i % (R / 8), key = k0 + kk;
      bf16x8_t v = {};
      if (key < kend) v = *reinterpret_cast<const bf16x8_t*>(p.cr + b * p.srcb + (long)key * p.srct + 8 * ch);
      *reinterpret_cast<bf16x8_t*>(rimg + kk * RS + 8 * ch) = v;
    }
    __syncthreads();
    // ---- 1. S tile: wave w -> keys 16w .. 16w+15; A = Q rows (lane l16 = row), B = key rows
    {
      f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
      const bf16* qrow = qimg + l16 * QS + 8 * g4;
      const bf16* crow = cimg + (16 * wave + l16) * CS + 8 * g4;
      const bf16* rrow = rimg + (16 * wave + l16) * RS + 8 * g4;
#pragma unroll
      for (int ks = 0; ks < C / 32; ++ks)
        s = mfma16(*reinterpret_cast<const bf16x8_t*>(qrow + 32 * ks),
                   *reinterpret_cast<const bf16x8_t*>(crow + 32 * ks), s);
#pragma unroll
      for (int ks = 0; ks < R / 32; ++ks)
        s = mfma16(*reinterpret_cast<const bf16x8_t*>(qrow + C + 32 * ks),
                   *reinterpret_cast<const bf16x8_t*>(rrow + 32 * ks), s);
      // C/D layout: column (key) = lane & 15, row = 4 (lane >> 4) + i
#pragma unroll
      for (int i = 0; i < 4; ++i) simg[(4 * g4 + i) * kMlaKT + 16 * wave + l16] = s[i];
    }
    __syncthreads();
    // ---- 2. online softmax (log2 domain) over the 64 keys of the tile
    {
      float v[4], tm = -INFINITY;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = k0 + sk + i;
        v[i] = (key < kend && key < lim) ? simg[srw * kMlaKT + sk + i] * p.scale_log2 : -INFINITY;
        tm = fmaxf(tm, v[i]);
      }
#pragma unroll
      for (int o2 = 1; o2 < 16; o2 <<= 1) tm = fmaxf(tm, __shfl_xor(tm, o2, 64));
      const float mo = mrow[srw];
      const float mn = fmaxf(mo, tm);
      const float alpha = (mn == -INFINITY) ? 1.f : __builtin_amdgcn_exp2f(mo - mn);
      float ps = 0.f;
      bf16x4 pv;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float e = (v[i] == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(v[i] - mn);
        pv[i] = (bf16)e;
        ps += e;
      }
      *reinterpret_cast<bf16x4*>(pimg + srw * PS + sk) = pv;
#pragma unroll
      for (int o2 = 1; o2 < 16; o2 <<= 1) ps += __shfl_xor(ps, o2, 64);
      __syncthreads();  // every thread of the row has read mrow before it changes
      if ((tid & 15) == 0) {
        lrow[srw] = lrow[srw] * alpha + ps;
        mrow[srw] = mn;
        arow[srw] = alpha;
      }
    }
    __syncthreads();
    // ---- 3. O (16 rows x C/4 cols per wave) = alpha O + P C_tile
    {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float a = arow[4 * g4 + i];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) o[nt][i] *= a;
      }
      typedef __attribute__((address_space(3))) s16x4m lds_s4;
      const int q = l16 >> 2, pp = l16 & 3;
#pragma unroll
      for (int kst = 0; kst < kMlaKT / 32; ++kst) {
        // A = P[row l16][keys 32 kst + 8 g4 .. +8]
        const bf16x8_t pa = *reinterpret_cast<const bf16x8_t*>(pimg + l16 * PS + 32 * kst + 8 * g4);
        const int kr0 = 32 * kst + 8 * g4 + q;  // first of this lane's two tr rows
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const int col = NCW * wave + 16 * nt + 4 * pp;
          const s16x4m a4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(cimg + kr0 * CS + col));
          const s16x4m b4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(cimg + (kr0 + 4) * CS + col));
          const bf16x4 av = __builtin_bit_cast(bf16x4, a4), bv = __builtin_bit_cast(bf16x4, b4);
          const bf16x8_t bfr = __builtin_shufflevector(av, bv, 0, 1, 2, 3, 4, 5, 6, 7);
          o[nt] = mfma16(pa, bfr, o[nt]);
        }
      }
    }
  }
  __syncthreads();
  // ---- epilogue: rows 4 g4 + i, columns NCW w + 16 nt + l16
  if (p.nsplit == 1) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = r0 + 4 * g4 + i;
      if (row >= p.rows) continue;
      const float l = lrow[4 * g4 + i];
      const float inv = l > 0.f ? 1.f / l : 0.f;
      const int t = row / p.H, h = row % p.H;
      bf16* dst = p.out + b * p.sob + t * p.sot + h * p.soh;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) dst[NCW * wave + 16 * nt + l16] = (bf16)(o[nt][i] * inv);
    }
  } else {
    const long base = ((long)split * p.B + b) * p.rows;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = r0 + 4 * g4 + i;
      if (row >= p.rows) continue;
      float* dst = p.part_o + (base + row) * C;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) dst[NCW * wave + 16 * nt + l16] = o[nt][i];
    }
    if (tid < kMlaRB && r0 + tid < p.rows) {
      p.part_ml[(base + r0 + tid) * 2] = mrow[tid];
      p.part_ml[(base + r0 + tid) * 2 + 1] = lrow[tid];
    }
  }
}

// combine the splits: O = sum_s O_s 2^(m_s - M) / sum_s l_s 2^(m_s - M)
template <int C>
__global__ __launch_bounds__(256) void mla_merge_kernel(MlaParams p) {
  const long row = blockIdx.x;  // (b, row)
  const int b = row / p.rows, r = row % p.rows;
  float M = -INFINITY;
  for (int s = 0; s < p.nsplit; ++s) M = fmaxf(M, p.part_ml[(((long)s * p.B + b) * p.rows + r) * 2]);
  float L = 0.f;
  for (int s = 0; s < p.nsplit; ++s) {
    const float* ml = p.part_ml + (((long)s * p.B + b) * p.rows + r) * 2;
    if (ml[0] != -INFINITY) L += ml[1] * __builtin_amdgcn_exp2f(ml[0] - M);
  }
  const float inv = L > 0.f ? 1.f / L : 0.f;
  const int t = r / p.H, h = r % p.H;
  bf16* dst = p.out + b * p.sob + t * p.sot + h * p.soh;
  for (int c = threadIdx.x; c < C; c += 256) {
    float acc = 0.f;
    for (int s = 0; s < p.nsplit; ++s) {
      const long base = ((long)s * p.B + b) * p.rows + r;
      const float m = p.part_ml[base * 2];
      if (m != -INFINITY) acc += p.part_o[base * C + c] * __builtin_amdgcn_exp2f(m - M);
    }
    dst[c] = (bf16)(acc * inv);
  }
}

// q [B,T,H,C] (absorbed nope query), qr [B,T,H,R], cc [B,Smax,C], cr [B,Smax,R] (caches;
// row stride free, inner dim contiguous). Keys [0, kv_len) are valid; query token t sits at
// cache row kv_len - T + t (causal). kv_len_t (device int32 [1]) overrides kv_len (graph mode,
// then max_len bounds the split grid). Returns o_lat [B,T,H,C] bf16.
at::Tensor mla_decode(const at::Tensor& q, const at::Tensor& qr, const at::Tensor& cc, const at::Tensor& cr,
                      double scale, int64_t kv_len, const c10::optional<at::Tensor>& kv_len_t, int64_t nsplit_req) {
  for (auto* t : {&q, &qr, &cc, &cr})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->stride(-1) == 1,
                "mla_decode: bf16 HIP tensors, last dim contiguous");
  TORCH_CHECK(q.dim() == 4 && qr.dim() == 4 && cc.dim() == 3 && cr.dim() == 3, "mla_decode: ranks 4,4,3,3");
  const int B = q.size(0), T = q.size(1), H = q.size(2), C = q.size(3), R = qr.size(3), Smax = cc.size(1);
  TORCH_CHECK(cc.size(2) == C && cr.size(2) == R && qr.size(1) == T && qr.size(2) == H && cc.size(0) == B,
              "mla_decode: shape mismatch");
  for (auto* t : {&q, &qr})
    TORCH_CHECK(t->stride(0) % 8 == 0 && t->stride(1) % 8 == 0 && t->stride(2) % 8 == 0 &&
                (uintptr_t)t->data_ptr() % 16 == 0, "mla_decode: 16-byte aligned rows");
  for (auto* t : {&cc, &cr})
    TORCH_CHECK(t->stride(0) % 8 == 0 && t->stride(1) % 8 == 0 && (uintptr_t)t->data_ptr() % 16 == 0,
                "mla_decode: 16-byte aligned cache rows");
  const bool dev_len = kv_len_t.has_value();
  if (dev_len) TORCH_CHECK(kv_len_t->is_cuda() && kv_len_t->scalar_type() == at::kInt, "kv_len_t: int32 device");
  const int Sbound = dev_len ? Smax : (int)kv_len;
  TORCH_CHECK(Sbound <= Smax && T <= Sbound, "mla_decode: kv_len out of range");
  DeviceGuard g(q.device());
  auto out = at::empty({B, T, H, C}, q.options());
  MlaParams p{};
  p.q = (const bf16*)q.data_ptr(); p.qr = (const bf16*)qr.data_ptr();
  p.cc = (const bf16*)cc.data_ptr(); p.cr = (const bf16*)cr.data_ptr(); p.out = (bf16*)out.data_ptr();
  p.kv_len_ptr = dev_len ? kv_len_t->data_ptr<int>() : nullptr;
  p.kv_len = (int)kv_len;
  p.B = B; p.T = T; p.H = H; p.rows = T * H;
  p.sqb = q.stride(0); p.sqt = q.stride(1); p.sqh = q.stride(2);
  p.srb = qr.stride(0); p.srt = qr.stride(1); p.srh = qr.stride(2);
  p.scb = cc.stride(0); p.sct = cc.stride(1); p.srcb = cr.stride(0); p.srct = cr.stride(1);
  p.sob = out.stride(0); p.sot = out.stride(1); p.soh = out.stride(2);
  p.scale_log2 = (float)(scale * 1.4426950408889634);
  const int ntiles = cdiv(Sbound, kMlaKT);
  const int nrb = cdiv(p.rows, kMlaRB);
  // splits: enough workgroups to cover the chip at small batch, >= 2 tiles per split
  // splits: at small batch a block streams few tiles serially and the tile load latency is the
  // cost, so spread the key range up to one tile per split until the grid covers the chip
  int nsplit = nsplit_req > 0 ? (int)nsplit_req : std::max(1, std::min(ntiles, 256 / std::max(1, B * nrb)));
  nsplit = std::max(1, std::min(nsplit, ntiles));
  p.tiles_per_split = cdiv(ntiles, nsplit);
  nsplit = cdiv(ntiles, p.tiles_per_split);
  p.nsplit = nsplit;
  at::Tensor part;
  if (nsplit > 1) {
    part = at::empty({(long)nsplit * B * p.rows * (C + 2)}, q.options().dtype(at::kFloat));
    p.part_o = part.data_ptr<float>();
    p.part_ml = p.part_o + (long)nsplit * B * p.rows * C;
  }
  if (B * T * H == 0) return out;
  auto st = stream();
  dim3 grid(B * nrb, nsplit);
#define MLA_L(CV, RV)                                                              \
  do {                                                                             \
    mla_decode_kernel<CV, RV><<<grid, 256, 0, st>>>(p);                            \
    if (nsplit > 1) mla_merge_kernel<CV><<<B * p.rows, 256, 0, st>>>(p);           \
  } while (0)
  // kv_lora in {64, 128, 256, 512} x rope in {32, 64}: every preset (tiny, V2-Lite, V3)
  if (R == 64) {
    if (C == 512) MLA_L(512, 64);
    else if (C == 256) MLA_L(256, 64);
    else if (C == 128) MLA_L(128, 64);
    else if (C == 64) MLA_L(64, 64);
    else TORCH_CHECK(false, "mla_decode: kv_lora must be 64, 128, 256 or 512");
  } else if (R == 32) {
    if (C == 512) MLA_L(512, 32);
    else if (C == 256) MLA_L(256, 32);
    else if (C == 128) MLA_L(128, 32);
    else if (C == 64) MLA_L(64, 32);
    else TORCH_CHECK(false, "mla_decode: kv_lora must be 64, 128, 256 or 512");
  } else {
    TORCH_CHECK(false, "mla_decode: rope dim must be 32 or 64");
  }
#undef MLA_L
  SPA_LAUNCH_CHECK();
  return out;
}

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.def("mla_decode(Tensor q, Tensor qr, Tensor cc, Tensor cr, float scale, int kv_len, Tensor? kv_len_t=None, "
        "int nsplit=0) -> Tensor");
}
TORCH_LIBRARY_IMPL(spa, CUDA, m) { m.impl("mla_decode", &spa::mla_decode); }
