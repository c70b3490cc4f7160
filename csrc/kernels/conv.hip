// Implicit-GEMM 2-D convolution on MFMA (gfx950), K20: AlexNet convs (alexnet/alexnet.py:11-25)
// and the ViT patch embedding (vision transformer/ViT.ipynb:186). No column buffer is ever
// materialised: the activation operand of each GEMM is gathered tile-by-tile straight from the
// image into LDS, with zero fill for padding taps.
//
//   fwd    Y [N*OH*OW, OC]   = X~ [N*OH*OW, K] . Wp [OC, K]^T              (+ bias)
//   dgrad  dX [N*H*W, Cp]    = dY~ [N*H*W, KH*KW*OC] . Wr [KH*KW*OC, Cp]
//   wgrad  dW [OC, K]        = dY [N*OH*OW, OC]^T . X~ [N*OH*OW, K]        (split over rows)
//
// X~ / dY~ are the implicit im2col views. The K order of X~ is chosen so that 8 consecutive
// columns are 8 contiguous, 16-byte-aligned elements of the image:
//   * NHWC image (channels padded to Cp % 8 == 0), K = (kh, kw, c): the default layout -- a
//     conv net stays channels-last end to end (LRN / max-pool have NHWC kernels in misc.hip);
//   * NCHW image, K = (c, kh, kw), when KW, the W stride, the W padding and W are multiples of 8:
//     the ViT patchify (k = s = 16) reads the NCHW image directly, no layout pass at all.
// A per-8-column table ktab (int4: element offset, dh, dw) turns any column group into one
// address + two bounds checks, so the gather costs one 16-byte load and ~6 VALU ops per chunk;
// row decompositions (m -> n, i, j) use multiply-high division by runtime constants.
//
// Tiles: 128 x 128 x 32, 4 waves of 64 x 64 (2 x 2 v_mfma_f32_32x32x16_bf16 per 16-k step), LDS
// double-buffered through registers with one barrier per k-step, images and operand reads from
// gemm_common.h (K-contiguous images for the gathered / weight-row operands, K-strided images read
// with ds_read_b64_tr_b16 where the reduction runs over rows of the source).
// wgrad splits the N*OH*OW reduction over blockIdx.y into fp32 partials; a reduce kernel sums
// them and writes the gradient straight into the parameter's [OC, C, KH, KW] layout.
#include "spa_common.h"
#include "gemm_common.h"

SPA_DEBUG_TU("conv.hip")

namespace spa {

struct ConvGeo {
  int M, N, K;                       // GEMM dims (wgrad: M = OC, N = conv K, K = rows)
  const bf16* g;                     // gathered image
  long gN;                           // elements per image of g
  int gH, gW, sH, sW;                // bounds and element strides of h / w in g
  FastDiv dR, dC;                    // row m -> (n, r = i*J + j): dR divides by I*J, dC by J
  int rsh, rsw, rph, rpw;            // h0 = i*rsh - rph, w0 = j*rsw - rpw
  int ssh, ssw;                      // strided dgrad: tap (h, w) valid iff h % ssh == 0 ...
  const int4* ktab;                  // per 8-column group: (offset, dh, dw, -)
  const bf16* d;                     // dense operand
  long ldd;
  const int* btab;                   // dgrad: per-k row offset into the packed weights
  bf16* out;
  float* part;
  const bf16* bias;
  int kchunk;                        // wgrad: rows per split
  long gnumel;                       // elements of g (debug-build gather guard)
};

constexpr int CBM = 128, CBN = 128, CBK = 32, CNT = 256;

// MODE 0 fwd, 1 dgrad (stride 1), 2 dgrad (strided), 3 wgrad
template <int MODE>
__global__ __launch_bounds__(CNT, 2) void conv_gemm_kernel(ConvGeo p) {
  constexpr int BM = CBM, BN = CBN, BK = CBK, NT = CNT;
  constexpr int TM = 64, TN = 64, IM = 2, IN = 2;
  constexpr int AEL = BM * BK, BEL = BN * BK;
  constexpr int CA = AEL / 8 / NT, CB = BEL / 8 / NT;
  constexpr bool A_KC = MODE != 3, B_KC = MODE == 0;
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * (AEL + BEL)];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int nnt = (p.N + BN - 1) / BN;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int n0 = (lid % nnt) * BN, m0 = (lid / nnt) * BM;
  const int kbeg = MODE == 3 ? blockIdx.y * p.kchunk : 0;
  const int kend = MODE == 3 ? min(p.K, kbeg + p.kchunk) : p.K;

  // ---- per-thread fixed state of the gathered operand
  long gbase[2];
  int gh[2], gw[2];
  bool gv[2];
  int4 gt = make_int4(0, 0, 0, 0);
  auto decomp = [&](int m, long& base, int& h0, int& w0) {
    const int n = fdiv(m, p.dR);
    const int r = m - n * p.dR.d;
    const int i = fdiv(r, p.dC);
    const int j = r - i * p.dC.d;
    h0 = i * p.rsh - p.rph;
    w0 = j * p.rsw - p.rpw;
    base = (long)n * p.gN + (MODE == 2 ? 0L : (long)h0 * p.sH + (long)w0 * p.sW);
  };
  if (MODE != 3) {
#pragma unroll
    for (int c = 0; c < CA; ++c) {
      const int m = m0 + ((tid + c * NT) >> 2);
      gv[c] = m < p.M;
      decomp(gv[c] ? m : 0, gbase[c], gh[c], gw[c]);
    }
  } else {
    const int gn = n0 + (tid & 15) * 8;
    if (gn < p.N) gt = p.ktab[gn >> 3];
  }

  bf16x8 ra[CA], rb[CB];
  auto gather = [&](long base, int h0, int w0, int4 t, bool ok) -> bf16x8 {
    const int h = h0 + t.y, w = w0 + t.z;
    if (MODE == 2) {
      ok = ok && h >= 0 && w >= 0 && h % p.ssh == 0 && w % p.ssw == 0 && h / p.ssh < p.gH && w / p.ssw < p.gW;
      if (ok) SPA_DBG_CHECK(base + (long)(h / p.ssh) * p.sH + (long)(w / p.ssw) * p.sW + t.x + 7, p.gnumel);
      return ok ? *reinterpret_cast<const bf16x8*>(p.g + base + (long)(h / p.ssh) * p.sH + (long)(w / p.ssw) * p.sW + t.x)
                : bf16x8{};
    }
    ok = ok && (unsigned)h < (unsigned)p.gH && (unsigned)w < (unsigned)p.gW;
    if (ok) SPA_DBG_CHECK(base + t.x + 7, p.gnumel);   // debug build: the tap lies inside the image
    return ok ? *reinterpret_cast<const bf16x8*>(p.g + base + t.x) : bf16x8{};
  };
  auto load_tiles = [&](int kk) {
#pragma unroll
    for (int c = 0; c < CA; ++c) {
      const int idx = tid + c * NT;
      if (MODE != 3) {                      // gathered rows, K-contiguous
        const int gk = kk + (idx & 3) * 8;
        const bool ok = gv[c] && gk < kend;
        ra[c] = gather(gbase[c], gh[c], gw[c], ok ? p.ktab[gk >> 3] : make_int4(0, 0, 0, 0), ok);
      } else {                              // dY [rows][OC], K-strided: (row, 8 channels)
        const int gk = kk + (idx >> 4), gm = m0 + (idx & 15) * 8;
        ra[c] = (gk < kend && gm < p.M) ? *reinterpret_cast<const bf16x8*>(p.d + (long)gk * p.ldd + gm) : bf16x8{};
      }
    }
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      const int idx = tid + c * NT;
      if (MODE == 0) {                      // packed weights [OC][K]
        const int gn = n0 + (idx >> 2), gk = kk + (idx & 3) * 8;
        rb[c] = (gn < p.N && gk < kend) ? *reinterpret_cast<const bf16x8*>(p.d + (long)gn * p.ldd + gk) : bf16x8{};
      } else if (MODE != 3) {               // weight rows k = (kh, kw, oc), 8 channels
        const int gk = kk + (idx >> 4), gn = n0 + (idx & 15) * 8;
        rb[c] = (gk < kend && gn < p.N) ? *reinterpret_cast<const bf16x8*>(p.d + p.btab[gk] + gn) : bf16x8{};
      } else {                              // gathered X~ rows (reduction), fixed column group
        const int gk = kk + (idx >> 4), gn = n0 + (idx & 15) * 8;
        bool ok = gk < kend && gn < p.N;
        long base = 0;
        int h0 = 0, w0 = 0;
        decomp(ok ? gk : 0, base, h0, w0);
        rb[c] = gather(base, h0, w0, gt, ok);
      }
    }
  };
  auto store_tiles = [&](int buf) {
    bf16* At = smem + buf * (AEL + BEL);
    bf16* Bt = At + AEL;
#pragma unroll
    for (int c = 0; c < CA; ++c) {
      const int idx = tid + c * NT;
      if (A_KC) {
        const int r = idx >> 2, u = (idx & 3) * 2;
        *reinterpret_cast<bf16x4*>(At + kc_off<BK>(r, u)) = __builtin_shufflevector(ra[c], ra[c], 0, 1, 2, 3);
        *reinterpret_cast<bf16x4*>(At + kc_off<BK>(r, u + 1)) = __builtin_shufflevector(ra[c], ra[c], 4, 5, 6, 7);
      } else {
        *reinterpret_cast<bf16x8*>(At + ks_off<BM>(idx >> 4, idx & 15)) = ra[c];
      }
    }
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      const int idx = tid + c * NT;
      if (B_KC) {
        const int r = idx >> 2, u = (idx & 3) * 2;
        *reinterpret_cast<bf16x4*>(Bt + kc_off<BK>(r, u)) = __builtin_shufflevector(rb[c], rb[c], 0, 1, 2, 3);
        *reinterpret_cast<bf16x4*>(Bt + kc_off<BK>(r, u + 1)) = __builtin_shufflevector(rb[c], rb[c], 4, 5, 6, 7);
      } else {
        *reinterpret_cast<bf16x8*>(Bt + ks_off<BN>(idx >> 4, idx & 15)) = rb[c];
      }
    }
  };

  f32x16 acc[IN][IM];
#pragma unroll
  for (int i = 0; i < IN; ++i)
#pragma unroll
    for (int j = 0; j < IM; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int kt = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  const int l32 = lane & 31, hh = lane >> 5;
  if (kt > 0) {
    load_tiles(kbeg);
    store_tiles(0);
    if (kt > 1) load_tiles(kbeg + BK);
  }
  __syncthreads();
  for (int t = 0; t < kt; ++t) {
    const int buf = t & 1;
    if (t + 1 < kt) {
      store_tiles(buf ^ 1);
      if (t + 2 < kt) load_tiles(kbeg + (t + 2) * BK);
    }
    const bf16* At = smem + buf * (AEL + BEL);
    const bf16* Bt = At + AEL;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      bf16x8 af[IM], bfr[IN];
#pragma unroll
      for (int j = 0; j < IM; ++j) {
        const int mrow = wm * TM + j * 32;
        af[j] = A_KC ? ld_kc<BK>(At, mrow + l32, s, hh) : ld_ks<BM>(At, mrow, s, lane);
      }
#pragma unroll
      for (int i = 0; i < IN; ++i) {
        const int ncol = wn * TN + i * 32;
        bfr[i] = B_KC ? ld_kc<BK>(Bt, ncol + l32, s, hh) : ld_ks<BN>(Bt, ncol, s, lane);
      }
#pragma unroll
      for (int i = 0; i < IN; ++i)
#pragma unroll
        for (int j = 0; j < IM; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[i], af[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  // ---- epilogue (C^T tiles: lane owns column m = l32, rows n = 8g + 4hh + {0..3})
#pragma unroll
  for (int i = 0; i < IN; ++i)
#pragma unroll
    for (int j = 0; j < IM; ++j) {
      const int gm = m0 + wm * TM + j * 32 + l32;
      if (gm >= p.M) continue;
      if (MODE == 3) SPA_DBG_CHECK(blockIdx.y * p.kchunk, p.K);   // debug build: a live split
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int gn = n0 + wn * TN + i * 32 + 8 * g + 4 * hh;
        if (gn >= p.N) continue;
        if (MODE == 3) {
          f32x4 v;
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = acc[i][j][4 * g + q];
          *reinterpret_cast<f32x4*>(p.part + ((long)blockIdx.y * p.M + gm) * p.N + gn) = v;
        } else {
          bf16x4 w4;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            float v = acc[i][j][4 * g + q];
            if (MODE == 0 && p.bias) v += (float)p.bias[gn + q];
            w4[q] = (bf16)v;
          }
          *reinterpret_cast<bf16x4*>(p.out + (long)gm * p.N + gn) = w4;
        }
      }
    }
}

// ---------------------------------------------------------------------------- layout kernels
// any-strided 4-D [N, C, H, W] (NCHW or channels-last storage, bf16 / fp32) -> NHWC bf16 with the
// channel dim zero-padded to Cp; one thread per 8 output channels (16-byte store)
template <typename T>
__global__ __launch_bounds__(256) void to_nhwc_kernel(const T* __restrict__ x, bf16* __restrict__ y, int N, int C,
                                                      int H, int W, int Cp, long sn, long sc, long sh, long sw) {
  const int oct = Cp / 8;
  const long total = (long)N * H * W * oct;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int o = i % oct;
    const long pix = i / oct;
    const int w = pix % W, h = (pix / W) % H, n = pix / ((long)W * H);
    const T* src = x + n * sn + h * sh + w * sw;
    bf16x8 v;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = o * 8 + q;
      v[q] = c < C ? (bf16)(float)src[c * sc] : (bf16)0.f;
    }
    *reinterpret_cast<bf16x8*>(y + pix * Cp + o * 8) = v;
  }
}
// NHWC [N, H, W, Cp] -> contiguous NCHW [N, C, H, W] (drops padded channels)
__global__ __launch_bounds__(256) void from_nhwc_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int N,
                                                        int C, int H, int W, int Cp) {
  const long total = (long)N * C * H * W;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long hw = i % ((long)H * W);
    const long nc = i / ((long)H * W);
    const int c = nc % C, n = nc / C;
    y[i] = x[((long)n * H * W + hw) * Cp + c];
  }
}
// weight [OC, C, KH, KW] -> packed [OC, KH, KW, Cp] bf16 (padded channels zero)
template <typename T>
__global__ __launch_bounds__(256) void pack_weight_kernel(const T* __restrict__ w, bf16* __restrict__ out, int OC,
                                                          int C, int KH, int KW, int Cp) {
  const long total = (long)OC * KH * KW * Cp;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c = i % Cp;
    const long r = i / Cp;
    const int kw = r % KW, kh = (r / KW) % KH, oc = r / ((long)KW * KH);
    out[i] = c < C ? (bf16)(float)w[(((long)oc * C + c) * KH + kh) * KW + kw] : (bf16)0.f;
  }
}
// sum wgrad partials [S, OC, Kc] -> dW [OC, C, KH, KW] (param layout); Kc order (kh, kw, cp) when
// nhwc else (c, kh, kw)
template <typename OT>
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, OT* __restrict__ dw, int S,
                                                           int OC, int C, int KH, int KW, int Cp, int nhwc) {
  const long Kc = nhwc ? (long)KH * KW * Cp : (long)C * KH * KW;
  const long total = (long)OC * C * KH * KW;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int kw = i % KW, kh = (i / KW) % KH;
    const int c = (i / ((long)KW * KH)) % C;
    const long oc = i / ((long)KW * KH * C);
    const long col = nhwc ? ((long)kh * KW + kw) * Cp + c : i % Kc;
    float s = 0.f;
    for (int q = 0; q < S; ++q) s += part[((long)q * OC + oc) * Kc + col];
    dw[i] = (OT)s;
  }
}
// bias grad: column sums of dY [rows, OC]; block (x: 32 channel octets, y: row split), 8 row lanes
__global__ __launch_bounds__(256) void bias_part_kernel(const bf16* __restrict__ dy, float* __restrict__ part,
                                                        int rows, int OC, int chunk) {
  __shared__ float red[8][256 + 8];
  const int oc8 = blockIdx.x * 32 + (threadIdx.x & 31), rl = threadIdx.x >> 5;
  const int r0 = blockIdx.y * chunk, r1 = min(rows, r0 + chunk);
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (oc8 * 8 < OC)
    for (int r = r0 + rl; r < r1; r += 8) {
      float f[8];
      load8(dy + (long)r * OC + oc8 * 8, f);
#pragma unroll
      for (int q = 0; q < 8; ++q) s[q] += f[q];
    }
#pragma unroll
  for (int q = 0; q < 8; ++q) red[rl][(threadIdx.x & 31) * 8 + q] = s[q];
  __syncthreads();
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col < OC) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) t += red[q][threadIdx.x];
    part[(long)blockIdx.y * OC + col] = t;
  }
}
template <typename OT>
__global__ __launch_bounds__(256) void bias_reduce_kernel(const float* __restrict__ part, OT* __restrict__ db, int S,
                                                          int OC) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= OC) return;
  float s = 0.f;
  for (int q = 0; q < S; ++q) s += part[(long)q * OC + c];
  db[c] = (OT)s;
}

// ---------------------------------------------------------------------------- host
static int grid1(long n) { return (int)std::max<long>(1, std::min<long>((n + 255) / 256, 16384)); }

at::Tensor conv_to_nhwc(const at::Tensor& x, int64_t Cp) {
  SPA_CHECK_CUDA(x);
  TORCH_CHECK(x.dim() == 4 && Cp % 8 == 0 && Cp >= x.size(1), "conv_to_nhwc: 4-D input, Cp % 8 == 0");
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  DeviceGuard g(x.device());
  auto y = at::empty({N, H, W, Cp}, x.options().dtype(at::kBFloat16));
  const long total = (long)N * H * W * (Cp / 8);
  if (total == 0) return y;
#define TN(TT)                                                                                                \
  to_nhwc_kernel<TT><<<grid1(total), 256, 0, stream()>>>((const TT*)x.data_ptr(), (bf16*)y.data_ptr(), N, C, H, W, \
                                                         Cp, x.stride(0), x.stride(1), x.stride(2), x.stride(3))
  if (x.scalar_type() == at::kBFloat16) TN(bf16); else if (x.scalar_type() == at::kFloat) TN(float);
  else TORCH_CHECK(false, "conv_to_nhwc: bf16/fp32");
#undef TN
  SPA_LAUNCH_CHECK();
  return y;
}

at::Tensor conv_from_nhwc(const at::Tensor& x, int64_t C) {
  SPA_CHECK_CUDA(x);
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous() && x.scalar_type() == at::kBFloat16);
  const int N = x.size(0), H = x.size(1), W = x.size(2), Cp = x.size(3);
  TORCH_CHECK(C <= Cp);
  DeviceGuard g(x.device());
  auto y = at::empty({N, C, H, W}, x.options());
  const long total = (long)N * C * H * W;
  if (total == 0) return y;
  from_nhwc_kernel<<<grid1(total), 256, 0, stream()>>>((const bf16*)x.data_ptr(), (bf16*)y.data_ptr(), N, C, H, W, Cp);
  SPA_LAUNCH_CHECK();
  return y;
}

at::Tensor conv_pack_weight(const at::Tensor& w_, int64_t Cp) {
  auto w = w_.contiguous();
  SPA_CHECK_CUDA(w);
  TORCH_CHECK(w.dim() == 4 && Cp % 8 == 0 && Cp >= w.size(1));
  const int OC = w.size(0), C = w.size(1), KH = w.size(2), KW = w.size(3);
  DeviceGuard g(w.device());
  auto out = at::empty({OC, KH, KW, Cp}, w.options().dtype(at::kBFloat16));
  const long total = out.numel();
  if (total == 0) return out;
  if (w.scalar_type() == at::kBFloat16)
    pack_weight_kernel<bf16><<<grid1(total), 256, 0, stream()>>>((const bf16*)w.data_ptr(), (bf16*)out.data_ptr(), OC,
                                                                 C, KH, KW, Cp);
  else
    pack_weight_kernel<float><<<grid1(total), 256, 0, stream()>>>(w.data_ptr<float>(), (bf16*)out.data_ptr(), OC, C,
                                                                  KH, KW, Cp);
  SPA_LAUNCH_CHECK();
  return out;
}

// geo = [nhwc, N, C, H, W, Cp, OC, KH, KW, sh, sw, ph, pw, OH, OW]
struct Geo {
  int nhwc, N, C, H, W, Cp, OC, KH, KW, sh, sw, ph, pw, OH, OW;
  explicit Geo(const std::vector<int64_t>& v) {
    TORCH_CHECK(v.size() == 15, "conv geo: 15 ints");
    nhwc = v[0]; N = v[1]; C = v[2]; H = v[3]; W = v[4]; Cp = v[5]; OC = v[6]; KH = v[7]; KW = v[8];
    sh = v[9]; sw = v[10]; ph = v[11]; pw = v[12]; OH = v[13]; OW = v[14];
    TORCH_CHECK(OH == (H + 2 * ph - KH) / sh + 1 && OW == (W + 2 * pw - KW) / sw + 1, "conv geo: output size");
    TORCH_CHECK(OC % 8 == 0, "conv: out channels must be a multiple of 8");
    if (nhwc) {
      TORCH_CHECK(Cp % 8 == 0 && Cp >= C, "conv: NHWC channels padded to a multiple of 8");
    } else {
      TORCH_CHECK(Cp == C && KW % 8 == 0 && sw % 8 == 0 && pw % 8 == 0 && W % 8 == 0,
                  "conv: NCHW gather needs KW, stride_w, pad_w and W multiples of 8");
    }
  }
  long K() const { return (long)KH * KW * Cp; }
  long rows() const { return (long)N * OH * OW; }
};

static void fill_gather(ConvGeo& p, const Geo& G, const at::Tensor& x) {
  p.g = (const bf16*)x.data_ptr();
  p.gnumel = x.numel();
  p.gN = (long)G.Cp * G.H * G.W;
  p.gH = G.H; p.gW = G.W;
  p.sH = G.nhwc ? G.W * G.Cp : G.W;
  p.sW = G.nhwc ? G.Cp : 1;
  p.dR = make_fastdiv(G.OH * G.OW);
  p.dC = make_fastdiv(G.OW);
  p.rsh = G.sh; p.rsw = G.sw; p.rph = G.ph; p.rpw = G.pw;
  p.ssh = p.ssw = 1;
}

static void check_x(const at::Tensor& x, const Geo& G) {
  SPA_CHECK_CUDA(x);
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.is_contiguous(), "conv: bf16 contiguous gathered image");
  if (G.nhwc) {
    TORCH_CHECK(x.dim() == 4 && x.size(0) == G.N && x.size(1) == G.H && x.size(2) == G.W && x.size(3) == G.Cp,
                "conv: NHWC image shape");
  } else {
    TORCH_CHECK(x.dim() == 4 && x.size(0) == G.N && x.size(1) == G.C && x.size(2) == G.H && x.size(3) == G.W,
                "conv: NCHW image shape");
  }
  TORCH_CHECK(x.numel() < (1L << 31) && G.rows() < (1L << 31), "conv: < 2^31 elements / rows");
}

// x: gathered image (NHWC [N,H,W,Cp] or NCHW [N,C,H,W]); wp [OC, K] in the same K order;
// ktab int32 [K/8, 4]; returns Y NHWC [N, OH, OW, OC]
at::Tensor conv_fwd(const at::Tensor& x, const at::Tensor& wp, const at::Tensor& ktab,
                    const c10::optional<at::Tensor>& bias, std::vector<int64_t> geo) {
  const Geo G(geo);
  check_x(x, G);
  const long K = G.K();
  TORCH_CHECK(wp.scalar_type() == at::kBFloat16 && wp.is_contiguous() && wp.numel() == (long)G.OC * K, "conv: wp");
  TORCH_CHECK(ktab.scalar_type() == at::kInt && ktab.is_contiguous() && ktab.numel() == K / 8 * 4, "conv: ktab");
  if (bias) TORCH_CHECK(bias->scalar_type() == at::kBFloat16 && bias->numel() == G.OC && bias->is_contiguous());
  DeviceGuard g(x.device());
  auto y = at::empty({G.N, G.OH, G.OW, G.OC}, x.options());
  if (G.rows() == 0) return y;
  ConvGeo p{};
  fill_gather(p, G, x);
  p.M = G.rows(); p.N = G.OC; p.K = K;
  p.ktab = (const int4*)ktab.data_ptr<int>();
  p.d = (const bf16*)wp.data_ptr(); p.ldd = K;
  p.out = (bf16*)y.data_ptr();
  p.bias = bias ? (const bf16*)bias->data_ptr() : nullptr;
  const int grid = cdiv(p.M, CBM) * cdiv(p.N, CBN);
  conv_gemm_kernel<0><<<grid, CNT, 0, stream()>>>(p);
  SPA_LAUNCH_CHECK();
  return y;
}

// dy NHWC [N, OH, OW, OC]; wp packed NHWC [OC, KH, KW, Cp]; ktab [KH*KW*OC/8, 4] over dY~ columns
// (kh, kw, oc); btab int32 [KH*KW*OC] row offsets into wp; returns dX NHWC [N, H, W, Cp]
at::Tensor conv_dgrad(const at::Tensor& dy, const at::Tensor& wp, const at::Tensor& ktab, const at::Tensor& btab,
                      std::vector<int64_t> geo) {
  const Geo G(geo);
  TORCH_CHECK(G.nhwc, "conv_dgrad: NHWC geometry");
  SPA_CHECK_CUDA(dy);
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && dy.is_contiguous() && dy.numel() == G.rows() * G.OC, "conv: dy");
  TORCH_CHECK(wp.scalar_type() == at::kBFloat16 && wp.is_contiguous() && wp.numel() == (long)G.OC * G.K());
  const long Kd = (long)G.KH * G.KW * G.OC;
  TORCH_CHECK(ktab.numel() == Kd / 8 * 4 && btab.numel() == Kd && btab.scalar_type() == at::kInt);
  TORCH_CHECK((long)G.N * G.H * G.W < (1L << 31) && dy.numel() < (1L << 31));
  DeviceGuard g(dy.device());
  auto dx = at::empty({G.N, G.H, G.W, G.Cp}, dy.options());
  if (dx.numel() == 0) return dx;
  ConvGeo p{};
  p.M = G.N * G.H * G.W; p.N = G.Cp; p.K = Kd;
  p.g = (const bf16*)dy.data_ptr();
  p.gnumel = dy.numel();
  p.gN = (long)G.OH * G.OW * G.OC;
  p.gH = G.OH; p.gW = G.OW;
  p.sH = G.OW * G.OC; p.sW = G.OC;
  p.dR = make_fastdiv(G.H * G.W);
  p.dC = make_fastdiv(G.W);
  p.rsh = 1; p.rsw = 1; p.rph = -G.ph; p.rpw = -G.pw;   // h0 = ih + ph
  p.ssh = G.sh; p.ssw = G.sw;
  p.ktab = (const int4*)ktab.data_ptr<int>();
  p.d = (const bf16*)wp.data_ptr(); p.ldd = 0;
  p.btab = btab.data_ptr<int>();
  p.out = (bf16*)dx.data_ptr();
  const int grid = cdiv(p.M, CBM) * cdiv(p.N, CBN);
  if (G.sh == 1 && G.sw == 1) conv_gemm_kernel<1><<<grid, CNT, 0, stream()>>>(p);
  else conv_gemm_kernel<2><<<grid, CNT, 0, stream()>>>(p);
  SPA_LAUNCH_CHECK();
  return dx;
}

// dy NHWC [N, OH, OW, OC]; x gathered image as in conv_fwd; returns (dW [OC, C, KH, KW] of
// w_dtype, dB [OC] of w_dtype or empty)
std::vector<at::Tensor> conv_wgrad(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& ktab,
                                   std::vector<int64_t> geo, bool want_bias, at::ScalarType w_dtype, int64_t splits) {
  const Geo G(geo);
  check_x(x, G);
  SPA_CHECK_CUDA(dy);
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && dy.is_contiguous() && dy.numel() == G.rows() * G.OC, "conv: dy");
  const long K = G.K();
  TORCH_CHECK(ktab.numel() == K / 8 * 4);
  TORCH_CHECK(w_dtype == at::kBFloat16 || w_dtype == at::kFloat);
  DeviceGuard g(x.device());
  auto st = stream();
  auto opts = x.options();
  auto dw = at::empty({G.OC, G.C, G.KH, G.KW}, opts.dtype(w_dtype));
  auto db = want_bias ? at::empty({G.OC}, opts.dtype(w_dtype)) : at::Tensor();
  const long rows = G.rows();
  const int tiles = cdiv(G.OC, CBM) * cdiv(K, CBN);
  // ~2048 blocks, >= 512 rows per split, and the fp32 partial slab kept to <= 64 MiB
  const long slab = (long)G.OC * K * 4;
  int S = splits > 0 ? (int)splits
                     : std::max(1, std::min<int>(std::min<int>(cdiv(2048, tiles), cdiv(rows, 512)),
                                                 (int)std::max<long>(1, (64L << 20) / slab)));
  const int kchunk = cdiv(cdiv(rows, S), CBK) * CBK;
  S = std::max(1, cdiv(rows, kchunk));
  auto part = at::empty({S, G.OC, K}, opts.dtype(at::kFloat));
  ConvGeo p{};
  fill_gather(p, G, x);
  p.M = G.OC; p.N = K; p.K = rows;
  p.ktab = (const int4*)ktab.data_ptr<int>();
  p.d = (const bf16*)dy.data_ptr(); p.ldd = G.OC;
  p.part = part.data_ptr<float>();
  p.kchunk = kchunk;
  if (rows > 0) {
    conv_gemm_kernel<3><<<dim3(tiles, S), CNT, 0, st>>>(p);
  } else {
    part.zero_();
  }
  const long tot = dw.numel();
  if (w_dtype == at::kBFloat16)
    wgrad_reduce_kernel<bf16><<<grid1(tot), 256, 0, st>>>(p.part, (bf16*)dw.data_ptr(), S, G.OC, G.C, G.KH, G.KW, G.Cp,
                                                          G.nhwc);
  else
    wgrad_reduce_kernel<float><<<grid1(tot), 256, 0, st>>>(p.part, dw.data_ptr<float>(), S, G.OC, G.C, G.KH, G.KW,
                                                           G.Cp, G.nhwc);
  if (want_bias) {
    const int Sb = std::max(1, std::min<int>(64, cdiv(rows, 1024)));
    const int chunk = std::max<int>(1, cdiv(rows, Sb));
    auto bpart = at::empty({Sb, G.OC}, opts.dtype(at::kFloat));
    bias_part_kernel<<<dim3(cdiv(G.OC, 256), Sb), 256, 0, st>>>((const bf16*)dy.data_ptr(), bpart.data_ptr<float>(),
                                                               (int)rows, G.OC, chunk);
    if (w_dtype == at::kBFloat16)
      bias_reduce_kernel<bf16><<<cdiv(G.OC, 256), 256, 0, st>>>(bpart.data_ptr<float>(), (bf16*)db.data_ptr(), Sb, G.OC);
    else
      bias_reduce_kernel<float><<<cdiv(G.OC, 256), 256, 0, st>>>(bpart.data_ptr<float>(), db.data_ptr<float>(), Sb,
                                                                  G.OC);
  }
  SPA_LAUNCH_CHECK();
  return {dw, db};
}

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.def("conv_to_nhwc(Tensor x, int Cp) -> Tensor");
  m.def("conv_from_nhwc(Tensor x, int C) -> Tensor");
  m.def("conv_pack_weight(Tensor w, int Cp) -> Tensor");
  m.def("conv_fwd(Tensor x, Tensor wp, Tensor ktab, Tensor? bias, int[] geo) -> Tensor");
  m.def("conv_dgrad(Tensor dy, Tensor wp, Tensor ktab, Tensor btab, int[] geo) -> Tensor");
  m.def("conv_wgrad(Tensor dy, Tensor x, Tensor ktab, int[] geo, bool want_bias, ScalarType w_dtype, int splits=0) -> Tensor[]");
}
TORCH_LIBRARY_IMPL(spa, CUDA, m) {
  m.impl("conv_to_nhwc", &spa::conv_to_nhwc);
  m.impl("conv_from_nhwc", &spa::conv_from_nhwc);
  m.impl("conv_pack_weight", &spa::conv_pack_weight);
  m.impl("conv_fwd", &spa::conv_fwd);
  m.impl("conv_dgrad", &spa::conv_dgrad);
  m.impl("conv_wgrad", &spa::conv_wgrad);
}
