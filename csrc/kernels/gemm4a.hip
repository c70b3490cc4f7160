// Grouped / dense bf16 GEMM, third generation: the hipBLASLt tile shape (256 x 256 C tile, 4 waves,
// one per SIMD, each owning a 128 x 128 quadrant = 64 16x16 MFMA tiles = 256 fp32 accumulators per
// lane) with the accumulators PINNED in the accumulator register file.
//
// Why: written with __builtin_amdgcn_mfma_*, hipcc splits 256 loop-carried accumulators per lane
// over VGPRs and AGPRs and re-homes them every trip (148-460 v_accvgpr moves per 128 MFMAs,
// profiles/r5_gemm4w_hipblaslt_shape_probe.txt), so this shape ran 1,108 TF against hipBLASLt's
// 1,712 at 8192^3. Here every MFMA is an inline-asm v_mfma_f32_16x16x32_bf16 whose C/D operand is an
// "+a" (AGPR) constraint: the register allocator must keep each accumulator quad in a[...] at every
// MFMA, so the loop carries them there with no copies; A / B fragments stay in VGPRs (ds_read_b128
// destinations, waited for by hipcc's own lgkmcnt bookkeeping, which sees the asm operands).
//
// Pipeline (per 32-deep K slice, one s_barrier each): a 4-stage LDS ring filled by
// buffer_load ... lds (16 B per lane, lane-linear images, swizzle in the per-lane SOURCE address)
// three slices ahead; the wave's 16 fragments of slice t+1 are read (ds_read_b128) into the other
// register set while the 64 MFMAs of slice t run, interleaved one read per 4 MFMAs with the 8 DMA
// pieces of slice t+3 spread over the stream. A counted vmcnt before each barrier retires exactly
// the slice the next one reads; all LDS is one array and every barrier is a bare s_barrier.
//
// Modes (grouped_gemm8's contract, csrc/kernels/gemm8.hip):
//   0 fwd   Y[M, N]  = X[M, K] W_e[N, K]^T        rows grouped by offsets (E = 1: dense X W^T)
//   1 dX    dX[M, N] = dY[M, K] W_e[K, N]          rows grouped (W_e stored [K=Nw][N=Kw])
//   2 dW    dW_e[N, K] = dY_e[T, N]^T X_e[T, K]   reduction rows grouped (token segments);
//           PART: the "experts" are token slices of one dense product, fp32 partials (wgrad4a)
//
// LDS images of one operand slice (lane-linear DMA destinations; the swizzle is an involution
// applied to the per-lane SOURCE address and to the read address):
//   K-contiguous [256 rows][32 k], 64-B rows: 16-B chunk c of row r at r * 64 + 16 * (c ^ ((r >> 2) & 3))
//     -- the 16 lanes of a ds_read_b128 quarter (16 consecutive rows, one chunk) hit 16 distinct
//     16-B bank groups;
//   K-strided [32 k][256 cols], 512-B rows: chunk c of k-row r at r * 512 + 16 * (c ^ f(r)),
//     f(r) = ((r & 3) << 2) | ((r >> 2) & 3) -- read with ds_read_b64_tr_b16 (gemm8's recipe).
#include "gemm_common.h"

#include <string>
#include <type_traits>

SPA_DEBUG_TU("gemm4a.hip")

namespace spa {

namespace g4 {

constexpr int BM = 256, BN = 256, BK = 32, NT = 256, NS = 4;
constexpr int IMG = 256 * BK * 2;             // one operand slice image (16 KiB)
constexpr int STAGE = 2 * IMG;                // A + B of one slice (32 KiB)
constexpr int RING = NS * STAGE;              // 128 KiB
constexpr int ERS = 256 * 2 + 16;             // epilogue C image row stride (bytes)
constexpr int SMEM = (RING > 256 * ERS ? RING : 256 * ERS) + 64;

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, long bytes) {
  const long nb = bytes < 0 ? 0 : (bytes > 0xFFFFFFFFL ? 0xFFFFFFFFL : bytes);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)(unsigned)nb, 0x00020000);
}
// byte offset (from the slice origin in global memory) of DMA piece j (0..3) of this thread, 16-B
// slot q = j * 256 + tid:
//   K-contiguous: row q >> 2, physical chunk q & 3, logical chunk (q & 3) ^ ((row >> 2) & 3)
//   K-strided:    k-row q >> 5, physical chunk q & 31, logical chunk (q & 31) ^ f(row)
__device__ __forceinline__ int ksw(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
__device__ __forceinline__ unsigned dma_off(bool kc, int tid, int j, long ld) {
  const int q = j * NT + tid;
  if (kc) {
    const int r = q >> 2, c = (q & 3) ^ ((r >> 2) & 3);
    return (unsigned)((r * ld + 8 * c) * 2);
  }
  const int r = q >> 5, c = (q & 31) ^ ksw(r);
  return (unsigned)((r * ld + 8 * c) * 2);
}
typedef __attribute__((address_space(3))) s16x4_t lds_s4;
// 16x16x32 operand of image columns col0 .. col0+15 from a K-strided image (gemm8 rd_ks, 512-B rows)
__device__ __forceinline__ bf16x8 rd_ks(const char* img, int col0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int ch = (col0 >> 3) + (p >> 1);
  const int ra = 8 * g + q, rb = ra + 4;
  const s16x4_t a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + ra * 512 + 16 * (ch ^ ksw(ra)) + 8 * (p & 1)));
  const s16x4_t b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + rb * 512 + 16 * (ch ^ ksw(rb)) + 8 * (p & 1)));
  const bf16x4 av = __builtin_bit_cast(bf16x4, a), bv = __builtin_bit_cast(bf16x4, b);
  return __builtin_shufflevector(av, bv, 0, 1, 2, 3, 4, 5, 6, 7);
}

}  // namespace g4

#define G4_MFMA(ACC, A, B) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(ACC) : "v"(A), "v"(B))
// first slice: C = inline constant 0, so every definition of an accumulator is an AGPR-constrained
// asm output (a C++ zero-init is a VGPR def: the loop-carried PHIs then live in VGPRs and are
// copied into AGPRs around every MFMA)
#define G4_MFMA0(ACC, A, B) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(ACC) : "v"(A), "v"(B))

// block -> output tile: (expert, row tile, column tile) and, in mode 2, the expert's token range.
// Modes 0 / 1: inclusive scan of the experts' row-tile counts (one expert per thread). Mode 2: heavy
// experts first, dealt to the XCDs in snake order (gemm8.hip mode 2); PART: plain order. Uses the
// first E4 ints of smem (before the ring is filled) and scratch[0..15]; false: no tile for this block.
struct G4Tile {
  int e;
  long m0, mend, n0, k0, kend;
  const bf16* Bp;
  bf16* Cp;
};
template <int MODE, bool PART>
__device__ __forceinline__ bool g4_map(G4Tile& out, char* smem, int* scratch, const int* __restrict__ offsets, int E,
                                       int M, int N, long strideB, long strideC, int gm, const bf16* B, bf16* C) {
  using namespace g4;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nnt = (N + BN - 1) / BN;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  int nt = lid % nnt;
  int mt = lid / nnt;
  int e = 0;
  long m0 = 0, mend = M, k0 = 0, kend = 0;
  const bf16* Bp = B;
  bf16* Cp = C;
  if (MODE != 2) {
    // tile -> (expert, row tile): inclusive scan of the experts' row-tile counts (one per thread).
    // The grid is sized for the worst case (every expert ragged); the REAL tiles R = rows x nnt take
    // the lowest block ids and the XCD remap runs over R, so no real tile waits behind an empty
    // block for a second dispatch round (the remap over the whole grid had scattered the empty
    // blocks: at 4096^3 16 real tiles landed past the 256 CUs and the kernel ran two rounds)
    int* wsum = scratch + 8;
    const int o0 = tid < E ? offsets[tid] : 0, o1 = tid < E ? offsets[tid + 1] : 0;
    const int tiles = (o1 - o0 + BM - 1) / BM;
    int inc = tiles;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(inc, o, 64);
      if (lane >= o) inc += v;
    }
    if (lane == 63) wsum[wave] = inc;
    if (tid == 0) scratch[0] = -1;
    __syncthreads();
    int pre = inc - tiles, rows = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
      const int v = wsum[w];
      pre += w < wave ? v : 0;
      rows += v;
    }
    const int R = rows * nnt;
    if ((int)blockIdx.x >= R) return false;                  // uniform: empty blocks exit together
    const int lid = xcd_remap(blockIdx.x, R);
    nt = lid % nnt;
    mt = lid / nnt;
    if (gm > 1) {   // groups of gm row tiles x all column tiles (L2 reuse of B panels), dense only
      const int g = lid / (gm * nnt), r = lid % (gm * nnt);
      const int gs = min(gm, rows - g * gm);
      mt = g * gm + r % gs;
      nt = r / gs;
    }
    if (tid < E && tiles > 0 && mt >= pre && mt < pre + tiles) {
      scratch[0] = tid; scratch[1] = mt - pre; scratch[2] = o0; scratch[3] = o1;
    }
    __syncthreads();
    e = __builtin_amdgcn_readfirstlane(scratch[0]);
    if (e < 0) return false;
    mt = __builtin_amdgcn_readfirstlane(scratch[1]);
    m0 = __builtin_amdgcn_readfirstlane(scratch[2]) + (long)mt * BM;
    mend = __builtin_amdgcn_readfirstlane(scratch[3]);
    Bp = B + e * strideB;
  } else {
    const int nmt = (M + BM - 1) / BM;
    const int per_e = nmt * nnt;
    if constexpr (!PART) {
      // heavy experts first, dealt to the XCDs in snake order (gemm8.hip mode 2: every expert owns
      // the same output tiles but a tile's work is its token count)
      int* cnt = reinterpret_cast<int*>(smem);
      const int E4 = (E + 3) & ~3;
      const int o0 = tid < E ? offsets[tid] : 0, o1 = tid < E ? offsets[tid + 1] : 0;
      if (tid < E4) cnt[tid] = o1 - o0;
      __syncthreads();
      const int4* cnt4 = reinterpret_cast<const int4*>(cnt);
      long tot = 0;
      int mx = 0;
#pragma unroll 4
      for (int j = 0; j < E4 / 4; ++j) {
        const int4 v = cnt4[j];
        tot += (long)v.x + v.y + v.z + v.w;
        mx = max(max(mx, max(v.x, v.y)), max(v.z, v.w));
      }
      const bool snake = E % 8 == 0 && (long)mx * E <= 2 * tot;
      int pos, r;
      if (snake) {
        const int x = blockIdx.x % 8, j = blockIdx.x / 8, u = j / per_e;
        r = j % per_e;
        pos = u * 8 + ((u & 1) ? 7 - x : x);
      } else {
        pos = blockIdx.x / per_e;
        r = blockIdx.x % per_e;
      }
      if (pos >= E) return false;
      nt = r % nnt;
      mt = r / nnt;
      if (tid < E) {
        const int c = o1 - o0;
        int rank = 0;
#pragma unroll 4
        for (int j = 0; j < E4 / 4; ++j) {
          const int4 v = cnt4[j];
          rank += (v.x > c) || (v.x == c && 4 * j < tid);
          rank += (v.y > c) || (v.y == c && 4 * j + 1 < tid);
          rank += (v.z > c) || (v.z == c && 4 * j + 2 < tid);
          rank += (v.w > c) || (v.w == c && 4 * j + 3 < tid);
        }
        if (rank == pos) { scratch[0] = tid; scratch[2] = o0; scratch[3] = o1; }
      }
      __syncthreads();
      e = __builtin_amdgcn_readfirstlane(scratch[0]);
      __syncthreads();   // the count image lives in the ring the prologue DMA fills
    } else {
      e = blockIdx.x / per_e;
      if (e >= E) return false;
      const int r = blockIdx.x % per_e;
      nt = r % nnt;
      mt = r / nnt;
      if (tid == 0) { scratch[2] = offsets[e]; scratch[3] = offsets[e + 1]; }
      __syncthreads();
    }
    m0 = (long)mt * BM;
    k0 = __builtin_amdgcn_readfirstlane(scratch[2]);
    kend = __builtin_amdgcn_readfirstlane(scratch[3]);
    Cp = C + e * strideC;
  }
  out.e = e;
  out.m0 = m0;
  out.mend = mend;
  out.n0 = (long)nt * BN;
  out.k0 = k0;
  out.kend = kend;
  out.Bp = Bp;
  out.Cp = Cp;
  return true;
}

// epilogue of both kernels: PART -> fp32 partials straight from the fragments; else C^T fragments ->
// padded bf16 row image [256][256] in LDS -> 16-B global stores (+ the old value when accumulate)
template <int MODE, bool PART>
__device__ __forceinline__ void g4_epilogue(f32x4 (&acc)[8][8], char* smem, bf16* C, bf16* Cp, int e, long m0,
                                            long n0, long rowlim, int M, int N, long ldc, long strideC,
                                            int accumulate, long a_rows) {
  using namespace g4;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  if constexpr (PART) {
    // fp32 partials straight from the fragments (16 B per lane along a C row)
    float* Cf = reinterpret_cast<float*>(C) + (long)e * strideC;
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const long gmr = m0 + wm * 128 + 16 * i + (lane & 15);
        const long gn = n0 + wn * 128 + 16 * j + 4 * (lane >> 4);
        if (gmr < M && gn < N && SPA_DBG_OK(gn + 3, ldc)) *reinterpret_cast<f32x4*>(Cf + gmr * ldc + gn) = acc[j][i];
      }
    return;
  }
  // ---- epilogue: C^T fragments -> padded bf16 row image [256][256] in LDS -> 16-B global stores
  // accumulate: this thread's 32 old C chunks are requested first (128 VGPRs, free once the main
  // loop is done), so their latency hides under the image build and its barrier; read inside the
  // store loop they cost one memory round trip per unrolled group of 4 (8 per tile), which at the
  // expert dW's ~768-deep reductions was as long as a third of the tile's MFMA work
  bf16x8 old[32];
  if (accumulate) {
#pragma unroll
    for (int c = 0; c < 32; ++c) {
      const int idx = tid + c * NT, r = idx >> 5, ch = idx & 31;
      const long gmr = m0 + r;
      const long gn = n0 + ch * 8;
      bf16x8 o;
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = (bf16)0.f;
      if (gmr < rowlim && gn < N) o = *reinterpret_cast<const bf16x8*>(Cp + gmr * ldc + gn);
      old[c] = o;
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const f32x4 v = acc[j][i];
      bf16x4 w4;
#pragma unroll
      for (int q = 0; q < 4; ++q) w4[q] = (bf16)v[q];
      const int r = wm * 128 + 16 * i + (lane & 15);
      const int cn = wn * 128 + 16 * j + 4 * (lane >> 4);
      *reinterpret_cast<bf16x4*>(smem + r * ERS + cn * 2) = w4;
    }
  __syncthreads();
  if (accumulate) {
#pragma unroll
    for (int c = 0; c < 32; ++c) {
      const int idx = tid + c * NT, r = idx >> 5, ch = idx & 31;
      const long gmr = m0 + r;
      const long gn = n0 + ch * 8;
      if (gmr < rowlim && gn < N && SPA_DBG_OK(gmr, MODE == 2 ? M : a_rows) & SPA_DBG_OK(gn + 7, ldc)) {
        bf16x8 v = *reinterpret_cast<const bf16x8*>(smem + r * ERS + ch * 16);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = (bf16)((float)v[q] + (float)old[c][q]);
        *reinterpret_cast<bf16x8*>(Cp + gmr * ldc + gn) = v;
      }
    }
    return;
  }
  // write only: the round-5 loop (a fully unrolled one measured 5 % slower here)
#pragma unroll 4
  for (int c = 0; c < 32; ++c) {
    const int idx = tid + c * NT, r = idx >> 5, ch = idx & 31;
    const long gmr = m0 + r;
    const long gn = n0 + ch * 8;
    if (gmr < rowlim && gn < N && SPA_DBG_OK(gmr, MODE == 2 ? M : a_rows) & SPA_DBG_OK(gn + 7, ldc))
      *reinterpret_cast<bf16x8*>(Cp + gmr * ldc + gn) = *reinterpret_cast<const bf16x8*>(smem + r * ERS + ch * 16);
  }
}

template <int MODE, int SCHED = 0, bool PART = false>
__global__ __launch_bounds__(256, 1) void gemm4a_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                        bf16* __restrict__ C, const int* __restrict__ offsets, int E,
                                                        int M, int N, int K, long lda, long ldb, long ldc,
                                                        long strideB, long strideC, int accumulate, long a_rows,
                                                        long b_rows, int gm) {
  using namespace g4;
  constexpr bool A_KC = MODE != 2, B_KC = MODE == 0;
  // SCHED (profiling ablations, SPA_G4_SCHED; 2-5 compute wrong results by construction):
  //   0 DMA spread over the MFMA stream, 1 DMA after it, 2 no DMA / vmcnt in the loop,
  //   3 no fragment reads in the loop, 4 MFMAs only (no DMA, reads, barriers), 5 no DMA, no barrier
  constexpr bool LOOP_DMA = SCHED <= 1 || SCHED == 3, LOOP_RD = SCHED != 3 && SCHED != 4;
  constexpr bool LOOP_BAR = SCHED != 4 && SCHED != 5;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];
  int* scratch = reinterpret_cast<int*>(smem + SMEM - 64);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  G4Tile tl;
  if (!g4_map<MODE, PART>(tl, smem, scratch, offsets, E, M, N, strideB, strideC, gm, B, C)) return;
  const int e = tl.e;
  const long m0 = tl.m0, mend = tl.mend, k0 = tl.k0, kend = MODE == 2 ? tl.kend : K;
  const bf16* Bp = tl.Bp;
  bf16* Cp = tl.Cp;
  SPA_DBG_CHECK(e, E);
  SPA_DBG_ASSERT(MODE == 2 ? kend <= a_rows && kend <= b_rows : mend <= a_rows && m0 < mend,
                 MODE == 2 ? kend : mend, a_rows);
  const long n0 = tl.n0;
  const int ktiles = kend > k0 ? (int)((kend - k0 + BK - 1) / BK) : 0;
  unsigned voA[4], voB[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    voA[j] = dma_off(A_KC, tid, j, lda);
    voB[j] = dma_off(B_KC, tid, j, ldb);
  }
  // readable extents (elements): whole operands, or up to the expert's last token (dW)
  const long limA = MODE == 2 ? kend * lda : a_rows * lda;
  const long limB = MODE == 2 ? kend * ldb : b_rows * ldb;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);

  // DMA piece j (0..3 A, 4..7 B) of slice t into its stage
  auto dma = [&](int t, int j) {
    char* dst = smem + (t & (NS - 1)) * STAGE + (j >> 2) * IMG + (j & 3) * (NT * 16) + wave_u * 1024;
    const long kk = k0 + (long)t * BK;
    const bool ja = j < 4;
    const bf16* base = ja ? A : Bp;
    const long origin = ja ? (A_KC ? m0 * lda + kk : kk * lda + m0) : (B_KC ? n0 * ldb + kk : kk * ldb + n0);
    const long lim = ja ? limA : limB;
    const __amdgpu_buffer_rsrc_t rs = rsrc(base + origin, (lim - origin) * 2);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)dst, 16, ja ? voA[j & 3] : voB[j & 3], 0, 0, 0);
  };
  // K-contiguous fragment row r of an image (r = 16 * frag + (lane & 15)), logical chunk lane >> 4
  const int rl = lane & 15, chunk = (lane >> 4) ^ ((rl >> 2) & 3);
  const int offA = (wm * 128 + rl) * 64 + 16 * chunk, offB = (wn * 128 + rl) * 64 + 16 * chunk;
  // K-strided fragment f (image columns 16 f ..): lane (g, q, p) reads k-rows ra = 8 g + q and ra + 4
  // at chunk ch = (w << 4) | (f << 1) | (p >> 1) -- disjoint bits, so ch ^ sw(r) = c ^ (f << 1) with the
  // per-lane c = ((w << 4) | (p >> 1)) ^ sw(r); the byte address is then row + 16 (c ^ (f << 1)).
  const int kg = lane >> 4, kq = (lane & 15) >> 2, kp = lane & 3;
  const int ra = 8 * kg + kq;
  int ksA = (((wm << 4) | (kp >> 1)) ^ ksw(ra)) | ((((wm << 4) | (kp >> 1)) ^ ksw(ra + 4)) << 8);
  int ksB = (((wn << 4) | (kp >> 1)) ^ ksw(ra)) | ((((wn << 4) | (kp >> 1)) ^ ksw(ra + 4)) << 8);
  const int krow = ra * 512 + 8 * (kp & 1);
  auto rd = [&](int st, int which, int f) -> bf16x8 {   // stage st (mod NS), which 0: A frag f, 1: B frag f
    const char* img = smem + (st & (NS - 1)) * STAGE + which * IMG;
    if ((which ? B_KC : A_KC)) return *reinterpret_cast<const bf16x8*>(img + (which ? offB : offA) + f * 1024);
    const int cc = which ? ksB : ksA;
    const int ca = (cc & 255) ^ (f << 1), cb = (cc >> 8) ^ (f << 1);
    const s16x4_t x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + krow + 16 * ca));
    const s16x4_t y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + krow + 2048 + 16 * cb));
    const bf16x4 xv = __builtin_bit_cast(bf16x4, x), yv = __builtin_bit_cast(bf16x4, y);
    return __builtin_shufflevector(xv, yv, 0, 1, 2, 3, 4, 5, 6, 7);
  };

  f32x4 acc[8][8];   // [n frag j][m frag i]: C^T tiles (rows n, cols m); defined by slice 0
  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];

  // prologue: slices 0..2 in flight, slice 0 retired, its fragments read. DMA and fragment reads
  // run unconditionally past the last slice: a phantom slice's pieces land in a stage nobody reads
  // again (zero-filled past the operand), so the loop carries no branches and vmcnt stays 8. An
  // empty reduction (ktiles 0: an expert without tokens in dW) runs slice 0 on zero-filled images.
#pragma unroll
  for (int j = 0; j < 8; ++j) dma(0, j);
#pragma unroll
  for (int j = 0; j < 8; ++j) dma(1, j);
#pragma unroll
  for (int j = 0; j < 8; ++j) dma(2, j);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int f = 0; f < 8; ++f) { fa0[f] = rd(0, 0, f); fb0[f] = rd(0, 1, f); }
  if constexpr (!LOOP_RD) {
#pragma unroll
    for (int f = 0; f < 8; ++f) { fa1[f] = rd(1, 0, f); fb1[f] = rd(1, 1, f); }
  }

  // one slice: 64 MFMAs on (fa, fb) = slice t, fragments of slice t+1 into (na, nb), DMA of t+3
  // (t is a multiple of 4 plus the compile-time U, so every LDS offset is an immediate)
  auto slice = [&](int t, auto U, auto F0, bf16x8 (&fa)[8], bf16x8 (&fb)[8], bf16x8 (&na)[8], bf16x8 (&nb)[8]) {
    constexpr int u = decltype(U)::value;
    constexpr bool first = decltype(F0)::value;
    if constexpr (!A_KC) asm volatile("" : "+v"(ksA));
    if constexpr (!B_KC) asm volatile("" : "+v"(ksB));
#pragma unroll
    for (int g = 0; g < 16; ++g) {            // 16 groups of 4 MFMAs: n frag j = g >> 1, m frags 4 (g & 1) ..
      const int j = g >> 1;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = 4 * (g & 1) + q;
        if constexpr (first) G4_MFMA0(acc[j][i], fb[j], fa[i]);
        else G4_MFMA(acc[j][i], fb[j], fa[i]);
      }
      __builtin_amdgcn_sched_barrier(0);
      // one fragment read per group (A frags first)
      if constexpr (LOOP_RD) {
        if (g < 8) na[g] = rd(u + 1, 0, g);
        else nb[g - 8] = rd(u + 1, 1, g - 8);
      }
      if ((SCHED == 0 || SCHED == 3) && (g & 1)) dma(t + 3, g >> 1);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (SCHED == 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) dma(t + 3, j);
    }
    if constexpr (LOOP_DMA) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // retire slice t+2; younger: slice t+3
    if constexpr (LOOP_BAR) __builtin_amdgcn_s_barrier();
  };
  using U0 = std::integral_constant<int, 0>;
  using U1 = std::integral_constant<int, 1>;
  using U2 = std::integral_constant<int, 2>;
  using U3 = std::integral_constant<int, 3>;
  using T1 = std::true_type;
  using T0 = std::false_type;
  slice(0, U0{}, T1{}, fa0, fb0, fa1, fb1);
  for (int t = 1; t < ktiles; t += 4) {
    slice(t, U1{}, T0{}, fa1, fb1, fa0, fb0);
    if (t + 1 >= ktiles) break;
    slice(t + 1, U2{}, T0{}, fa0, fb0, fa1, fb1);
    if (t + 2 >= ktiles) break;
    slice(t + 2, U3{}, T0{}, fa1, fb1, fa0, fb0);
    if (t + 3 >= ktiles) break;
    slice(t + 3, U0{}, T0{}, fa0, fb0, fa1, fb1);
  }
  // drain the phantom DMA before the epilogue reuses the ring; an MFMA's result may not be read
  // (v_accvgpr_read) within its 8-pass latency by compiler code
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
  __syncthreads();
  g4_epilogue<MODE, PART>(acc, smem, C, Cp, e, m0, n0, MODE == 2 ? (long)M : mend, M, N, ldc, strideC, accumulate,
                          a_rows);
}



// ---------------------------------------------------------------------------------------------
// gemm4r: the same 4-wave 256 x 256 tile, AGPR-pinned accumulators, with hipBLASLt's staging
// (read from its gfx950 MT256x256x64 kernels: DTL off, one LDS buffer, prefetch 2): 64-deep K tiles
// go HBM -> VGPRs (buffer_load_dwordx4, 16 per wave per tile = 64 staging VGPRs) -> LDS
// (ds_write_b128), two barriers per tile. Why not LDS-DMA: each buffer_load ... lds issue holds the
// issuing wave for ~60-185 cycles, and at one wave per SIMD that is MFMA time -- gemm4a with its
// DMA removed runs 1,673 TF at 8192^3, with it 1,180 (profiles/r6_gemm4a_ablations.txt). A register
// load issues in a few cycles; its ds_write (13) fits an MFMA gap.
//   phase 1 (K half 0): 64 MFMAs on F0, the 16 K-half-1 fragments of this tile read into F1
//   lgkmcnt(0) + barrier: every wave is done reading this tile
//   phase 2 (K half 1): 64 MFMAs on F1; groups 0-7 write the staged next tile to LDS and reload the
//     staging registers with the tile after it; lgkmcnt(0) + barrier after group 11; groups 12-15
//     read the next tile's K-half-0 fragments into F0
// LDS images as gemm8 (64-deep tiles): K-contiguous [256][64] (128-B rows, chunk c of row r at
// r * 128 + 16 (c ^ ((r >> 1) & 7))), K-strided [64][256] (512-B rows, chunk c ^ f(r)).
template <int MODE, bool PART = false, int POL = 0>
__global__ __launch_bounds__(256, 1) void gemm4r_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                        bf16* __restrict__ C, const int* __restrict__ offsets, int E,
                                                        int M, int N, int K, long lda, long ldb, long ldc,
                                                        long strideB, long strideC, int accumulate, long a_rows,
                                                        long b_rows, int gm) {
  using namespace g4;
  constexpr bool A_KC = MODE != 2, B_KC = MODE == 0;
  constexpr int TK = 64, TIMG = 256 * TK * 2;   // 64-deep tile, one operand image (32 KiB)
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];
  int* scratch = reinterpret_cast<int*>(smem + SMEM - 64);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  G4Tile tl;
  if (!g4_map<MODE, PART>(tl, smem, scratch, offsets, E, M, N, strideB, strideC, gm, B, C)) return;
  const int e = tl.e;
  const long m0 = tl.m0, mend = tl.mend, n0 = tl.n0, k0 = tl.k0, kend = MODE == 2 ? tl.kend : K;
  const bf16* Bp = tl.Bp;
  bf16* Cp = tl.Cp;
  SPA_DBG_CHECK(e, E);
  SPA_DBG_ASSERT(MODE == 2 ? kend <= a_rows && kend <= b_rows : mend <= a_rows && m0 < mend,
                 MODE == 2 ? kend : mend, a_rows);
  const int ktiles = kend > k0 ? (int)((kend - k0 + TK - 1) / TK) : 0;
  __syncthreads();   // g4_map's count image (mode 2) is overwritten by the first LDS writes

  // ---- global -> VGPR staging: 8 loads per operand per wave, instruction q = 4 j + wave
  //   K-contiguous: rows 8q .. 8q+7 (lane: row 8q + l/8, 16-B chunk l%8), soffset 8q*ld*2
  //   K-strided:    k-rows 2q, 2q+1 (lane: k-row 2q + l/32, chunk l%32), soffset 2q*ld*2
  // the tile advance moves the descriptor base; the range check zero-fills past the operand (modes
  // 0/1: its last row; mode 2: the expert's last token)
  auto lane_voff = [&](bool kc, long ld) -> unsigned {
    return kc ? (unsigned)(((lane >> 3) * ld + 8 * (lane & 7)) * 2) : (unsigned)(((lane >> 5) * ld + 8 * (lane & 31)) * 2);
  };
  const unsigned voA = lane_voff(A_KC, lda), voB = lane_voff(B_KC, ldb);
  const long limA = MODE == 2 ? kend * lda : a_rows * lda;
  const long limB = MODE == 2 ? kend * ldb : b_rows * ldb;
  // tile origins (elements) and per-tile advance
  const long oA = A_KC ? m0 * lda + k0 : k0 * lda + m0, oB = B_KC ? n0 * ldb + k0 : k0 * ldb + n0;
  const long stA = A_KC ? TK : TK * lda, stB = B_KC ? TK : TK * ldb;
  auto load = [&](int t, int j) -> bf16x8 {   // slot j (0..7 A, 8..15 B) of tile t
    const bool ja = j < 8;
    const int q = 4 * (j & 7) + wave;
    const bool kc = ja ? A_KC : B_KC;
    const long ld = ja ? lda : ldb;
    const long org = (ja ? oA : oB) + (long)t * (ja ? stA : stB);
    const long lim = ja ? limA : limB;
    const __amdgpu_buffer_rsrc_t rs = rsrc((ja ? A : Bp) + org, (lim - org) * 2);
    const int soff = (int)((kc ? 8 * q : 2 * q) * ld * 2);
    // cache policy (POL, profiling: 1 = A sc0 sc1 / B sc1 as hipBLASLt's NTA3/NTB2 kernels, 2 = swapped)
    constexpr int PA = POL == 1 ? 17 : POL == 2 ? 16 : 0, PB = POL == 1 ? 16 : POL == 2 ? 17 : 0;
    if (ja) return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, voA, soff, PA));
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, voB, soff, PB));
  };
  // LDS write address of slot j (see the image layouts above)
  auto waddr = [&](int j) -> int {
    const bool ja = j < 8;
    const int q = 4 * (j & 7) + wave;
    const int img = ja ? 0 : TIMG;
    if (ja ? A_KC : B_KC) {
      const int r = 8 * q + (lane >> 3), c = lane & 7;
      return img + r * 128 + 16 * (c ^ ((r >> 1) & 7));
    }
    const int r = 2 * q + (lane >> 5), c = lane & 31;
    return img + r * 512 + 16 * (c ^ ksw(r));
  };
  // fragment reads: K-contiguous operand frag f (rows 16 f + l%16 of the wave's 128), k-slice s
  const int rl = lane & 15, g4l = lane >> 4, xs = (rl >> 1) & 7;
  auto kc_addr = [&](int w, int s) -> int {   // + 2048 f
    return (w * 128 + rl) * 128 + 16 * ((4 * s + g4l) ^ xs);
  };
  const int kcA0 = kc_addr(wm, 0), kcA1 = kc_addr(wm, 1), kcB0 = TIMG + kc_addr(wn, 0), kcB1 = TIMG + kc_addr(wn, 1);
  // K-strided operand frag f (image columns w*128 + 16 f ..), k-slice s: lane (g, q, p) reads k-rows
  // ra = 32 s + 8 g + q and ra + 4 at chunk ((w << 4) | (f << 1) | (p >> 1)) ^ f(r)
  const int kq = rl >> 2, kp = lane & 3;
  auto ks_c = [&](int w, int r) { return (((w << 4) | (kp >> 1)) ^ ksw(r)); };
  int ksA[2], ksB[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const int ra = 32 * s2 + 8 * g4l + kq;
    ksA[s2] = ks_c(wm, ra) | (ks_c(wm, ra + 4) << 8);
    ksB[s2] = ks_c(wn, ra) | (ks_c(wn, ra + 4) << 8);
  }
  const int krow = (8 * g4l + kq) * 512 + 8 * (kp & 1);
  auto rd = [&](int which, int s, int f) -> bf16x8 {
    const bool kc = which ? B_KC : A_KC;
    if (kc) {
      const int base = which ? (s ? kcB1 : kcB0) : (s ? kcA1 : kcA0);
      return *reinterpret_cast<const bf16x8*>(smem + base + 2048 * f);
    }
    const char* img = smem + (which ? TIMG : 0) + 32 * 512 * s + krow;
    const int cc = which ? ksB[s] : ksA[s];
    const int ca = (cc & 255) ^ (f << 1), cb = (cc >> 8) ^ (f << 1);
    const s16x4_t x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + 16 * ca));
    const s16x4_t y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + 2048 + 16 * cb));
    return __builtin_shufflevector(__builtin_bit_cast(bf16x4, x), __builtin_bit_cast(bf16x4, y), 0, 1, 2, 3, 4, 5, 6, 7);
  };
  auto lds_bar = [&]() {   // this wave's LDS ops done, then the block barrier (no vmcnt: loads stay in flight)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  f32x4 acc[8][8];   // [n frag j][m frag i]: C^T tiles; defined by the first tile's MFMAs
  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8], stg[16];

  // prologue: tile 0 -> LDS, tile 1 -> staging registers, tile 0's K-half-0 fragments
#pragma unroll
  for (int j = 0; j < 16; ++j) stg[j] = load(0, j);
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    *reinterpret_cast<bf16x8*>(smem + waddr(j)) = stg[j];
    stg[j] = load(1, j);
  }
  lds_bar();
#pragma unroll
  for (int f = 0; f < 8; ++f) { fa0[f] = rd(0, 0, f); fb0[f] = rd(1, 0, f); }

  // one memory instruction per MFMA gap (hipBLASLt's placement: an MFMA of 16x16x32 holds the wave's
  // vector issue for 8 of its 16 cycles, so one read / write / load beside it is nearly free, a burst
  // of them is not). MFMA m of a phase: n frag j = m / 8, m frag i = m % 8.
  auto tile = [&](int t, auto F0) {
    constexpr bool first = decltype(F0)::value;
    if constexpr (!A_KC) asm volatile("" : "+v"(ksA[0]), "+v"(ksA[1]));
    if constexpr (!B_KC) asm volatile("" : "+v"(ksB[0]), "+v"(ksB[1]));
    // ---- phase 1: K half 0 on (fa0, fb0); the 16 K-half-1 fragments into (fa1, fb1), one per MFMA
#pragma unroll
    for (int m = 0; m < 64; ++m) {
      const int j = m >> 3, i = m & 7;
      if constexpr (first) G4_MFMA0(acc[j][i], fb0[j], fa0[i]);
      else G4_MFMA(acc[j][i], fb0[j], fa0[i]);
      if (m < 16) {
        __builtin_amdgcn_sched_barrier(0);
        if (m < 8) fa1[m] = rd(0, 1, m);
        else fb1[m - 8] = rd(1, 1, m - 8);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    lds_bar();
    // ---- phase 2: K half 1 on (fa1, fb1); staged tile t+1 -> LDS (slot s at MFMA 3 s), tile t+2 ->
    // staging (at 3 s + 1); barrier after MFMA 47; the next tile's K half 0 fragments at 48..63 in
    // the order its first MFMAs consume them (fb0[0], fa0[0..7], fb0[1..7])
#pragma unroll
    for (int m = 0; m < 64; ++m) {
      const int j = m >> 3, i = m & 7;
      G4_MFMA(acc[j][i], fb1[j], fa1[i]);
      __builtin_amdgcn_sched_barrier(0);
      if (m < 48) {
        const int sl = m / 3;
        if (m % 3 == 0) *reinterpret_cast<bf16x8*>(smem + waddr(sl)) = stg[sl];
        else if (m % 3 == 1) stg[sl] = load(t + 2, sl);
        else if (m == 47) lds_bar();
      } else {
        const int r = m - 48;
        if (r == 0) fb0[0] = rd(1, 0, 0);
        else if (r <= 8) fa0[r - 1] = rd(0, 0, r - 1);
        else fb0[r - 8] = rd(1, 0, r - 8);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  tile(0, std::true_type{});
  for (int t = 1; t < ktiles; ++t) tile(t, std::false_type{});
  // the staging loads of the last tiles (phantom, never read) and the LDS reads drain before the
  // epilogue reuses LDS; an MFMA's result may not be read within its 8-pass latency
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
  __syncthreads();
  g4_epilogue<MODE, PART>(acc, smem, C, Cp, e, m0, n0, MODE == 2 ? (long)M : mend, M, N, ldc, strideC, accumulate,
                          a_rows);
}


// ---------------------------------------------------------------------------------------------
// gemm4d: the structure of hipBLASLt's fastest gfx950 bf16 kernel for this tile (its hand-written
// "Custom_..._MT256x256x64_MI16x16x1" assembly, read from the shipped code object): LDS-DMA into TWO
// 64-deep tile buffers, two tiles ahead, one DMA piece per ~3 MFMAs of the first K half, three
// barriers per tile. The DMA pieces of a tile share one descriptor per operand (advanced once per
// tile), one lane offset VGPR and per-piece scalar offsets, so a piece issues with nothing to wait
// for -- gemm4a's DMA recomputed a descriptor per piece, and its 32-deep 4-stage ring waited on
// vmcnt twice as often.
//   tile t (buffer b = t & 1), MFMAs 0..63 on F0 (K half 0), 64..127 on F1 (K half 1):
//     m 0..15   read F1 (tile t, buffer b)
//     m 16      lgkmcnt(0) + barrier: every wave is done reading buffer b
//     m 18..63  DMA tile t+2 into buffer b (16 pieces, one per 3 MFMAs)
//     m 96      vmcnt(16) (tile t+1 landed; tile t+2's pieces stay in flight) + barrier
//     m 97..112 read F0 (tile t+1, buffer b^1)
template <int MODE, bool PART = false>
__global__ __launch_bounds__(256, 1) void gemm4d_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                        bf16* __restrict__ C, const int* __restrict__ offsets, int E,
                                                        int M, int N, int K, long lda, long ldb, long ldc,
                                                        long strideB, long strideC, int accumulate, long a_rows,
                                                        long b_rows, int gm) {
  using namespace g4;
  constexpr bool A_KC = MODE != 2, B_KC = MODE == 0;
  constexpr int TK = 64, TIMG = 256 * TK * 2, TBUF = 2 * TIMG;   // one operand image 32 KiB, a buffer 64 KiB
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];
  int* scratch = reinterpret_cast<int*>(smem + SMEM - 64);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  G4Tile tl;
  if (!g4_map<MODE, PART>(tl, smem, scratch, offsets, E, M, N, strideB, strideC, gm, B, C)) return;
  const int e = tl.e;
  const long m0 = tl.m0, mend = tl.mend, n0 = tl.n0, k0 = tl.k0, kend = MODE == 2 ? tl.kend : K;
  const bf16* Bp = tl.Bp;
  bf16* Cp = tl.Cp;
  SPA_DBG_CHECK(e, E);
  SPA_DBG_ASSERT(MODE == 2 ? kend <= a_rows && kend <= b_rows : mend <= a_rows && m0 < mend,
                 MODE == 2 ? kend : mend, a_rows);
  const int ktiles = kend > k0 ? (int)((kend - k0 + TK - 1) / TK) : 0;
  __syncthreads();   // g4_map's count image (mode 2) lives where the first DMA lands

  // ---- DMA geometry. Piece j (0..7) of an operand for this wave is wave-instruction q = 4 j + wave
  // of the block: K-contiguous rows 8q .. 8q+7 / K-strided k-rows 2q, 2q+1 -> LDS bytes q*1024 of
  // the image (lane l at + 16 l). Source: the lane's offset within the piece (the swizzle of a
  // K-strided k-row 8j + 2w + l/32 depends on j's parity) + the piece's offset.
  auto lane_src = [&](bool kc, long ld, int par) -> unsigned {
    if (kc) {
      const int u = lane >> 3, r = 8 * wave + u;          // rows of q = wave (j = 0); swizzle depends on q & 1 only
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      return (unsigned)((u * ld + 8 * c) * 2);
    }
    const int h = lane >> 5, r = 8 * par + 2 * wave + h;  // k-row of piece j with j & 1 = par (j = par)
    const int c = (lane & 31) ^ ksw(r);
    return (unsigned)((h * ld + 8 * c) * 2);
  };
  // per-piece lane offsets (the piece's scalar offset folded in: a non-constant soffset operand of
  // __builtin_amdgcn_raw_ptr_buffer_load_lds makes hipcc's host pass drop the kernel instantiation)
  auto soff = [&](bool kc, long ld, int j) -> unsigned { return (unsigned)((kc ? 8 : 2) * (4 * j + wave) * ld * 2); };
  unsigned voA[8], voB[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    voA[j] = lane_src(A_KC, lda, j & 1) + soff(A_KC, lda, j);
    voB[j] = lane_src(B_KC, ldb, j & 1) + soff(B_KC, ldb, j);
  }
  const long limA = MODE == 2 ? kend * lda : a_rows * lda;
  const long limB = MODE == 2 ? kend * ldb : b_rows * ldb;
  const long oA = A_KC ? m0 * lda + k0 : k0 * lda + m0, oB = B_KC ? n0 * ldb + k0 : k0 * ldb + n0;
  const long stA = A_KC ? TK : TK * lda, stB = B_KC ? TK : TK * ldb;
  // descriptor inputs of the current tile (base, bytes) per operand; the descriptors themselves are
  // built at each piece from these (a pure op: hipcc keeps one per tile). A descriptor-typed local
  // captured by the lambdas made the host pass drop the kernel's instantiation (undefined launch stub).
  const bf16* pA = A;
  const bf16* pB = Bp;
  long nA = 0, nB = 0;
  auto set_rsrc = [&](int t) {   // tile t's descriptor inputs (once per tile per operand)
    const long a0 = oA + (long)t * stA, b0 = oB + (long)t * stB;
    pA = A + a0;
    pB = Bp + b0;
    nA = (limA - a0) * 2;
    nB = (limB - b0) * 2;
  };
  auto piece = [&](int buf, int j) {   // piece j (0..7 A, 8..15 B) of the tile whose descriptors are set
    const bool ja = j < 8;
    const int jj = j & 7;
    char* dst = smem + buf * TBUF + (ja ? 0 : TIMG) + (4 * jj + wave) * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(ja ? rsrc(pA, nA) : rsrc(pB, nB), (lds_void*)dst, 16,
                                             ja ? voA[jj] : voB[jj], 0, 0, 0);
  };

  // ---- fragment reads (gemm4r's image layouts at a buffer offset)
  const int rl = lane & 15, g4l = lane >> 4, xs = (rl >> 1) & 7;
  auto kc_addr = [&](int w, int s) -> int { return (w * 128 + rl) * 128 + 16 * ((4 * s + g4l) ^ xs); };
  const int kcA0 = kc_addr(wm, 0), kcA1 = kc_addr(wm, 1), kcB0 = TIMG + kc_addr(wn, 0), kcB1 = TIMG + kc_addr(wn, 1);
  const int kq = rl >> 2, kp = lane & 3;
  auto ks_c = [&](int w, int r) { return (((w << 4) | (kp >> 1)) ^ ksw(r)); };
  int ksA[2], ksB[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const int ra = 32 * s2 + 8 * g4l + kq;
    ksA[s2] = ks_c(wm, ra) | (ks_c(wm, ra + 4) << 8);
    ksB[s2] = ks_c(wn, ra) | (ks_c(wn, ra + 4) << 8);
  }
  const int krow = (8 * g4l + kq) * 512 + 8 * (kp & 1);
  auto rd = [&](int buf, int which, int s, int f) -> bf16x8 {
    const bool kc = which ? B_KC : A_KC;
    if (kc) {
      const int base = which ? (s ? kcB1 : kcB0) : (s ? kcA1 : kcA0);
      return *reinterpret_cast<const bf16x8*>(smem + buf * TBUF + base + 2048 * f);
    }
    const char* img = smem + buf * TBUF + (which ? TIMG : 0) + 32 * 512 * s + krow;
    const int cc = which ? ksB[s] : ksA[s];
    const int ca = (cc & 255) ^ (f << 1), cb = (cc >> 8) ^ (f << 1);
    const s16x4_t x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + 16 * ca));
    const s16x4_t y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + 2048 + 16 * cb));
    return __builtin_shufflevector(__builtin_bit_cast(bf16x4, x), __builtin_bit_cast(bf16x4, y), 0, 1, 2, 3, 4, 5, 6, 7);
  };
  auto bar = [&]() {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  f32x4 acc[8][8];
  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];

  // prologue: tiles 0 and 1 in flight, tile 0 retired, its K-half-0 fragments
  set_rsrc(0);
#pragma unroll
  for (int j = 0; j < 16; ++j) piece(0, j);
  set_rsrc(1);
#pragma unroll
  for (int j = 0; j < 16; ++j) piece(1, j);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  bar();
#pragma unroll
  for (int f = 0; f < 8; ++f) { fb0[f] = rd(0, 1, 0, f); fa0[f] = rd(0, 0, 0, f); }

  auto tile = [&](int t, auto BUF, auto F0) {
    constexpr int b = decltype(BUF)::value;
    constexpr bool first = decltype(F0)::value;
    if constexpr (!A_KC) asm volatile("" : "+v"(ksA[0]), "+v"(ksA[1]));
    if constexpr (!B_KC) asm volatile("" : "+v"(ksB[0]), "+v"(ksB[1]));
#pragma unroll
    for (int m = 0; m < 64; ++m) {
      const int j = m >> 3, i = m & 7;
      if constexpr (first) G4_MFMA0(acc[j][i], fb0[j], fa0[i]);
      else G4_MFMA(acc[j][i], fb0[j], fa0[i]);
      __builtin_amdgcn_sched_barrier(0);
      if (m < 16) {
        if (m < 8) fb1[m] = rd(b, 1, 1, m);
        else fa1[m - 8] = rd(b, 0, 1, m - 8);
      } else if (m == 16) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's reads of buffer b done
        bar();
        set_rsrc(t + 2);
      } else if (m >= 18 && (m - 18) % 3 == 0) {
        piece(b, (m - 18) / 3);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int m = 0; m < 64; ++m) {
      const int j = m >> 3, i = m & 7;
      G4_MFMA(acc[j][i], fb1[j], fa1[i]);
      __builtin_amdgcn_sched_barrier(0);
      if (m == 32) {
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");    // tile t+1 landed (this wave's pieces)
        bar();                                               // ... and every wave's
      } else if (m > 32 && m <= 48) {
        const int r = m - 33;                                // next tile's K half 0, in consumption order
        if (r < 8) fb0[r] = rd(b ^ 1, 1, 0, r);
        else fa0[r - 8] = rd(b ^ 1, 0, 0, r - 8);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  using B0 = std::integral_constant<int, 0>;
  using B1 = std::integral_constant<int, 1>;
  tile(0, B0{}, std::true_type{});
  for (int t = 1; t < ktiles; t += 2) {
    tile(t, B1{}, std::false_type{});
    if (t + 1 >= ktiles) break;
    tile(t + 1, B0{}, std::false_type{});
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
  __syncthreads();
  g4_epilogue<MODE, PART>(acc, smem, C, Cp, e, m0, n0, MODE == 2 ? (long)M : mend, M, N, ldc, strideC, accumulate,
                          a_rows);
}

#undef G4_MFMA
#undef G4_MFMA0

static int g4_group(int E) {
  const char* e = getenv("SPA_G4_GM");
  return E > 1 ? 1 : (e ? std::max(1, atoi(e)) : 4);
}
static int g4_sched() {
  const char* e = getenv("SPA_G4_SCHED");
  return e ? atoi(e) : 0;
}
static int g4_pol() {
  const char* e = getenv("SPA_G4_POL");
  return e ? atoi(e) : 0;
}
// SPA_G4_IMPL: "ring" = the 32-deep 4-stage LDS-DMA ring (gemm4a_kernel), "reg" = register staging
// (gemm4r_kernel); default: two 64-deep LDS-DMA buffers (gemm4d_kernel). The 64-deep kernels need the
// reduction dim % 64 in modes 0 / 1.
static int g4_impl() {
  const char* e = getenv("SPA_G4_IMPL");
  if (!e) return 2;
  const std::string v(e);
  return v == "ring" ? 0 : v == "reg" ? 1 : 2;
}


// grouped_gemm8's contract (csrc/kernels/gemm8.hip): modes 0 / 1 need the reduction dim % 32 and
// N % 8; mode 2 N, K % 8 (any token counts)
at::Tensor gemm4a(const at::Tensor& a, const at::Tensor& w, const at::Tensor& offsets, int64_t mode,
                  const c10::optional<at::Tensor>& out_, bool accumulate, int64_t impl_) {
  // impl: -1 = SPA_G4_IMPL / default (two-buffer LDS-DMA), 0 ring, 1 register staging, 2 two-buffer DMA
  const int impl = impl_ >= 0 ? (int)impl_ : g4_impl();
  TORCH_CHECK(a.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16, "gemm4a: bf16");
  TORCH_CHECK(a.is_contiguous() && w.is_contiguous() && offsets.scalar_type() == at::kInt && offsets.is_cuda());
  const int E = offsets.numel() - 1;
  TORCH_CHECK(E >= 1 && E <= 256, "gemm4a: 1..256 experts");
  TORCH_CHECK((uintptr_t)a.data_ptr() % 16 == 0 && (uintptr_t)w.data_ptr() % 16 == 0, "gemm4a: 16-B aligned");
  DeviceGuard g(a.device());
  auto st = stream();
  const int sch = g4_sched();
  if (mode == 0 || mode == 1) {
    TORCH_CHECK(w.dim() == 3 && w.size(0) == E);
    const int M = a.size(0), Nw = w.size(1), Kw = w.size(2);
    const int N = mode == 0 ? Nw : Kw, K = mode == 0 ? Kw : Nw;
    TORCH_CHECK(a.size(1) == K, "gemm4a: A/W shape mismatch");
    TORCH_CHECK(K % 32 == 0 && N % 8 == 0, "gemm4a: reduction % 32, output cols % 8");
    TORCH_CHECK((long)(M + 256) * K * 2 < (1L << 32) && (long)(Nw + 256) * Kw * 2 < (1L << 32),
                "gemm4a: operands < 4 GiB");
    auto out = out_ ? *out_ : at::empty({M, N}, a.options());
    if (M == 0) return out;
    TORCH_CHECK(out.is_contiguous() && out.size(0) == M && out.size(1) == N);
    if (K == 0) {
      if (!accumulate) out.zero_();
      return out;
    }
    const int grid = (cdiv(M, 256) + E) * cdiv(N, 256);
    if (impl == 2) {
      TORCH_CHECK(K % 64 == 0, "gemm4a: reduction % 64");
#define G4D(MD) gemm4d_kernel<MD><<<grid, 256, 0, st>>>((const bf16*)a.data_ptr(), (const bf16*)w.data_ptr(),         \
                                                       (bf16*)out.data_ptr(), offsets.data_ptr<int>(), E, M, N, K, K, \
                                                       Kw, N, (long)Nw * Kw, 0, accumulate ? 1 : 0, M, Nw, g4_group(E))
      if (mode == 0) G4D(0); else G4D(1);
#undef G4D
      SPA_LAUNCH_CHECK();
      return out;
    }
    if (impl == 1) {
      TORCH_CHECK(K % 64 == 0, "gemm4a (register-staged): reduction % 64");
      const int pol = g4_pol();
      if (mode == 0 && pol == 1)
        gemm4r_kernel<0, false, 1><<<grid, 256, 0, st>>>((const bf16*)a.data_ptr(), (const bf16*)w.data_ptr(),
                                               (bf16*)out.data_ptr(), offsets.data_ptr<int>(), E, M, N, K, K, Kw, N,
                                               (long)Nw * Kw, 0, accumulate ? 1 : 0, M, Nw, g4_group(E));
      else if (mode == 0 && pol == 2)
        gemm4r_kernel<0, false, 2><<<grid, 256, 0, st>>>((const bf16*)a.data_ptr(), (const bf16*)w.data_ptr(),
                                               (bf16*)out.data_ptr(), offsets.data_ptr<int>(), E, M, N, K, K, Kw, N,
                                               (long)Nw * Kw, 0, accumulate ? 1 : 0, M, Nw, g4_group(E));
      else if (mode == 0)
        gemm4r_kernel<0><<<grid, 256, 0, st>>>((const bf16*)a.data_ptr(), (const bf16*)w.data_ptr(),
                                               (bf16*)out.data_ptr(), offsets.data_ptr<int>(), E, M, N, K, K, Kw, N,
                                               (long)Nw * Kw, 0, accumulate ? 1 : 0, M, Nw, g4_group(E));
      else
        gemm4r_kernel<1><<<grid, 256, 0, st>>>((const bf16*)a.data_ptr(), (const bf16*)w.data_ptr(),
                                               (bf16*)out.data_ptr(), offsets.data_ptr<int>(), E, M, N, K, K, Kw, N,
                                               (long)Nw * Kw, 0, accumulate ? 1 : 0, M, Nw, g4_group(E));
      SPA_LAUNCH_CHECK();
      return out;
    }
#define G4_L(MD, S)                                                                                                 \
  gemm4a_kernel<MD, S><<<grid, 256, 0, st>>>((const bf16*)a.data_ptr(), (const bf16*)w.data_ptr(),                  \
                                             (bf16*)out.data_ptr(), offsets.data_ptr<int>(), E, M, N, K, K, Kw, N,   \
                                             (long)Nw * Kw, 0, accumulate ? 1 : 0, M, Nw, g4_group(E))
    if (mode == 0) {
      switch (sch) {
        case 1: G4_L(0, 1); break;
        case 2: G4_L(0, 2); break;
        case 3: G4_L(0, 3); break;
        case 4: G4_L(0, 4); break;
        case 5: G4_L(0, 5); break;
        default: G4_L(0, 0);
      }
    }
    else { if (sch == 1) G4_L(1, 1); else G4_L(1, 0); }
#undef G4_L
    SPA_LAUNCH_CHECK();
    return out;
  }
  TORCH_CHECK(mode == 2, "gemm4a: mode 0/1/2");
  const int N = a.size(1), K = w.size(1), T = a.size(0);
  TORCH_CHECK(w.dim() == 2 && w.size(0) == T && N % 8 == 0 && K % 8 == 0);
  TORCH_CHECK((long)(T + 64) * (N + 256) * 2 < (1L << 32) && (long)(T + 64) * (K + 256) * 2 < (1L << 32),
              "gemm4a: operands < 4 GiB");
  auto out = out_ ? *out_ : at::empty({E, N, K}, a.options());
  TORCH_CHECK(out.is_contiguous() && out.numel() == (long)E * N * K);
  const int grid = E * cdiv(N, 256) * cdiv(K, 256);
  if (impl == 2)
    gemm4d_kernel<2><<<grid, 256, 0, st>>>((const bf16*)a.data_ptr(), (const bf16*)w.data_ptr(),
                                           (bf16*)out.data_ptr(), offsets.data_ptr<int>(), E, N, K, 0, N, K, K, 0,
                                           (long)N * K, accumulate ? 1 : 0, T, T, 1);
  else if (impl == 1)
    gemm4r_kernel<2><<<grid, 256, 0, st>>>((const bf16*)a.data_ptr(), (const bf16*)w.data_ptr(),
                                           (bf16*)out.data_ptr(), offsets.data_ptr<int>(), E, N, K, 0, N, K, K, 0,
                                           (long)N * K, accumulate ? 1 : 0, T, T, 1);
  else if (sch == 1)
    gemm4a_kernel<2, 1><<<grid, 256, 0, st>>>((const bf16*)a.data_ptr(), (const bf16*)w.data_ptr(),
                                              (bf16*)out.data_ptr(), offsets.data_ptr<int>(), E, N, K, 0, N, K, K, 0,
                                              (long)N * K, accumulate ? 1 : 0, T, T, 1);
  else
    gemm4a_kernel<2, 0><<<grid, 256, 0, st>>>((const bf16*)a.data_ptr(), (const bf16*)w.data_ptr(),
                                              (bf16*)out.data_ptr(), offsets.data_ptr<int>(), E, N, K, 0, N, K, K, 0,
                                              (long)N * K, accumulate ? 1 : 0, T, T, 1);
  SPA_LAUNCH_CHECK();
  return out;
}

// fp32 partials of a dense weight gradient split over S token slices (wgrad8's contract, gemm8.hip):
// part[s] = dy[slice s]^T x[slice s], [S, N, K] fp32, on the register-staged kernel's mode 2
void launch_gemm4r_wgrad_part(const bf16* dy, const bf16* x, float* part, const int* offsets, int S, int N, int K,
                              long lda, long ldb, long T, hipStream_t st) {
  const int grid = S * cdiv(N, 256) * cdiv(K, 256);
  gemm4r_kernel<2, true><<<grid, 256, 0, st>>>(dy, x, reinterpret_cast<bf16*>(part), offsets, S, N, K, 0, lda, ldb,
                                               K, 0, (long)N * K, 0, T, T, 1);
}

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.def("gemm4a(Tensor a, Tensor w, Tensor offsets, int mode, Tensor(a!)? out, bool accumulate=False, int impl=-1) -> Tensor");
}
TORCH_LIBRARY_IMPL(spa, CUDA, m) {
  m.impl("gemm4a", &spa::gemm4a);
}
