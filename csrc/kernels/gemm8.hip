// Grouped MoE GEMM, second generation: 256 x 256 x 64 tiles, 8 waves, operands DMA'd straight
// from HBM into LDS (buffer_load ... lds, 16 B per lane), four phases per K-tile with counted
// vmcnt waits so four half-tiles stay in flight across the raw barriers.
//
// Modes (same contract as grouped_gemm in moe.hip):
//   0 fwd   Y[M, N]  = X[M, K] W_e[N, K]^T        rows grouped by offsets
//   1 dX    dX[M, N] = dY[M, K] W_e[K, N]          rows grouped (W_e stored [K=Nw][N=Kw])
//   2 dW    dW_e[N, K] = dY_e[T, N]^T X_e[T, K]   reduction rows grouped (token segments)
//
// Block 512 threads = 8 waves as 2 (M) x 4 (N). The 256 x 256 C tile is split into two
// 128-row A halves and two 128-col B halves; wave (wm, wn) owns rows {h*128 + wm*64 + [0,64)} and
// cols {h*128 + wn*32 + [0,32)} of both halves, so each of its four quadrants (mh, nh) reads one
// A half and one B half. Per K-tile the wave computes its quadrants in the order
// (0,0) (0,1) (1,1) (1,0) -- 16 v_mfma_f32_16x16x32_bf16 each -- while the block stages the
// four halves of a K-tile up to two K-tiles ahead (schedule at the main loop: none in the phase
// that reads 12 fragments, one each in phases 2 and 3, two in phase 4):
//
//   phase: ds_read this quadrant's new fragments | DMA 0-2 halves | [vmcnt] | s_barrier |
//          lgkmcnt(0) | 16 MFMA | s_barrier
//
// Waves 4-7 run one barrier behind waves 0-3 (an extra s_barrier before the loop), so on every
// SIMD -- which holds wave w and wave w+4 -- one wave reads LDS / issues DMA while the other runs
// its MFMA cluster. A wait in phase p still precedes every reader of phase p+1 by a barrier in
// both groups, and every restage is >= 2 phases after the last read (one barrier of slack for
// the stagger).
//
// The counted waits (vmcnt 8 / 8 / 10 after phases 1, 2 and 4) retire exactly the half the next
// phase reads (B1, A1, then A0 + B0 of the next tile); every half is restaged >= 2 phases after
// its last read. All LDS is one array and every barrier is a bare s_barrier, so no implicit
// vmcnt(0) drains the DMA queue inside the loop.
//
// LDS images (lane-linear DMA destinations; the swizzle lives in the per-lane SOURCE address
// and the matching read address, an involution):
//   K-contiguous half [128 rows][64 k]: 16-B chunk c of row r at r*128 + 16*(c ^ ((r >> 1) & 7))
//     -- ds_read_b128 row reads of 16 consecutive rows hit 16 distinct bank slots;
//   K-strided half [64 k][128 cols]: chunk c of k-row r at r*256 + 16*(c ^ f(r)),
//     f(r) = ((r & 3) << 2) | ((r >> 2) & 3) -- read with ds_read_b64_tr_b16 (conflict-free).
// Out-of-range rows / columns / tokens read as zero through the buffer descriptor range check
// (dW descriptors start at the expert's first token and end at its last).
#include "gemm_common.h"

#include <map>
#include <mutex>
#include <tuple>
#include <vector>

SPA_DEBUG_TU("gemm8.hip")

namespace spa {

namespace g8 {

constexpr int BM = 256, BN = 256, BK = 64, NT = 512;
constexpr int HALF = 128 * 64 * 2;            // bytes per half-tile image (16 KiB)
constexpr int STAGE = 4 * HALF;               // A0 A1 B0 B1 of one K-tile (64 KiB)

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) s16x4_t lds_s4;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, long bytes) {
  const long nb = bytes < 0 ? 0 : (bytes > 0xFFFFFFFFL ? 0xFFFFFFFFL : bytes);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)(unsigned)nb, 0x00020000);
}

// Per-thread byte offset of the j-th (0, 1) 16-B DMA piece of a half image, relative to the
// half's origin in global memory. Fixed for the whole kernel: the tile-dependent part of every
// address lives in the (scalar) buffer descriptor base, so the K loop does no VALU address math.
//   K-contiguous half [128 rows][64 k]: slot q -> row q >> 3, chunk (q & 7) ^ ((row >> 1) & 7)
//   K-strided half    [64 k][128 cols]: slot q -> k-row q >> 4, chunk (q & 15) ^ f(row)
__device__ __forceinline__ unsigned dma_off(bool kc, int tid, int j, long ld) {
  const int q = j * NT + tid;
  if (kc) {
    const int r = q >> 3, c = (q & 7) ^ ((r >> 1) & 7);
    return (unsigned)((r * ld + 8 * c) * 2);
  }
  const int r = q >> 4, c = (q & 15) ^ (((r & 3) << 2) | ((r >> 2) & 3));
  return (unsigned)((r * ld + 8 * c) * 2);
}
// DMA one half image: origin = element offset of its first (row, k) in `base`, limit = elements
// readable before the range check zero-fills. lds_wave = this wave's 1 KiB slice of the half.
__device__ __forceinline__ void stage_half(const bf16* base, long origin, long limit, char* lds_wave,
                                           const unsigned (&vo)[2]) {
  const __amdgpu_buffer_rsrc_t rs = rsrc(base + origin, (limit - origin) * 2);
#pragma unroll
  for (int j = 0; j < 2; ++j)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(lds_wave + j * (NT * 16)), 16, vo[j], 0, 0, 0);
}

// 16x16x32 operand (16 rows of the half starting at row0, k-slice s of the 64-k tile) from a
// K-contiguous image: lane l -> row row0 + (l & 15), k 32 s + 8 (l >> 4) .. +7
__device__ __forceinline__ bf16x8 rd_kc(const char* half, int row0, int s, int lane) {
  const int r = row0 + (lane & 15), c = 4 * s + (lane >> 4);
  return *reinterpret_cast<const bf16x8*>(half + r * 128 + 16 * (c ^ ((r >> 1) & 7)));
}
// same operand from a K-strided image (rows of the operand = image columns col0 .. col0+15)
__device__ __forceinline__ bf16x8 rd_ks(const char* half, int col0, int s, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int ch = (col0 >> 3) + (p >> 1);
  const int ra = 32 * s + 8 * g + q, rb = ra + 4;
  const int fa = ((ra & 3) << 2) | ((ra >> 2) & 3), fb = ((rb & 3) << 2) | ((rb >> 2) & 3);
  const s16x4_t a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(half + ra * 256 + 16 * (ch ^ fa) + 8 * (p & 1)));
  const s16x4_t b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(half + rb * 256 + 16 * (ch ^ fb) + 8 * (p & 1)));
  const bf16x4 av = __builtin_bit_cast(bf16x4, a), bv = __builtin_bit_cast(bf16x4, b);
  return __builtin_shufflevector(av, bv, 0, 1, 2, 3, 4, 5, 6, 7);
}

}  // namespace g8

#define G8_WAIT_VM(N) \
  do {                \
    if (ABL != 3) asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); \
  } while (0)
#define G8_WAIT_LGKM0()                                \
  do {                                                 \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
    __builtin_amdgcn_sched_barrier(0);                 \
  } while (0)

// SPA_G8_STAMP=1 (profiling build only, tools/build_variant.sh): wave 0 of each block records
// s_memtime segment lengths of its tile -- mapping, prologue (first DMA issue to landed), K-loop,
// epilogue -- plus its K-tile count into g8_stamp[block % G8_NSTAMP] (read by the g8_stamps op)
#ifndef SPA_G8_STAMP
#define SPA_G8_STAMP 0
#endif
constexpr int G8_NSTAMP = 16384;
#if SPA_G8_STAMP
__device__ long long g8_stamp[G8_NSTAMP * 8];
#define G8_T(i) g8t[i] = (long long)__builtin_amdgcn_s_memtime()
#else
#define G8_T(i) \
  do {          \
  } while (0)
#endif

// ABL: ablation switch for profiling only (tools/bench_moe.py --ablate): 0 normal, 1 no DMA
// (compute on whatever LDS holds), 2 no LDS fragment reads, 3 no vmcnt waits (1-3 on the
// round-2 schedule), 8 the round-2 schedule itself (A/B reference); env value 4 selects the ILV schedule (DMA pieces issued between the MFMAs of each cluster). Measured at
// 8192^3 (tools/bench_moe.py, profiles/r2_gemm8_ablation.txt): ILV 764 TF vs 1113 TF for the
// shipped schedule -- a DMA piece's issue stalls the issuing wave's own MFMA stream. 1-3 give wrong
// results by construction and are never selected by the op unless SPA_GG8_ABLATE is set.
// PART (mode 2 only): the "experts" are token slices of one dense dW product (split-K) and each
// writes its fp32 partial [M, N] at C + e * strideC floats, summed by wgrad_reduce_kernel.
template <int MODE, int ABL = 0, bool ILV = false, bool PART = false>
__global__ __launch_bounds__(512, 1) void grouped_gemm8_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                               bf16* __restrict__ C, const int* __restrict__ offsets,
                                                               int E, int M, int N, int K, long lda, long ldb, long ldc,
                                                               long strideB, long strideC, int accumulate, long a_rows,
                                                               long b_rows, int gm = 1, int tailr = 0) {
  using namespace g8;
  constexpr bool A_KC = MODE != 2, B_KC = MODE == 0;
  // ONE LDS array (a second __shared__ object can make hipcc drain the DMA queue before ds_reads);
  // the tile -> expert scan scratch sits past the two stages, where no DMA lands
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE + 64];
  int* scratch = reinterpret_cast<int*>(smem + 2 * STAGE);   // [0] expert, [1] tile, [8..15] wave sums
#if SPA_G8_STAMP
  long long g8t[5] = {0, 0, 0, 0, 0};
#endif
  G8_T(0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int nnt = (N + BN - 1) / BN;
  int nt = 0, mt = 0;
  if (MODE == 2) {
    const int lid = xcd_remap(blockIdx.x, gridDim.x);
    nt = lid % nnt;
    mt = lid / nnt;
  }
  int e = 0;
  bool tail = false;
  long m0 = 0, mend = M, k0 = 0, kend = K;
  const bf16* Bp = B;
  bf16* Cp = C;
  if (MODE != 2) {
    int* wsum = scratch + 8;
    // the expert's row range travels through LDS with its id (no second global round trip). The
    // grid is sized for the worst case (every expert ragged): the REAL tiles R = rows x nnt take the
    // lowest block ids and the XCD remap runs over R (a remap over the whole grid scattered the
    // empty blocks, and real tiles landed behind them in an extra dispatch round)
    const int o0 = tid < E ? offsets[tid] : 0, o1 = tid < E ? offsets[tid + 1] : 0;
    const int cnt = o1 - o0, rem = cnt & (BM - 1);
    // tail tiles: an expert's last <= tailr (<= TR) rows past a multiple of 256 go to a 64-row tile
    // (below) instead of a 256-row one paid in full -- at dsv3_style routing half the experts end
    // 1-55 rows past a multiple of 256, 15 % of the grid (tools/bench_gg_counts.py)
    const bool tl = rem > 0 && rem <= tailr;
    const int tiles = (cnt >> 8) + (rem > 0 && !tl ? 1 : 0);
    const int pk = tiles + (tl ? 1 << 20 : 0);   // row tiles | tail tiles << 20, scanned together
    int inc = pk;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(inc, o, 64);
      if (lane >= o) inc += v;
    }
    if (lane == 63) wsum[wave] = inc;
    if (tid == 0) scratch[0] = -1;
    __syncthreads();
    int pre = inc - pk, rows = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
      const int v = wsum[w];
      pre += w < wave ? v : 0;
      rows += v;
    }
    const int pre_t = pre >> 20, tails = rows >> 20;
    pre &= (1 << 20) - 1;
    rows &= (1 << 20) - 1;
    const int R = rows * nnt;
    if ((int)blockIdx.x >= R + tails * nnt) return;
    tail = (int)blockIdx.x >= R;
    if (!tail) {
      const int lid = xcd_remap(blockIdx.x, R);
      nt = lid % nnt;
      mt = lid / nnt;
      if (gm > 1) {   // groups of gm row tiles x all column tiles (L2 / MALL reuse of B panels)
        const int g = lid / (gm * nnt), r = lid % (gm * nnt);
        const int gs = min(gm, rows - g * gm);
        mt = g * gm + r % gs;
        nt = r / gs;
      }
      if (tid < E && tiles > 0 && mt >= pre && mt < pre + tiles) {
        scratch[0] = tid; scratch[1] = mt - pre; scratch[2] = o0; scratch[3] = o1;
      }
    } else {          // tail tile j of the tail experts (in expert order), column tile nt
      const int t = blockIdx.x - R, j = t / nnt;
      nt = t % nnt;
      if (tid < E && tl && pre_t == j) {
        scratch[0] = tid; scratch[1] = cnt >> 8; scratch[2] = o0; scratch[3] = o1;
      }
    }
    __syncthreads();
    e = __builtin_amdgcn_readfirstlane(scratch[0]);
    if (e < 0) return;
    mt = __builtin_amdgcn_readfirstlane(scratch[1]);
    m0 = __builtin_amdgcn_readfirstlane(scratch[2]) + (long)mt * BM;
    mend = __builtin_amdgcn_readfirstlane(scratch[3]);
    Bp = B + e * strideB;
  } else {
    const int nmt = (M + BM - 1) / BM;
    e = mt / nmt;
    mt = mt % nmt;
    if (e >= E) return;
    if constexpr (!PART && ABL != 8) {   // (ABL 8 = the round-2 kernel: expert-major order)
      // Heavy experts first. Every expert owns the same number of output tiles but a tile's work
      // is its expert's token count, and routing is rarely balanced: the expert-major order ran a
      // dsv3_style step's dW at 507 TF (750 on balanced routing) and 400-440 TF at a 9x hot expert
      // (profiles/r3_gemm8_dw_order_ab.txt). Position pos takes the expert of count rank pos
      // (descending, ties by index). Block -> pos: with E % 8 == 0 and no expert above twice the
      // mean, each XCD (block i runs on XCD i % 8) owns E / 8 whole experts -- their tiles share
      // dY_e / X_e in its L2 -- dealt from the ranking in snake order (ranks 0-7 to XCDs 0-7, 8-15
      // to 7-0, ...), heaviest first on each; otherwise (a hot expert would pin its XCD) plain
      // dispatch order, which spreads every expert's tiles over all XCDs. Counts are staged in the
      // not yet used stage area; the choice is the same in every block.
      // (counts zero-padded to a multiple of 4 and read as int4: the one-int-per-iteration loops
      // below waited out an LDS round trip per expert, ~2K cycles of the tile's ~7.7K mapping)
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
      const int per_e = nmt * nnt;
      int pos, r;
      if (snake) {
        const int x = blockIdx.x % 8, j = blockIdx.x / 8, u = j / per_e;
        r = j % per_e;
        pos = u * 8 + ((u & 1) ? 7 - x : x);
      } else {
        pos = blockIdx.x / per_e;
        r = blockIdx.x % per_e;
      }
      nt = r % nnt;
      mt = r / nnt;
      if (tid < E) {
        const int c = o1 - o0;
        int rank = 0;
#pragma unroll 4
        for (int j = 0; j < E4 / 4; ++j) {   // (zero padding never outranks: c >= 0, index > tid)
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
    } else {
      if (tid == 0) { scratch[2] = offsets[e]; scratch[3] = offsets[e + 1]; }
      __syncthreads();
    }
    m0 = (long)mt * BM;
    Cp = C + e * strideC;
  }
  if (MODE == 2) {   // the expert's token range is the reduction range (staged in LDS with its id)
    k0 = __builtin_amdgcn_readfirstlane(scratch[2]);
    kend = __builtin_amdgcn_readfirstlane(scratch[3]);
  }
  // debug build: the tile -> (expert, row tile) scan and the group offsets name real rows
  SPA_DBG_CHECK(e, E);
  SPA_DBG_ASSERT(offsets[e] >= 0 && offsets[e] <= offsets[e + 1], offsets[e], offsets[e + 1]);
  SPA_DBG_ASSERT(MODE == 2 ? kend <= a_rows && kend <= b_rows : mend <= a_rows && m0 < mend, MODE == 2 ? kend : mend, a_rows);
  const int n0 = nt * BN;
  const int ktiles = kend > k0 ? (int)((kend - k0 + BK - 1) / BK) : 0;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  unsigned voA[2], voB[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    voA[j] = dma_off(A_KC, tid, j, lda);
    voB[j] = dma_off(B_KC, tid, j, ldb);
  }
  // readable extents (elements): whole operands, or up to the expert's last token (dW)
  const long limA = MODE == 2 ? kend * lda : a_rows * lda;
  const long limB = MODE == 2 ? kend * ldb : b_rows * ldb;

  // half images of stage s: A0 A1 B0 B1
  auto half = [&](int s, int which) -> char* { return smem + s * STAGE + which * HALF; };
  auto stage = [&](int t, int which) {       // which: 0 A0, 1 A1, 2 B0, 3 B1
    if (ABL == 1) return;
    char* dst = half(t & 1, which) + wave_u * 1024;
    const long kk = k0 + (long)t * BK;       // absolute reduction index of the tile
    if (which < 2) {
      const long r = m0 + 128 * which;
      stage_half(A, A_KC ? r * lda + kk : kk * lda + r, limA, dst, voA);
    } else {
      const long c = n0 + 128 * (which - 2);
      stage_half(Bp, B_KC ? c * ldb + kk : kk * ldb + c, limB, dst, voB);
    }
  };
  auto stage_piece = [&](int t, int which, int j) {   // one of the two DMA pieces of a half
    if (ABL == 1) return;
    char* dst = half(t & 1, which) + wave_u * 1024 + j * (NT * 16);
    const long kk = k0 + (long)t * BK;
    const bf16* base;
    long origin, limit;
    unsigned vo;
    if (which < 2) {
      const long r = m0 + 128 * which;
      base = A; origin = A_KC ? r * lda + kk : kk * lda + r; limit = limA; vo = voA[j];
    } else {
      const long c = n0 + 128 * (which - 2);
      base = Bp; origin = B_KC ? c * ldb + kk : kk * ldb + c; limit = limB; vo = voB[j];
    }
    const __amdgpu_buffer_rsrc_t rs = rsrc(base + origin, (limit - origin) * 2);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)dst, 16, vo, 0, 0, 0);
  };

  f32x4 acc[8][4];   // [m frag: mh*4 + i][n frag: nh*2 + j], C^T tiles (rows n, cols m)
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[4][2], b0f[2][2], b1f[2][2];     // one A half, BOTH B halves in registers
  bool do_reads = true;                      // ablation 2: fragments read in the first K-tile only

  auto read_a = [&](const char* h) {
    if (!do_reads) return;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        af[i][s] = A_KC ? rd_kc(h, wm * 64 + 16 * i, s, lane) : rd_ks(h, wm * 64 + 16 * i, s, lane);
  };
  auto read_b = [&](const char* h, bf16x8 (&bf)[2][2]) {
    if (!do_reads) return;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        bf[j][s] = B_KC ? rd_kc(h, wn * 32 + 16 * j, s, lane) : rd_ks(h, wn * 32 + 16 * j, s, lane);
  };
  // MFMA cluster with the phase's two DMA pieces issued between MFMAs 4|5 and 10|11, so their
  // (long) address-processing issue overlaps this wave's own MFMAs (st_t < 0: nothing to stage)
  auto mfma_qs = [&](int mh, int nh, const bf16x8 (&bf)[2][2], int st_t, int st_w) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[mh * 4 + i][nh * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][s], af[i][s], acc[mh * 4 + i][nh * 2 + j], 0, 0, 0);
          const int idx = s * 8 + i * 2 + j;
          if ((idx == 4 || idx == 10) && st_t >= 0) {
            __builtin_amdgcn_sched_barrier(0);
            stage_piece(st_t, st_w, idx == 4 ? 0 : 1);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
    __builtin_amdgcn_s_setprio(0);
  };
  auto mfma_q = [&](int mh, int nh, const bf16x8 (&bf)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[mh * 4 + i][nh * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][s], af[i][s], acc[mh * 4 + i][nh * 2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // Schedule (K-tile t lives in stage t & 1). Reads: P1 A0 + B0, P2 B1, P3 A1, P4 none (B0
  // still in registers). A half is free 2 phases after its last read, so tile t+2 refills the
  // stage of tile t while t is still being computed:
  //   P1 stages B1(t+1)   P2 A1(t+1)   P3 A0(t+2)   P4 B0(t+2)
  // => 4 halves (8 DMA per thread) stay in flight across every wait; each half has 5-6 phases
  // between issue and first read. Waits (end of P1, P2, P4) retire exactly the next reader's half.
  if constexpr (MODE != 2 && ABL == 0 && !ILV) {
    if (__builtin_amdgcn_readfirstlane((int)tail)) {
      // Tail tile: rows [m0, mend) (<= TR = 64) x 256 columns, 3-stage ring of 40 KiB K-tiles (A: 64
      // rows, one DMA piece per thread; B0 / B1: the usual 128-column halves), two K-tiles in flight:
      // 16 MFMAs per wave per K-tile are too few to cover a one-deep prefetch's latency. Wave (tm, wn)
      // owns rows tm * 32 + [0, 32), cols 64 wn + [0, 64); the tail blocks run last, in the grid's
      // final partial dispatch round.
      constexpr int TS = 8192 + 2 * HALF;
      const int tm = wave >> 2;
      f32x4 tacc[2][4];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) tacc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      auto tstage = [&](int t) {
        char* dst = smem + (t % 3) * TS + wave_u * 1024;
        const long kk = k0 + (long)t * BK;
        {
          const long origin = m0 * lda + kk;       // A is K-contiguous in modes 0 and 1
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc(A + origin, (limA - origin) * 2), (lds_void*)dst, 16, voA[0], 0, 0, 0);
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const long c = n0 + 128 * h;
          const long origin = B_KC ? c * ldb + kk : kk * ldb + c;
          const __amdgpu_buffer_rsrc_t rs = rsrc(Bp + origin, (limB - origin) * 2);
#pragma unroll
          for (int j = 0; j < 2; ++j)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + 8192 + h * HALF + j * (NT * 16)), 16, voB[j], 0, 0, 0);
        }
      };
      if (ktiles > 0) tstage(0);
      if (ktiles > 1) tstage(1);
      for (int t = 0; t < ktiles; ++t) {
        const char* ts = smem + (t % 3) * TS;
        if (t + 2 < ktiles) { tstage(t + 2); G8_WAIT_VM(10); } else if (t + 1 < ktiles) { G8_WAIT_VM(5); } else { G8_WAIT_VM(0); }
        __builtin_amdgcn_s_barrier();
        bf16x8 ta[2][2], tb[4][2];
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
#pragma unroll
          for (int i = 0; i < 2; ++i) ta[i][ss] = rd_kc(ts, tm * 32 + 16 * i, ss, lane);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int c = 64 * wn + 16 * j;
            const char* hb = ts + 8192 + (c >> 7) * HALF;
            tb[j][ss] = B_KC ? rd_kc(hb, c & 127, ss, lane) : rd_ks(hb, c & 127, ss, lane);
          }
        }
        G8_WAIT_LGKM0();
#pragma unroll
        for (int ss = 0; ss < 2; ++ss)
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              tacc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tb[j][ss], ta[i][ss], tacc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_barrier();
      }
      // C^T fragments: lane holds C[row0 + (lane & 15)][col0 + 4 (lane >> 4) + q], 8 B per lane
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const long gm = m0 + tm * 32 + 16 * i + (lane & 15);
          const int gn = n0 + 64 * wn + 16 * j + 4 * (lane >> 4);
          if (gm < mend && gn < N && SPA_DBG_OK(gm, M) & SPA_DBG_OK(gn + 3, ldc)) {
            bf16* cp = Cp + gm * ldc + gn;
            const f32x4 v = tacc[i][j];
            bf16x4 w4;
            if (accumulate) {
              const bf16x4 o = *reinterpret_cast<const bf16x4*>(cp);
#pragma unroll
              for (int q = 0; q < 4; ++q) w4[q] = (bf16)(v[q] + (float)o[q]);
            } else {
#pragma unroll
              for (int q = 0; q < 4; ++q) w4[q] = (bf16)v[q];
            }
            *reinterpret_cast<bf16x4*>(cp) = w4;
          }
        }
      return;
    }
  }
  const bool late = __builtin_amdgcn_readfirstlane(wave) >= 4;   // scalar branch, not an EXEC mask
  if (ILV) {
    // (measured slower; kept for the A/B) DMA issue inside the MFMA clusters (after the phase's first barrier): with the stagger a
    // half waited for at the end of phase q may be read from phase q+2 on, so the waits run one
    // phase earlier than the reads need: end of P1 -> A1(t) (read P3), end of P3 -> A0, B0(t+1)
    // (read P1 next), end of P4 -> B1(t+1) (read P2 next); 3 halves stay in flight.
    if (ktiles > 0) {
      stage(0, 0); stage(0, 2); stage(0, 3); stage(0, 1);
      if (ktiles > 1) { stage(1, 0); stage(1, 2); G8_WAIT_VM(6); } else { G8_WAIT_VM(2); }  // A0 B0 B1 (0)
      __builtin_amdgcn_s_barrier();
      if (late) __builtin_amdgcn_s_barrier();
    }
    for (int t = 0; t < ktiles; ++t) {
      const int s = t & 1;
      const bool n1 = t + 1 < ktiles, n2 = t + 2 < ktiles;
      do_reads = ABL != 2 || t == 0;
      // ---- phase 1: quadrant (0,0); stages B1(t+1)
      read_a(half(s, 0));
      read_b(half(s, 2), b0f);
      __builtin_amdgcn_s_barrier();
      G8_WAIT_LGKM0();
      mfma_qs(0, 0, b0f, n1 ? t + 1 : -1, 3);
      if (n1) { G8_WAIT_VM(6); } else { G8_WAIT_VM(0); }                    // retire A1(t)
      __builtin_amdgcn_s_barrier();
      // ---- phase 2: quadrant (0,1); stages A1(t+1)
      read_b(half(s, 3), b1f);
      __builtin_amdgcn_s_barrier();
      G8_WAIT_LGKM0();
      mfma_qs(0, 1, b1f, n1 ? t + 1 : -1, 1);
      __builtin_amdgcn_s_barrier();
      // ---- phase 3: quadrant (1,1); stages A0(t+2)
      read_a(half(s, 1));
      __builtin_amdgcn_s_barrier();
      G8_WAIT_LGKM0();
      mfma_qs(1, 1, b1f, n2 ? t + 2 : -1, 0);
      if (n1) { if (n2) { G8_WAIT_VM(6); } else { G8_WAIT_VM(4); } }        // retire A0, B0(t+1)
      __builtin_amdgcn_s_barrier();
      // ---- phase 4: quadrant (1,0), no LDS reads; stages B0(t+2)
      __builtin_amdgcn_s_barrier();
      mfma_qs(1, 0, b0f, n2 ? t + 2 : -1, 2);
      if (n1) { if (n2) { G8_WAIT_VM(6); } else { G8_WAIT_VM(2); } }        // retire B1(t+1)
      __builtin_amdgcn_s_barrier();
    }
  } else if (ABL == 0) {
    // Shipped schedule ("schedule 2"): no DMA in the phase that reads 12 fragments (P1: A0 + B0).
    // B1(t+2) moves from P1(t+1) to P4(t) next to B0(t+2) (B1(t) was last read in P2(t): 2
    // phases, the minimum that A0's restage already uses), so the phases carry reads / DMA halves
    // 12/0, 4/1, 8/1, 0/2 instead of 12/1, 4/1, 8/1, 0/1, and up to 5 halves stay in flight.
    // ABBA vs the previous schedule (tools/bench_gemm8_dense.py --ab 8,
    // profiles/r3_gemm8_schedule2_ab.txt): dense 8192^3 +3-8 %, grouped dX +10-11 %, fwd and dW
    // +1-3 %. Rejected in the same A/B: A0(t+2) also in P4 (12/0 4/1 8/0 0/3: -2..-5 %) and a
    // second A fragment set with A0(t+1) read in P4 (4/1 4/1 8/1 8/1: -3..-14 %); later A/Bs: the
    // MFMA clusters without s_setprio(1) -13..-19 %, P1 reading B0 before A0 with an lgkmcnt(8)
    // before its barrier -1..-2 % (profiles/r3_gemm8_schedule2_ab.txt).
    //   P1 -        P2 A1(t+1)   P3 A0(t+2)   P4 B0(t+2) B1(t+2)
    // Waits: end of P1 retires B1(t) (younger: A1(t) + A0 B0 B1(t+1)), end of P2 A1(t) (younger:
    // A0 B0 B1 A1(t+1)), end of P4 A0, B0(t+1) (younger: B1 A1(t+1) + A0 B0 B1(t+2)).
    G8_T(1);
    if (ktiles > 0) {
      stage(0, 0); stage(0, 2); stage(0, 3); stage(0, 1);
      if (ktiles > 1) { stage(1, 0); stage(1, 2); stage(1, 3); G8_WAIT_VM(10); } else { G8_WAIT_VM(4); }  // A0, B0 (0)
      __builtin_amdgcn_s_barrier();
      if (late) __builtin_amdgcn_s_barrier();
    }
    G8_T(2);
    for (int t = 0; t < ktiles; ++t) {
      const int s = t & 1;
      const bool n1 = t + 1 < ktiles, n2 = t + 2 < ktiles;
      // ---- phase 1: quadrant (0,0), no DMA
      read_a(half(s, 0));
      read_b(half(s, 2), b0f);
      if (n1) { G8_WAIT_VM(8); } else { G8_WAIT_VM(2); }                       // retire B1(t)
      __builtin_amdgcn_s_barrier();
      G8_WAIT_LGKM0();
      mfma_q(0, 0, b0f);
      __builtin_amdgcn_s_barrier();
      // ---- phase 2: quadrant (0,1)
      read_b(half(s, 3), b1f);
      if (n1) { stage(t + 1, 1); G8_WAIT_VM(8); } else { G8_WAIT_VM(0); }      // retire A1(t)
      __builtin_amdgcn_s_barrier();
      G8_WAIT_LGKM0();
      mfma_q(0, 1, b1f);
      __builtin_amdgcn_s_barrier();
      // ---- phase 3: quadrant (1,1)
      read_a(half(s, 1));
      if (n2) stage(t + 2, 0);
      __builtin_amdgcn_s_barrier();
      G8_WAIT_LGKM0();
      mfma_q(1, 1, b1f);
      __builtin_amdgcn_s_barrier();
      // ---- phase 4: quadrant (1,0) -- no LDS reads
      if (n2) { stage(t + 2, 2); stage(t + 2, 3); G8_WAIT_VM(10); }             // retire A0, B0(t+1)
      else if (n1) { G8_WAIT_VM(4); }
      __builtin_amdgcn_s_barrier();
      mfma_q(1, 0, b0f);
      __builtin_amdgcn_s_barrier();
    }
  } else {
  if (ktiles > 0) {
    stage(0, 0); stage(0, 2); stage(0, 3); stage(0, 1);
    if (ktiles > 1) { stage(1, 0); stage(1, 2); G8_WAIT_VM(8); } else { G8_WAIT_VM(4); }   // A0, B0 (0)
    __builtin_amdgcn_s_barrier();
    if (late) __builtin_amdgcn_s_barrier();
  }
  for (int t = 0; t < ktiles; ++t) {
    const int s = t & 1;
    const bool n1 = t + 1 < ktiles, n2 = t + 2 < ktiles;
    do_reads = ABL != 2 || t == 0;
    // ---- phase 1: quadrant (0,0)
    read_a(half(s, 0));
    read_b(half(s, 2), b0f);
    if (n1) { stage(t + 1, 3); G8_WAIT_VM(8); } else { G8_WAIT_VM(2); }      // retire B1(t)
    __builtin_amdgcn_s_barrier();
    G8_WAIT_LGKM0();
    mfma_q(0, 0, b0f);
    __builtin_amdgcn_s_barrier();
    // ---- phase 2: quadrant (0,1)
    read_b(half(s, 3), b1f);
    if (n1) { stage(t + 1, 1); G8_WAIT_VM(8); } else { G8_WAIT_VM(0); }      // retire A1(t)
    __builtin_amdgcn_s_barrier();
    G8_WAIT_LGKM0();
    mfma_q(0, 1, b1f);
    __builtin_amdgcn_s_barrier();
    // ---- phase 3: quadrant (1,1)
    read_a(half(s, 1));
    if (n2) stage(t + 2, 0);
    __builtin_amdgcn_s_barrier();
    G8_WAIT_LGKM0();
    mfma_q(1, 1, b1f);
    __builtin_amdgcn_s_barrier();
    // ---- phase 4: quadrant (1,0) -- no LDS reads
    if (n2) { stage(t + 2, 2); G8_WAIT_VM(8); }                              // retire A0, B0(t+1)
    else if (n1) { G8_WAIT_VM(0); }
    __builtin_amdgcn_s_barrier();
    mfma_q(1, 0, b0f);
    __builtin_amdgcn_s_barrier();
  }
  }
  if (ktiles > 0 && !late) __builtin_amdgcn_s_barrier();   // equal barrier counts on exit
  G8_T(3);
  if constexpr (PART) {
    // fp32 partials straight from the fragments: 16 rows x 64 contiguous bytes per store
    float* Cf = reinterpret_cast<float*>(C) + (long)e * strideC;
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int nh = 0; nh < 2; ++nh)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const long gm = m0 + mh * 128 + wm * 64 + 16 * i + (lane & 15);
            const int gn = n0 + nh * 128 + wn * 32 + 16 * j + 4 * (lane >> 4);
            if (gm < M && gn < N && SPA_DBG_OK(gn + 3, ldc)) *reinterpret_cast<f32x4*>(Cf + gm * ldc + gn) = acc[mh * 4 + i][nh * 2 + j];
          }
#if SPA_G8_STAMP
    if (ABL == 0 && tid == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      G8_T(4);
      long long* st = g8_stamp + (blockIdx.x % G8_NSTAMP) * 8;
      st[0] = g8t[1] - g8t[0]; st[1] = g8t[2] - g8t[1]; st[2] = g8t[3] - g8t[2]; st[3] = g8t[4] - g8t[3];
      st[4] = ktiles; st[5] = 10 + MODE;
    }
#endif
    return;
  }
  // ---- epilogue through LDS, one 128-row half at a time: C^T fragments (n = 4 (l >> 4) + q,
  // m = l & 15) -> padded row image (528-B rows: the 16 rows of a fragment store land on 16
  // distinct bank pairs) -> whole-row 16-byte global stores (a per-lane 8-byte store at a row
  // stride would touch 16 cache lines per instruction)
  constexpr int RS = 256 * 2 + 16;
  // accumulate: all 16 old-value chunks of this thread are loaded up front (buffer loads, zero past
  // the tile's rows / columns), so their latency overlaps the image writes; one load-wait-add-store
  // per chunk made the epilogue 30.7K cycles against 6.5K without accumulate (profiles/r5_gemm8_stamps.txt)
  const long rowlim = MODE == 2 ? (long)M : mend;
  const bool pre = accumulate && rowlim * ldc * 2 < 0x7fffffffL;
  bf16x8 old[2][8];
  if (pre) {
    const __amdgpu_buffer_rsrc_t cr = rsrc(Cp, rowlim * ldc * 2);
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const int idx = tid + c * NT, r = idx >> 5, ch = idx & 31;
        const long gm = m0 + mh * 128 + r;
        const int gn = n0 + ch * 8;
        const unsigned off = gn < N ? (unsigned)((gm * ldc + gn) * 2) : 0x80000000u;
        old[mh][c] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(cr, off, 0, 0));
      }
  }
  __syncthreads();
#pragma unroll
  for (int mh = 0; mh < 2; ++mh) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int nh = 0; nh < 2; ++nh)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const f32x4 v = acc[mh * 4 + i][nh * 2 + j];
          bf16x4 w4;
#pragma unroll
          for (int q = 0; q < 4; ++q) w4[q] = (bf16)v[q];
          const int r = wm * 64 + 16 * i + (lane & 15);
          const int cn = nh * 128 + wn * 32 + 16 * j + 4 * (lane >> 4);
          *reinterpret_cast<bf16x4*>(smem + r * RS + cn * 2) = w4;
        }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int idx = tid + c * NT, r = idx >> 5, ch = idx & 31;
      const long gm = m0 + mh * 128 + r;
      const int gn = n0 + ch * 8;
      if ((MODE == 2 ? gm < M : gm < mend) && gn < N && SPA_DBG_OK(gm, M) & SPA_DBG_OK(gn + 7, ldc)) {
        bf16x8 v = *reinterpret_cast<const bf16x8*>(smem + r * RS + ch * 16);
        bf16* cp = Cp + gm * ldc + gn;
        if (accumulate) {
          const bf16x8 o = pre ? old[mh][c] : *reinterpret_cast<const bf16x8*>(cp);
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] = (bf16)((float)v[q] + (float)o[q]);
        }
        *reinterpret_cast<bf16x8*>(cp) = v;
      }
    }
    __syncthreads();
  }
#if SPA_G8_STAMP
  if (ABL == 0 && tid == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the epilogue's stores left
    G8_T(4);
    long long* st = g8_stamp + (blockIdx.x % G8_NSTAMP) * 8;
    st[0] = g8t[1] - g8t[0]; st[1] = g8t[2] - g8t[1]; st[2] = g8t[3] - g8t[2]; st[3] = g8t[4] - g8t[3];
    st[4] = ktiles; st[5] = MODE;
  }
#endif
}

// out[i] (+)= sum_s part[s, i] over n elements (n % 4 == 0), bf16 or fp32 out
template <typename OT>
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, OT* __restrict__ out, long n,
                                                           int S, int accumulate) {
  for (long i = ((long)blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += (long)gridDim.x * 1024) {
    f32x4 a = *reinterpret_cast<const f32x4*>(part + i);
    for (int s = 1; s < S; ++s) a += *reinterpret_cast<const f32x4*>(part + (long)s * n + i);
    if constexpr (sizeof(OT) == 4) {
      if (accumulate) a += *reinterpret_cast<const f32x4*>(out + i);
      *reinterpret_cast<f32x4*>(out + i) = a;
    } else {
      bf16x4 o;
      if (accumulate) {
        const bf16x4 old = *reinterpret_cast<const bf16x4*>(out + i);
#pragma unroll
        for (int q = 0; q < 4; ++q) a[q] += (float)old[q];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = (bf16)a[q];
      *reinterpret_cast<bf16x4*>(out + i) = o;
    }
  }
}

void launch_gemm4r_wgrad_part(const bf16* dy, const bf16* x, float* part, const int* offsets, int S, int N, int K,
                              long lda, long ldb, long T, hipStream_t st);
// SPA_WGRAD_G4=0: the partial products on this file's 8-phase kernel instead of gemm4a.hip's gemm4r
static bool wgrad_g4() {
  const char* e = getenv("SPA_WGRAD_G4");
  return !(e && e[0] == '0');
}

// Dense weight gradient out[N, K] (+)= dy[T, N]^T x[T, K] on the 8-phase kernel's token-major
// (mode 2) path, split over tokens into S slices so that S x tiles fills the chip; fp32
// partials, deterministic reduce. For the T >> N, K products (ViT-B/16: T = 50432, N, K
// 768..3072) where hipBLASLt's direct TN form runs 230-600 TF
// (profiles/r2_wgrad_layouts_vit_llama.txt). out: bf16 or fp32 (a main_grad), contiguous.
at::Tensor wgrad8(const at::Tensor& dy, const at::Tensor& x, const c10::optional<at::Tensor>& out_, bool accumulate,
                  int64_t splits) {
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && x.scalar_type() == at::kBFloat16, "wgrad8: bf16 operands");
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && dy.size(0) == x.size(0), "wgrad8: dy [T, N], x [T, K]");
  TORCH_CHECK(dy.stride(1) == 1 && x.stride(1) == 1, "wgrad8: unit column stride");
  const long T = dy.size(0);
  const int N = dy.size(1), K = x.size(1);
  const long lda = dy.stride(0), ldb = x.stride(0);
  TORCH_CHECK(N % 8 == 0 && K % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0, "wgrad8: dims and row strides % 8");
  TORCH_CHECK((uintptr_t)dy.data_ptr() % 16 == 0 && (uintptr_t)x.data_ptr() % 16 == 0, "wgrad8: 16-B aligned");
  TORCH_CHECK((T + 64) * (lda + 256) * 2 < (1L << 32) && (T + 64) * (ldb + 256) * 2 < (1L << 32),
              "wgrad8: operands < 4 GiB");
  DeviceGuard g(dy.device());
  auto out = out_ ? *out_ : at::empty({N, K}, dy.options());
  TORCH_CHECK(out.is_contiguous() && out.numel() == (long)N * K &&
                  (out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat),
              "wgrad8: out [N, K] bf16/fp32 contiguous");
  if (N == 0 || K == 0) return out;
  auto st = stream();
  const int tiles = cdiv(N, 256) * cdiv(K, 256);
  int S = (int)splits;
  if (S <= 0) S = std::max(1, 256 / tiles);              // one wave of blocks over 256 CUs
  S = (int)std::max<long>(1, std::min<long>(S, T / 512));  // >= 8 k-iterations per slice
  const long chunk = ((T + S - 1) / S + 63) / 64 * 64;
  S = (int)((T + chunk - 1) / chunk);
  if (S == 0) {
    if (!accumulate) out.zero_();
    return out;
  }
  // slice offsets live on the device, one tensor per (device, T, S): the upload (a synchronising
  // pageable copy) happens on first use only, never per backward
  static std::map<std::tuple<int, long, int>, at::Tensor> offs_cache;
  static std::mutex offs_mu;
  at::Tensor offsets;
  {
    std::lock_guard<std::mutex> lk(offs_mu);
    auto key = std::make_tuple((int)dy.get_device(), T, S);
    auto it = offs_cache.find(key);
    if (it == offs_cache.end()) {
      std::vector<int> off(S + 1);
      for (int i = 0; i <= S; ++i) off[i] = (int)std::min<long>(T, (long)i * chunk);
      it = offs_cache.emplace(key, at::from_blob(off.data(), {S + 1}, at::kInt).to(dy.device())).first;
    }
    offsets = it->second;
  }
  auto part = at::empty({S, N, K}, dy.options().dtype(at::kFloat));
  if (wgrad_g4())   // the register-staged 4-wave kernel (gemm4a.hip): grouped dW +11 % over this one
    launch_gemm4r_wgrad_part((const bf16*)dy.data_ptr(), (const bf16*)x.data_ptr(), part.data_ptr<float>(),
                             offsets.data_ptr<int>(), S, N, K, lda, ldb, T, st);
  else
    grouped_gemm8_kernel<2, 0, false, true><<<S * tiles, 512, 0, st>>>(
        (const bf16*)dy.data_ptr(), (const bf16*)x.data_ptr(), reinterpret_cast<bf16*>(part.data_ptr<float>()),
        offsets.data_ptr<int>(), S, N, K, 0, lda, ldb, K, 0, (long)N * K, 0, T, T);
  SPA_LAUNCH_CHECK();
  const long n = (long)N * K;
  const int rb = (int)std::min<long>((n / 4 + 255) / 256, 4096);
  if (out.scalar_type() == at::kFloat)
    wgrad_reduce_kernel<float><<<rb, 256, 0, st>>>(part.data_ptr<float>(), out.data_ptr<float>(), n, S,
                                                   accumulate ? 1 : 0);
  else
    wgrad_reduce_kernel<bf16><<<rb, 256, 0, st>>>(part.data_ptr<float>(), (bf16*)out.data_ptr(), n, S,
                                                  accumulate ? 1 : 0);
  SPA_LAUNCH_CHECK();
  return out;
}

static int ablation() {
  const char* e = getenv("SPA_GG8_ABLATE");
  return e ? atoi(e) : 0;
}
// SPA_GG8_TAIL (read per call): an expert's last rows past a multiple of 256 go to a 64-row tail
// tile when there are at most this many (default 64, the tail tile's capacity; 0: always a full tile)
static int g8_tail() {
  const char* e = getenv("SPA_GG8_TAIL");
  return e ? std::max(0, std::min(64, atoi(e))) : 64;
}
// SPA_G8_GM (read per call): row tiles per tile group of a dense (E = 1) forward / dX grid
// (default 4: 4 x 8 tiles per XCD wave instead of 1 x 32 -- dense 8192^3 +5 % fwd, +14 % dX);
// grouped GEMMs keep the row-major order (the grouping measured -3 % on their forward)
static int g8_group(int E) {
  const char* e = getenv("SPA_G8_GM");
  return E > 1 ? 1 : (e ? std::max(1, atoi(e)) : 4);
}
// same contract as grouped_gemm (moe.hip); requires the reduction dim % 64 == 0 in modes 0/1
// and N, K % 8 == 0
at::Tensor grouped_gemm8(const at::Tensor& a, const at::Tensor& w, const at::Tensor& offsets, int64_t mode,
                         const c10::optional<at::Tensor>& out_, bool accumulate) {
  TORCH_CHECK(a.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16, "grouped_gemm8: bf16");
  TORCH_CHECK(a.is_contiguous() && w.is_contiguous() && offsets.scalar_type() == at::kInt);
  const int E = offsets.numel() - 1;
  TORCH_CHECK(E >= 1 && E <= 512, "grouped_gemm8: 1..512 experts");
  TORCH_CHECK((uintptr_t)a.data_ptr() % 16 == 0 && (uintptr_t)w.data_ptr() % 16 == 0, "grouped_gemm8: 16-B aligned");
  DeviceGuard g(a.device());
  auto st = stream();
  if (mode == 0 || mode == 1) {
    TORCH_CHECK(w.dim() == 3 && w.size(0) == E);
    const int M = a.size(0), Nw = w.size(1), Kw = w.size(2);
    const int N = mode == 0 ? Nw : Kw, K = mode == 0 ? Kw : Nw;
    TORCH_CHECK(a.size(1) == K, "grouped_gemm8: A/W shape mismatch");
    TORCH_CHECK(K % 64 == 0 && N % 8 == 0, "grouped_gemm8: reduction % 64, output cols % 8");
    TORCH_CHECK((long)(M + 256) * K * 2 < (1L << 32) && (long)(Nw + 256) * Kw * 2 < (1L << 32),
                "grouped_gemm8: operands < 4 GiB");
    auto out = out_ ? *out_ : at::empty({M, N}, a.options());
    if (M == 0) return out;
    TORCH_CHECK(out.is_contiguous() && out.size(0) == M && out.size(1) == N);
    const int grid = (cdiv(M, 256) + E) * cdiv(N, 256);
#define G8_L(MD, AB)                                                                                          \
  if (abl == 4) grouped_gemm8_kernel<MD, 0, true><<<grid, 512, 0, st>>>(                                     \
      (const bf16*)a.data_ptr(), (const bf16*)w.data_ptr(), (bf16*)out.data_ptr(), offsets.data_ptr<int>(), E, M,  \
      N, K, K, Kw, N, (long)Nw * Kw, 0, accumulate ? 1 : 0, M, Nw, g8_group(E));                      \
  else grouped_gemm8_kernel<MD, AB><<<grid, 512, 0, st>>>((const bf16*)a.data_ptr(), (const bf16*)w.data_ptr(),     \
                                                     (bf16*)out.data_ptr(), offsets.data_ptr<int>(), E, M, N, K, K, \
                                                     Kw, N, (long)Nw * Kw, 0, accumulate ? 1 : 0, M, Nw, g8_group(E), \
                                                     abl == 0 ? g8_tail() : 0)
    const int abl = ablation();
    if (mode == 0) {
      if (abl == 1) { G8_L(0, 1); } else if (abl == 2) { G8_L(0, 2); } else if (abl == 3) { G8_L(0, 3); } else if (abl == 8) { G8_L(0, 8); } else { G8_L(0, 0); }
    } else {
      if (abl == 1) { G8_L(1, 1); } else if (abl == 2) { G8_L(1, 2); } else if (abl == 3) { G8_L(1, 3); } else if (abl == 8) { G8_L(1, 8); } else { G8_L(1, 0); }
    }
#undef G8_L
    SPA_LAUNCH_CHECK();
    return out;
  }
  TORCH_CHECK(mode == 2, "grouped_gemm8: mode 0/1/2");
  const int N = a.size(1), K = w.size(1), T = a.size(0);
  TORCH_CHECK(w.size(0) == T && N % 8 == 0 && K % 8 == 0);
  TORCH_CHECK((long)(T + 64) * (N + 256) * 2 < (1L << 32) && (long)(T + 64) * (K + 256) * 2 < (1L << 32),
              "grouped_gemm8: operands < 4 GiB");
  auto out = out_ ? *out_ : at::empty({E, N, K}, a.options());
  TORCH_CHECK(out.is_contiguous() && out.numel() == (long)E * N * K);
  const int grid = E * cdiv(N, 256) * cdiv(K, 256);
#define G8_L2(AB)                                                                                             \
  if (abl == 4) grouped_gemm8_kernel<2, 0, true><<<grid, 512, 0, st>>>(                                      \
      (const bf16*)a.data_ptr(), (const bf16*)w.data_ptr(), (bf16*)out.data_ptr(), offsets.data_ptr<int>(), E, N,  \
      K, 0, N, K, K, 0, (long)N * K, accumulate ? 1 : 0, T, T);                                     \
  else grouped_gemm8_kernel<2, AB><<<grid, 512, 0, st>>>((const bf16*)a.data_ptr(), (const bf16*)w.data_ptr(),      \
                                                    (bf16*)out.data_ptr(), offsets.data_ptr<int>(), E, N, K, 0, N, K, \
                                                    K, 0, (long)N * K, accumulate ? 1 : 0, T, T)
  const int abl = ablation();
  if (abl == 1) { G8_L2(1); } else if (abl == 2) { G8_L2(2); } else if (abl == 3) { G8_L2(3); } else if (abl == 8) { G8_L2(8); } else { G8_L2(0); }
#undef G8_L2
  SPA_LAUNCH_CHECK();
  return out;
}

// profiling build (SPA_G8_STAMP=1): the per-block segment stamps since the last call, then cleared
// [G8_NSTAMP, 8] int64 (mapping, prologue, K-loop, epilogue cycles, K-tiles, mode); empty otherwise
at::Tensor g8_stamps() {
#if SPA_G8_STAMP
  auto out = at::empty({G8_NSTAMP, 8}, at::TensorOptions().dtype(at::kLong));
  TORCH_CHECK(hipDeviceSynchronize() == hipSuccess && hipMemcpyFromSymbol(out.data_ptr(), HIP_SYMBOL(g8_stamp),
              sizeof(long long) * G8_NSTAMP * 8, 0, hipMemcpyDeviceToHost) == hipSuccess, "g8_stamps: copy failed");
  void* sym = nullptr;   // read-and-clear: the next launch's blocks are the only live entries
  TORCH_CHECK(hipGetSymbolAddress(&sym, HIP_SYMBOL(g8_stamp)) == hipSuccess &&
              hipMemset(sym, 0, sizeof(long long) * G8_NSTAMP * 8) == hipSuccess, "g8_stamps: clear failed");
  return out;
#else
  return at::Tensor();
#endif
}

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.def("g8_stamps() -> Tensor", &spa::g8_stamps);
  m.def("grouped_gemm8(Tensor a, Tensor w, Tensor offsets, int mode, Tensor(a!)? out, bool accumulate) -> Tensor");
  m.def("wgrad8(Tensor dy, Tensor x, Tensor(a!)? out, bool accumulate, int splits) -> Tensor");
}
TORCH_LIBRARY_IMPL(spa, CUDA, m) {
  m.impl("grouped_gemm8", &spa::grouped_gemm8);
  m.impl("wgrad8", &spa::wgrad8);
}
