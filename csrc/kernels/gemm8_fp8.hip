// Block-scaled fp8 (e4m3) grouped GEMM on the 8-phase LDS-DMA schedule of gemm8.hip, with
// v_mfma_scale_f32_16x16x128_f8f6f4 (E8M0 scales applied by the matrix core).
//
// Why a second fp8 kernel: the register-staged 256 x 256 kernel of moe_fp8.hip reads 1.5 KB of LDS
// per 32x32x64 MFMA and writes every staged byte through VGPRs -- about 128 B/clk/CU of LDS
// traffic at full MFMA rate, i.e. LDS-bound at 1.2-1.5 PF. Here a K-tile is 128 BYTES per row
// (128 e4m3 values), so the LDS images, the DMA pieces, the swizzle and the phase schedule are
// byte-for-byte those of the bf16 kernel (64 bf16 per row): per phase a wave runs 8 MFMAs of 32
// cycles (the bf16 kernel: 16 of 16 cycles) on the same LDS bytes, i.e. twice the FLOPs per staged
// byte and per LDS read at the same issue cadence.
//
// Two operand kinds, both K-contiguous (the quantizers produce the transposed images):
//   WG = false (forward / dX):  Y[M, N] = (A[M, K] * sa) (B_e[N, K] * sb_e)^T, rows of A grouped by
//       expert offsets; sa: 1 x 128 activation tiles, sb: 128 x 128 weight blocks.
//   WG = true (weight gradient): C_e[M, N] (+)= A[:, seg_e] B[:, seg_e]^T over expert e's padded
//       token segment [poff[e], poff[e+1]); both operands with per-row 128 x 1 token tiles.
// Scales travel with their K-tile: the host transposes them to k-tile-major byte arrays
// ([KB][rows], rows padded to 16) so the 256 row scales of one tile are contiguous, and waves 0 / 1
// DMA them (one 16-B piece per lane, 1 KiB slot) right before the tile's A0 half -- older than A0 in
// the wave's vmcnt order, so the counted wait that retires A0 retires them too (the extra op only
// makes the other counted waits of those two waves stricter).
//
// MFMA lane maps (16x16x128, e4m3): operand lane l holds row (l & 15), bytes 32 (l >> 4) .. +31 of
// the 128-byte K-tile; the scale VGPR of lane l applies to row (l & 15). Instruction A = the B-side
// fragment (rows n), instruction B = the A-side fragment (rows m): acc[i][j] is a C^T tile with
// m = 16 i + (l & 15), n = 16 j + 4 (l >> 4) + q -- the accumulator layout of gemm8.hip.
#include "act_common.h"
#include "gemm_common.h"

SPA_DEBUG_TU("gemm8_fp8.hip")

namespace spa {

namespace g8f {

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int BM = 256, BN = 256, BK = 128, NT = 512;
constexpr int HALF = 128 * BK;                 // bytes per half-tile image (16 KiB)
constexpr int SCL = 2048;                      // per stage: A-scale slot (1 KiB) + B-scale slot
constexpr int STAGE = 4 * HALF + SCL;          // A0 A1 B0 B1 + scales

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, long bytes) {
  const long nb = bytes < 0 ? 0 : (bytes > 0xFFFFFFFFL ? 0xFFFFFFFFL : bytes);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)(unsigned)nb, 0x00020000);
}
// K-contiguous half [128 rows][128 B]: DMA slot q -> row q >> 3, chunk (q & 7) ^ ((row >> 1) & 7)
__device__ __forceinline__ unsigned dma_off(int tid, int j, long ld) {
  const int q = j * NT + tid;
  const int r = q >> 3, c = (q & 7) ^ ((r >> 1) & 7);
  return (unsigned)(r * ld + 16 * c);
}
// 16x16x128 operand: rows row0 .. row0 + 15 of a half image, lane l -> row (l & 15), bytes
// 32 (l >> 4) .. +31 (two swizzled 16-B chunks). Read as bf16x8 like gemm8.hip: with int4 loads
// hipcc could not tell the reads from the in-flight LDS-DMA writes and put a vmcnt(0) -- a drain
// of the whole DMA pipeline -- before every phase's first ds_read
__device__ __forceinline__ i32x8 rd_op(const char* half, int row0, int lane) {
  const int r = row0 + (lane & 15), c = 2 * (lane >> 4), sw = (r >> 1) & 7;
  const bf16x8 a = *reinterpret_cast<const bf16x8*>(half + r * BK + 16 * (c ^ sw));
  const bf16x8 b = *reinterpret_cast<const bf16x8*>(half + r * BK + 16 * ((c + 1) ^ sw));
  typedef int i32x4_ __attribute__((ext_vector_type(4)));
  const i32x4_ ai = __builtin_bit_cast(i32x4_, a), bi = __builtin_bit_cast(i32x4_, b);
  return __builtin_shufflevector(ai, bi, 0, 1, 2, 3, 4, 5, 6, 7);
}

}  // namespace g8f

#define G8F_WAIT_VM(N) asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory")
#define G8F_WAIT_LGKM0()                               \
  do {                                                 \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
    __builtin_amdgcn_sched_barrier(0);                 \
  } while (0)

// A [a_rows, lda] e4m3 (K-contiguous); B [.., ldb] e4m3 (WG = false: expert e at B + e * strideB,
// rows n); sAt [KB][ldsa] / sBt (WG: [KB][ldsb]; else [E][KB][ldsb] weight-block scales): E8M0
// bytes, k-tile major. offsets: expert row offsets (WG = false) or padded token offsets (WG).
// C: bf16 [M, N] (WG = false) or [E, M, N] bf16 / fp32 (out_f32), accumulate in place if asked.
template <bool WG>
__global__ __launch_bounds__(512, 1) void gemm8_fp8_kernel(const uint8_t* __restrict__ A,
                                                           const uint8_t* __restrict__ B,
                                                           const uint8_t* __restrict__ sAt,
                                                           const uint8_t* __restrict__ sBt, void* __restrict__ C,
                                                           const int* __restrict__ offsets, int E, int M, int N,
                                                           int K, long lda, long ldb, long strideB, long a_rows,
                                                           long b_rows, int KB, long ldsa, long ldsb, long sa_bytes,
                                                           long sb_bytes, int accumulate, int out_f32, int tailr = 0) {
  using namespace g8f;
  // ONE LDS array: a second __shared__ object can make hipcc drain the DMA queue before ds_reads
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE + 64];
  int* scratch = reinterpret_cast<int*>(smem + 2 * STAGE);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int nnt = (N + BN - 1) / BN;
  int lid = xcd_remap(blockIdx.x, gridDim.x);
  int nt = lid % nnt;
  int mt = lid / nnt;
  int e = 0;
  bool tail = false;
  long m0 = 0, mend = M, k0 = 0, kend = K;
  if (!WG) {
    int* wsum = scratch + 8;
    const int cnt = tid < E ? offsets[tid + 1] - offsets[tid] : 0, rem = cnt & (BM - 1);
    // tail tiles (gemm8.hip): an expert's last <= tailr rows past a multiple of 256 run on a 64-row tile
    const bool tl = rem > 0 && rem <= tailr;
    const int tiles = (cnt >> 8) + (rem > 0 && !tl ? 1 : 0);
    const int pk = tiles + (tl ? 1 << 20 : 0);   // row tiles | tail tiles << 20
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
    for (int w = 0; w < 8; ++w) {
      const int v = wsum[w];
      pre += w < wave ? v : 0;
      rows += v;
    }
    const int pre_t = pre >> 20, tails = rows >> 20;
    pre &= (1 << 20) - 1;
    rows &= (1 << 20) - 1;
    // real tiles on the lowest block ids, XCD remap over them only (gemm8.hip: the empty blocks of
    // the worst-case grid must not push real tiles into another dispatch round); tail tiles last
    const int R = rows * nnt;
    if ((int)blockIdx.x >= R + tails * nnt) return;
    tail = (int)blockIdx.x >= R;
    if (!tail) {
      lid = xcd_remap(blockIdx.x, R);
      nt = lid % nnt;
      mt = lid / nnt;
      if (tid < E && tiles > 0 && mt >= pre && mt < pre + tiles) { scratch[0] = tid; scratch[1] = mt - pre; }
    } else {
      const int t = blockIdx.x - R, j = t / nnt;
      nt = t % nnt;
      if (tid < E && tl && pre_t == j) { scratch[0] = tid; scratch[1] = cnt >> 8; }
    }
    __syncthreads();
    e = __builtin_amdgcn_readfirstlane(scratch[0]);
    if (e < 0) return;
    mt = __builtin_amdgcn_readfirstlane(scratch[1]);
    m0 = __builtin_amdgcn_readfirstlane(offsets[e]) + (long)mt * BM;
    mend = __builtin_amdgcn_readfirstlane(offsets[e + 1]);
  } else {
    const int nmt = (M + BM - 1) / BM;
    e = mt / nmt;
    mt = mt % nmt;
    if (e >= E) return;
    m0 = (long)mt * BM;
    k0 = __builtin_amdgcn_readfirstlane(offsets[e]);
    kend = __builtin_amdgcn_readfirstlane(offsets[e + 1]);
  }
  const int n0 = nt * BN;
  // debug build: the tile -> (expert, row tile) scan and the group offsets name real rows
  SPA_DBG_CHECK(e, E);
  SPA_DBG_ASSERT(offsets[e] >= 0 && offsets[e] <= offsets[e + 1], offsets[e], offsets[e + 1]);
  // (WG: the token range runs along the rows of the transposed K-contiguous images, stride lda / ldb)
  SPA_DBG_ASSERT(WG ? kend <= lda && kend <= ldb : mend <= a_rows && m0 < mend, WG ? kend : mend, WG ? lda : a_rows);
  const uint8_t* Bp = WG ? B : B + e * strideB;
  const int ktiles = kend > k0 ? (int)((kend - k0 + BK - 1) / BK) : 0;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  unsigned voA[2], voB[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    voA[j] = dma_off(tid, j, lda);
    voB[j] = dma_off(tid, j, ldb);
  }
  const long limA = a_rows * lda, limB = b_rows * ldb;
  // scale images: A rows m0 .. m0+255 and B rows n0 .. n0+255 (WG) / weight blocks n0/128 + {0,1}
  // start at byte (origin & 15) of their 1 KiB slot (16-B aligned DMA source)
  const long nb0 = WG ? n0 : n0 / 128;
  const int dA = (int)(m0 & 15), dB = (int)(nb0 & 15);

  auto half = [&](int s, int which) -> char* { return smem + s * STAGE + which * HALF; };
  auto stage = [&](int t, int which) {       // which: 0 A0 (+ the tile's scales), 1 A1, 2 B0, 3 B1
    char* dst = half(t & 1, which) + wave_u * 1024;
    const long kk = k0 + (long)t * BK;       // absolute reduction index (bytes) of the tile
    const int kb = (int)(kk / BK);
    if (which == 0 && wave_u < 2) {
      // wave 0: A scales, wave 1: B scales of tile t (one 16-B piece per lane)
      const uint8_t* sb = wave_u == 0 ? sAt + (long)kb * ldsa + (m0 & ~15L)
                                      : sBt + ((WG ? 0L : (long)e * KB) + kb) * ldsb + (nb0 & ~15L);
      const long lim = wave_u == 0 ? sa_bytes - (long)(sb - sAt) : sb_bytes - (long)(sb - sBt);
      const __amdgpu_buffer_rsrc_t rs = rsrc(sb, lim);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(smem + (t & 1) * STAGE + 4 * HALF + wave_u * 1024),
                                               16, (unsigned)(lane * 16), 0, 0, 0);
    }
    const bool isA = which < 2;
    const long origin = isA ? (m0 + 128 * which) * lda + kk : (n0 + 128 * (which - 2)) * ldb + kk;
    const uint8_t* base = isA ? A : Bp;
    const __amdgpu_buffer_rsrc_t rs = rsrc(base + origin, (isA ? limA : limB) - origin);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + j * (NT * 16)), 16, isA ? voA[j] : voB[j], 0, 0, 0);
  };

  f32x4 acc[8][4];   // [m frag: mh*4 + i][n frag: nh*2 + j], C^T tiles (rows n, cols m)
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  i32x8 af[4], b0f[2], b1f[2];
  int sca[2][4], scb[2][2];                  // [mh][i] / [nh][j] E8M0 bytes of the current tile

  auto read_a = [&](const char* h) {
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = rd_op(h, wm * 64 + 16 * i, lane);
  };
  auto read_b = [&](const char* h, i32x8 (&bf)[2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j) bf[j] = rd_op(h, wn * 32 + 16 * j, lane);
  };
  auto read_scales = [&](int s) {
    const uint8_t* sa = reinterpret_cast<const uint8_t*>(smem + s * STAGE + 4 * HALF) + dA;
    const uint8_t* sb = reinterpret_cast<const uint8_t*>(smem + s * STAGE + 4 * HALF + 1024) + dB;
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int i = 0; i < 4; ++i) sca[mh][i] = sa[mh * 128 + wm * 64 + 16 * i + (lane & 15)];
#pragma unroll
    for (int nh = 0; nh < 2; ++nh)
#pragma unroll
      for (int j = 0; j < 2; ++j) scb[nh][j] = WG ? sb[nh * 128 + wn * 32 + 16 * j + (lane & 15)] : sb[nh];
  };
  auto mfma_q = [&](int mh, int nh, const i32x8 (&bf)[2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[mh * 4 + i][nh * 2 + j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
            bf[j], af[i], acc[mh * 4 + i][nh * 2 + j], 0, 0, 0, scb[nh][j], 0, sca[mh][i]);
    // pin the cluster to its phase: hipcc otherwise sinks the (side-effect free) scaled MFMAs
    // out of the phase, past the barriers, into one block at the end of the K-tile
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(acc[mh * 4 + i][nh * 2 + j]));
    __builtin_amdgcn_s_setprio(0);
  };

  // Schedule (gemm8.hip): K-tile t lives in stage t & 1. Reads: P1 A0 + B0 + the tile's scales,
  // P2 B1, P3 A1, P4 none. Stages, S2 (forward / dX: gemm8.hip's shipped schedule): P1 none, P2
  // A1(t+1), P3 A0(t+2) (+ scales), P4 B0(t+2) and B1(t+2), waits vmcnt 8 / 8 / 10; otherwise (Wgrad:
  // the round-2 schedule, 3 % faster there, profiles/r3_gemm8_schedule2_ab.txt) P1 B1(t+1), P2
  // A1(t+1), P3 A0(t+2), P4 B0(t+2), waits 8 / 8 / 8. Waits (end of P1, P2, P4) retire exactly the
  // next reader's half (waves 0 / 1 count one scale piece more per A0 half, so their waits are one
  // piece stricter); waves 4-7 run one barrier behind waves 0-3.
  if constexpr (!WG) {
    if (__builtin_amdgcn_readfirstlane((int)tail)) {
      // Tail tile (gemm8.hip): rows [m0, mend) (<= 64) x 256 columns, 3-stage ring of 42 KiB K-tiles
      // (A: 64 rows, one DMA piece per thread; B0 / B1 halves; the tile's scale slots, waves 0 / 1);
      // wave (tm, wn) owns rows tm * 32 + [0, 32), cols 64 wn + [0, 64): 8 scaled MFMAs per K-tile
      constexpr int TS = 8192 + 2 * HALF + SCL;
      const int tm = wave >> 2;
      f32x4 tacc[2][4];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) tacc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      auto tstage = [&](int t) {
        char* dst = smem + (t % 3) * TS;
        const long kk = k0 + (long)t * BK;
        const int kb = (int)(kk / BK);
        if (wave_u < 2) {   // wave 0: A scales, wave 1: B scales of tile t
          const uint8_t* sb = wave_u == 0 ? sAt + (long)kb * ldsa + (m0 & ~15L) : sBt + ((long)e * KB + kb) * ldsb + (nb0 & ~15L);
          const long lim = wave_u == 0 ? sa_bytes - (long)(sb - sAt) : sb_bytes - (long)(sb - sBt);
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc(sb, lim), (lds_void*)(dst + 8192 + 2 * HALF + wave_u * 1024), 16,
                                                   (unsigned)(lane * 16), 0, 0, 0);
        }
        {
          const long origin = m0 * lda + kk;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc(A + origin, limA - origin), (lds_void*)(dst + wave_u * 1024), 16, voA[0], 0, 0, 0);
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const long origin = (n0 + 128 * h) * ldb + kk;
          const __amdgpu_buffer_rsrc_t rs = rsrc(Bp + origin, limB - origin);
#pragma unroll
          for (int j = 0; j < 2; ++j)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + 8192 + h * HALF + wave_u * 1024 + j * (NT * 16)), 16,
                                                     voB[j], 0, 0, 0);
        }
      };
      const bool sw = wave_u < 2;             // waves 0 / 1 issue one scale piece more per stage
      if (ktiles > 0) tstage(0);
      if (ktiles > 1) tstage(1);
      for (int t = 0; t < ktiles; ++t) {
        const char* ts = smem + (t % 3) * TS;
        if (t + 2 < ktiles) {
          tstage(t + 2);
          if (sw) { G8F_WAIT_VM(12); } else { G8F_WAIT_VM(10); }
        } else if (t + 1 < ktiles) {
          if (sw) { G8F_WAIT_VM(6); } else { G8F_WAIT_VM(5); }
        } else {
          G8F_WAIT_VM(0);
        }
        __builtin_amdgcn_s_barrier();
        i32x8 ta[2], tb[4];
        int tsa[2], tsb[4];
        const uint8_t* sa = reinterpret_cast<const uint8_t*>(ts + 8192 + 2 * HALF) + dA;
        const uint8_t* sbp = reinterpret_cast<const uint8_t*>(ts + 8192 + 2 * HALF + 1024) + dB;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          ta[i] = rd_op(ts, tm * 32 + 16 * i, lane);
          tsa[i] = sa[tm * 32 + 16 * i + (lane & 15)];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = 64 * wn + 16 * j;
          tb[j] = rd_op(ts + 8192 + (c >> 7) * HALF, c & 127, lane);
          tsb[j] = sbp[c >> 7];
        }
        G8F_WAIT_LGKM0();
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            tacc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(tb[j], ta[i], tacc[i][j], 0, 0, 0, tsb[j], 0, tsa[i]);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(tacc[i][j]));
        __builtin_amdgcn_s_barrier();
      }
      bf16* Cb = reinterpret_cast<bf16*>(C);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const long gm = m0 + tm * 32 + 16 * i + (lane & 15);
          const int gn = n0 + 64 * wn + 16 * j + 4 * (lane >> 4);
          if (gm < mend && gn < N && SPA_DBG_OK(gn + 3, N)) {
            bf16* cp = Cb + gm * N + gn;
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
  constexpr bool S2 = !WG;
  const bool late = __builtin_amdgcn_readfirstlane(wave) >= 4;
  if (ktiles > 0) {
    stage(0, 0); stage(0, 2); stage(0, 3); stage(0, 1);
    if (ktiles > 1) {
      stage(1, 0); stage(1, 2);
      if (S2) { stage(1, 3); G8F_WAIT_VM(10); } else { G8F_WAIT_VM(8); }                    // A0, B0 (0)
    } else {
      G8F_WAIT_VM(4);
    }
    __builtin_amdgcn_s_barrier();
    if (late) __builtin_amdgcn_s_barrier();
  }
  for (int t = 0; t < ktiles; ++t) {
    const int s = t & 1;
    const bool n1 = t + 1 < ktiles, n2 = t + 2 < ktiles;
    // ---- phase 1: quadrant (0,0)
    read_a(half(s, 0));
    read_b(half(s, 2), b0f);
    read_scales(s);
    if (n1) { if (!S2) stage(t + 1, 3); G8F_WAIT_VM(8); } else { G8F_WAIT_VM(2); }   // retire B1(t)
    __builtin_amdgcn_s_barrier();
    G8F_WAIT_LGKM0();
    mfma_q(0, 0, b0f);
    __builtin_amdgcn_s_barrier();
    // ---- phase 2: quadrant (0,1)
    read_b(half(s, 3), b1f);
    if (n1) { stage(t + 1, 1); G8F_WAIT_VM(8); } else { G8F_WAIT_VM(0); }      // retire A1(t)
    __builtin_amdgcn_s_barrier();
    G8F_WAIT_LGKM0();
    mfma_q(0, 1, b1f);
    __builtin_amdgcn_s_barrier();
    // ---- phase 3: quadrant (1,1)
    read_a(half(s, 1));
    if (n2) stage(t + 2, 0);
    __builtin_amdgcn_s_barrier();
    G8F_WAIT_LGKM0();
    mfma_q(1, 1, b1f);
    __builtin_amdgcn_s_barrier();
    // ---- phase 4: quadrant (1,0) -- no LDS reads
    if (n2) {                                                                  // retire A0, B0(t+1)
      stage(t + 2, 2);
      if (S2) { stage(t + 2, 3); G8F_WAIT_VM(10); } else { G8F_WAIT_VM(8); }
    } else if (n1) {
      if (S2) { G8F_WAIT_VM(4); } else { G8F_WAIT_VM(0); }
    }
    __builtin_amdgcn_s_barrier();
    mfma_q(1, 0, b0f);
    __builtin_amdgcn_s_barrier();
  }
  if (ktiles > 0 && !late) __builtin_amdgcn_s_barrier();   // equal barrier counts on exit

  if constexpr (WG) {
    if (out_f32) {
      // fp32 [E, M, N] straight from the fragments (16 rows x 64 contiguous bytes per store)
      float* Cf = reinterpret_cast<float*>(C) + (long)e * M * N;
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
              if (gm < M && gn < N && SPA_DBG_OK(gn + 3, N)) {
                f32x4 v = acc[mh * 4 + i][nh * 2 + j];
                f32x4* cp = reinterpret_cast<f32x4*>(Cf + gm * N + gn);
                if (accumulate) v += *cp;
                *cp = v;
              }
            }
      return;
    }
  }
  // ---- bf16 epilogue through LDS, one 128-row half at a time (gemm8.hip): C^T fragments ->
  // padded row image -> whole-row 16-byte global stores
  bf16* Cb = reinterpret_cast<bf16*>(C) + (WG ? (long)e * M * N : 0L);
  const long mlim = WG ? (long)M : mend;
  constexpr int RS = 256 * 2 + 16;
  __syncthreads();
#pragma unroll
  for (int mh = 0; mh < 2; ++mh) {
    // accumulate: the half's 8 old chunks of this thread are requested before its image is built
    // (the store loop's loads could not move above the stores before them -- the row stride is not a
    // constant -- so each chunk paid a memory round trip; gemm4a.hip g4_epilogue, r6_gemm4_acc_epilogue)
    bf16x8 old[8];
    if (accumulate) {
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const int idx = tid + c * NT, r = idx >> 5, ch = idx & 31;
        const long gm = m0 + mh * 128 + r;
        const int gn = n0 + ch * 8;
        bf16x8 o;
#pragma unroll
        for (int q = 0; q < 8; ++q) o[q] = (bf16)0.f;
        if (gm < mlim && gn < N) o = *reinterpret_cast<const bf16x8*>(Cb + gm * N + gn);
        old[c] = o;
      }
    }
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
      if (gm < mlim && gn < N && SPA_DBG_OK(gn + 7, N)) {
        bf16x8 v = *reinterpret_cast<const bf16x8*>(smem + r * RS + ch * 16);
        bf16* cp = Cb + gm * N + gn;
        if (accumulate) {
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] = (bf16)((float)v[q] + (float)old[c][q]);
        }
        *reinterpret_cast<bf16x8*>(cp) = v;
      }
    }
    __syncthreads();
  }
}

// byte matrix [R, C] (row stride ld_in) -> [C, ldo] with ldo >= R (padding left as is): the
// k-tile-major scale images of the kernel above; 64 x 64 tiles through LDS
__global__ __launch_bounds__(256) void scale_t_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                      long R, int Cc, long ld_in, long ldo, long batch_in,
                                                      long batch_out) {
  __shared__ uint8_t tile[64][65];
  const long r0 = (long)blockIdx.x * 64;
  const int c0 = blockIdx.y * 64;
  in += blockIdx.z * batch_in;
  out += blockIdx.z * batch_out;
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int r = i >> 6, c = i & 63;
    tile[r][c] = (r0 + r < R && c0 + c < Cc) ? in[(r0 + r) * ld_in + c0 + c] : (uint8_t)0;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int c = i >> 6, r = i & 63;
    if (c0 + c < Cc && r0 + r < ldo) out[(long)(c0 + c) * ldo + r0 + r] = tile[r][c];
  }
}

static at::Tensor scale_t(const at::Tensor& s, long R, int Cc, int batch) {
  // s viewed as [batch][R][Cc] -> [batch][Cc][ldo], ldo = R rounded up to 16 (+16 slack so a
  // 16-B DMA piece never needs the range check to stay inside the allocation)
  const long ldo = (R + 15) / 16 * 16;
  auto out = at::empty({(long)batch * Cc * ldo + 16}, s.options());
  if (R > 0 && Cc > 0)
    scale_t_kernel<<<dim3((unsigned)((ldo + 63) / 64), (unsigned)((Cc + 63) / 64), (unsigned)batch), 256, 0, stream()>>>(
        s.data_ptr<uint8_t>(), out.data_ptr<uint8_t>(), R, Cc, Cc, ldo, R * Cc, (long)Cc * ldo);
  SPA_LAUNCH_CHECK();
  return out;
}

// Same contract as grouped_gemm_fp8_blk (moe_fp8.hip): xq [M, K] e4m3 + sx [M, K/128] E8M0,
// wq [E, N, K] e4m3 + sw [E, N/128, K/128] -> y [M, N] bf16
at::Tensor gemm8_fp8_blk(const at::Tensor& xq, const at::Tensor& sx, const at::Tensor& wq, const at::Tensor& sw,
                         const at::Tensor& offsets) {
  TORCH_CHECK(xq.scalar_type() == at::kFloat8_e4m3fn && wq.scalar_type() == at::kFloat8_e4m3fn, "e4m3 operands");
  TORCH_CHECK(sx.scalar_type() == at::kByte && sw.scalar_type() == at::kByte, "E8M0 (uint8) scales");
  TORCH_CHECK(xq.is_contiguous() && wq.is_contiguous() && sx.is_contiguous() && sw.is_contiguous());
  TORCH_CHECK(offsets.scalar_type() == at::kInt);
  const int E = offsets.numel() - 1;
  TORCH_CHECK(E >= 1 && E <= 512 && wq.dim() == 3 && wq.size(0) == E, "gemm8_fp8_blk: 1..512 experts");
  const int M = xq.size(0), K = xq.size(1), N = wq.size(1);
  TORCH_CHECK(wq.size(2) == K && K % 128 == 0 && N % 8 == 0, "gemm8_fp8_blk: K % 128, N % 8");
  const int KB = K / 128, NB = (N + 127) / 128;
  TORCH_CHECK(sx.numel() == (long)M * KB && sw.numel() == (long)E * NB * KB, "gemm8_fp8_blk: scale shapes");
  TORCH_CHECK((long)(M + 256) * K < (1L << 32) && (long)(N + 256) * K < (1L << 32), "gemm8_fp8_blk: operands < 4 GiB");
  TORCH_CHECK((uintptr_t)xq.data_ptr() % 16 == 0 && (uintptr_t)wq.data_ptr() % 16 == 0, "gemm8_fp8_blk: 16-B aligned");
  DeviceGuard g(xq.device());
  auto out = at::empty({M, N}, xq.options().dtype(at::kBFloat16));
  if (M == 0) return out;
  auto sat = scale_t(sx, M, KB, 1);            // [KB][ldsa]
  auto sbt = scale_t(sw, NB, KB, E);           // [E][KB][ldsb]
  const long ldsa = (M + 15) / 16 * 16, ldsb = (NB + 15) / 16 * 16;
  const int grid = (cdiv(M, 256) + E) * cdiv(N, 256);
  const char* te = getenv("SPA_GG8_TAIL");      // as gemm8.hip: tail tiles for <= 64 trailing rows
  const int tailr = te ? std::max(0, std::min(64, atoi(te))) : 64;
  gemm8_fp8_kernel<false><<<grid, 512, 0, stream()>>>(
      (const uint8_t*)xq.data_ptr(), (const uint8_t*)wq.data_ptr(), sat.data_ptr<uint8_t>(), sbt.data_ptr<uint8_t>(),
      out.data_ptr(), offsets.data_ptr<int>(), E, M, N, K, K, K, (long)N * K, M, N, KB, ldsa, ldsb,
      sat.numel(), sbt.numel(), 0, 0, tailr);
  SPA_LAUNCH_CHECK();
  return out;
}

// Same contract as wgrad_fp8_blk (moe_fp8.hip): dW_e [M, N] (+)= aq[:, seg_e] bq[:, seg_e]^T for the
// quant_t_fp8_seg images aq [M, ld], bq [N, ld] (scales [rows, ld/128]); out [E, M, N] bf16 / fp32
at::Tensor wgrad8_fp8_blk(const at::Tensor& aq, const at::Tensor& sa, const at::Tensor& bq, const at::Tensor& sb,
                          const at::Tensor& poff, const c10::optional<at::Tensor>& out_, bool accumulate) {
  TORCH_CHECK(aq.scalar_type() == at::kFloat8_e4m3fn && bq.scalar_type() == at::kFloat8_e4m3fn, "e4m3 operands");
  TORCH_CHECK(sa.scalar_type() == at::kByte && sb.scalar_type() == at::kByte, "E8M0 (uint8) scales");
  TORCH_CHECK(aq.is_contiguous() && bq.is_contiguous() && sa.is_contiguous() && sb.is_contiguous());
  TORCH_CHECK(poff.scalar_type() == at::kInt, "wgrad8_fp8_blk: int32 padded offsets");
  const int E = poff.numel() - 1;
  const int M = aq.size(0), N = bq.size(0);
  const long ld = aq.size(1);
  TORCH_CHECK(bq.size(1) == ld && ld % 128 == 0 && N % 8 == 0, "wgrad8_fp8_blk: shapes");
  TORCH_CHECK(sa.size(0) == M && sb.size(0) == N && sa.size(1) == ld / 128 && sb.size(1) == ld / 128,
              "wgrad8_fp8_blk: scale shapes");
  TORCH_CHECK((long)(M + 256) * ld < (1L << 32) && (long)(N + 256) * ld < (1L << 32), "wgrad8_fp8_blk: operands < 4 GiB");
  TORCH_CHECK((uintptr_t)aq.data_ptr() % 16 == 0 && (uintptr_t)bq.data_ptr() % 16 == 0, "wgrad8_fp8_blk: 16-B aligned");
  DeviceGuard g(aq.device());
  auto out = out_ ? *out_ : at::empty({E, M, N}, aq.options().dtype(at::kBFloat16));
  TORCH_CHECK(out.is_contiguous() && out.numel() == (long)E * M * N &&
                  (out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat),
              "wgrad8_fp8_blk: out [E, M, N] bf16/fp32 contiguous");
  if (E == 0 || M == 0 || N == 0) return out;
  const int KB = (int)(ld / 128);
  auto sat = scale_t(sa, M, KB, 1);            // [KB][ldsa]
  auto sbt = scale_t(sb, N, KB, 1);            // [KB][ldsb]
  const long ldsa = (M + 15) / 16 * 16, ldsb = (N + 15) / 16 * 16;
  const int grid = E * cdiv(M, 256) * cdiv(N, 256);
  gemm8_fp8_kernel<true><<<grid, 512, 0, stream()>>>(
      (const uint8_t*)aq.data_ptr(), (const uint8_t*)bq.data_ptr(), sat.data_ptr<uint8_t>(), sbt.data_ptr<uint8_t>(),
      out.data_ptr(), poff.data_ptr<int>(), E, M, N, 0, ld, ld, 0, M, N, KB, ldsa, ldsb, sat.numel(), sbt.numel(),
      accumulate ? 1 : 0, out.scalar_type() == at::kFloat ? 1 : 0);
  SPA_LAUNCH_CHECK();
  return out;
}

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.def("gemm8_fp8_blk(Tensor xq, Tensor sx, Tensor wq, Tensor sw, Tensor offsets) -> Tensor");
  m.def("wgrad8_fp8_blk(Tensor aq, Tensor sa, Tensor bq, Tensor sb, Tensor poff, Tensor(a!)? out, bool accumulate) -> Tensor");
}
TORCH_LIBRARY_IMPL(spa, CUDA, m) {
  m.impl("gemm8_fp8_blk", &spa::gemm8_fp8_blk);
  m.impl("wgrad8_fp8_blk", &spa::wgrad8_fp8_blk);
}
