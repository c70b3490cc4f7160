// Device helpers shared by the flash-attention kernels (attention.hip) and the wide-head
// kernels (attention_wide.hip): MFMA 32x32x16 bf16 wrappers, the accumulator -> operand
// packing, the swizzled LDS images with row (ds_read_b128) and transposed
// (ds_read_b64_tr_b16) reads, and the register-staged tile loader.
#pragma once
#include "spa_common.h"
#include <type_traits>

namespace spa {

// LDS image row width for a head dim: 192-wide rows are staged in 256-wide image rows
template <int HD> constexpr int img_w() { return HD == 192 ? 256 : HD; }

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

// deferred-rescale threshold in log2 units (T13): P = 2^(s*c - m) <= 2^8
constexpr float kRescaleThr = 8.f;

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }
// max of x over lanes l and l^32 (one v_permlane32_swap, no LDS)
__device__ __forceinline__ float halfmax(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float halfsum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z[i] = (bf16)0.f;
  return z;
}
__device__ __forceinline__ f32x16 splat16(float v) {
  f32x16 a;
#pragma unroll
  for (int r = 0; r < 16; ++r) a[r] = v;
  return a;
}
// accumulator registers 8s..8s+7 -> bf16 operand fragment (permuted k order)
__device__ __forceinline__ bf16x8 pack_acc(const f32x16& a, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (bf16)a[8 * s + j];
  return r;
}

// ---- swizzled row-major [rows][HD] bf16 LDS images -------------------------
template <int HD>
__device__ __forceinline__ int swz(int r) {
  if constexpr (HD >= 128) return ((r & 3) << 2) | ((r >> 2) & 3);
  else return (((r >> 1) & 1) << 2) | ((r >> 2) & 3);
}
template <int HD>
__device__ __forceinline__ int img_off(int r, int ch) {  // element offset of 16B chunk ch of row r
  return r * HD + 8 * (ch ^ swz<HD>(r));
}
// A/B operand "X^T" for one 16-deep k-step, where X is the row-major image with
// rows = k index, columns = output index. Lane l gets X[r0 + 16s + perm(j)][c0 + (l&31)].
template <int HD>
__device__ __forceinline__ bf16x8 rd_tr(const bf16* img, int rbase, int c0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3, hh = lane >> 5;
  const int c = c0 + 16 * (g & 1) + 4 * pp;  // column (element) this lane addresses
  const int ch = c >> 3, within = c & 7;
  const int ra = rbase + 4 * hh + q, rb = ra + 8;
  typedef __attribute__((address_space(3))) s16x4 lds_s4;
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s4*)(img + ra * HD + 8 * (ch ^ swz<HD>(ra)) + within));
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_s4*)(img + rb * HD + 8 * (ch ^ swz<HD>(rb)) + within));
  // whole-vector bit casts: element-wise short->bf16 inserts miscompile (duplicated dwords)
  const bf16x4 av = __builtin_bit_cast(bf16x4, a), bv = __builtin_bit_cast(bf16x4, b);
  return __builtin_shufflevector(av, bv, 0, 1, 2, 3, 4, 5, 6, 7);
}

// Per-lane LDS element offsets, computed once per kernel (the swizzle term is
// invariant under the +32-row / +16-row steps of the loops, which become
// immediate offsets): row reads (row = lane&31, chunk = 2ks + half) and the
// two halves of each transposed read (k-step rows 0..15, d-tile dt).
// The swizzle XORs the low 4 bits of the 16-B chunk index, so at HD = 256 the offsets of chunks
// 16..31 are those of chunks 0..15 plus 128 elements: only the first 8 row / 4 transposed
// offsets are kept in registers, the rest are immediates (16 fewer VGPRs per image at HD 256).
template <int N>
struct LdsOffs {            // operator[k] = v[k % N] + (k / N) * 128 elements (k a constant)
  int v[N];
  __device__ __forceinline__ int operator[](int k) const { return v[k % N] + (k / N) * 128; }
};
template <int HD>
struct LdsOff {
  static constexpr int NR = HD / 16 > 8 ? 8 : HD / 16, NTR = HD / 32 > 4 ? 4 : HD / 32;
  LdsOffs<NR> row;
  LdsOffs<NTR> tra, trb;
  __device__ __forceinline__ void init(int lane) {
    static_assert(HD <= 256, "LdsOff: the +128 offset rule holds up to 32 chunks per row");
    const int l32 = lane & 31, hh = lane >> 5, g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
#pragma unroll
    for (int ks = 0; ks < NR; ++ks) row.v[ks] = l32 * HD + 8 * ((2 * ks + hh) ^ swz<HD>(l32));
    const int ra = 4 * hh + q, rb = ra + 8;
#pragma unroll
    for (int dt = 0; dt < NTR; ++dt) {
      const int c = 32 * dt + 16 * (g & 1) + 4 * pp;
      const int ch = c >> 3, within = c & 7;
      tra.v[dt] = ra * HD + 8 * (ch ^ swz<HD>(ra)) + within;
      trb.v[dt] = rb * HD + 8 * (ch ^ swz<HD>(rb)) + within;
    }
    SPA_DBG_LDS(row.v[NR - 1] + 7, 32 * HD);
    SPA_DBG_LDS(trb.v[NTR - 1] + 3, 16 * HD);
  }
};
__device__ __forceinline__ bf16x8 ld_row(const bf16* img, int off) {
  return *reinterpret_cast<const bf16x8*>(img + off);
}
__device__ __forceinline__ bf16x8 ld_tr(const bf16* img, int offa, int offb) {
  typedef __attribute__((address_space(3))) s16x4 lds_s4;
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + offa));
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + offb));
  const bf16x4 av = __builtin_bit_cast(bf16x4, a), bv = __builtin_bit_cast(bf16x4, b);
  return __builtin_shufflevector(av, bv, 0, 1, 2, 3, 4, 5, 6, 7);
}
template <int V> using IC = std::integral_constant<int, V>;

// Instruction order for an MFMA chain whose operands come from LDS (sched_group_barrier masks:
// 0x100 DS read, 0x008 MFMA): PRE + AHEAD * PER reads first, then (1 MFMA, PER reads) for the
// next N - AHEAD MFMAs, then the last AHEAD MFMAs -- each MFMA's operand was requested AHEAD
// MFMAs earlier, so the counted lgkmcnt waits overlap LDS latency with the chain instead of the
// default schedule's read -> lgkmcnt(0) -> MFMA serialisation. Place right after the chain.
template <int N, int PER, int AHEAD, int PRE = 0>
__device__ __forceinline__ void chain_sched() {
  __builtin_amdgcn_sched_group_barrier(0x100, PRE + AHEAD * PER, 0);
#pragma unroll
  for (int i = 0; i < N - AHEAD; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, PER, 0);
  }
  __builtin_amdgcn_sched_group_barrier(0x008, AHEAD, 0);
}

// 32-bit LDS address of a pointer into __shared__ memory (a generic pointer to LDS carries the
// LDS offset in its low 32 bits), made provably wave-uniform for an "s" asm operand
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)p);
}
// 16 B per lane of a buffer straight into LDS (lane i -> lds + 16 i) as inline asm: hipcc neither
// counts it (the caller's own s_waitcnt vmcnt(N) retires it) nor makes later ds_reads wait vmcnt(0)
// for it. M0 carries the LDS base and is restored.
// NT: non-temporal (streamed once; keeps the L2 for data that is re-read, e.g. a shared K tile)
template <bool NT = false>
__device__ __forceinline__ void dma16_asm(__amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned lds) {
  unsigned keep;
  if constexpr (NT)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen nt lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(rs), "s"(lds) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(rs), "s"(lds) : "memory");
}

// Register-staged tile loader: ROWS x HDC bf16 tile of a strided tensor -> regs -> LDS image
// with IW-element rows (IW = img_w<HDC>, >= HDC).
// Global side: one buffer descriptor per tile (scalar work), its range ending at the
// tensor's last valid row, so rows >= nrows load as zeros without a branch. The per-lane
// byte offsets and LDS offsets are loop invariant (computed once).
// Thread -> chunk map: W = min(IW/8, 16) lanes share a row, a lane takes the chunk
// columns ch, ch+16, ... of its row (IW = 256: two; chunks >= HDC/8 of a 192-wide row are
// never loaded) and rows rr, rr+R, ... (R = NT/W, a multiple of 16). The XOR swizzle only
// touches the low 4 chunk bits and repeats every 16 rows, so all of a lane's LDS offsets are
// one register + immediates; on the global side each row pass gets its own scalar descriptor
// and the column step is the instruction offset.
template <int HDC, int ROWS, int NT>
struct TileLoader {
  static constexpr int IW = img_w<HDC>();
  static constexpr int CPR = IW / 8;                   // 16B chunks per image row
  static constexpr int W = CPR < 16 ? CPR : 16;        // lanes per row
  static constexpr int NC = CPR / W;                   // column chunks per lane (16 apart)
  static constexpr int R = NT / W;                     // rows between a lane's row passes
  static constexpr int NP = ROWS / R;                  // row passes
  static constexpr int CH = NP * NC;
  static_assert(R % 16 == 0 && ROWS % R == 0 && NP >= 1, "tile/threads mismatch");
  bf16x8 r[CH];
  int voff;  // byte offset of this lane's first chunk within its row pass
  int loff;  // element offset of this lane's first chunk in the LDS image
  int ch;    // this lane's first chunk column
  __device__ __forceinline__ void init(long stride, int tid) {
    const int rr = tid / W;
    ch = tid % W;
    voff = (int)(((long)rr * stride + ch * 8) * 2);
    loff = img_off<IW>(rr, ch);
  }
  __device__ __forceinline__ bool valid(int j) const { return HDC == IW || ch + 16 * j < HDC / 8; }
  __device__ __forceinline__ void load(const bf16* base, long stride, int row0, int nrows) {
#pragma unroll
    for (int ps = 0; ps < NP; ++ps) {
      const int r0 = row0 + ps * R;
      const int left = nrows - r0;
      const int bytes = left > 0 ? (int)(((long)(left - 1) * stride + HDC) * 2) : 0;
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc((void*)(base + (long)r0 * stride), 0, bytes, 0x00020000);
#pragma unroll
      for (int j = 0; j < NC; ++j)
        if (valid(j))
          r[ps * NC + j] =
              __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, voff + 256 * j, 0, 0));
    }
  }
  __device__ __forceinline__ void store(bf16* img) const {
    // debug build: this lane's last 16-B chunk ends inside the ROWS x IW image
    SPA_DBG_LDS(loff + (NP - 1) * R * IW + 128 * (NC - 1) + 7, ROWS * IW);
#pragma unroll
    for (int ps = 0; ps < NP; ++ps)
#pragma unroll
      for (int j = 0; j < NC; ++j)
        if (valid(j)) *reinterpret_cast<bf16x8*>(img + loff + ps * R * IW + 128 * j) = r[ps * NC + j];
  }
};


}  // namespace spa
