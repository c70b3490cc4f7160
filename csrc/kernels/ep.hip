// Expert-parallel row regroup (parallel/expert_parallel.py).
//
// After the dispatch all-to-all, a rank holds the rows sent to its El local experts in
// (source rank, local expert) order -- the order the P senders packed them. The grouped
// expert GEMM wants them (local expert, source rank)-major, and the combine all-to-all
// wants the inverse. Round 1 built that permutation on the host (a Python double loop of
// torch.arange slices, 2*P*El host ops per MoE layer per step, plus two index_select
// copies). Here ONE launch does both: every block rebuilds the two exclusive prefix sums
// of the received-count matrix rc [P, El] in LDS (P*El <= 1024 counts, a 256-thread
// block scan), each wave takes one row, finds its (src, expert) segment by binary search
// in LDS, and copies the row with 16-byte vector loads/stores. Rows are opaque bytes
// (bf16 activations, fp8 payloads, fp32 scales all go through the same kernel).
//
// to_em = 1: y[expert-major position of j] = x[j]   (dispatch side)
// to_em = 0: y[j] = x[expert-major position of j]   (combine side; also the backward)
#include "spa_common.h"

SPA_DEBUG_TU("ep.hip")

namespace spa {

constexpr int kRegroupMaxSeg = 1024;

// exclusive scan of v over the block (256 threads, each owning up to 4 consecutive items)
__device__ __forceinline__ void block_excl_scan4(const int* in, int* out, int n, int* wsum) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  int v[4], s = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int i = 4 * t + k;
    v[k] = i < n ? in[i] : 0;
    s += v[k];
  }
  // inclusive wave scan of the per-thread sums
  int inc = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  int base = 0;
  for (int k = 0; k < w; ++k) base += wsum[k];
  int run = base + inc - s;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int i = 4 * t + k;
    if (i < n) out[i] = run;
    run += v[k];
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void ep_regroup_kernel(const char* __restrict__ x, char* __restrict__ y, long R,
                                                         int row_bytes, const int64_t* __restrict__ rc, int P, int El,
                                                         int to_em) {
  __shared__ int cnt_sm[kRegroupMaxSeg], cnt_em[kRegroupMaxSeg];
  __shared__ int sm[kRegroupMaxSeg], em_k[kRegroupMaxSeg];
  __shared__ int wsum[8];
  const int nseg = P * El;
  for (int i = threadIdx.x; i < nseg; i += 256) {
    const int c = (int)rc[i];               // i = s*El + e  (src-major)
    const int s = i / El, e = i % El;
    cnt_sm[i] = c;
    cnt_em[e * P + s] = c;                  // expert-major index
  }
  __syncthreads();
  block_excl_scan4(cnt_sm, sm, nseg, wsum);
  block_excl_scan4(cnt_em, em_k, nseg, wsum + 4);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long j = (long)blockIdx.x * 4 + wave;
  if (j >= R) return;
  // last segment whose src-major start <= j (empty segments share their successor's start;
  // upper_bound picks the last of equal starts, which is the non-empty one)
  int lo = 0, hi = nseg;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (sm[mid] <= j) lo = mid + 1; else hi = mid;
  }
  const int seg = lo - 1;
  const int s = seg / El, e = seg % El;
  const long dest = (long)em_k[e * P + s] + (j - sm[seg]);
  const long src_row = to_em ? j : dest, dst_row = to_em ? dest : j;
  // debug build: the counts sum to R, so every row lands in a segment and every destination exists
  if (!(SPA_DBG_OK(seg, nseg) & SPA_DBG_OK(dest, R))) return;
  const char* src = x + src_row * (long)row_bytes;
  char* dst = y + dst_row * (long)row_bytes;
  for (int o = lane * 16; o < row_bytes; o += 64 * 16)
    *reinterpret_cast<int4*>(dst + o) = *reinterpret_cast<const int4*>(src + o);
}

at::Tensor ep_regroup(const at::Tensor& x, const at::Tensor& rc, int64_t P, int64_t El, bool to_em) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous(), "ep_regroup: x must be a contiguous HIP tensor");
  TORCH_CHECK(rc.is_cuda() && rc.scalar_type() == at::kLong && rc.numel() == P * El, "ep_regroup: rc [P*El] int64");
  TORCH_CHECK(P * El <= kRegroupMaxSeg, "ep_regroup: at most 1024 (rank, expert) segments");
  const long R = x.size(0);
  const long row_bytes = R ? x.numel() / R * x.element_size() : 0;
  TORCH_CHECK(row_bytes % 16 == 0 && ((uintptr_t)x.data_ptr() % 16) == 0, "ep_regroup: rows must be 16-byte multiples");
  auto y = at::empty_like(x);
  if (R == 0) return y;
  DeviceGuard g(x.device());
  const int grid = cdiv(R, 4);
  ep_regroup_kernel<<<grid, 256, 0, stream()>>>((const char*)x.data_ptr(), (char*)y.data_ptr(), R, (int)row_bytes,
                                                rc.data_ptr<int64_t>(), (int)P, (int)El, to_em ? 1 : 0);
  SPA_LAUNCH_CHECK();
  return y;
}

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.def("ep_regroup(Tensor x, Tensor rc, int P, int El, bool to_em) -> Tensor");
}
TORCH_LIBRARY_IMPL(spa, CUDA, m) { m.impl("ep_regroup", &spa::ep_regroup); }
