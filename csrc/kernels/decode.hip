// Split-K decode attention for KV-cached generation on gfx950.
//
// The reference re-runs the whole prefix for every generated token (gpt/gpt-jax.ipynb:821-829,
// llama3/LLaMA-jax.ipynb:499-511, gemma/gemma.ipynb:608-630, deepseekv3/deepseekv3.ipynb:
// 1849-1873); the framework keeps a KV cache, so each step is a few query rows against a
// long cache: memory-bound, and with B * Hkv far below the CU count a per-head kernel would
// leave most of the chip idle. This kernel splits the KEY axis instead:
//
//   grid = (B * Hkv, nsplit); block = 4 waves. A block takes the R = G * Tq query rows that
//   share kv-head hk (G = H / Hkv: GQA / MQA rows are processed together, so every K/V byte
//   is read once per block) against keys [s * chunk, (s + 1) * chunk).
//   Lanes: hd / 4 lanes per key (4 bf16 of the head dim each: one 8-byte load per lane per
//   key row, 64 / (hd/4) keys per wave step). Each lane group keeps its own online-softmax
//   state (m, l, o[4]) per row; groups are merged with v_permlane32_swap / LDS at the end.
//   The split's (m, l, o) go to fp32 partials; attn_decode_combine_kernel merges the splits
//   and writes bf16 out + lse (an in-launch merge by the last-arriving split block is kept
//   behind SPA_DECODE_FUSED=1: its cross-XCD release/acquire fences measured slower).
// Causal: query row t sits at position Tk - Tq + t (the cache holds the prefix plus the new
// tokens); keys beyond a row's position are masked.
#include "spa_common.h"

#include <map>
#include <mutex>

namespace spa {

struct DecodeParams {
  const bf16* q; const bf16* k; const bf16* v;
  float* opart; float* mpart; float* lpart;  // [nsplit][B][Tq][H][hd], [nsplit][B][Tq][H]
  bf16* out; float* lse;
  const int* kv_len;  // optional device-side cache length (HIP-graph replay); else Tk
  int* arrivals;      // [B * Hkv] split-arrival counters (zero between launches)
  int B, Tq, Tk, H, Hkv, nsplit, chunk;
  long sqb, sqt, sqh, skb, skt, skh, svb, svt, svh, sob, sot, soh;
  float scale_log2;
  bool causal;
};

constexpr int kMaxRows = 16;
constexpr int kKeysPerLoad = 8;
// keys one 4-wave block covers per load batch: 4 waves x (64 / (hd / 4)) lane groups x 8
constexpr int keys_per_batch(int hd) { return 4 * (256 / hd) * kKeysPerLoad; }

template <int HD, int R, bool FUSED>
__global__ __launch_bounds__(256) void attn_decode_kernel(DecodeParams p) {
  constexpr int KL = HD / 4;        // lanes per key
  constexpr int KPW = 64 / KL;      // keys per wave step
  constexpr int NG = 4 * KPW;       // lane groups per block
  constexpr int KPL = kKeysPerLoad; // keys per lane group per load batch
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int sub = lane % KL, grp = wave * KPW + lane / KL;
  const int bh = blockIdx.x, split = blockIdx.y;
  const int hk = bh % p.Hkv, b = bh / p.Hkv;
  const int G = p.H / p.Hkv;
  const int rows = G * p.Tq;
  const int Tk = p.kv_len ? min(*p.kv_len, p.Tk) : p.Tk;
  const int k0 = split * p.chunk, k1 = min(Tk, k0 + p.chunk);

  // query slices (pre-scaled to log2 units), rows r = t * G + g  (head hk*G + g, token t)
  float qv[R][4];
  int qpos[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int t = r / G, g = r % G;
    qpos[r] = p.causal ? Tk - p.Tq + t : Tk;
    if (r < rows) {
      const bf16* qp = p.q + b * p.sqb + (long)t * p.sqt + (long)(hk * G + g) * p.sqh + 4 * sub;
      const bf16x4 x = *reinterpret_cast<const bf16x4*>(qp);
#pragma unroll
      for (int j = 0; j < 4; ++j) qv[r][j] = (float)x[j] * p.scale_log2;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) qv[r][j] = 0.f;
      qpos[r] = -1;  // never visible
    }
  }
  float m[R], l[R], o[R][4];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    m[r] = -INFINITY; l[r] = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[r][j] = 0.f;
  }
  const bf16* kb = p.k + b * p.skb + hk * p.skh + 4 * sub;
  const bf16* vb = p.v + b * p.svb + hk * p.svh + 4 * sub;
  // Batches of KPL keys per lane group: every K/V load of a batch is issued before any is
  // consumed (one HBM round trip per batch, 2 * KPL loads in flight per lane), and the batch
  // shares one online-softmax rescale per row. Keys past the split end are clamped on load
  // and masked in the softmax. (One key per round trip measured 24.6 us per layer at a
  // 1K-token cache: pure latency.)
  for (int base = k0; base < k1; base += NG * KPL) {
    bf16x4 kx[KPL], vx[KPL];
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
      const long kk = min(base + j * NG + grp, k1 - 1);
      kx[j] = *reinterpret_cast<const bf16x4*>(kb + kk * p.skt);
      vx[j] = *reinterpret_cast<const bf16x4*>(vb + kk * p.svt);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float s[KPL];
      float mx = m[r];
#pragma unroll
      for (int j = 0; j < KPL; ++j) {
        float d = qv[r][0] * (float)kx[j][0];
#pragma unroll
        for (int e = 1; e < 4; ++e) d = fmaf(qv[r][e], (float)kx[j][e], d);
#pragma unroll
        for (int w = KL / 2; w > 0; w >>= 1) d += __shfl_xor(d, w, KL);
        const int key = base + j * NG + grp;
        s[j] = (key >= k1 || key > qpos[r]) ? -INFINITY : d;
        mx = fmaxf(mx, s[j]);
      }
      if (mx == -INFINITY) continue;  // nothing visible yet for this row
      const float alpha = __builtin_amdgcn_exp2f(m[r] - mx);  // m = -inf -> 0
      l[r] *= alpha;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[r][e] *= alpha;
#pragma unroll
      for (int j = 0; j < KPL; ++j) {
        const float pj = __builtin_amdgcn_exp2f(s[j] - mx);
        l[r] += pj;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[r][e] = fmaf(pj, (float)vx[j][e], o[r][e]);
      }
      m[r] = mx;
    }
  }
  // merge the NG lane groups: in-wave groups through shuffles, then waves through LDS
  __shared__ float sm[4][R], sl[4][R], so[4][R][HD];
#pragma unroll
  for (int r = 0; r < R; ++r) {
#pragma unroll
    for (int w = KL; w < 64; w <<= 1) {
      const float m2 = __shfl_xor(m[r], w, 64), l2 = __shfl_xor(l[r], w, 64);
      const float mn = fmaxf(m[r], m2);
      const float a1 = mn == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m[r] - mn);
      const float a2 = mn == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m2 - mn);
      l[r] = l[r] * a1 + l2 * a2;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[r][j] = o[r][j] * a1 + __shfl_xor(o[r][j], w, 64) * a2;
      m[r] = mn;
    }
    if (lane < KL) {
#pragma unroll
      for (int j = 0; j < 4; ++j) so[wave][r][4 * sub + j] = o[r][j];
      if (sub == 0) { sm[wave][r] = m[r]; sl[wave][r] = l[r]; }
    }
  }
  __syncthreads();
  // rows x hd outputs of this split: thread -> (row, 4-element slice)
  for (int i = tid; i < rows * KL; i += 256) {
    const int r = i / KL, s4 = i % KL;
    float mn = -INFINITY;
#pragma unroll
    for (int w = 0; w < 4; ++w) mn = fmaxf(mn, sm[w][r]);
    float lt = 0.f, ot[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float a = mn == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(sm[w][r] - mn);
      lt += sl[w][r] * a;
#pragma unroll
      for (int j = 0; j < 4; ++j) ot[j] += so[w][r][4 * s4 + j] * a;
    }
    const int t = r / G, hq = hk * G + r % G;
    const long row = (((long)split * p.B + b) * p.Tq + t) * p.H + hq;
    f32x4 w4;
#pragma unroll
    for (int j = 0; j < 4; ++j) w4[j] = ot[j];
    *reinterpret_cast<f32x4*>(p.opart + row * HD + 4 * s4) = w4;
    if (s4 == 0) { p.mpart[row] = mn; p.lpart[row] = lt; }
  }
  if constexpr (!FUSED) return;  // attn_decode_combine_kernel merges the splits
  // Split-K fix-up in the same launch: the last of the nsplit blocks of this (b, kv head) to
  // arrive merges every split's partials (saves the separate combine launch, which measured
  // 10.4 us per layer at a 1K cache -- a latency chain over the splits with 4 blocks in flight).
  // Release (L2 write-back only) by every wave after its partial stores, before the arrival
  // counter moves; acquire (L2 invalidate only) in the last block before it reads partials
  // written through other XCDs' L2s. Measured (LLaMA3-8B graph decode, B=1, same box):
  // 252 tok/s fused vs 278 with the separate combine launch -- the L2 write-back / invalidate
  // cost more than the launch it saves; hence off by default.
  __shared__ int last;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __syncthreads();
  if (tid == 0) {
    const int old = atomicAdd(p.arrivals + bh, 1);
    last = old == p.nsplit - 1;
    if (last) p.arrivals[bh] = 0;  // every split has arrived: re-arm for the next launch
  }
  __syncthreads();
  if (!last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const long nrows = (long)p.B * p.Tq * p.H;
  for (int i = tid; i < rows * KL; i += 256) {
    const int r = i / KL, s4 = i % KL;
    const int t = r / G, hq = hk * G + r % G;
    const long row = ((long)b * p.Tq + t) * p.H + hq;
    float mn = -INFINITY;
    for (int s = 0; s < p.nsplit; ++s) mn = fmaxf(mn, __builtin_nontemporal_load(p.mpart + s * nrows + row));
    float lt = 0.f, ot[4] = {0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < p.nsplit; ++s) {
      const float ms = __builtin_nontemporal_load(p.mpart + s * nrows + row);
      const float a = ms == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(ms - mn);
      lt += __builtin_nontemporal_load(p.lpart + s * nrows + row) * a;
      const f32x4 x = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p.opart + (s * nrows + row) * HD + 4 * s4));
#pragma unroll
      for (int j = 0; j < 4; ++j) ot[j] += x[j] * a;
    }
    const float inv = lt > 0.f ? 1.f / lt : 0.f;
    bf16x4 w;
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = (bf16)(ot[j] * inv);
    *reinterpret_cast<bf16x4*>(p.out + b * p.sob + t * p.sot + hq * p.soh + 4 * s4) = w;
    if (s4 == 0)
      p.lse[((long)b * p.H + hq) * p.Tq + t] = lt > 0.f ? (mn + __log2f(lt)) * 0.69314718055994531f : INFINITY;
  }
}

// Split merge, one block per (b, t, h) row: the block max of the split maxima first, then each
// of the 4 waves folds every 4th split (hd spread over the lanes, 4 splits' loads in flight),
// and the waves are summed through LDS. The latency chain is ~nsplit / 16 round trips; the
// first version (one thread per 4 outputs, all splits in sequence) measured 10.4 us per layer
// at 17 splits.
template <int HD>
__global__ __launch_bounds__(256) void attn_decode_combine_kernel(DecodeParams p) {
  constexpr int E = HD / 64;  // outputs per lane
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long nrows = (long)p.B * p.Tq * p.H;
  const long row = blockIdx.x;
  __shared__ float red[4];
  __shared__ float sacc[4][HD + 1];
  float mx = -INFINITY;
  for (int s = tid; s < p.nsplit; s += 256) mx = fmaxf(mx, p.mpart[s * nrows + row]);
  mx = block_max<256>(mx, red);
  float lt = 0.f, acc[E];
#pragma unroll
  for (int e = 0; e < E; ++e) acc[e] = 0.f;
  if (mx != -INFINITY) {
#pragma unroll 4
    for (int s = wave; s < p.nsplit; s += 4) {
      const float ms = p.mpart[s * nrows + row];
      const float a = ms == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(ms - mx);
      lt += p.lpart[s * nrows + row] * a;
      const float* src = p.opart + (s * nrows + row) * HD + lane * E;
      if constexpr (E == 1) {
        acc[0] += src[0] * a;
      } else if constexpr (E == 2) {
        const f32x2 x = *reinterpret_cast<const f32x2*>(src);
        acc[0] += x[0] * a; acc[1] += x[1] * a;
      } else {
        const f32x4 x = *reinterpret_cast<const f32x4*>(src);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] += x[e] * a;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) sacc[wave][lane * E + e] = acc[e];
  if (lane == 0) sacc[wave][HD] = lt;
  __syncthreads();
  if (wave != 0) return;
  const float L = sacc[0][HD] + sacc[1][HD] + sacc[2][HD] + sacc[3][HD];
  const float inv = L > 0.f ? 1.f / L : 0.f;
  const long h = row % p.H, t = (row / p.H) % p.Tq, b = row / ((long)p.H * p.Tq);
  bf16* dst = p.out + b * p.sob + t * p.sot + h * p.soh + lane * E;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int d = lane * E + e;
    dst[e] = (bf16)((sacc[0][d] + sacc[1][d] + sacc[2][d] + sacc[3][d]) * inv);
  }
  if (lane == 0) p.lse[(b * p.H + h) * p.Tq + t] = L > 0.f ? (mx + __log2f(L)) * 0.69314718055994531f : INFINITY;
}

// Split-arrival counters, one set per (device, stream): zeroed once, left at zero by every
// launch (the last block of each kv group re-arms its counter), so no per-call memset and a
// captured hipGraph can replay the kernel as is. Launches on one stream are serialised, so
// they never share a counter concurrently.
static int* arrival_counters(const at::Tensor& like, hipStream_t st, int n) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, at::Tensor> bufs;
  std::lock_guard<std::mutex> lock(mu);
  auto& t = bufs[{like.get_device(), st}];
  if (!t.defined() || t.numel() < n)
    t = at::zeros({std::max(n, 4096)}, like.options().dtype(at::kInt));
  return t.data_ptr<int>();
}

// q [B, Tq, H, hd] (Tq * H / Hkv <= 16), k/v [B, Tk, Hkv, hd] strided (cache views); with
// kv_len (device int32) k/v are the full cache buffers and only rows [0, *kv_len) count, so a
// decode step can be captured once in a hipGraph and replayed at every position.
// Returns (out [B, Tq, H, hd] bf16, lse [B, H, Tq] fp32).
std::vector<at::Tensor> attn_decode(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, double scale,
                                    bool causal, int64_t nsplit_req, const c10::optional<at::Tensor>& kv_len) {
  for (auto* t : {&q, &k, &v}) {
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->dim() == 4, "attn_decode: bf16 [B,T,H,hd]");
    TORCH_CHECK(t->stride(3) == 1 && t->stride(2) % 4 == 0 && t->stride(1) % 4 == 0 && t->stride(0) % 4 == 0 &&
                    ((uintptr_t)t->data_ptr() % 8) == 0,
                "attn_decode: rows must be 8-byte aligned and contiguous in hd");
  }
  const int B = q.size(0), Tq = q.size(1), H = q.size(2), HD = q.size(3);
  const int Tk = k.size(1), Hkv = k.size(2);
  TORCH_CHECK(k.size(0) == B && v.size(0) == B && v.size(1) == Tk && v.size(2) == Hkv && k.size(3) == HD &&
              v.size(3) == HD && H % Hkv == 0, "attn_decode: shape mismatch");
  TORCH_CHECK(Tq <= Tk, "attn_decode: the cache must hold the query tokens");
  const int rows = Tq * (H / Hkv);
  TORCH_CHECK(rows <= kMaxRows, "attn_decode: Tq * H / Hkv must be <= 16 (use flash attention for prefill)");
  DeviceGuard g(q.device());
  auto out = at::empty({B, Tq, H, HD}, q.options());
  auto lse = at::empty({B, H, Tq}, q.options().dtype(at::kFloat));
  if (B * Tq * H == 0) return {out, lse};
  // split the keys so the grid covers the chip ~2x, each split a whole number of load
  // batches (hd 128: 64 keys = 8 lane groups x 8 keys in flight)
  const int kpb = keys_per_batch(HD);
  int nsplit = (int)nsplit_req;
  int chunk;
  if (nsplit <= 0) {
    const int want = std::max(1, 512 / std::max(1, B * Hkv));
    nsplit = std::max(1, std::min(want, cdiv(Tk, kpb)));
    chunk = cdiv(cdiv(Tk, nsplit), kpb) * kpb;
  } else {
    chunk = cdiv(Tk, nsplit);
  }
  nsplit = cdiv(Tk, chunk);
  auto part = at::empty({(long)nsplit * B * Tq * H * (HD + 2)}, q.options().dtype(at::kFloat));
  DecodeParams p{};
  p.q = (const bf16*)q.data_ptr(); p.k = (const bf16*)k.data_ptr(); p.v = (const bf16*)v.data_ptr();
  p.opart = part.data_ptr<float>();
  p.mpart = p.opart + (long)nsplit * B * Tq * H * HD;
  p.lpart = p.mpart + (long)nsplit * B * Tq * H;
  p.out = (bf16*)out.data_ptr(); p.lse = lse.data_ptr<float>();
  p.B = B; p.Tq = Tq; p.Tk = Tk; p.H = H; p.Hkv = Hkv; p.nsplit = nsplit; p.chunk = chunk;
  p.sqb = q.stride(0); p.sqt = q.stride(1); p.sqh = q.stride(2);
  p.skb = k.stride(0); p.skt = k.stride(1); p.skh = k.stride(2);
  p.svb = v.stride(0); p.svt = v.stride(1); p.svh = v.stride(2);
  p.sob = out.stride(0); p.sot = out.stride(1); p.soh = out.stride(2);
  p.scale_log2 = (float)(scale * 1.4426950408889634);
  p.causal = causal;
  if (kv_len.has_value()) {  // k/v are the whole cache; the valid length lives on the device
    TORCH_CHECK(kv_len->is_cuda() && kv_len->scalar_type() == at::kInt && kv_len->numel() >= 1,
                "attn_decode: kv_len must be a device int32 tensor");
    p.kv_len = kv_len->data_ptr<int>();
  }
  auto st = stream();
  const char* env = getenv("SPA_DECODE_FUSED");
  const bool fused = env ? atoi(env) != 0 : false;  // in-launch merge measured slower (see kernel)
  if (fused) p.arrivals = arrival_counters(q, st, B * Hkv);
  const dim3 grid(B * Hkv, nsplit);
  const int nrows = B * Tq * H;
#define SPA_DECODE_ROWS(HDV, F)                                                                    \
  {                                                                                                \
    if (rows <= 4) attn_decode_kernel<HDV, 4, F><<<grid, 256, 0, st>>>(p);                         \
    else if (rows <= 8) attn_decode_kernel<HDV, 8, F><<<grid, 256, 0, st>>>(p);                    \
    else attn_decode_kernel<HDV, 16, F><<<grid, 256, 0, st>>>(p);                                  \
  }
#define SPA_DECODE_LAUNCH(HDV)                                                                      \
  {                                                                                                \
    if (fused) SPA_DECODE_ROWS(HDV, true)                                                          \
    else {                                                                                         \
      SPA_DECODE_ROWS(HDV, false)                                                                  \
      attn_decode_combine_kernel<HDV><<<nrows, 256, 0, st>>>(p);                \
    }                                                                                              \
  }
  if (HD == 64) SPA_DECODE_LAUNCH(64)
  else if (HD == 128) SPA_DECODE_LAUNCH(128)
  else if (HD == 256) SPA_DECODE_LAUNCH(256)
  else TORCH_CHECK(false, "attn_decode: head dim must be 64, 128 or 256");
#undef SPA_DECODE_LAUNCH
#undef SPA_DECODE_ROWS
  SPA_LAUNCH_CHECK();
  return {out, lse};
}

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.def("attn_decode(Tensor q, Tensor k, Tensor v, float scale, bool causal, int nsplit, Tensor? kv_len=None) -> Tensor[]");
}
TORCH_LIBRARY_IMPL(spa, CUDA, m) { m.impl("attn_decode", &spa::attn_decode); }
