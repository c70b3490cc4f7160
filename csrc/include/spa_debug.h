// Device-side bounds guards for the debug build of the extension (SPA_DEBUG_BOUNDS=1).
//
// Build:  tools/build_variant.sh dbg -DSPA_DEBUG_BOUNDS=1        -> ab/_C_dbg.so
// Use:    SPA_EXT_SO=ab/_C_dbg.so SPA_DEBUG_SYNC=1 python ...     (ops/_ext.py)
//
// In the release build every macro below is empty (SPA_DBG_OK is the constant `true`), so the
// shipped kernels carry no extra instruction. In the debug build a guard that fails does NOT trap
// (a trap is a GPU fault, and a faulting kernel can take the whole machine down on this pool): it
// records the first violation of its translation unit -- file, line, block, thread, the offending
// index and its limit -- in a per-TU __device__ record with one vector atomic, prints it once with
// device printf, and the guarded store is skipped (SPA_DBG_OK returns false). The host reads and
// clears the records with torch.ops.spa.debug_bounds_report(); ops/_ext.py calls it after every
// op when SPA_DEBUG_SYNC=1 and raises naming the op, so a bad tile coordinate is localised to
// (op, file:line, block, thread, index) from one run, without rocgdb.
//
// Guard kinds:
//   SPA_DBG_CHECK(i, n)        record if i is outside [0, n)
//   SPA_DBG_ASSERT(c, a, b)    record if the condition c is false (a, b: values to report)
//   SPA_DBG_OK(i, n)           SPA_DBG_CHECK + returns whether i is inside: `if (SPA_DBG_OK(o, n)) *p = v;`
//   SPA_DBG_LDS(off, n)        LDS element offset inside the kernel's n-element __shared__ image
// Each .hip file that uses them names itself once at namespace scope: SPA_DEBUG_TU("attention.hip").
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#ifndef SPA_DEBUG_BOUNDS
#define SPA_DEBUG_BOUNDS 0
#endif

namespace spa {
namespace dbg {

struct Record {
  unsigned hits;   // violations seen since the last report
  int line;
  int bx, by, bz, tid;
  int kind;        // 0 index, 1 assert, 2 LDS
  long long idx, lim;
};

// host registry of the per-TU records (csrc/kernels/debug.hip)
typedef void (*ReadFn)(Record* out, bool reset);
int register_tu(const char* file, ReadFn fn);
bool enabled();

}  // namespace dbg
}  // namespace spa

#if SPA_DEBUG_BOUNDS

namespace spa {
namespace dbg {
// internal linkage: one record per translation unit (no relocatable device code needed)
static __device__ Record g_rec;

__device__ __noinline__ static void fail(int line, int kind, long long idx, long long lim) {
  if (atomicAdd(&g_rec.hits, 1u) == 0u) {
    g_rec.line = line;
    g_rec.kind = kind;
    g_rec.bx = blockIdx.x;
    g_rec.by = blockIdx.y;
    g_rec.bz = blockIdx.z;
    g_rec.tid = threadIdx.x;
    g_rec.idx = idx;
    g_rec.lim = lim;
    printf("SPA_DEBUG_BOUNDS line %d kind %d block (%d,%d,%d) thread %d: %lld vs limit %lld\n", line, kind,
           (int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z, (int)threadIdx.x, idx, lim);
  }
}
__device__ __forceinline__ static bool ok(long long i, long long n, int line, int kind) {
  if (i >= 0 && i < n) return true;
  fail(line, kind, i, n);
  return false;
}
}  // namespace dbg
}  // namespace spa

#define SPA_DBG_CHECK(i, n) ((void)::spa::dbg::ok((long long)(i), (long long)(n), __LINE__, 0))
#define SPA_DBG_OK(i, n) (::spa::dbg::ok((long long)(i), (long long)(n), __LINE__, 0))
#define SPA_DBG_LDS(off, n) ((void)::spa::dbg::ok((long long)(off), (long long)(n), __LINE__, 2))
#define SPA_DBG_ASSERT(c, a, b) \
  ((c) ? (void)0 : ::spa::dbg::fail(__LINE__, 1, (long long)(a), (long long)(b)))
#define SPA_DEBUG_TU(name)                                                                    \
  namespace spa { namespace dbg { namespace {                                                 \
  void read_tu(Record* out, bool reset) {                                                     \
    (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rec), sizeof(Record), 0, hipMemcpyDeviceToHost); \
    if (reset && out->hits) {                                                                 \
      Record z{};                                                                             \
      (void)hipMemcpyToSymbol(HIP_SYMBOL(g_rec), &z, sizeof(Record), 0, hipMemcpyHostToDevice); \
    }                                                                                         \
  }                                                                                           \
  const int registered_tu = register_tu(name, &read_tu);                                      \
  } } }

#else

#define SPA_DBG_CHECK(i, n) ((void)0)
#define SPA_DBG_OK(i, n) (true)
#define SPA_DBG_LDS(off, n) ((void)0)
#define SPA_DBG_ASSERT(c, a, b) ((void)0)
#define SPA_DEBUG_TU(name)

#endif
