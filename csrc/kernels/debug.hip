// Host side of the device bounds guards (csrc/include/spa_debug.h): the registry of per-TU
// violation records and the two ops that expose it,
//   torch.ops.spa.debug_bounds_enabled() -> bool   (true only in a -DSPA_DEBUG_BOUNDS=1 build)
//   torch.ops.spa.debug_bounds_report(reset) -> str (one line per TU with a violation, "" if clean)
#include "spa_common.h"
#include "spa_debug.h"

#include <mutex>
#include <sstream>
#include <string>
#include <vector>

namespace spa {
namespace dbg {

namespace {
struct Entry {
  const char* file;
  ReadFn fn;
};
std::vector<Entry>& registry() {
  static std::vector<Entry> r;
  return r;
}
std::mutex& registry_mu() {
  static std::mutex m;
  return m;
}
}  // namespace

int register_tu(const char* file, ReadFn fn) {
  std::lock_guard<std::mutex> g(registry_mu());
  registry().push_back({file, fn});
  return (int)registry().size();
}

bool enabled() { return SPA_DEBUG_BOUNDS != 0; }

static const char* kind_name(int k) { return k == 1 ? "assert" : k == 2 ? "lds-offset" : "index"; }

std::string report(bool reset) {
  std::lock_guard<std::mutex> g(registry_mu());
  std::ostringstream os;
  for (const Entry& e : registry()) {
    Record r{};
    e.fn(&r, reset);
    if (r.hits == 0) continue;
    os << e.file << ":" << r.line << " " << kind_name(r.kind) << " " << r.idx << " outside [0, " << r.lim
       << ") block (" << r.bx << "," << r.by << "," << r.bz << ") thread " << r.tid << " (" << r.hits
       << " violations)\n";
  }
  return os.str();
}

}  // namespace dbg

static bool debug_bounds_enabled() { return dbg::enabled(); }
static std::string debug_bounds_report(bool reset) {
  if (!dbg::enabled()) return std::string();
  (void)hipDeviceSynchronize();
  return dbg::report(reset);
}

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.def("debug_bounds_enabled() -> bool", &spa::debug_bounds_enabled);
  m.def("debug_bounds_report(bool reset=True) -> str", &spa::debug_bounds_report);
}
