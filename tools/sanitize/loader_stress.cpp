// Host-side sanitizer stress test of the native token loader (csrc/runtime/token_loader.cpp).
//
// Built twice by tests/test_sanitizers_cpu.py -- with -fsanitize=address,undefined and with
// -fsanitize=thread -- and run on the CPU: producer threads filling the ring while the
// consumer seeks backwards and forwards, destruction with workers parked on a full ring,
// tensor and mmap'ed file sources, both window orders. Every batch is checked against the
// stateless batch_at() and against the id stream (ids are their own positions, so y = x + 1).
// GPU code is not sanitized (not available on this pool); this covers the host runtime.
#include "../../csrc/runtime/token_loader.cpp"

#include <cstdio>
#include <cstdlib>

static int check(spa::TokenLoader& L, int steps, int seek_every) {
  for (int i = 0; i < steps; ++i) {
    if (seek_every && i % seek_every == seek_every - 1) L.seek((i * 7) % 50);
    const int64_t pos = L.position();
    at::Tensor b = L.next();
    at::Tensor ref = L.batch_at(pos);
    if (!at::equal(b, ref)) {
      std::fprintf(stderr, "batch %ld differs from batch_at\n", (long)pos);
      return 1;
    }
    if (!at::equal(b[1], b[0] + 1)) {
      std::fprintf(stderr, "batch %ld: targets are not the next tokens\n", (long)pos);
      return 1;
    }
  }
  return 0;
}

int main() {
  const int64_t n = 200000;
  at::Tensor ids = at::arange(0, n, at::TensorOptions().dtype(at::kInt));
  for (int rep = 0; rep < 4; ++rep) {
    spa::TokenLoader L("", 4, ids, /*B=*/8, /*T=*/64, /*seed=*/rep, /*rank=*/rep % 2, /*world=*/2,
                       /*threads=*/4, /*depth=*/6, /*pin=*/false, /*sequential=*/rep % 2 == 1);
    if (check(L, 300, rep == 0 ? 0 : 23)) return 1;
  }
  {  // destroyed while every worker is parked on a full ring
    spa::TokenLoader L("", 4, ids, 4, 32, 7, 0, 1, 3, 2, false, false);
    (void)L.next();
  }
  // mmap'ed uint16 file source
  const char* path = "/tmp/spa_loader_stress.bin";
  {
    FILE* f = std::fopen(path, "wb");
    if (!f) return 2;
    for (int64_t i = 0; i < 60000; ++i) {
      const uint16_t v = (uint16_t)i;
      std::fwrite(&v, 2, 1, f);
    }
    std::fclose(f);
  }
  {
    spa::TokenLoader L(path, 2, at::Tensor(), 4, 128, 3, 0, 1, 2, 4, false, true);
    if (check(L, 200, 17)) return 1;
  }
  std::remove(path);
  std::puts("loader stress ok");
  return 0;
}
