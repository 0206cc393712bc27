// Host-side stress test of the paged-KV BlockAllocator, built with AddressSanitizer +
// UndefinedBehaviorSanitizer by tests/test_native_sanitizers.py (sanitizers
// on host code).  Random allocate / commit / release sequences with shared prompt prefixes;
// checks the refcount and free-count invariants after every operation.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <stdexcept>
#include <vector>

#include "runtime/block_allocator.h"

using k8sllm::BlockAllocator;

#define CHECK(c)                                                            \
  do {                                                                      \
    if (!(c)) {                                                             \
      std::fprintf(stderr, "CHECK failed: %s (line %d)\n", #c, __LINE__); \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

int main() {
  const int nb = 257, bs = 16;
  BlockAllocator a(nb, bs, true);
  std::mt19937 rng(12345);
  std::vector<int32_t> system(40 * bs);
  for (size_t i = 0; i < system.size(); ++i) system[i] = (int32_t)(i * 7 + 3);
  struct Seq { std::vector<int32_t> blocks, toks; };
  std::vector<Seq> live;
  long ops = 0, fails = 0;
  for (int it = 0; it < 20000; ++it) {
    const int op = rng() % 3;
    if (op < 2) {
      Seq s;
      const int shared = (int)(rng() % system.size());
      s.toks.assign(system.begin(), system.begin() + shared);
      const int extra = 1 + (int)(rng() % 300);
      for (int i = 0; i < extra; ++i) s.toks.push_back((int32_t)(rng() % 128000));
      const int total = (int)s.toks.size() + (int)(rng() % 64);
      const bool can = a.can_allocate(s.toks, total);
      try {
        auto al = a.allocate(s.toks, total);
        CHECK(can);
        CHECK((int)al.blocks.size() == (total + bs - 1) / bs);
        // full shared blocks, then at most block_size - 1 copied positions; the last prompt token is never cached
        CHECK((al.cached_tokens - al.copy_tokens) % bs == 0 && al.cached_tokens < (int)s.toks.size());
        CHECK(al.copy_tokens >= 0 && al.copy_tokens < bs);
        CHECK(al.copy_tokens == 0 || (al.copy_src >= 0 && al.copy_src < nb));
        for (int b : al.blocks) CHECK(al.copy_tokens == 0 || b != al.copy_src);
        for (int b : al.blocks) CHECK(b >= 0 && b < nb && a.refcount(b) >= 1);
        s.blocks = al.blocks;
        a.commit_prefix(s.blocks, s.toks, (int)s.toks.size());
        live.push_back(std::move(s));
      } catch (const std::runtime_error&) {
        CHECK(!can);
        ++fails;
      }
    } else if (!live.empty()) {
      const size_t i = rng() % live.size();
      a.release(live[i].blocks);
      live.erase(live.begin() + (long)i);
    }
    int held = 0;
    std::vector<int> seen(nb, 0);
    for (const auto& s : live)
      for (int b : s.blocks) ++seen[b];
    for (int b = 0; b < nb; ++b) {
      CHECK(a.refcount(b) == seen[b]);
      held += seen[b] > 0;
    }
    CHECK(a.num_free() == nb - held);
    ++ops;
  }
  for (const auto& s : live) a.release(s.blocks);
  CHECK(a.num_free() == nb);
  a.reset_prefix_cache();
  CHECK(a.num_cached() == 0 && a.num_free() == nb);
  std::printf("ok ops=%ld alloc_failures=%ld hits=%llu queries=%llu\n", ops, fails,
              (unsigned long long)a.hits(), (unsigned long long)a.queries());
  return 0;
}
