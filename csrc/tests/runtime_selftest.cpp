// Host-only self-test of the native runtime (tokenizer, paged-KV block allocator, Go JSON
// string encoder), built with -fsanitize=address,undefined by tests/test_runtime_native.py
// (sanitizers on the host code; no GPU involved). Multi-threaded allocator
// churn exercises the mutex paths. Exit code 0 = all checks passed.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../runtime/block_allocator.h"
#include "../runtime/gojson.h"
#include "../runtime/tokenizer.h"

static int failures = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                       \
    }                                                                   \
  } while (0)

static void test_tokenizer() {
  for (int64_t V : {1024, 32000, 128256}) {
    llmc::SyntheticTokenizer t(V);
    std::mt19937 rng(static_cast<unsigned>(V));
    for (int it = 0; it < 200; ++it) {
      // random UTF-8-ish text incl. multi-byte sequences and raw bytes
      std::string s;
      const int n = rng() % 300;
      for (int i = 0; i < n; ++i) {
        const unsigned r = rng() % 10;
        if (r < 6) s.push_back(static_cast<char>('a' + rng() % 26));
        else if (r < 7) s.push_back(' ');
        else if (r < 8) s += "\xc3\xa9";       // é
        else if (r < 9) s += "\xe2\x82\xac";   // €
        else s.push_back(static_cast<char>(rng() % 256));
      }
      const std::vector<int32_t> ids = t.encode(s);
      for (int32_t id : ids) CHECK(id >= 0 && id < V - 2);
      CHECK(t.decode(ids.data(), static_cast<int64_t>(ids.size())) == s);
    }
    for (int32_t id = 0; id < V; id += 97) (void)t.piece(id);
  }
}

static void test_allocator() {
  llmc::BlockAllocator a(4096, 64);
  CHECK(a.num_free() == 4096);
  CHECK(a.blocks_for(0) == 0 && a.blocks_for(1) == 1 && a.blocks_for(64) == 1 && a.blocks_for(65) == 2);
  std::vector<std::thread> th;
  for (int w = 0; w < 8; ++w) {
    th.emplace_back([&a, w]() {
      std::mt19937 rng(static_cast<unsigned>(w));
      std::vector<std::vector<int32_t>> held;
      for (int it = 0; it < 2000; ++it) {
        if (held.empty() || rng() % 2) {
          auto b = a.allocate(1 + rng() % 16);
          if (!b.empty()) held.push_back(std::move(b));
        } else {
          const size_t k = rng() % held.size();
          if (rng() % 4 == 0) {
            a.incref(held[k]);
            a.free(held[k]);
          }
          a.free(held[k]);
          held.erase(held.begin() + static_cast<long>(k));
        }
      }
      for (auto& b : held) a.free(b);
    });
  }
  for (auto& t : th) t.join();
  CHECK(a.num_free() == 4096);
  CHECK(a.allocate(5000).empty());
}

static void test_gojson() {
  CHECK(llmc::go_json_string("a\"b\\c") == "\"a\\\"b\\\\c\"");
  CHECK(llmc::go_json_string("<&>") == "\"\\u003c\\u0026\\u003e\"");
  CHECK(llmc::go_json_string(std::string("\x01", 1)) == "\"\\u0001\"");
  CHECK(llmc::go_json_string("\xff") == "\"\\ufffd\"");
  CHECK(llmc::go_json_string("\xe2\x80\xa8") == "\"\\u2028\"");
  std::mt19937 rng(7);
  for (int it = 0; it < 2000; ++it) {
    std::string s;
    const int n = rng() % 64;
    for (int i = 0; i < n; ++i) s.push_back(static_cast<char>(rng() % 256));
    const std::string j = llmc::go_json_string(s);
    CHECK(j.size() >= 2 && j.front() == '"' && j.back() == '"');
  }
}

int main() {
  test_tokenizer();
  test_allocator();
  test_gojson();
  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("runtime selftest ok\n");
  return 0;
}
