// The host-only C++ of libdeltareplay under the sanitizers (tests/test_host_sanitizers.py; SURVEY.md
// §5: "TSAN/ASAN builds of the host library"): the LogSegment listing (log_segment.cpp), the Parquet
// footer / page-header planner and the small-column host decoder (parquet_meta.cpp), the host JSON DOM
// (json_host.cpp) and the host SNAPPY decoder (snappy_host.cpp) -- everything the library runs on the
// CPU between the C ABI and the device.
//
//   host_sanitize <tables dir> <threads> <snappy samples dir>
//
// Every table under <tables dir> (a directory holding _delta_log) is listed, every checkpoint footer
// parsed, every column chunk's pages walked and decoded on the host, every commit line parsed; then
// every input is mutated (truncations, byte flips, random bytes) and fed again, where only the
// library's own errors (dr::Error) may come back. With <threads> > 1 the same work runs on that many
// threads at once, each with its own data (the C ABI's contract: distinct contexts are independent),
// which is what the ThreadSanitizer build checks. Prints "ok <items>" and exits 0.
#include <dirent.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../delta_amd/csrc/common.h"
#include "../../delta_amd/csrc/json_host.h"
#include "../../delta_amd/csrc/log_segment.h"
#include "../../delta_amd/csrc/parquet_meta.h"
#include "../../delta_amd/csrc/snappy_host.h"

using namespace dr;

static std::vector<std::string> list_dir(const std::string& d) {
  std::vector<std::string> out;
  if (DIR* dir = opendir(d.c_str())) {
    while (dirent* e = readdir(dir))
      if (e->d_name[0] != '.') out.push_back(e->d_name);
    closedir(dir);
  }
  return out;
}

static std::atomic<uint64_t> g_items{0};

// Footer + pages + host decode of one checkpoint image; dr::Error is the only allowed failure.
static void checkpoint_image(const std::vector<uint8_t>& f) {
  try {
    pq::FileMeta m = pq::parse_footer(f.data(), f.size());
    for (const pq::RowGroup& rg : m.row_groups) {
      int64_t row_base = 0;
      for (const pq::ColumnChunk& cc : rg.cols) {
        const pq::Leaf* leaf = m.leaf(cc.path);
        if (!leaf) continue;
        try {
          (void)pq::walk_pages(f.data(), f.size(), cc);
          pq::HostColumn hc = pq::decode_column_host(f.data(), f.size(), cc, *leaf);
          (void)pq::sparse_entries(f.data(), f.size(), cc, *leaf, 1, row_base);
          g_items += hc.def.size() + 1;
        } catch (const Error&) {
        }
      }
      row_base += rg.num_rows;
    }
  } catch (const Error&) {
  }
}

static void json_text(const std::string& text) {
  size_t at = 0;
  while (at < text.size()) {
    size_t nl = text.find('\n', at);
    if (nl == std::string::npos) nl = text.size();
    JVal v;
    std::string err;
    if (json_parse(text.data() + at, nl - at, &v, &err)) {
      const std::string back = json_dump(v);
      JVal v2;
      if (!json_parse(back.data(), back.size(), &v2)) {
        std::fprintf(stderr, "json_dump output does not parse: %s\n", back.c_str());
        std::abort();
      }
      if (const JVal* add = v.get("add"))
        if (const JVal* sz = add->get("size"))
          if (sz->is_int()) (void)sz->as_int();
    }
    ++g_items;
    at = nl + 1;
  }
}

static void snappy_image(const std::vector<uint8_t>& in) {
  uint64_t n = 0;
  if (!snappy_uncompressed_length(in.data(), in.size(), &n) || n > (64u << 20)) return;
  std::vector<uint8_t> out(n + 1);
  (void)snappy_decompress(in.data(), in.size(), out.data(), n);
  ++g_items;
}

// Truncations, byte flips and random overwrites of `src`, each handed to `fn`.
template <class F>
static void mutations(const std::vector<uint8_t>& src, std::mt19937_64& rng, int rounds, F fn) {
  if (src.empty()) return;
  for (int r = 0; r < rounds; ++r) {
    std::vector<uint8_t> m = src;
    switch (r % 4) {
      case 0: m.resize(rng() % m.size()); break;
      case 1: for (int k = 0; k < 8; ++k) m[rng() % m.size()] ^= uint8_t(1u << (rng() % 8)); break;
      case 2: {
        const size_t at = rng() % m.size(), len = std::min<size_t>(m.size() - at, 1 + rng() % 64);
        for (size_t k = 0; k < len; ++k) m[at + k] = uint8_t(rng());
        break;
      }
      default: m.erase(m.begin() + long(rng() % m.size())); break;
    }
    fn(m);
  }
}

static void work(const std::string& tables, const std::string& samples, uint64_t seed) {
  std::mt19937_64 rng(seed);
  for (const std::string& t : list_dir(tables)) {
    const std::string log = tables + "/" + t + "/_delta_log";
    try {
      LogSegmentInfo seg = get_log_segment(log, -1);
      for (const SegFile& c : seg.checkpoint) {
        const std::vector<uint8_t> f = read_file(log + "/" + c.name);
        checkpoint_image(f);
        mutations(f, rng, 24, [](const std::vector<uint8_t>& m) { checkpoint_image(m); });
      }
      for (const SegFile& d : seg.deltas) {
        const std::vector<uint8_t> f = read_file(log + "/" + d.name);
        json_text(std::string(f.begin(), f.end()));
        mutations(f, rng, 24, [](const std::vector<uint8_t>& m) { json_text(std::string(m.begin(), m.end())); });
      }
      for (int64_t v = 0; v <= seg.version; ++v) (void)get_log_segment(log, v);
      ++g_items;
    } catch (const Error&) {
    }
  }
  for (const std::string& s : list_dir(samples)) {
    const std::vector<uint8_t> f = read_file(samples + "/" + s);
    snappy_image(f);
    mutations(f, rng, 48, [](const std::vector<uint8_t>& m) { snappy_image(m); });
  }
}

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: host_sanitize <tables dir> <threads> <snappy samples dir>\n");
    return 2;
  }
  const std::string tables = argv[1], samples = argv[3];
  const int threads = std::max(1, std::atoi(argv[2]));
  std::vector<std::thread> ts;
  for (int k = 0; k < threads; ++k) ts.emplace_back(work, tables, samples, uint64_t(0xDE17A + k));
  for (std::thread& th : ts) th.join();
  std::printf("ok %llu\n", (unsigned long long)g_items.load());
  return 0;
}
