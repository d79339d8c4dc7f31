// libdeltareplay: host orchestration of the device replay and the C ABI (include/deltareplay.h).
//
// One dr_ctx owns a HIP stream and a caching device allocator. dr_stage copies a LogSegment's
// bytes into HBM and plans the checkpoint page decode; dr_replay_staged runs K1 (JSON), K2
// (Parquet), canonicalisation, K3 (hash partition) and K4 (per-bucket last-writer-wins) on the
// device and keeps the reconstructed state resident until dr_state_release.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <dlfcn.h>
#include <sys/mman.h>
#include <unistd.h>
#include <sys/stat.h>
#include <fcntl.h>
#include <thread>

#include <algorithm>
#include <cmath>
#include <atomic>
#include <functional>
#include <type_traits>
#include <cstring>
#include <cctype>
#include <cerrno>
#include <cstdlib>
#include <cstdio>
#include <map>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "common.h"
#include "json_host.h"
#include "kernels.h"
#include "log_segment.h"
#include "parquet_meta.h"

// ---- stage ranges (SURVEY.md §5 tracing) --------------------------------------------------------------
// roctx ranges around the replay's stages -- parse.json, decode.checkpoint, canonicalize,
// hash.partition, reduce, compact, exchange, filter, export, checkpoint.write, apply -- under a
// top-level range per C-ABI operation, the counterpart of the reference's recordDeltaOperation around
// "delta.log.update" / "delta.checkpoint" (D/metering/DeltaLogging.scala:58-108). Off unless DR_ROCTX is
// set (rocprofv3 --marker-trace shows them); the library dlopens rocprofiler-sdk's roctx on first use,
// so it carries no link dependency. A replay enqueues all its kernels before one host round trip, so a
// range spans its stage's enqueues; DR_ROCTX=sync closes every range with a stream synchronize, which
// makes the ranges the stages' device time (and serialises K1 with K2).
namespace trace {
struct Api {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
};
static int mode() {
  static const int m = [] {
    const char* e = std::getenv("DR_ROCTX");
    return !e || !*e || std::strcmp(e, "0") == 0 ? 0 : std::strcmp(e, "sync") == 0 ? 2 : 1;
  }();
  return m;
}
static const Api& api() {
  static const Api a = [] {
    Api x;
    if (!mode()) return x;
    void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("libroctx64.so.4", RTLD_NOW | RTLD_LOCAL);
    if (!h) return x;
    x.push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
    x.pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
    if (!x.push || !x.pop) x = Api{};
    return x;
  }();
  return a;
}
}  // namespace trace
struct StageRange {
  hipStream_t s;
  bool on;
  explicit StageRange(const char* name, hipStream_t stream = nullptr) : s(stream), on(trace::mode() && trace::api().push) {
    if (on) trace::api().push(name);
  }
  ~StageRange() {
    if (!on) return;
    if (trace::mode() == 2 && s) (void)hipStreamSynchronize(s);
    trace::api().pop();
  }
  StageRange(const StageRange&) = delete;
  StageRange& operator=(const StageRange&) = delete;
};
// a range over the rest of the enclosing scope
#define DR_STAGE_CAT2(a, b) a##b
#define DR_STAGE_CAT(a, b) DR_STAGE_CAT2(a, b)
#define DR_STAGE(name, stream) StageRange DR_STAGE_CAT(dr_stage_range_, __LINE__)(name, stream)


using namespace dr;

#define HIP_OK_NOTHROW(x) (void)(x)  // (destructor paths: a failed call is left to the next checked one)
#define HIP_OK(x)                                                                                  \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) fail(DR_E_DEVICE, fmt("%s failed: %s", #x, hipGetErrorString(e_)));      \
  } while (0)

// ---------------------------------------------------------------------------------------------------
// context + caching allocator
// ---------------------------------------------------------------------------------------------------
struct dr_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;  // K1 line parsing, overlapped with the checkpoint decode
  std::string err;
  bool timing = false;
  std::string timing_only;  // non-empty: only this kernel gets an event pair (dr_set_timing_only)
  // Path-changing options, set per context through dr_ctx_set_option (include/deltareplay.h; the
  // reference's per-session DeltaSQLConf, D/sources/DeltaSQLConf.scala:29): no process-global state
  // picks a code path.
  struct Options {
    int64_t overlap = 0;       // DR_OPT_OVERLAP: K1 line parsing on stream2 beside the checkpoint decode
                               // (r06: step equal either way, 9.14-9.20 vs 9.17 ms; off keeps each
                               // kernel's events its own)
    int64_t split = 1;         // DR_OPT_SPLIT: k_bucket_split for large replays (0: K4 sub-passes)
    int64_t bucket_bits = -1;  // DR_OPT_BUCKET_BITS: cap on K3's bucket bits (-1: automatic)
    int64_t filter_eval = 0;   // DR_OPT_FILTER_EVAL: 0 dictionary codes, 1 typed leaves, 2 generic interpreter
    int64_t apply_full = 0;    // DR_OPT_APPLY_FULL: dr_state_apply always through K3/K4
    int64_t canon_hint = -1;   // DR_OPT_CANON_HINT: arena bytes standing in for the first replay's sizing
    int64_t json_staged = 0;   // DR_OPT_JSON_STAGED: every segment through the staged K1 kernel
    int64_t host_cache_bytes = int64_t(64) << 30;  // DR_OPT_HOST_CACHE_BYTES: pinned blocks kept for reuse
  } opt;
  // Every entry point that takes this context (or a state, range, shard or communicator of it) holds
  // this lock for the call: a context may be shared by host threads (several Spark tasks of one
  // executor exporting ranges of one state), and the calls then run one at a time.
  std::recursive_mutex api_mu;
  struct Mark {
    std::string name;
    hipEvent_t ev;
    int s;  // 0: stream, 1: stream2
  };
  std::vector<Mark> marks;
  struct KMark {  // one kernel launch, bracketed by an event pair on its stream
    std::string name;
    hipEvent_t a, b;
  };
  std::vector<KMark> kmarks;
  std::vector<std::pair<std::string, float>> timings;
  std::multimap<size_t, void*> free_blocks;
  std::unordered_map<void*, size_t> sizes;
  std::mutex mu;
  // pinned bounce slots of the staging readers (two per reader thread, created on the first large
  // staging and kept for the context's life): a chunk is read into a slot, copied to the pageable
  // host copy, and DMA'd to HBM from the slot; an event per slot guards its reuse
  static constexpr size_t kBounceBytes = size_t(8) << 20;
  std::vector<uint8_t*> bounce;
  std::vector<hipEvent_t> bounce_ev;
  void ensure_bounce(size_t slots) {
    while (bounce.size() < slots) {
      void* p = nullptr;
      if (hipHostMalloc(&p, kBounceBytes, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        fail(DR_E_OOM, "pinned staging slot");
      }
      hipEvent_t e;
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
        (void)hipHostFree(p);
        fail(DR_E_DEVICE, "staging event");
      }
      bounce.push_back(static_cast<uint8_t*>(p));
      bounce_ev.push_back(e);
    }
  }

  // pinned readback words: a replay queues every kernel first and then copies its counters, error
  // codes and the non-file line list here in one round trip (one stream sync per replay)
  static constexpr size_t kPinWords = 8192;
  uint64_t* hpin = nullptr;
  uint64_t* pinned() {
    if (!hpin) {
      void* p = nullptr;
      // coherent: a kernel's stores reach it without a copy engine (launch_readback, the flag)
      if (hipHostMalloc(&p, kPinWords * sizeof(uint64_t), hipHostMallocCoherent) != hipSuccess) {
        (void)hipGetLastError();
        fail(DR_E_OOM, "pinned readback words");
      }
      hpin = static_cast<uint64_t*>(p);
      // hipHostMalloc does not promise zeroed memory: the completion word must not already hold the
      // first sequence number a readback waits for
      std::memset(hpin, 0, kPinWords * sizeof(uint64_t));
      void* d = nullptr;
      HIP_OK(hipHostGetDevicePointer(&d, p, 0));
      hpin_dev = static_cast<uint64_t*>(d);
    }
    return hpin;
  }
  uint64_t* hpin_dev = nullptr;  // the same words as a kernel writes them (launch_readback)
  uint64_t* pinned_dev() {
    (void)pinned();
    return hpin_dev;
  }
  // the readback completion word (the pinned block's last) and its sequence
  static constexpr size_t kPinFlag = kPinWords - 1;
  uint64_t pin_seq = 0;
  // Waits for a readback launched with {flag, seq}: a spin on the pinned word (a stream synchronize
  // sleeps and wakes ~10 us after the kernel ends), with a stream synchronize after 1 s of spinning
  // (and to surface any launch error).
  void wait_readback(uint64_t seq) {
    const volatile uint64_t* f = pinned() + kPinFlag;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t k = 0; *f != seq; ++k) {
      if ((k & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) {
        HIP_OK(hipStreamSynchronize(stream));
        if (*f != seq) fail(DR_E_INTERNAL, "readback completion word not written");
        break;
      }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
  }

  // DR_POISON=1 (tests): every block handed out is filled with 0xA5 first, so a kernel that reads
  // memory it never wrote sees the same garbage whatever the context ran before (a block reused
  // from free_blocks otherwise holds whatever its last owner left). The fill is ordered after all
  // queued work and before all later work: a released block may still be read by kernels queued on
  // the context's streams (stream order makes that safe for the next owner), and the null stream is
  // not ordered with the context's non-blocking streams.
  static bool poison() {
    static const bool on = std::getenv("DR_POISON") != nullptr;
    return on;
  }
  // (the whole block: a reused block can be up to 2n + 1 MiB, and a read past n must not see history)
  void* poisoned(void* p, size_t n) {
    if (poison() && p) {
      size_t blk = n;
      {
        std::lock_guard<std::mutex> g(mu);
        auto it = sizes.find(p);
        if (it != sizes.end()) blk = it->second;
      }
      HIP_OK(hipDeviceSynchronize());
      HIP_OK(hipMemset(p, 0xA5, blk));
      HIP_OK(hipDeviceSynchronize());
    }
    return p;
  }
  void* alloc(size_t n) {
    n = (n + 255) & ~size_t(255);
    if (n == 0) n = 256;
    void* p = nullptr;
    {
      std::lock_guard<std::mutex> g(mu);
      auto it = free_blocks.lower_bound(n);
      if (it != free_blocks.end() && it->first <= 2 * n + (1 << 20)) {
        p = it->second;
        free_blocks.erase(it);
      }
    }
    if (p) return poisoned(p, n);
    if (hipMalloc(&p, n) != hipSuccess) {
      (void)hipGetLastError();
      trim();
      if (hipMalloc(&p, n) != hipSuccess) {
        (void)hipGetLastError();
        fail(DR_E_OOM, fmt("device allocation of %zu bytes failed", n));
      }
    }
    {
      std::lock_guard<std::mutex> g(mu);
      sizes[p] = n;
    }
    return poisoned(p, n);
  }
  void release(void* p) {
    if (!p) return;
    if (poison()) {  // quarantined until the API call ends (check_quarantine)
      size_t n = 0;
      {
        std::lock_guard<std::mutex> g(mu);
        n = sizes[p];
      }
      HIP_OK_NOTHROW(hipDeviceSynchronize());
      HIP_OK_NOTHROW(hipMemset(p, 0xA5, n));
      HIP_OK_NOTHROW(hipDeviceSynchronize());
      std::lock_guard<std::mutex> g(mu);
      quarantine.push_back(p);
      return;
    }
    std::lock_guard<std::mutex> g(mu);
    free_blocks.emplace(sizes[p], p);
  }
  // DR_POISON: blocks released during an API call, filled with 0xA5 at release. When the call ends
  // (guard) every one must still hold only 0xA5 -- a write after release is a kernel queued after the
  // block was handed back, i.e. a buffer that did not live as long as the launch using it -- and then
  // joins the free list. (Blocks over 4 MiB: their first and last 64 KiB.)
  std::vector<void*> quarantine;
  std::string check_quarantine() {
    std::vector<void*> q;
    {
      std::lock_guard<std::mutex> g(mu);
      q.swap(quarantine);
    }
    if (q.empty()) return "";
    std::string bad;
    if (hipDeviceSynchronize() != hipSuccess) bad = "device error before the quarantine check";
    std::vector<uint8_t> h;
    for (void* p : q) {
      size_t n;
      {
        std::lock_guard<std::mutex> g(mu);
        n = sizes[p];
      }
      const size_t win = size_t(64) << 10;
      const std::pair<size_t, size_t> spans[2] = {{0, n <= (size_t(4) << 20) ? n : win},
                                                  {n <= (size_t(4) << 20) ? n : n - win, n}};
      for (const auto& sp : spans) {
        if (sp.second <= sp.first || !bad.empty()) continue;
        h.resize(sp.second - sp.first);
        if (hipMemcpy(h.data(), static_cast<uint8_t*>(p) + sp.first, h.size(), hipMemcpyDeviceToHost) != hipSuccess) {
          bad = "quarantine read failed";
          break;
        }
        for (size_t k = 0; k < h.size(); ++k)
          if (h[k] != 0xA5) {
            bad = fmt("device block of %zu bytes written after its release (byte %zu = 0x%02x)", n, sp.first + k, h[k]);
            break;
          }
      }
      std::lock_guard<std::mutex> g(mu);
      free_blocks.emplace(n, p);
    }
    return bad;
  }
  // pinned host blocks (hipHostMalloc) for the export columns, cached like the device blocks: a
  // released state's block serves the next export of a similar size without pinning pages again
  std::multimap<size_t, void*> host_free;
  std::unordered_map<void*, size_t> host_sizes;
  void* host_alloc(size_t n) {
    n = (n + 4095) & ~size_t(4095);
    if (n == 0) n = 4096;
    {
      std::lock_guard<std::mutex> g(mu);
      auto it = host_free.lower_bound(n);
      if (it != host_free.end() && it->first <= 2 * n + (size_t(16) << 20)) {
        void* p = it->second;
        host_free_bytes -= it->first;
        host_free.erase(it);
        return p;
      }
    }
    void* p = nullptr;
    if (hipHostMalloc(&p, n, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      host_trim();
      if (hipHostMalloc(&p, n, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        fail(DR_E_OOM, fmt("pinned host allocation of %zu bytes failed", n));
      }
    }
    std::lock_guard<std::mutex> g(mu);
    host_sizes[p] = n;
    return p;
  }
  // The cache of released blocks stays within opt.host_cache_bytes (a large single-part
  // checkpoint's block no longer stays pinned until the context ends): a released block evicts the
  // largest cached ones until it fits (the newest block is the likeliest to be asked for again: the
  // next range or part of the same size), and a block larger than the bound is unpinned at once.
  size_t host_free_bytes = 0;
  void host_release(void* p) {
    if (!p) return;
    std::vector<void*> drop;
    {
      std::lock_guard<std::mutex> g(mu);
      const size_t n = host_sizes[p];
      const size_t cap = size_t(std::max<int64_t>(opt.host_cache_bytes, 0));
      if (n > cap) {
        drop.push_back(p);
        host_sizes.erase(p);
      } else {
        while (host_free_bytes + n > cap && !host_free.empty()) {
          auto it = std::prev(host_free.end());
          host_free_bytes -= it->first;
          host_sizes.erase(it->second);
          drop.push_back(it->second);
          host_free.erase(it);
        }
        host_free.emplace(n, p);
        host_free_bytes += n;
      }
    }
    for (void* q : drop) (void)hipHostFree(q);
  }
  void host_trim() {
    std::lock_guard<std::mutex> g(mu);
    for (auto& kv : host_free) {
      (void)hipHostFree(kv.second);
      host_sizes.erase(kv.second);
    }
    host_free.clear();
    host_free_bytes = 0;
  }
  void trim() {
    std::lock_guard<std::mutex> g(mu);
    for (auto& kv : free_blocks) {
      (void)hipFree(kv.second);
      sizes.erase(kv.second);
    }
    free_blocks.clear();
  }
  // A stage's time is the interval since the previous mark on the same stream (a stream's first
  // mark only opens its timeline).
  // timing events are pooled: creating and destroying four per replay cost the bench's timed steps
  // more than the events themselves
  std::vector<hipEvent_t> ev_pool;
  hipEvent_t get_event() {
    if (!ev_pool.empty()) {
      hipEvent_t e = ev_pool.back();
      ev_pool.pop_back();
      return e;
    }
    hipEvent_t e;
    HIP_OK(hipEventCreate(&e));
    return e;
  }
  void put_event(hipEvent_t e) { ev_pool.push_back(e); }
  void mark(const char* name, int on = 0) {
    if (!timing || !timing_only.empty()) return;  // stage marks only in the per-kernel table mode
    hipEvent_t e = get_event();
    HIP_OK(hipEventRecord(e, on ? stream2 : stream));
    marks.push_back(Mark{name, e, on});
  }
  // The launch hook (kernels.h): an event pair carried by each selected launch of the call.
  static bool on_launch(void* user, const char* kernel, hipEvent_t* start, hipEvent_t* stop) {
    dr_ctx* c = static_cast<dr_ctx*>(user);
    KMark k{kernel_name(kernel), nullptr, nullptr};
    if (!(c->timing_only.empty() || k.name == c->timing_only)) return false;
    k.a = c->get_event();
    k.b = c->get_event();
    *start = k.a;
    *stop = k.b;
    c->kmarks.push_back(k);
    return true;
  }
  // "(dev::k_gather<uint64_t, uint32_t>)" -> "k_gather"
  static std::string kernel_name(const char* k) {
    std::string n(k);
    size_t a = n.rfind("::");
    if (a != std::string::npos) n = n.substr(a + 2);
    size_t b = n.find_first_of("<)");
    if (b != std::string::npos) n = n.substr(0, b);
    while (!n.empty() && n[0] == '(') n = n.substr(1);
    return n;
  }
  void begin_call() {
    if (timing) set_launch_hook(&dr_ctx::on_launch, this);
  }
  // Stage intervals, then one entry per kernel launch ("name", or "name#k" for its k-th launch
  // in the call, k >= 2).
  void collect_timings() {
    set_launch_hook(nullptr, nullptr);
    timings.clear();
    for (auto& m : marks) HIP_OK(hipEventSynchronize(m.ev));
    for (size_t i = 1; i < marks.size(); ++i) {
      size_t k = i;
      while (k > 0 && marks[k - 1].s != marks[i].s) --k;
      if (k == 0) continue;
      float ms = 0;
      HIP_OK(hipEventElapsedTime(&ms, marks[k - 1].ev, marks[i].ev));
      timings.emplace_back(marks[i].name, ms);
    }
    for (auto& m : marks) put_event(m.ev);
    marks.clear();
    std::map<std::string, int> seen;
    for (auto& k : kmarks) {
      HIP_OK(hipEventSynchronize(k.b));
      float ms = 0;
      HIP_OK(hipEventElapsedTime(&ms, k.a, k.b));
      const int n = ++seen[k.name];
      timings.emplace_back(n == 1 ? k.name : k.name + "#" + std::to_string(n), ms);
      put_event(k.a);
      put_event(k.b);
    }
    kmarks.clear();
    for (auto& kv : stats) timings.emplace_back(kv.first, float(kv.second));
    stats.clear();
  }
  // counters of the call that are reported with its timings (stat.* entries: counts, not ms)
  std::vector<std::pair<std::string, double>> stats;
  void drop_timings() {
    set_launch_hook(nullptr, nullptr);
    stats.clear();
    for (auto& m : marks) put_event(m.ev);
    marks.clear();
    for (auto& k : kmarks) {
      put_event(k.a);
      put_event(k.b);
    }
    kmarks.clear();
  }
};

// RAII device buffer from the context cache.
template <typename T>
struct DBuf {
  dr_ctx* ctx = nullptr;
  T* p = nullptr;
  size_t n = 0;
  DBuf() = default;
  DBuf(dr_ctx* c, size_t count) : ctx(c), n(count) { p = static_cast<T*>(c->alloc(std::max<size_t>(count, 1) * sizeof(T))); }
  DBuf(const DBuf&) = delete;
  DBuf& operator=(const DBuf&) = delete;
  DBuf(DBuf&& o) noexcept { *this = std::move(o); }
  DBuf& operator=(DBuf&& o) noexcept {
    reset();
    ctx = o.ctx; p = o.p; n = o.n; own = o.own;
    o.p = nullptr; o.n = 0;
    return *this;
  }
  ~DBuf() { reset(); }
  void reset() {
    if (p && ctx && own) ctx->release(p);
    p = nullptr;
    n = 0;
    own = true;
  }
  // a non-owning view of the first `count` elements of another buffer
  void view(const DBuf& o, size_t count) {
    reset();
    ctx = o.ctx; p = o.p; n = count; own = false;
  }
  bool own = true;
  void zero(hipStream_t s) { if (p) HIP_OK(hipMemsetAsync(p, 0, std::max<size_t>(n, 1) * sizeof(T), s)); }
};

template <typename T>
static T d2h_one(const T* p, hipStream_t s) {
  T v;
  HIP_OK(hipMemcpyAsync(&v, p, sizeof(T), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  return v;
}

template <typename T>
static std::vector<T> d2h(const T* p, size_t n, hipStream_t s) {
  std::vector<T> v(n);
  if (n) {
    HIP_OK(hipMemcpyAsync(v.data(), p, n * sizeof(T), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
  }
  return v;
}

// ---------------------------------------------------------------------------------------------------
// staged segment
// ---------------------------------------------------------------------------------------------------
struct JsonFileRec { int64_t version; uint64_t off, len; };

struct CkPart {
  uint64_t off = 0, len = 0;   // within the concatenated checkpoint bytes
  pq::FileMeta meta;
  uint64_t row_base = 0;
  int32_t rg_lo = 0, rg_hi = -1;   // row groups [rg_lo, rg_hi) of this part are staged (-1: all)
  uint64_t rows = 0;               // rows in the staged row groups
  size_t rg_end() const { return rg_hi < 0 ? meta.row_groups.size() : std::min<size_t>(size_t(rg_hi), meta.row_groups.size()); }
};

struct NonFileAction {
  int kind;                    // dev::K_METADATA / K_TXN / K_PROTOCOL
  uint64_t order;              // action index (replay order)
  std::string json;            // {"metaData":{...}} etc.
  std::shared_ptr<const JVal> val;  // inner object (shared: a state's winners are copied per apply)
};

// Hot checkpoint columns decoded on the device.
enum HotCol { HC_ADD_PATH = 0, HC_ADD_SIZE = 1, HC_RM_PATH = 2, HC_RM_DELTS = 3, HC_N = 4 };
static const char* kHotPath[HC_N] = {"add.path", "add.size", "remove.path", "remove.deletionTimestamp"};

// Decode plan of a set of checkpoint leaf columns: page table, SNAPPY plan and scratch, PLAIN
// BYTE_ARRAY boundary scratch, decompressed-page arena. Built once at staging, reused per replay.
struct PagePlan {
  std::vector<std::string> paths;        // leaf column paths, output slot = index
  std::vector<int> max_def, max_rep;
  std::vector<bool> present;
  std::vector<uint64_t> levels;          // per column: rows (flat) or level entries (repeated)
  std::vector<PageDesc> pages;
  DBuf<PageDesc> d_pages;
  uint32_t dict_entries = 0;
  DBuf<uint8_t> d_arena;
  // SNAPPY plan + persistent scratch
  std::vector<SnapPage> snap_pages;
  std::vector<uint32_t> chunk_base, block_page, chunk_page;
  std::vector<CopyJob> copy_jobs;
  uint32_t nchunks = 0;
  DBuf<SnapPage> d_snap;
  DBuf<uint32_t> d_chunk_base, d_block_page, d_chunk_page;
  DBuf<CopyJob> d_copy;
  DBuf<uint32_t> s_spec_exit, s_vis, s_entry, s_spec_first, s_assumed, s_region, s_chunk_out, s_chunk_out_start,
      s_chunk_elems, s_pages_bad, s_block_chunk, s_page_mark;
  DBuf<uint8_t> s_chunk_flag;
  DBuf<unsigned long long> s_region_count;
  std::vector<uint32_t> wg_chunk0;
  DBuf<uint32_t> d_wg_chunk0;
  uint64_t snap_in_bytes = 0, snap_out_bytes = 0, copy_bytes = 0;
  uint64_t snap_elements = 0;  // SNAPPY elements of the pages (known after a timed replay)
  // PLAIN BYTE_ARRAY boundary scratch (k_ba_bounds)
  uint32_t ba_pages = 0;
  uint64_t ba_vals = 0;
  std::vector<uint2> ba_tiles;
  DBuf<uint2> d_ba_tiles;
  DBuf<uint32_t> s_ba_vals, s_ba_ok, s_ba_count, s_ba_tile_cnt;
  DBuf<uint64_t> s_ba_tile_off, s_ba_kept;
  DBuf<uint32_t> s_ba_link;
};

// Host copy of a staged segment's bytes (the host side keeps them: checkpoint footers / page headers
// for planning, non-file JSON lines, dr_parse_commits' line views). Large stagings are pinned
// (hipHostMalloc), so the chunked H2D copies that overlap the file reads are plain DMA; small ones
// (a streaming tail's commit) are ordinary heap memory. `n` bytes are the payload; the allocation
// holds `pad` more zero bytes.
struct HostBytes {
  uint8_t* p = nullptr;
  size_t n = 0, cap = 0;
  bool pinned = false;
  HostBytes() = default;
  HostBytes(const HostBytes&) = delete;
  HostBytes& operator=(const HostBytes&) = delete;
  ~HostBytes() { release(); }
  void release() {
    if (p) {
      if (pinned) (void)hipHostFree(p);
      else std::free(p);
    }
    p = nullptr;
    n = cap = 0;
  }
  void alloc(size_t bytes, size_t pad, bool pin) {
    release();
    cap = bytes + pad;
    pinned = pin;
    if (pin && hipHostMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(cap, 1), hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      p = nullptr;
      pinned = false;
    }
    if (!p && cap >= (size_t(64) << 20)) {  // large: 2 MiB-aligned, transparent huge pages (fewer faults)
      if (posix_memalign(reinterpret_cast<void**>(&p), size_t(2) << 20, cap) != 0) p = nullptr;
      if (p) (void)madvise(p, cap, MADV_HUGEPAGE);
    }
    if (!p) p = static_cast<uint8_t*>(std::malloc(std::max<size_t>(cap, 1)));
    if (!p) fail(DR_E_OOM, fmt("host staging buffer of %zu bytes", cap));
    n = bytes;
    if (pad) memset(p + bytes, 0, pad);
  }
  uint8_t* data() { return p; }
  const uint8_t* data() const { return p; }
  size_t size() const { return n; }
  uint8_t& operator[](size_t i) { return p[i]; }
  const uint8_t& operator[](size_t i) const { return p[i]; }
};

struct StagedData {
  dr_ctx* ctx = nullptr;
  HostBytes h_json, h_pq;
  DBuf<uint8_t> d_json, d_pq;
  std::vector<JsonFileRec> jfiles;
  std::vector<CkPart> parts;
  uint64_t ck_rows = 0;
  uint64_t json_lines = 0;                // newline bytes in h_json (every file newline-terminated)
  int64_t ck_version = -1;
  int64_t version = -1;
  PagePlan hot;                           // the four hot leaf columns, decoded by every replay
  bool has_col[HC_N] = {false, false, false, false};
  int max_def[HC_N] = {0, 0, 0, 0};
  int add_def = 1, rm_def = 1;
  std::vector<NonFileAction> ck_nonfile;  // protocol/metaData/txn rows of the checkpoint
  std::unique_ptr<PagePlan> pv;           // add.partitionValues map columns (planned on first filter)
  std::unique_ptr<PagePlan> mt;           // add.modificationTime (planned on first scan order)
  std::unique_ptr<PagePlan> exp[2];       // the export's add / remove leaves (planned on first export)
  std::mutex pv_mu;
  // canonicalisation arena bytes the last replay of this segment needed (-1: none yet). A capacity
  // hint only: the next replay sizes its arena from it instead of reading the special-path counters
  // back before K3; an arena that turns out too small is detected at the end and the replay redone.
  std::atomic<int64_t> canon_need{-1};
};

struct dr_staged {
  std::shared_ptr<StagedData> d;
};

// Host vectors the export copies into: no value-initialisation (the D2H copy overwrites every
// element; zero-filling gigabytes first doubled the export time).
template <typename T>
struct NoInitAlloc : std::allocator<T> {
  template <typename U>
  struct rebind { using other = NoInitAlloc<U>; };
  NoInitAlloc() = default;
  template <typename U>
  NoInitAlloc(const NoInitAlloc<U>&) {}
  template <typename U>
  void construct(U* p) noexcept { ::new (static_cast<void*>(p)) U; }
  template <typename U, typename... A>
  void construct(U* p, A&&... a) { ::new (static_cast<void*>(p)) U(std::forward<A>(a)...); }
};
template <typename T>
using hvec = std::vector<T, NoInitAlloc<T>>;

struct DevExport;  // the device export columns of one side (defined with export_device)

// One side of dr_state_export on the host: every column a slice of one pinned block (the context's
// cache), filled by asynchronous copies from the device export and one stream synchronisation.
struct ExportCols {
  bool built = false;
  int64_t n = 0;
  dr_ctx* ctx = nullptr;
  std::vector<void*> blocks;  // pinned blocks (the context's cache) holding the columns
  int64_t *path_off = nullptr, *size = nullptr, *mtime = nullptr, *delts = nullptr, *stats_off = nullptr,
          *pv_entry_off = nullptr, *pv_key_off = nullptr, *pv_val_off = nullptr, *tags_entry_off = nullptr,
          *tags_key_off = nullptr, *tags_val_off = nullptr;
  uint8_t *path_bytes = nullptr, *delts_valid = nullptr, *efm = nullptr, *stats_bytes = nullptr, *stats_null = nullptr,
          *pv_null = nullptr, *pv_key_bytes = nullptr, *pv_val_bytes = nullptr, *pv_val_null = nullptr,
          *tags_null = nullptr, *tags_key_bytes = nullptr, *tags_val_bytes = nullptr, *tags_val_null = nullptr;
  ExportCols() = default;
  ExportCols(const ExportCols&) = delete;
  ExportCols& operator=(const ExportCols&) = delete;
  ~ExportCols() {
    if (ctx)
      for (void* b : blocks) ctx->host_release(b);
  }
};

// D2H into a host vector without initialising it first.
template <typename T, typename H>
static void d2h_into(H& out, const T* p, size_t n, hipStream_t s) {
  out.resize(n);
  if (n) {
    HIP_OK(hipMemcpyAsync(out.data(), p, n * sizeof(T), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
  }
}

// The chain of states that dr_state_apply grows from one full replay: an
// append-only action store (the base's survivors, then every applied tail), the device path index
// over it (k_index.hip) and, per applied tail, the undo log that turns the index back into any older
// state's view. Every state of the chain reads the store through views; only the head moves.
struct IncChain {
  dr_ctx* ctx = nullptr;
  uint64_t n = 0, cap = 0;  // actions in the store, capacity
  DBuf<uint8_t> kind, flags;
  DBuf<uint64_t> key, path_ptr, src_off;
  DBuf<uint32_t> path_len, src_len;
  DBuf<int64_t> size, delts;
  DBuf<uint16_t> src_id;
  uint64_t tcap = 0, used = 0;  // table slots (power of two), occupied slots
  DBuf<unsigned long long> keys;
  DBuf<uint32_t> vals;
  DBuf<ulonglong2> tomb_list;  // tombstone candidates of the head, {action, deletionTimestamp} (stale entries are skipped)
  uint64_t tomb_n = 0, tomb_cap = 0;
  struct Undo {
    DBuf<uint2> e;
    uint64_t n = 0;
  };
  std::vector<Undo> undo;  // undo[g - 1] turns generation g back into g - 1
  uint32_t head = 0;
  std::vector<std::shared_ptr<StagedData>> sources;
  std::vector<std::shared_ptr<DBuf<uint8_t>>> arenas;
  DBuf<unsigned long long> ctr;
};

struct ExpDecoded;

struct dr_state {
  dr_ctx* ctx = nullptr;
  // a state of an apply chain: its actions are the store's first n_actions, its survivor lists are
  // built from the index on first use (ensure_ready)
  std::shared_ptr<IncChain> chain;
  uint32_t gen = 0, nsrc = 0;
  bool lists_ready = true;
  bool ordered = false;  // survivor lists sorted by action index (order_lists, on first use)
  std::shared_ptr<StagedData> staged;
  // the staged segments the action records point into: {staged} for a replay; for a state built
  // by dr_state_apply, its base's sources plus the applied tail (only sources[0] can hold
  // checkpoint rows). src_id (empty: every action is from sources[0]) names each action's source.
  std::vector<std::shared_ptr<StagedData>> sources;
  DBuf<uint16_t> src_id;
  bool sharded = false;  // a rank's part of a sharded replay (source-side survivors, owner-side counters)
  int64_t cutoff = INT64_MIN;  // minFileRetentionTimestamp the survivors were selected with
  uint64_t n_actions = 0;
  // resident action arrays
  DBuf<uint8_t> kind, flags;
  DBuf<uint64_t> key, path_ptr, src_off;
  DBuf<uint32_t> path_len, src_len;
  DBuf<int64_t> size, delts;
  DBuf<uint64_t> path_ref;  // packed path references written by K1 / K2 / k_canon (parse_launch's states only)
  std::vector<std::shared_ptr<DBuf<uint8_t>>> arenas;  // canonical special paths (path_ptr targets)
  DBuf<uint32_t> live, tomb;   // survivor action indices (hash order per bucket)
  uint64_t n_live = 0, n_tomb = 0;
  dr_counts counts{};
  // a rank of the library's sharded replay: its own counters before the all-reduce (what the
  // torch driver's local state reports), for per-rank roofline accounting
  dr_counts local_counts{};
  bool has_local_counts = false;
  std::string nonfile_json;
  std::vector<NonFileAction> nonfile;  // winners: protocol, metadata, txns
  ExportCols exp[2];
  // K5 cache: partition columns of the live AddFiles cast to their types (k_pv_extract), built on
  // the first dr_filter that references each (name, type) and reused by every later one
  struct PvCol {
    std::string name;
    int32_t type;
    DBuf<uint32_t> w32;
    DBuf<int64_t> w64;
    DBuf<uint64_t> sptr;
    DBuf<uint32_t> slen;
    DBuf<uint8_t> isnull;
    DBuf<uint64_t> s8;
    DBuf<int64_t> w64hi;  // DECIMAL: high 64 bits of the unscaled value
    // K5 dictionary (built on the first leaf-form filter that reads the column): u16 code per live
    // file, code 0 = NULL; rep[c] = a row holding code c's value. dict: -1 not built, 0 none, 1 ok
    int dict = -1;
    uint32_t ncode = 0;
    DBuf<uint16_t> code;
    DBuf<uint32_t> rep;
  };
  std::vector<std::unique_ptr<PvCol>> pv_cols;
  std::vector<std::shared_ptr<DBuf<uint8_t>>> pv_arenas;  // unescaped string values
  // export: the checkpoint's add / remove leaves, decoded on the first export of each side
  std::shared_ptr<ExpDecoded> exp_dec[2];
  // the materialised state (dr_state_materialize): every field of both sides extracted on the device
  // and kept resident -- the reference's cached SingleAction rows (D/util/StateCache.scala:45-68)
  std::shared_ptr<DevExport> dexp[2];
};

// ---------------------------------------------------------------------------------------------------
// checkpoint planning (host)
// ---------------------------------------------------------------------------------------------------
static int leaf_def_of(const pq::Leaf& l, int depth) { return l.def_of[size_t(depth)]; }

static std::string render_protocol(const std::vector<pq::Entry>& rd, const std::vector<pq::Entry>& wr, size_t i,
                                   size_t j) {
  JVal o;
  o.t = JVal::OBJ;
  JVal a; a.t = JVal::NUM; a.s = std::to_string(rd[i].ival);
  JVal b; b.t = JVal::NUM; b.s = std::to_string(wr[j].ival);
  o.o.emplace_back("minReaderVersion", a);
  o.o.emplace_back("minWriterVersion", b);
  return json_dump(o);
}

// Decodes protocol / metaData / txn rows of one checkpoint part on the host (run-wise, so the
// all-null runs of a 10M-row checkpoint cost nothing). Rows are reported in row order.
static void decode_ck_nonfile(StagedData& s, CkPart& part, uint64_t base_action) {
  const uint8_t* file = s.h_pq.data() + part.off;
  const pq::FileMeta& m = part.meta;
  int64_t rg_base = 0;
  for (size_t gi = size_t(part.rg_lo); gi < part.rg_end(); ++gi) {
    const pq::RowGroup& rg = m.row_groups[gi];
    auto col = [&](const std::string& path) -> const pq::ColumnChunk* {
      for (auto& c : rg.cols) if (c.path == path) return &c;
      return nullptr;
    };
    // Collect entries per column keyed by row.
    struct Field { std::string name; std::vector<pq::Entry> e; const pq::Leaf* leaf; };
    auto load = [&](const std::string& path, int thr_depth) -> std::vector<pq::Entry> {
      const pq::Leaf* l = m.leaf(path);
      const pq::ColumnChunk* c = col(path);
      if (!l || !c) return {};
      return pq::sparse_entries(file, part.len, *c, *l, leaf_def_of(*l, thr_depth),
                                int64_t(part.row_base) + rg_base);
    };
    std::map<int64_t, NonFileAction> rows;  // row -> action
    // protocol
    {
      auto rd = load("protocol.minReaderVersion", 0);
      auto wr = load("protocol.minWriterVersion", 0);
      for (size_t i = 0; i < rd.size(); ++i) {
        NonFileAction a;
        a.kind = 5;
        a.order = base_action + uint64_t(rd[i].row);
        JVal o; o.t = JVal::OBJ;
        JVal x; x.t = JVal::NUM; x.s = std::to_string(rd[i].has_value ? rd[i].ival : 0);
        o.o.emplace_back("minReaderVersion", x);
        int64_t wv = 0;
        for (auto& w : wr) if (w.row == rd[i].row && w.has_value) wv = w.ival;
        JVal y; y.t = JVal::NUM; y.s = std::to_string(wv);
        o.o.emplace_back("minWriterVersion", y);
        a.val = std::make_shared<const JVal>(o);
        a.json = "{\"protocol\":" + json_dump(o) + "}";
        rows[rd[i].row] = a;
      }
    }
    // txn
    {
      auto app = load("txn.appId", 0);
      auto ver = load("txn.version", 0);
      auto lu = load("txn.lastUpdated", 0);
      for (auto& e : app) {
        NonFileAction a;
        a.kind = 4;
        a.order = base_action + uint64_t(e.row);
        JVal o; o.t = JVal::OBJ;
        JVal id; if (e.has_value) { id.t = JVal::STR; id.s = e.sval; }
        o.o.emplace_back("appId", id);
        for (auto& v : ver) if (v.row == e.row) { JVal x; x.t = JVal::NUM; x.s = std::to_string(v.has_value ? v.ival : 0); o.o.emplace_back("version", x); }
        for (auto& v : lu) if (v.row == e.row && v.has_value) { JVal x; x.t = JVal::NUM; x.s = std::to_string(v.ival); o.o.emplace_back("lastUpdated", x); }
        a.val = std::make_shared<const JVal>(o);
        a.json = "{\"txn\":" + json_dump(o) + "}";
        rows[e.row] = a;
      }
    }
    // metaData
    {
      auto id = load("metaData.id", 0);
      if (!id.empty()) {
        auto name = load("metaData.name", 0);
        auto desc = load("metaData.description", 0);
        auto prov = load("metaData.format.provider", 0);
        auto ok = load("metaData.format.options.key_value.key", 2);
        auto ov = load("metaData.format.options.key_value.value", 2);
        auto schema = load("metaData.schemaString", 0);
        auto pcols = load("metaData.partitionColumns.list.element", 1);
        auto ck = load("metaData.configuration.key_value.key", 1);
        auto cv = load("metaData.configuration.key_value.value", 1);
        auto ct = load("metaData.createdTime", 0);
        auto str_at = [](const std::vector<pq::Entry>& v, int64_t row, JVal* out) {
          for (auto& e : v) if (e.row == row && e.has_value) { out->t = JVal::STR; out->s = e.sval; return true; }
          return false;
        };
        // map / list entries of one row: entries whose def reaches the key_value (or list) level
        auto map_of = [](const std::vector<pq::Entry>& ks, const std::vector<pq::Entry>& vs, int64_t row,
                         int entry_def, JVal* out) {
          out->t = JVal::OBJ;
          bool present = false;
          for (size_t i = 0; i < ks.size(); ++i) {
            if (ks[i].row != row) continue;
            present = true;
            if (ks[i].def < entry_def) continue;
            JVal v;
            if (i < vs.size() && vs[i].has_value) { v.t = JVal::STR; v.s = vs[i].sval; }
            out->o.emplace_back(ks[i].sval, v);
          }
          return present;
        };
        for (auto& e : id) {
          int64_t r = e.row;
          NonFileAction a;
          a.kind = 3;
          a.order = base_action + uint64_t(r);
          JVal o; o.t = JVal::OBJ;
          JVal v;
          if (e.has_value) { v.t = JVal::STR; v.s = e.sval; o.o.emplace_back("id", v); }
          if (str_at(name, r, &v)) o.o.emplace_back("name", v);
          v = JVal();
          if (str_at(desc, r, &v)) o.o.emplace_back("description", v);
          JVal fmtv; fmtv.t = JVal::OBJ;
          v = JVal();
          if (str_at(prov, r, &v)) fmtv.o.emplace_back("provider", v);
          JVal opts;
          const pq::Leaf* okl = m.leaf("metaData.format.options.key_value.key");
          map_of(ok, ov, r, okl ? okl->max_def : 0, &opts);
          fmtv.o.emplace_back("options", opts);
          o.o.emplace_back("format", fmtv);
          v = JVal();
          if (str_at(schema, r, &v)) o.o.emplace_back("schemaString", v);
          JVal pc; pc.t = JVal::ARR;
          const pq::Leaf* pcl = m.leaf("metaData.partitionColumns.list.element");
          for (auto& x : pcols) {
            if (x.row != r || !pcl || x.def < pcl->max_def - 1) continue;
            JVal s;
            if (x.has_value) { s.t = JVal::STR; s.s = x.sval; }
            pc.a.push_back(s);
          }
          o.o.emplace_back("partitionColumns", pc);
          JVal conf;
          const pq::Leaf* ckl = m.leaf("metaData.configuration.key_value.key");
          map_of(ck, cv, r, ckl ? ckl->max_def : 0, &conf);
          o.o.emplace_back("configuration", conf);
          for (auto& x : ct) if (x.row == r && x.has_value) { JVal n; n.t = JVal::NUM; n.s = std::to_string(x.ival); o.o.emplace_back("createdTime", n); }
          a.val = std::make_shared<const JVal>(o);
          a.json = "{\"metaData\":" + json_dump(o) + "}";
          rows[r] = a;
        }
      }
    }
    for (auto& kv : rows) s.ck_nonfile.push_back(kv.second);
    rg_base += rg.num_rows;
  }
}

// Page plan of `P.paths` over the staged row groups of every checkpoint part (host: footer +
// page headers), then the SNAPPY plan, arena and scratch (device).
static void plan_pages(StagedData& s, PagePlan& P) {
  const size_t nc = P.paths.size();
  P.max_def.assign(nc, 0);
  P.max_rep.assign(nc, 0);
  P.present.assign(nc, false);
  P.levels.assign(nc, 0);
  if (s.parts.empty()) return;
  const pq::FileMeta& m0 = s.parts[0].meta;
  for (size_t c = 0; c < nc; ++c) {
    const pq::Leaf* l = m0.leaf(P.paths[c]);
    P.present[c] = l != nullptr;
    if (l) { P.max_def[c] = l->max_def; P.max_rep[c] = l->max_rep; }
  }
  uint64_t arena = 0;
  uint32_t dict_pool = 0;
  std::vector<uint64_t> entry(nc, 0);   // level-entry cursor of repeated columns
  for (CkPart& part : s.parts) {
    const uint8_t* file = s.h_pq.data() + part.off;
    uint64_t rg_row = part.row_base;
    for (size_t gi = size_t(part.rg_lo); gi < part.rg_end(); ++gi) {
      const pq::RowGroup& rg = part.meta.row_groups[gi];
      for (size_t c = 0; c < nc; ++c) {
        if (!P.present[c]) continue;
        const pq::ColumnChunk* cc = nullptr;
        for (auto& x : rg.cols) if (x.path == P.paths[c]) cc = &x;
        if (!cc) continue;
        if (cc->codec != 0 && cc->codec != 1)
          fail(DR_E_UNSUPPORTED, fmt("checkpoint codec %d is not supported (column %s)", cc->codec, P.paths[c].c_str()));
        const pq::Leaf* l = part.meta.leaf(P.paths[c]);
        if (!l) fail(DR_E_PARQUET, fmt("checkpoint parts disagree on column %s", P.paths[c].c_str()));
        const bool repeated = l->max_rep > 0;
        int dict_idx = -1;
        uint64_t row = repeated ? entry[c] : rg_row;
        for (const pq::Page& p : pq::walk_pages(file, part.len, *cc)) {
          PageDesc d{};
          d.src = uint64_t(part.off + uint64_t(p.data_off));  // relocated below
          d.dst = arena;
          d.csize = uint32_t(p.compressed_size);
          d.usize = uint32_t(p.uncompressed_size);
          d.num_values = uint32_t(p.num_values);
          d.kind = p.page_type == pq::DICTIONARY_PAGE ? PG_DICT : p.page_type == pq::DATA_PAGE_V2 ? PG_DATA_V2 : PG_DATA_V1;
          d.encoding = p.encoding;
          d.codec = cc->codec;
          d.col = int32_t(c);
          d.phys = l->type;
          d.max_def = l->max_def;
          d.max_rep = l->max_rep;
          d.v2_def_len = p.v2_def_len;
          d.v2_rep_len = p.v2_rep_len;
          d.v2_compressed = p.v2_compressed;
          if (d.kind == PG_DICT) {
            dict_idx = int(P.pages.size());
            d.dict_base = dict_pool;
            dict_pool += d.num_values;
            d.dict = -1;
          } else {
            d.dict = dict_idx;
            d.row_base = row;
            row += p.num_values;
            if (d.encoding != 0 && d.encoding != 2 && d.encoding != 8 && !(d.encoding == 3 && l->type == 0))
              fail(DR_E_UNSUPPORTED, fmt("encoding %d not supported for %s", d.encoding, P.paths[c].c_str()));
          }
          arena += (uint64_t(d.usize) + 16 + 15) & ~uint64_t(15);
          if (d.phys == 6 && (d.kind == PG_DICT || d.encoding == 0)) {  // PLAIN byte arrays
            d.ba = 1;
            d.ba_slot = P.ba_pages++;
            d.ba_base = P.ba_vals;
            d.hit_base = P.ba_tiles.size();
            P.ba_vals += d.usize / 4 + 2;
            const uint32_t nt = uint32_t((uint64_t(d.usize) + 15) / ba_tile_bytes() + 1);
            for (uint32_t t = 0; t < nt; ++t) P.ba_tiles.push_back(make_uint2(uint32_t(P.pages.size()), t));
          }
          P.pages.push_back(d);
        }
        if (repeated) {
          entry[c] = row;
        } else if (row != rg_row + uint64_t(rg.num_rows)) {
          fail(DR_E_PARQUET, fmt("column %s: %llu levels for %lld rows", P.paths[c].c_str(),
                                 (unsigned long long)(row - rg_row), (long long)rg.num_rows));
        }
      }
      rg_row += uint64_t(rg.num_rows);
    }
  }
  for (size_t c = 0; c < nc; ++c) P.levels[c] = P.max_rep[c] > 0 ? entry[c] : s.ck_rows;
  P.dict_entries = dict_pool;
  // SNAPPY plan: preamble, speculation chunks and 64 KiB output blocks per page (k_snappy.hip)
  for (const PageDesc& d : P.pages) {
    const uint64_t lv = d.kind == PG_DATA_V2 ? uint64_t(d.v2_def_len + d.v2_rep_len) : 0;
    if (lv) P.copy_jobs.push_back(CopyJob{d.src, d.dst, lv});
    P.copy_bytes += lv;
    const bool compressed = d.codec == 1 && !(d.kind == PG_DATA_V2 && !d.v2_compressed);
    if (!compressed) {
      P.copy_jobs.push_back(CopyJob{d.src + lv, d.dst + lv, d.usize - lv});
      P.copy_bytes += d.usize - lv;
      continue;
    }
    const uint8_t* h = s.h_pq.data() + d.src + lv;
    uint64_t total = 0;
    uint32_t pre = 0;
    for (int sh = 0; pre < 5 && pre < d.csize - lv; sh += 7) {
      const uint8_t b = h[pre++];
      total |= uint64_t(b & 0x7f) << sh;
      if (!(b & 0x80)) break;
    }
    if (total != d.usize - lv) fail(DR_E_PARQUET, "snappy preamble does not match the page size");
    {
      // a page the compressor could not shrink is a run of literals (one per 64 KiB fragment):
      // those bytes are copied as they are (a long literal spans many speculation chunks, which
      // would send the page to the serial decoder)
      std::vector<CopyJob> lit;
      uint64_t ip = pre, op = 0;
      const uint64_t n_in = d.csize - lv;
      while (ip < n_in && op < total) {
        const uint8_t tag = h[ip];
        if (tag & 3) break;
        const uint32_t l6 = tag >> 2, nb = l6 < 60 ? 0 : l6 - 59;
        if (ip + 1 + nb > n_in) break;
        uint64_t len = l6 + 1;
        if (nb) {
          len = 0;
          for (uint32_t k = 0; k < nb; ++k) len |= uint64_t(h[ip + 1 + k]) << (8 * k);
          len += 1;
        }
        if (ip + 1 + nb + len > n_in || op + len > total) break;
        lit.push_back(CopyJob{d.src + lv + ip + 1 + nb, d.dst + lv + op, len});
        ip += 1 + nb + len;
        op += len;
      }
      if (ip == n_in && op == total) {
        P.copy_jobs.insert(P.copy_jobs.end(), lit.begin(), lit.end());
        P.copy_bytes += total;
        continue;
      }
    }
    SnapPage sp{d.src + lv + pre, d.dst + lv, uint32_t(d.csize - lv - pre), uint32_t(d.usize - lv),
                uint32_t(P.block_page.size())};
    P.chunk_base.push_back(P.nchunks);
    const uint32_t ncp = (sp.n_in + snappy_chunk_bytes() - 1) / snappy_chunk_bytes();
    P.chunk_page.insert(P.chunk_page.end(), ncp, uint32_t(P.snap_pages.size()));
    for (uint32_t j = 0; j < ncp; j += snappy_wg_chunks()) P.wg_chunk0.push_back(P.nchunks + j);
    P.nchunks += ncp;
    P.snap_in_bytes += sp.n_in;
    P.snap_out_bytes += sp.n_out;
    const uint32_t nb = (sp.n_out + 65535) / 65536;
    for (uint32_t k = 0; k < nb; ++k) P.block_page.push_back(uint32_t(P.snap_pages.size()));
    P.snap_pages.push_back(sp);
  }
  P.chunk_base.push_back(P.nchunks);
  P.d_arena = DBuf<uint8_t>(s.ctx, arena + 4096);
  const uint64_t pqb = reinterpret_cast<uint64_t>(s.d_pq.p), arb = reinterpret_cast<uint64_t>(P.d_arena.p);
  for (SnapPage& sp : P.snap_pages) { sp.in += pqb; sp.out += arb; }
  for (CopyJob& j : P.copy_jobs) { j.src += pqb; j.dst += arb; }
  auto up = [&](auto& dbuf, auto& vec) {
    using T = typename std::decay_t<decltype(vec)>::value_type;
    dbuf = DBuf<T>(s.ctx, vec.size());
    if (!vec.empty())
      HIP_OK(hipMemcpyAsync(dbuf.p, vec.data(), vec.size() * sizeof(T), hipMemcpyHostToDevice, s.ctx->stream));
  };
  up(P.d_snap, P.snap_pages);
  up(P.d_chunk_base, P.chunk_base);
  up(P.d_chunk_page, P.chunk_page);
  up(P.d_block_page, P.block_page);
  up(P.d_copy, P.copy_jobs);
  up(P.d_wg_chunk0, P.wg_chunk0);
  P.s_spec_exit = DBuf<uint32_t>(s.ctx, P.nchunks);
  P.s_vis = DBuf<uint32_t>(s.ctx, uint64_t(P.nchunks) * (snappy_chunk_bytes() / 32));
  P.s_entry = DBuf<uint32_t>(s.ctx, P.nchunks);
  P.s_spec_first = DBuf<uint32_t>(s.ctx, P.nchunks);
  P.s_assumed = DBuf<uint32_t>(s.ctx, P.nchunks);
  P.s_region = DBuf<uint32_t>(s.ctx, P.nchunks);
  P.s_block_chunk = DBuf<uint32_t>(s.ctx, P.block_page.size() + 1);
  P.s_chunk_flag = DBuf<uint8_t>(s.ctx, P.nchunks);
  P.s_region_count = DBuf<unsigned long long>(s.ctx, 1);
  P.s_chunk_out = DBuf<uint32_t>(s.ctx, P.nchunks);
  P.s_chunk_out_start = DBuf<uint32_t>(s.ctx, P.nchunks);
  P.s_chunk_elems = DBuf<uint32_t>(s.ctx, P.nchunks);
  P.s_pages_bad = DBuf<uint32_t>(s.ctx, P.snap_pages.size());
  P.s_page_mark = DBuf<uint32_t>(s.ctx, P.snap_pages.size());
  P.s_ba_vals = DBuf<uint32_t>(s.ctx, P.ba_vals);
  up(P.d_ba_tiles, P.ba_tiles);
  P.s_ba_tile_cnt = DBuf<uint32_t>(s.ctx, P.ba_tiles.size());
  P.s_ba_tile_off = DBuf<uint64_t>(s.ctx, P.ba_tiles.size() + 1);
  P.s_ba_kept = DBuf<uint64_t>(s.ctx, P.ba_tiles.size() * 256);
  P.s_ba_link = DBuf<uint32_t>(s.ctx, P.ba_tiles.size() * 3);
  P.s_ba_ok = DBuf<uint32_t>(s.ctx, P.ba_pages);
  P.s_ba_count = DBuf<uint32_t>(s.ctx, P.ba_pages);
  for (PageDesc& d : P.pages) {
    d.src = pqb + d.src;
    d.dst = arb + d.dst;
  }
  up(P.d_pages, P.pages);
}

// Inflate + decode every page of a plan into `pa.cols` (allocated by the caller for P.levels).
// Scan scratch for n counts (at least 2^23 entries). DR_SCAN_SCRATCH_MAX (test hook) caps the size,
// so a scan too large for its scratch is shown to fail loudly (launch_scan_u32 refuses it).
static uint64_t scan_scratch_for(uint64_t n) {
  uint64_t b = scan_scratch_bytes(std::max<uint64_t>(n, uint64_t(1) << 23));
  if (const char* cap = std::getenv("DR_SCAN_SCRATCH_MAX")) b = std::min<uint64_t>(b, std::strtoull(cap, nullptr, 10));
  return b;
}
static ScanScratch ss(const DBuf<uint8_t>& b) { return ScanScratch{b.p, b.n}; }

static void decode_pages(dr_ctx* ctx, PagePlan& P, ParquetArgs& pa, DBuf<uint64_t>& dict_ptr, DBuf<uint32_t>& dict_len,
                         DBuf<uint32_t>& err, void*) {
  hipStream_t stream = ctx->stream;
  // scan scratch for the plan's largest scan: SNAPPY chunk element counts, PLAIN BYTE_ARRAY tiles
  // (a 100M-row checkpoint has 26M chunks: a scratch sized for 2^23 entries was overrun)
  DBuf<uint8_t> own_scratch(ctx, scan_scratch_for(std::max<uint64_t>(P.nchunks, P.ba_tiles.size())));
  const ScanScratch scratch = ss(own_scratch);
  pa.pages = P.d_pages.p;
  pa.npages = uint32_t(P.pages.size());
  dict_ptr = DBuf<uint64_t>(ctx, P.dict_entries);
  dict_len = DBuf<uint32_t>(ctx, P.dict_entries);
  pa.dict_ptr = dict_ptr.p;
  pa.dict_len = dict_len.p;
  pa.error = err.p;
  pa.ba_vals = P.s_ba_vals.p;
  pa.ba_hit = nullptr;
  pa.ba_tiles = P.d_ba_tiles.p;
  pa.nba_tiles = uint32_t(P.ba_tiles.size());
  pa.ba_tile_cnt = P.s_ba_tile_cnt.p;
  pa.ba_tile_off = P.s_ba_tile_off.p;
  pa.ba_kept = P.s_ba_kept.p;
  pa.ba_link = P.s_ba_link.p;
  pa.ba_ok = P.s_ba_ok.p;
  pa.ba_count = P.s_ba_count.p;
  launch_page_copy(P.d_copy.p, uint32_t(P.copy_jobs.size()), stream);
  if (!P.snap_pages.empty()) {
    P.s_pages_bad.zero(stream);
    P.s_page_mark.zero(stream);
    P.s_chunk_flag.zero(stream);
    P.s_region_count.zero(stream);
    SnappyArgs sa{};
    sa.pages = P.d_snap.p;
    sa.npages = uint32_t(P.snap_pages.size());
    sa.chunk_base = P.d_chunk_base.p;
    sa.nchunks = P.nchunks;
    sa.spec_exit = P.s_spec_exit.p;
    sa.vis = P.s_vis.p;
    sa.entry = P.s_entry.p;
    sa.spec_first = P.s_spec_first.p;
    sa.assumed_exit = P.s_assumed.p;
    sa.chunk_flag = P.s_chunk_flag.p;
    sa.region = P.s_region.p;
    sa.region_count = P.s_region_count.p;
    sa.page_mark = P.s_page_mark.p;
    sa.chunk_out = P.s_chunk_out.p;
    sa.chunk_out_start = P.s_chunk_out_start.p;
    sa.chunk_elems = P.s_chunk_elems.p;
    sa.block_page = P.d_block_page.p;
    sa.block_chunk = P.s_block_chunk.p;
    sa.nblocks = uint32_t(P.block_page.size());
    sa.wg_chunk0 = P.d_wg_chunk0.p;
    sa.nwg = uint32_t(P.wg_chunk0.size());
    sa.pages_bad = P.s_pages_bad.p;
    sa.error = err.p;
    sa.chunk_page = P.d_chunk_page.p;
    DBuf<uint64_t> stamps, rstats;
    const bool dbg = std::getenv("DR_SNAP_DEBUG") != nullptr;
    if (dbg) {
      stamps = DBuf<uint64_t>(ctx, P.block_page.size() * 16);
      stamps.zero(stream);
      sa.stamps = stamps.p;
      rstats = DBuf<uint64_t>(ctx, uint64_t(P.nchunks) * 4 + 4);
      rstats.zero(stream);
      sa.rstats = rstats.p;
    }
    launch_snappy(sa, stream, scratch);
    if (ctx->timing && !P.snap_elements) {  // statistics, once (the first timed replay)
      const std::vector<uint32_t> el = d2h(P.s_chunk_elems.p, P.nchunks, stream);
      for (uint32_t v : el) P.snap_elements += v;
    }
    if (dbg) {
      std::vector<uint64_t> st = d2h(stamps.p, P.block_page.size() * 16, stream);
      // 16 stamp slots per block (k_snap_exec): slot 0 at entry, 15 at the end, the phases between;
      // the mean clocks from each stamped slot to the next stamped one
      double acc[16] = {0};
      size_t nb2 = 0;
      for (size_t q = 0; q < P.block_page.size(); ++q) {
        const uint64_t* x = &st[q * 16];
        if (!x[0] || !x[15]) continue;
        ++nb2;
        // slots 11-13: active 4-byte groups at the start of jumping rounds 1-3 (of 16384), 14: the
        // block's most rounds of a thread -- counters, not clocks
        for (int k = 11; k <= 14; ++k) acc[k] += double(x[k]);
        for (int k = 1, prev = 0; k < 16; ++k)
          if (x[k] && (k < 11 || k > 14)) {
            acc[k] += double(x[k] - x[prev]);
            prev = k;
          }
      }
      std::fprintf(stderr, "exec phases (clocks/block, %zu blocks):", nb2);
      for (int k = 1; k < 16; ++k)
        if (acc[k] != 0) {
          if (k >= 11 && k <= 13) std::fprintf(stderr, " active%d %.0f", k - 10, nb2 ? acc[k] / double(nb2) : 0.0);
          else if (k == 14) std::fprintf(stderr, " rounds %.2f", nb2 ? acc[k] / double(nb2) : 0.0);
          else std::fprintf(stderr, " [%d] %.0f", k, nb2 ? acc[k] / double(nb2) : 0.0);
        }
      std::fprintf(stderr, "\n");
      const unsigned long long nreg = d2h_one(P.s_region_count.p, stream);
      std::vector<uint32_t> pb = d2h(P.s_pages_bad.p, P.snap_pages.size(), stream);
      size_t nb = 0;
      std::map<uint32_t, size_t> why;
      for (size_t q = 0; q < pb.size(); ++q) {
        nb += pb[q] != 0;
        if (pb[q]) {
          if (why[pb[q]]++ < 3)
            std::fprintf(stderr, "snappy bad page %zu code %u: n_in %u n_out %u\n", q, pb[q],
                         P.snap_pages[q].n_in, P.snap_pages[q].n_out);
        }
      }
      for (auto& kv : why) std::fprintf(stderr, "snappy bad code %u: %zu pages\n", kv.first, kv.second);
      const size_t nr = size_t(nreg);
      std::fprintf(stderr, "snappy: pages %zu, pages with serially resolved regions %zu, bad %zu\n", P.snap_pages.size(), nr, nb);
      // chunks whose true entry is not their first speculatively visited position (re-walked by
      // k_snap_count), and pages holding at least one
      std::vector<uint32_t> ent = d2h(P.s_entry.p, P.nchunks, stream), sf = d2h(P.s_spec_first.p, P.nchunks, stream);
      size_t nx = 0, px = 0;
      for (size_t q = 0; q < P.snap_pages.size(); ++q) {
        size_t k = 0;
        for (uint32_t c = P.chunk_base[q]; c < P.chunk_base[q + 1]; ++c) k += ent[c] != sf[c];
        nx += k;
        px += k != 0;
      }
      std::fprintf(stderr, "snappy: chunks %u, entry != speculative first %zu (on %zu pages)\n", P.nchunks, nx, px);
      // pages resolved serially (one walk per region, in page order); DR_SNAP_DUMP=dir writes the
      // compressed input of the slowest
      std::vector<uint32_t> reg = d2h(P.s_region.p, nr, stream);
      std::vector<uint64_t> rs = d2h(rstats.p, nr * 4, stream);
      std::vector<size_t> ord(nr);
      for (size_t k = 0; k < nr; ++k) ord[k] = k;
      std::sort(ord.begin(), ord.end(), [&](size_t x, size_t y) { return rs[x * 4] > rs[y * 4]; });
      for (size_t k = 0; k < std::min<size_t>(nr, 8); ++k) {
        const size_t r = ord[k];
        const uint32_t q = reg[r];
        const SnapPage& pg = P.snap_pages[q];
        if (const char* dir = std::getenv("DR_SNAP_DUMP")) {
          std::vector<uint8_t> raw = d2h(reinterpret_cast<const uint8_t*>(pg.in), pg.n_in, stream);
          const std::string fn = std::string(dir) + "/slow_page" + std::to_string(q) + ".snappy";
          if (FILE* f = std::fopen(fn.c_str(), "wb")) {
            std::fwrite(raw.data(), 1, raw.size(), f);
            std::fclose(f);
          }
        }
        std::fprintf(stderr, "resolve page %u (%u chunks, n_in %u n_out %u): clocks %llu windows %llu walks %llu spans %llu\n",
                     q, P.chunk_base[q + 1] - P.chunk_base[q], pg.n_in, pg.n_out, (unsigned long long)rs[r * 4],
                     (unsigned long long)rs[r * 4 + 1], (unsigned long long)rs[r * 4 + 2], (unsigned long long)rs[r * 4 + 3]);
      }
    }
  }
  if (P.ba_pages) {
    launch_ba_bounds(pa, stream, scratch);
    if (std::getenv("DR_BA_DEBUG")) {
      std::vector<uint32_t> ok = d2h(P.s_ba_ok.p, P.ba_pages, stream);
      size_t n = 0;
      for (uint32_t v : ok) n += v != 0;
      std::fprintf(stderr, "ba bounds: %zu of %u pages validated\n", n, P.ba_pages);
      const std::vector<uint32_t> lk = d2h(P.s_ba_link.p, P.ba_tiles.size() * 3, stream);
      const std::vector<uint32_t> tc = d2h(P.s_ba_tile_cnt.p, P.ba_tiles.size(), stream);
      int shown = 0;
      for (size_t t = 0; t < P.ba_tiles.size() && shown < 40; ++t) {
        const PageDesc& pd = P.pages[P.ba_tiles[t].x];
        if (ok[pd.ba_slot]) continue;
        std::fprintf(stderr, "ba tile %zu page %u y %u usize %u kind %d: first %u lsucc %u bad %u count %u\n", t,
                     P.ba_tiles[t].x, P.ba_tiles[t].y, pd.usize, int(pd.kind), lk[3 * t], lk[3 * t + 1], lk[3 * t + 2],
                     tc[t]);
        ++shown;
      }
    }
  }
  launch_pq_dict(pa, stream);
  launch_pq_data(pa, stream);
}

static double now_s();

static void plan_checkpoint(StagedData& s) {
  const double t0 = now_s();
  uint64_t row_base = 0;
  for (CkPart& part : s.parts) {
    part.meta = pq::parse_footer(s.h_pq.data() + part.off, part.len);
    part.row_base = row_base;
    part.rows = 0;
    for (size_t gi = size_t(part.rg_lo); gi < part.rg_end(); ++gi) part.rows += uint64_t(part.meta.row_groups[gi].num_rows);
    row_base += part.rows;
  }
  s.ck_rows = row_base;
  if (s.parts.empty()) return;
  const pq::FileMeta& m0 = s.parts[0].meta;
  for (int c = 0; c < HC_N; ++c) {
    const pq::Leaf* l = m0.leaf(kHotPath[c]);
    s.has_col[c] = l != nullptr;
    if (l) {
      if (l->max_rep != 0) fail(DR_E_PARQUET, fmt("column %s is repeated", kHotPath[c]));
      s.max_def[c] = l->max_def;
      if (c == HC_ADD_PATH) s.add_def = l->def_of[0];
      if (c == HC_RM_PATH) s.rm_def = l->def_of[0];
    }
  }
  if (!s.has_col[HC_ADD_PATH]) fail(DR_E_PARQUET, "checkpoint has no add.path column");
  s.hot.paths.assign(kHotPath, kHotPath + HC_N);
  const double t1 = now_s();
  plan_pages(s, s.hot);
  const double t2 = now_s();
  for (CkPart& part : s.parts) decode_ck_nonfile(s, part, 0);  // entry rows already include part.row_base
  if (std::getenv("DR_STAGE_DEBUG"))
    std::fprintf(stderr, "plan_checkpoint: %zu parts, footers %.3f s, pages %.3f s (%zu pages), non-file rows %.3f s\n",
                 s.parts.size(), t1 - t0, t2 - t1, s.hot.pages.size(), now_s() - t2);
}

// One segment file to stage: caller-owned bytes (dr_stage) or a file the library reads itself
// (dr_stage_log / a shard's slice). rg_lo / rg_hi: stage only row groups [rg_lo, rg_hi) of a
// checkpoint part (a multi-GPU shard's slice of the checkpoint; -1 = to the end).
struct StageSrc {
  int64_t version = 0;
  int32_t kind = DR_FILE_JSON, part = 0;
  const uint8_t* data = nullptr;  // borrowed bytes, or null: read `path`
  uint64_t len = 0;
  std::string path;
  int32_t rg_lo = 0, rg_hi = -1;
};

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Staging: the files' bytes go into the host buffers (h_json: the commits concatenated, each
// newline-terminated; h_pq: the checkpoint parts, 16-byte aligned) and into HBM. Large stagings are
// cut into 32 MiB chunks that worker threads read (pread, or memcpy from caller bytes) in parallel,
// counting the JSON newlines as they go; each finished chunk's H2D copy is issued at once from the
// pinned buffer, so the DMA overlaps the remaining reads and the host planning of the checkpoint.
static std::shared_ptr<StagedData> stage_sources(dr_ctx* ctx, std::vector<StageSrc>& src) {
  const bool dbg = std::getenv("DR_STAGE_DEBUG") != nullptr;
  const double t0 = now_s();
  auto s = std::make_shared<StagedData>();
  s->ctx = ctx;
  struct FdGuard {
    std::vector<int> fds;
    ~FdGuard() { for (int fd : fds) if (fd >= 0) close(fd); }
  } fdg;
  fdg.fds.assign(src.size(), -1);
  // sizes (and, for files read here, whether the last byte is a newline)
  std::vector<uint8_t> ends_nl(src.size(), 0);
  for (size_t i = 0; i < src.size(); ++i) {
    StageSrc& f = src[i];
    if (f.data || f.path.empty()) {
      ends_nl[i] = f.len && f.data[f.len - 1] == '\n';
      continue;
    }
    const int fd = open(f.path.c_str(), O_RDONLY);
    if (fd < 0) fail(DR_E_IO, fmt("cannot open %s", f.path.c_str()));
    fdg.fds[i] = fd;
    struct stat stt;
    if (fstat(fd, &stt) != 0) fail(DR_E_IO, fmt("cannot stat %s", f.path.c_str()));
    f.len = uint64_t(stt.st_size);
    if (f.kind == DR_FILE_JSON && f.len) {
      uint8_t last = 0;
      if (pread(fd, &last, 1, off_t(f.len - 1)) != 1) fail(DR_E_IO, fmt("read failed on %s", f.path.c_str()));
      ends_nl[i] = last == '\n';
    }
  }
  // layout: JSON in the given order, checkpoint parts by part number
  std::vector<size_t> js, cks;
  for (size_t i = 0; i < src.size(); ++i) (src[i].kind == DR_FILE_CHECKPOINT ? cks : js).push_back(i);
  std::stable_sort(cks.begin(), cks.end(), [&](size_t a, size_t b) { return src[a].part < src[b].part; });
  std::vector<uint64_t> host_off(src.size(), 0), region(src.size(), 0);
  uint64_t json_len = 0, added_nl = 0;
  for (size_t i : js) {
    const StageSrc& f = src[i];
    host_off[i] = json_len;
    region[i] = f.len + (ends_nl[i] ? 0 : 1);
    added_nl += ends_nl[i] ? 0 : 1;
    json_len += region[i];
    s->jfiles.push_back(JsonFileRec{f.version, host_off[i], region[i]});
    s->version = std::max(s->version, f.version);
  }
  uint64_t pq_len = 0;
  for (size_t i : cks) {
    const StageSrc& f = src[i];
    host_off[i] = pq_len;
    region[i] = (f.len + 15) & ~uint64_t(15);
    pq_len += region[i];
    CkPart p;
    p.off = host_off[i];
    p.len = f.len;
    p.rg_lo = f.rg_lo;
    p.rg_hi = f.rg_hi;
    s->parts.push_back(p);
    s->ck_version = f.version;
    s->version = std::max(s->version, f.version);
  }
  const uint64_t total = json_len + pq_len;
  const bool big = total >= (uint64_t(64) << 20);
  // DR_STAGE_PINNED=1: the host copy itself pinned (one DMA per chunk straight from it; pinning
  // 2.6 GB costs ~0.2 s per staging); default: pageable host copy + the context's pinned bounce slots
  const char* pin_env = std::getenv("DR_STAGE_PINNED");
  const bool pin = big && pin_env && std::atoi(pin_env) != 0;
  s->h_json.alloc(json_len, 64, pin);
  s->h_pq.alloc(pq_len, 64, pin);
  for (size_t i : js) if (!ends_nl[i]) s->h_json[host_off[i] + src[i].len] = '\n';
  for (size_t i : cks) memset(s->h_pq.data() + host_off[i] + src[i].len, 0, region[i] - src[i].len);
  s->d_json = DBuf<uint8_t>(ctx, json_len + 64);
  s->d_pq = DBuf<uint8_t>(ctx, pq_len + 64);
  const int nthreads = big ? std::max(1, std::min<int>(16, int(std::thread::hardware_concurrency()))) : 0;
  const bool bounce = big && !pin;
  if (bounce) ctx->ensure_bounce(size_t(2 * nthreads));
  const double t_layout = now_s();
  // chunks: (source, offset in the file, length); the last chunk of a file also carries the file's
  // region padding (added newline / alignment zeroes) in its H2D copy
  struct Chunk { size_t f; uint64_t off, len, h2d_len; };
  const uint64_t CH = bounce ? uint64_t(dr_ctx::kBounceBytes) - 16 : uint64_t(32) << 20;
  std::vector<Chunk> chunks;
  for (size_t i = 0; i < src.size(); ++i) {
    uint64_t o = 0;
    do {
      const uint64_t l = std::min(CH, src[i].len - o);
      const bool last = o + l >= src[i].len;
      chunks.push_back(Chunk{i, o, l, last ? region[i] - o : l});
      o += l;
    } while (o < src[i].len);
  }
  std::atomic<uint64_t> newlines{added_nl};
  std::atomic<uint64_t> h2d{0};
  std::atomic<int> err_flag{0};
  std::string err_msg;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<size_t> done;
  std::atomic<size_t> next{0};
  auto host_ptr = [&](const Chunk& c) {
    const size_t i = c.f;
    return (src[i].kind == DR_FILE_CHECKPOINT ? s->h_pq.data() : s->h_json.data()) + host_off[i] + c.off;
  };
  auto dev_ptr = [&](const Chunk& c) {
    return (src[c.f].kind == DR_FILE_CHECKPOINT ? s->d_pq.p : s->d_json.p) + host_off[c.f] + c.off;
  };
  auto set_err = [&](const std::string& m) {
    std::lock_guard<std::mutex> g(mu);
    if (!err_flag.exchange(1)) err_msg = m;
  };
  // read `c` into dst (pread or memcpy from the caller's bytes)
  auto read_chunk = [&](const Chunk& c, uint8_t* dst) {
    const StageSrc& f = src[c.f];
    if (f.data) {
      if (c.len) memcpy(dst, f.data + c.off, c.len);
      return true;
    }
    uint64_t got = 0;
    while (got < c.len) {
      const ssize_t r = pread(fdg.fds[c.f], dst + got, c.len - got, off_t(c.off + got));
      if (r <= 0) {
        set_err(fmt("read failed on %s", f.path.c_str()));
        return false;
      }
      got += uint64_t(r);
    }
    return true;
  };
  // bounce mode: every worker reads into its own two pinned slots in turn, copies the chunk to the
  // host copy and issues the slot's DMA itself (disjoint regions, so the order does not matter)
  auto work_bounce = [&](int t) {
    if (hipSetDevice(ctx->device) != hipSuccess) { set_err("hipSetDevice failed in a staging worker"); return; }
    int turn = 0;
    for (size_t k; (k = next++) < chunks.size() && !err_flag.load();) {
      const Chunk& c = chunks[k];
      const size_t slot = size_t(2 * t + turn);
      turn ^= 1;
      if (hipEventSynchronize(ctx->bounce_ev[slot]) != hipSuccess) { set_err("staging slot wait failed"); return; }
      uint8_t* b = ctx->bounce[slot];
      if (!read_chunk(c, b)) return;
      uint8_t* dst = host_ptr(c);
      const uint64_t pad = c.h2d_len - c.len;  // the file region's padding, already in the host copy
      if (pad) memcpy(b + c.len, dst + c.len, pad);
      memcpy(dst, b, c.len);
      if (src[c.f].kind == DR_FILE_JSON) newlines += uint64_t(std::count(b, b + c.len, uint8_t('\n')));
      if (c.h2d_len) {
        if (hipMemcpyAsync(dev_ptr(c), b, c.h2d_len, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
            hipEventRecord(ctx->bounce_ev[slot], ctx->stream) != hipSuccess) {
          set_err("staging H2D copy failed");
          return;
        }
        h2d += c.h2d_len;
      }
    }
  };
  // direct mode: read into the host copy; the calling thread issues the finished chunks' copies
  auto work_direct = [&] {
    for (size_t k; (k = next++) < chunks.size();) {
      const Chunk& c = chunks[k];
      uint8_t* dst = host_ptr(c);
      if (!err_flag.load() && read_chunk(c, dst) && src[c.f].kind == DR_FILE_JSON)
        newlines += uint64_t(std::count(dst, dst + c.len, uint8_t('\n')));
      std::lock_guard<std::mutex> g(mu);
      done.push_back(k);
      cv.notify_one();
    }
  };
  std::vector<std::thread> pool;
  if (bounce) {
    for (int t = 0; t < nthreads; ++t) pool.emplace_back(work_bounce, t);
    for (auto& t : pool) t.join();
  } else {
    for (int t = 0; t < nthreads; ++t) pool.emplace_back(work_direct);
    if (!nthreads) work_direct();
    size_t issued = 0;
    try {
      while (issued < chunks.size()) {
        std::vector<size_t> batch;
        {
          std::unique_lock<std::mutex> g(mu);
          cv.wait(g, [&] { return !done.empty(); });
          batch.swap(done);
        }
        for (size_t k : batch) {
          const Chunk& c = chunks[k];
          if (c.h2d_len && !err_flag.load())
            HIP_OK(hipMemcpyAsync(dev_ptr(c), host_ptr(c), c.h2d_len, hipMemcpyHostToDevice, ctx->stream));
          h2d += c.h2d_len;
          ++issued;
        }
      }
    } catch (...) {
      err_flag = 1;  // the workers stop reading; join them before the buffers go away
      for (auto& t : pool) t.join();
      (void)hipStreamSynchronize(ctx->stream);
      throw;
    }
    for (auto& t : pool) t.join();
  }
  if (err_flag.load()) {
    (void)hipStreamSynchronize(ctx->stream);
    fail(DR_E_IO, err_msg);
  }
  HIP_OK(hipMemcpyAsync(s->d_json.p + json_len, s->h_json.data() + json_len, 64, hipMemcpyHostToDevice, ctx->stream));
  HIP_OK(hipMemcpyAsync(s->d_pq.p + pq_len, s->h_pq.data() + pq_len, 64, hipMemcpyHostToDevice, ctx->stream));
  s->json_lines = newlines.load();
  const double t_read = now_s();
  plan_checkpoint(*s);
  const double t_plan = now_s();
  HIP_OK(hipStreamSynchronize(ctx->stream));
  if (dbg)
    std::fprintf(stderr, "stage: %.1f MB (%.1f MB H2D, %s, %d threads, %zu chunks): layout %.3f s, read+h2d issue %.3f s, "
                 "plan %.3f s, h2d drain %.3f s, total %.3f s\n", double(total) / 1e6, double(h2d.load()) / 1e6,
                 s->h_json.pinned ? "pinned" : bounce ? "pageable + pinned bounce" : "pageable", nthreads, chunks.size(), t_layout - t0, t_read - t_layout, t_plan - t_read, now_s() - t_plan, now_s() - t0);
  return s;
}

static std::shared_ptr<StagedData> stage_files(dr_ctx* ctx, const dr_file* files, int32_t nfiles,
                                               const int32_t* rg_lo = nullptr, const int32_t* rg_hi = nullptr) {
  std::vector<StageSrc> src(size_t(std::max(nfiles, 0)));
  for (int32_t i = 0; i < nfiles; ++i) {
    src[size_t(i)].version = files[i].version;
    src[size_t(i)].kind = files[i].kind;
    src[size_t(i)].part = files[i].part;
    src[size_t(i)].data = files[i].data;
    src[size_t(i)].len = files[i].len;
    if (rg_lo) {
      src[size_t(i)].rg_lo = rg_lo[i];
      src[size_t(i)].rg_hi = rg_hi[i];
    }
  }
  return stage_sources(ctx, src);
}

// ---------------------------------------------------------------------------------------------------
// replay
// ---------------------------------------------------------------------------------------------------
// Buckets average <= 2048 file actions (the reduce keeps up to 3072 per pass in its 4096-slot LDS table), capped by the scatter's
// LDS cursors; larger buckets are reduced in sub-passes.
static int bucket_bits_for(const dr_ctx* ctx, uint64_t n) {
  int bits = 0;
  while ((n >> bits) > 2048 && bits < int(part_max_bucket_bits())) ++bits;
  // DR_OPT_BUCKET_BITS: fewer, larger buckets (the reducer's sub-pass paths on a small table)
  if (ctx->opt.bucket_bits >= 0) bits = std::min<int>(bits, int(ctx->opt.bucket_bits));
  return bits;
}

static void reduce_nonfile(dr_state& st, std::vector<NonFileAction>& acts, bool validate) {
  // InMemoryLogReplay.append for the non-path actions: last protocol, last metaData, last txn per
  // appId (D/actions/InMemoryLogReplay.scala:47-53).
  std::sort(acts.begin(), acts.end(), [](const NonFileAction& a, const NonFileAction& b) { return a.order < b.order; });
  const NonFileAction* prot = nullptr;
  const NonFileAction* meta = nullptr;
  std::vector<std::string> app_order;
  std::map<std::string, const NonFileAction*> txns;
  for (const NonFileAction& a : acts) {
    if (a.kind == 5) prot = &a;
    else if (a.kind == 3) meta = &a;
    else if (a.kind == 4) {
      const JVal* id = a.val->get("appId");
      std::string k = id && id->t == JVal::STR ? id->s : std::string();
      if (!txns.count(k)) app_order.push_back(k);
      txns[k] = &a;
    }
  }
  st.nonfile.clear();
  std::string out;
  if (prot) { st.nonfile.push_back(*prot); out += prot->json + "\n"; }
  if (meta) { st.nonfile.push_back(*meta); out += meta->json + "\n"; }
  for (auto& k : app_order) { st.nonfile.push_back(*txns[k]); out += txns[k]->json + "\n"; }
  st.nonfile_json = out;
  st.counts.num_protocol = prot ? 1 : 0;
  st.counts.num_metadata = meta ? 1 : 0;
  st.counts.num_set_transactions = int64_t(txns.size());
  if (validate && !prot)  // D/Snapshot.scala:154-162
    fail(DR_E_MISSING_PROTOCOL, action_not_found("protocol", st.counts.version));
  if (validate && !meta)  // D/Snapshot.scala:163-171
    fail(DR_E_MISSING_METADATA, action_not_found("metadata", st.counts.version));
}

// What parse_launch leaves for parse_finish: the device counters (0 special count, 1 special bytes,
// 2 non-file lines, 3 malformed lines, 4 canonicalisation arena fill, 5 lines deferred to the
// General walker, 7 checkpoint decode error) and the non-file line list, read back after the
// caller has queued the rest of its kernels.
struct ParsePending {
  DBuf<uint64_t> counters;
  DBuf<uint64_t> nonfile;   // {line, byte offset} pairs
  uint64_t R = 0, nlines = 0;
  uint64_t canon_cap = 0;   // arena bytes given to k_canon (0: no canonicalisation launched)
  const void* canon_arena = nullptr;  // that arena (st->arenas' last entry when launched)
  bool canonicalize = false;
  bool canon_sized = false; // the arena was sized from the counters (exact), not from a hint
  size_t pin_at = 0;        // where its words land in ctx->pinned()
  // the small tail's deferred post-parse launch (parse_launch's defer_tail): k_tail_post's work,
  // run by launch_apply_small or parse_flush_tail; every buffer tail_ja points at stays alive for it
  // (nl, hard, and off2's: a block released here is handed to the next allocation while the deferred
  // launch, queued after that allocation's users, still writes it)
  bool tail_deferred = false;
  bool parse_deferred = false;  // ... and the line walk too (launch_apply_commit / parse_flush_tail)
  JsonParseArgs tail_ja{};
  CanonArgs tail_cg{};
  DBuf<uint64_t> nl, hard, off2;
};
constexpr size_t kPinNonfile = 1024;  // non-file entries (pairs) read back with the counters

// K1 + K2 + canonicalisation, queued on the context's stream: fills st's per-action arrays
// (checkpoint rows first, then JSON lines). On the first replay of a segment the special-path
// counters are read back before k_canon (the arena is sized exactly); later replays size the arena
// from the segment's last need and queue K3/K4 without a round trip.
static ParsePending parse_launch(dr_ctx* ctx, const std::shared_ptr<StagedData>& sp, dr_state* st,
                                 bool canonicalize, bool defer_tail = false) {
  StagedData& s = *sp;
  hipStream_t stream = ctx->stream;
  ParsePending pp;
  // ---- K1a: newline index ----
  const uint64_t json_len = s.h_json.size();
  const uint64_t nbj = json_num_blocks(json_len);
  const bool one_block = nbj == 1;  // a streamed commit: index, placement and counter reset in one launch
  // K1 beside K2 on two streams: a checkpoint to decode and a JSON part of several index blocks
  // (r04: 10.43 -> 10.33 ms per config-3 step); small segments keep one stream and their fused paths
  const bool overlap = ctx->opt.overlap != 0 && s.ck_rows > 0 && nbj > 1;
  DBuf<uint32_t> jcounts(ctx, one_block ? 1 : nbj + 1);
  DBuf<uint64_t> joff(ctx, nbj + 1);
  DBuf<uint8_t> scratch(ctx, scan_scratch_for(nbj));
  DBuf<uint16_t> jslots(ctx, one_block ? 1 : json_slot_entries(json_len));
  // the line count is known from staging (no read-back between the index and the parse)
  const uint64_t nlines = nbj ? s.json_lines : 0;
  DBuf<uint64_t> nl(ctx, nlines);
  DBuf<uint64_t> counters(ctx, 8);  // 0 special count, 1 special bytes, 2 nonfile count, 3 errors, 4 canon fill,
                                     // 5 lines deferred to the General walker, 7 checkpoint decode error
  // a segment of one wave: the parse kernel indexes its newlines and clears the counters itself
  const bool fuse1 = one_block && s.json_lines && s.json_lines <= JSON_FUSE_MAX_LINES && !overlap &&
                     !std::getenv("DR_CHECK_LINES");
  if (one_block) {
    if (!fuse1) launch_json_index1(s.d_json.p, json_len, nl.p, joff.p, counters.p, 8, stream);
  } else {
    counters.zero(stream);
    if (nbj) {
      launch_json_index(s.d_json.p, json_len, jcounts.p, jslots.p, stream);
      launch_scan_u32(jcounts.p, joff.p, nbj, ss(scratch), stream);
    }
  }
  if (nbj && std::getenv("DR_CHECK_LINES") && d2h_one(joff.p + nbj, stream) != nlines)
    fail(DR_E_INTERNAL, "device newline count differs from the staged count");
  const uint64_t R = s.ck_rows, N = R + nlines;
  st->n_actions = N;
  st->kind = DBuf<uint8_t>(ctx, N);
  st->flags = DBuf<uint8_t>(ctx, N);
  st->key = DBuf<uint64_t>(ctx, N);
  st->path_ptr = DBuf<uint64_t>(ctx, N);
  st->path_len = DBuf<uint32_t>(ctx, N);
  st->size = DBuf<int64_t>(ctx, N);
  st->delts = DBuf<int64_t>(ctx, N);
  st->src_off = DBuf<uint64_t>(ctx, N);
  st->src_len = DBuf<uint32_t>(ctx, N);
  st->path_ref = DBuf<uint64_t>(ctx, N);
  DBuf<uint64_t> nonfile(ctx, 2 * nlines);
  ActionArrays act{st->kind.p, st->flags.p, st->key.p, st->path_ptr.p, st->path_len.p, st->size.p, st->delts.p,
                   st->src_off.p, st->src_len.p, st->path_ref.p};
  DBuf<uint64_t> hard(ctx, nlines);
  // For a segment with a checkpoint and a multi-block JSON part (`overlap`, on unless
  // DR_OPT_OVERLAP = 0), K1's line parsing runs on stream2 beside the checkpoint decode below (r04:
  // 10.43 -> 10.33 ms per config-3 step, k_snap_exec's time unchanged); stream waits for it before
  // anything reads the action arrays. The guard joins stream2 before any buffer it uses can be
  // released. Small segments run on one stream (and take the fused small-segment paths).
  struct Overlap {
    dr_ctx* c;
    hipEvent_t fork = nullptr, done = nullptr;
    ~Overlap() {
      (void)hipStreamSynchronize(c->stream2);
      if (fork) (void)hipEventDestroy(fork);
      if (done) (void)hipEventDestroy(done);
    }
  } ov{ctx};
  // a small commit-only segment (a streamed commit): the deferred lines and the canonicalisation
  // run as one single-workgroup launch at the canonicalisation point (k_tail_post)
  const bool tail_post = canonicalize && s.ck_rows == 0 && nlines && nlines <= JSON_TAIL_POST_MAX && !overlap;
  JsonParseArgs ja{};
  if (nlines) {
    hipStream_t s2 = overlap ? ctx->stream2 : stream;
    DR_STAGE("parse.json", s2);
    if (overlap) {
      HIP_OK(hipEventCreateWithFlags(&ov.fork, hipEventDisableTiming));
      HIP_OK(hipEventRecord(ov.fork, stream));
      HIP_OK(hipStreamWaitEvent(s2, ov.fork, 0));
    }
    if (!one_block) launch_json_place(s.d_json.p, json_len, jcounts.p, joff.p, jslots.p, nl.p, s2);
    ja = JsonParseArgs{s.d_json.p, nl.p, nlines, R, act.kind, act.flags, act.key, act.path_ptr, act.path_len,
                     act.size, act.delts, act.src_off, act.src_len, counters.p + 0, counters.p + 1, counters.p + 2,
                     nonfile.p, nlines, counters.p + 3, hard.p,
                     reinterpret_cast<unsigned long long*>(counters.p + 5)};
    ja.buf_len = json_len;
    ja.force_staged = ctx->opt.json_staged ? 1u : 0u;
    ja.path_ref = act.path_ref;
    if (fuse1) {
      ja.zero = counters.p;
      ja.nzero = 8;
      ja.off2 = joff.p;
      ja.nl_out = nl.p;
    }
    static unsigned long long* phase = nullptr;  // DR_JSON_PHASES=1: staged-kernel phase clocks
    static uint64_t phase_calls = 0;
    if (std::getenv("DR_JSON_PHASES")) {
      if (!phase) {
        HIP_OK(hipMalloc(&phase, 16 * sizeof(unsigned long long)));
        HIP_OK(hipMemset(phase, 0, 16 * sizeof(unsigned long long)));
      }
      ja.phase = phase;
      if (++phase_calls % 200 == 0) {
        unsigned long long h[16];
        HIP_OK(hipMemcpy(h, phase, sizeof(h), hipMemcpyDeviceToHost));
        if (h[4])
          std::fprintf(stderr, "k_json_lines<true> clocks per wave: stage %.0f tape %.0f walk %.0f (rounds %.0f, first round %.0f; tape scan %.0f emit %.0f) (%llu waves)\n",
                       double(h[0]) / double(h[4]), double(h[1]) / double(h[4]), double(h[2]) / double(h[4]),
                       double(h[3]) / double(h[4]), double(h[5]) / double(h[4]), double(h[6]) / double(h[4]),
                       double(h[7]) / double(h[4]), h[4]);
        if (h[8] + h[9] + h[10] + h[11])
          std::fprintf(stderr, "k_apply_commit apply clocks: post-parse %.0f append %.0f touch %.0f delta %.0f\n",
                       double(h[8]) / double(h[4]), double(h[9]) / double(h[4]), double(h[10]) / double(h[4]),
                       double(h[11]) / double(h[4]));
        if (h[12] + h[13])
          std::fprintf(stderr, "k_apply_commit clocks: stage %.0f newlines %.0f walk %.0f apply %.0f expiry %.0f readback %.0f\n",
                       double(h[0]) / double(h[4]), double(h[1]) / double(h[4]), double(h[2]) / double(h[4]),
                       double(h[6]) / double(h[4]), double(h[12]) / double(h[4]), double(h[13]) / double(h[4]));
      }
    }
    // an applied streamed commit: the walk runs in the apply's one launch (launch_apply_commit)
    if (defer_tail && fuse1 && tail_post) pp.parse_deferred = true;
    else launch_json_parse(ja, s2);
    if (!tail_post) launch_json_hard(ja, s2);
    if (overlap) {
      HIP_OK(hipEventCreateWithFlags(&ov.done, hipEventDisableTiming));
      HIP_OK(hipEventRecord(ov.done, s2));
    }
  }
  // ---- K2: checkpoint ----
  DBuf<uint8_t> cdefs;  // the hot columns' definition levels, R bytes each, zeroed in one fill
  DBuf<int64_t> cival[HC_N];
  DBuf<uint64_t> csptr[HC_N];
  DBuf<uint32_t> cslen[HC_N];
  DBuf<uint64_t> dict_ptr;
  DBuf<uint32_t> dict_len, pq_err;
  if (R) {
    DR_STAGE("decode.checkpoint", stream);
    ParquetArgs pa{};
    pa.ncols = HC_N;
    cdefs = DBuf<uint8_t>(ctx, uint64_t(HC_N) * R);
    cdefs.zero(stream);
    for (int c = 0; c < HC_N; ++c) {
      if (c == HC_ADD_PATH || c == HC_RM_PATH) {
        csptr[c] = DBuf<uint64_t>(ctx, R);
        cslen[c] = DBuf<uint32_t>(ctx, R);
      } else {
        cival[c] = DBuf<int64_t>(ctx, R);
      }
      pa.cols[c] = FlatColumn{cdefs.p + uint64_t(c) * R, nullptr, cival[c].p, csptr[c].p, cslen[c].p};
    }
    pq_err = DBuf<uint32_t>(ctx, 1);
    pq_err.zero(stream);
    decode_pages(ctx, s.hot, pa, dict_ptr, dict_len, pq_err, scratch.p);
    CkptAssembleArgs ca{};
    ca.add_path = pa.cols[HC_ADD_PATH];
    ca.add_size = pa.cols[HC_ADD_SIZE];
    ca.rm_path = pa.cols[HC_RM_PATH];
    ca.rm_delts = pa.cols[HC_RM_DELTS];
    ca.add_def = s.add_def;
    ca.rm_def = s.rm_def;
    ca.add_path_max = s.max_def[HC_ADD_PATH];
    ca.add_size_max = s.has_col[HC_ADD_SIZE] ? s.max_def[HC_ADD_SIZE] : 255;
    ca.rm_path_max = s.max_def[HC_RM_PATH];
    ca.rm_delts_max = s.has_col[HC_RM_DELTS] ? s.max_def[HC_RM_DELTS] : 255;
    ca.has_rm = s.has_col[HC_RM_PATH] ? 1 : 0;
    ca.nrows = R;
    ca.row_base = 0;
    ca.act = act;
    ca.special_count = counters.p + 0;
    ca.special_bytes = counters.p + 1;
    launch_ckpt_assemble(ca, stream);
  }
  if (ov.done) {
    HIP_OK(hipStreamWaitEvent(stream, ov.done, 0));
  }
  // the checkpoint decoder's error code rides in counters[7]: one read-back for both
  if (R) HIP_OK(hipMemcpyAsync(counters.p + 7, pq_err.p, sizeof(uint32_t), hipMemcpyDeviceToDevice, stream));
  // ---- canonicalisation of special paths ----
  if (canonicalize) {
    DR_STAGE("canonicalize", stream);
    int64_t hint = s.canon_need.load();
    // DR_OPT_CANON_HINT=<bytes> stands in for the first replay's exact sizing (an undersized hint
    // exercises the detect-and-redo path)
    if (hint < 0 && ctx->opt.canon_hint >= 0) hint = ctx->opt.canon_hint;
    uint64_t cap = 0;
    if (hint < 0 && R == 0 && json_len <= (uint64_t(64) << 20)) {
      // a commit-only segment (an applied tail, a streamed commit): the bound from its bytes -- every
      // special path is a line's path string, so sum(len + 8) <= bytes + 8 lines -- needs no read-back
      cap = 2 * json_len + 80 * nlines + 64;
      pp.canon_sized = true;
    } else if (hint < 0) {  // first replay of the segment: the exact arena from the counters
      const std::vector<uint64_t> cnt = d2h(counters.p, 2, stream);
      cap = cnt[0] ? cnt[1] * 2 + 64 * cnt[0] + 64 : 0;
      pp.canon_sized = true;
    } else {
      cap = uint64_t(hint);
    }
    if (cap) {
      st->arenas.push_back(std::make_shared<DBuf<uint8_t>>(ctx, cap));
      pp.canon_arena = st->arenas.back()->p;
      CanonArgs cg{act, N, st->arenas.back()->p, cap, counters.p + 4};
      if (tail_post && defer_tail) pp.tail_deferred = true, pp.tail_ja = ja, pp.tail_cg = cg;
      else if (tail_post) launch_tail_post(ja, cg, stream);
      else launch_canon(cg, stream);
    } else if (tail_post) {
      if (defer_tail) pp.tail_deferred = true, pp.tail_ja = ja, pp.tail_cg = CanonArgs{act, 0, nullptr, 0, counters.p + 4};
      else launch_json_hard(ja, stream);
    }
    pp.canon_cap = cap;
    pp.canonicalize = true;
  }
  pp.counters = std::move(counters);
  pp.nonfile = std::move(nonfile);
  if (pp.tail_deferred) {
    pp.nl = std::move(nl);
    pp.hard = std::move(hard);
    pp.off2 = std::move(joff);  // the fused walk's line count (fuse1: ja.off2)
  }
  pp.R = R;
  pp.nlines = nlines;
  return pp;
}

// Queues the copies of parse_launch's counters and the first non-file entries into the pinned
// words at `at` (no sync).
// With `rb`, the spans are added to a launch_readback instead of queued as copies.
static size_t parse_queue_readback(dr_ctx* ctx, ParsePending& pp, size_t at, ReadbackArgs* rb = nullptr,
                                   int* nrb = nullptr) {
  uint64_t* h = ctx->pinned() + at;
  pp.pin_at = at;
  const uint64_t k = std::min<uint64_t>(pp.nlines, kPinNonfile);
  if (rb) {
    uint64_t* d = ctx->pinned_dev() + at;
    rb->src[*nrb] = pp.counters.p, rb->dst[*nrb] = d, rb->n[(*nrb)++] = 8;
    if (k) rb->src[*nrb] = pp.nonfile.p, rb->dst[*nrb] = d + 8, rb->n[(*nrb)++] = uint32_t(2 * k);
  } else {
    HIP_OK(hipMemcpyAsync(h, pp.counters.p, 8 * sizeof(uint64_t), hipMemcpyDeviceToHost, ctx->stream));
    if (k) HIP_OK(hipMemcpyAsync(h + 8, pp.nonfile.p, 2 * k * sizeof(uint64_t), hipMemcpyDeviceToHost, ctx->stream));
  }
  return at + 8 + 2 * kPinNonfile;
}

// Launches a deferred post-parse step that no fused apply took.
static void parse_flush_tail(dr_ctx* ctx, ParsePending& pp) {
  if (!pp.tail_deferred) return;
  if (pp.parse_deferred) launch_json_parse(pp.tail_ja, ctx->stream);
  pp.parse_deferred = false;
  if (pp.tail_cg.n) launch_tail_post(pp.tail_ja, pp.tail_cg, ctx->stream);
  else launch_json_hard(pp.tail_ja, ctx->stream);
  pp.tail_deferred = false;
}

// After the stream has drained: error codes, counters and the non-file actions (protocol /
// metaData / txn, parsed on the host: checkpoint rows first, then JSON lines in order). Returns
// false when the canonicalisation arena sized from the segment's hint was too small (the caller
// redoes the replay; the hint now holds the exact need).
static bool parse_finish(dr_ctx* ctx, const std::shared_ptr<StagedData>& sp, dr_state* st, ParsePending& pp,
                         std::vector<NonFileAction>& nf) {
  StagedData& s = *sp;
  const uint64_t* cnt = ctx->pinned() + pp.pin_at;
  const uint64_t R = pp.R, nlines = pp.nlines, json_len = s.h_json.size();
  if (R && cnt[7] != 0) fail(DR_E_PARQUET, fmt("device checkpoint decode failed (code %u)", unsigned(cnt[7])));
  st->counts.malformed_lines = int64_t(cnt[3]);
  if (pp.canonicalize) {
    const uint64_t need = cnt[0] ? cnt[1] * 2 + 64 * cnt[0] + 64 : 0;
    if (!pp.canon_sized && (need > pp.canon_cap || cnt[4] > pp.canon_cap)) {
      s.canon_need.store(int64_t(need));
      return false;
    }
    s.canon_need.store(int64_t(need));
    // no special path: nothing points into the arena sized from the segment's bytes (a commit-only
    // segment's bound is ~2x its JSON) -- it is not kept for the life of the state
    if (cnt[0] == 0 && pp.canon_arena && !st->arenas.empty() && st->arenas.back()->p == pp.canon_arena)
      st->arenas.pop_back();
  }
  nf = s.ck_nonfile;
  const uint64_t nnf = std::min<uint64_t>(cnt[2], nlines);
  if (nnf) {
    std::vector<std::pair<uint64_t, uint64_t>> lines(nnf);  // (line, byte offset)
    if (nnf <= kPinNonfile) {
      for (uint64_t k = 0; k < nnf; ++k) lines[k] = {cnt[8 + 2 * k], cnt[8 + 2 * k + 1]};
    } else {
      const std::vector<uint64_t> all = d2h(pp.nonfile.p, 2 * nnf, ctx->stream);
      for (uint64_t k = 0; k < nnf; ++k) lines[k] = {all[2 * k], all[2 * k + 1]};
    }
    std::sort(lines.begin(), lines.end());
    for (uint64_t k = 0; k < nnf; ++k) {
      const uint64_t li = lines[k].first;
      const uint64_t b = lines[k].second;
      uint64_t e = b;
      while (e < json_len && s.h_json[e] != '\n') ++e;
      JVal v;
      std::string perr;
      if (!json_parse(reinterpret_cast<const char*>(s.h_json.data() + b), e - b, &v, &perr) || v.t != JVal::OBJ)
        continue;  // malformed non-file line: PERMISSIVE null row
      // unwrap priority among non-file kinds: metaData > txn > protocol
      const char* names[3] = {"metaData", "txn", "protocol"};
      const int kinds[3] = {3, 4, 5};
      for (int k2 = 0; k2 < 3; ++k2) {
        const JVal* x = v.get(names[k2]);
        if (x && x->t != JVal::NUL) {
          NonFileAction a;
          a.kind = kinds[k2];
          a.order = R + li;
          a.val = std::make_shared<const JVal>(*x);
          a.json = std::string("{\"") + names[k2] + "\":" + json_dump(*x) + "}";
          nf.push_back(std::move(a));
          break;
        }
      }
    }
  }
  return true;
}

// K1 + K2 + canonicalisation with the counters read back at once (callers that use the arrays on
// the host right away). An arena hint that proved too small redoes the parse with the exact size.
static void parse_actions(dr_ctx* ctx, const std::shared_ptr<StagedData>& sp, dr_state* st,
                          std::vector<NonFileAction>& nf, bool canonicalize = true) {
  for (;;) {
    ParsePending pp = parse_launch(ctx, sp, st, canonicalize);
    parse_queue_readback(ctx, pp, 0);
    HIP_OK(hipStreamSynchronize(ctx->stream));
    if (parse_finish(ctx, sp, st, pp, nf)) return;
    st->arenas.clear();
  }
}

// K3 (hash partition) + K4 (per-bucket last-writer-wins, retention) + compaction over st's action
// arrays, queued without a host round trip; reduce_finish reads the counters back.
struct ReducePending {
  DBuf<unsigned long long> totals;
  DBuf<unsigned long long> vstats;  // timed replays: the verifier's {pairs, path bytes}
  size_t pin_at = 0;
};

static ReducePending reduce_launch(dr_ctx* ctx, dr_state* st, int64_t cutoff, uint32_t flags = 0) {
  hipStream_t stream = ctx->stream;
  const uint64_t N = st->n_actions;
  // ---- K3: partition by hash bucket ----
  if (N >= (uint64_t(1) << 30)) fail(DR_E_UNSUPPORTED, "more than 2^30 actions in one replay shard");
  const int bits = bucket_bits_for(ctx, N);
  const uint32_t nb = 1u << bits;
  const uint32_t nt = part_tiles(N);
  const uint64_t ncell = uint64_t(nb) * nt;
  DBuf<uint32_t> tcnt(ctx, ncell);
  DBuf<uint64_t> toff(ctx, ncell + 1), boff(ctx, nb + 1);
  DBuf<uint8_t> pscratch(ctx, scan_scratch_for(ncell));
  // packed path references in action order for k_bucket_verify: written by the producers beside
  // path_ptr / path_len (parse_launch's states), else packed here by k_bucket_hist
  const bool have_ref = st->path_ref.p && st->path_ref.n >= N;
  DBuf<uint64_t> pref_own;
  if (!have_ref) pref_own = DBuf<uint64_t>(ctx, N);
  uint64_t* pref = have_ref ? st->path_ref.p : pref_own.p;
  PartitionArgs pa{st->kind.p, st->flags.p, st->key.p, st->size.p, st->delts.p, N, cutoff, bits, nt,
                   tcnt.p, toff.p, nullptr, have_ref ? nullptr : st->path_ptr.p, st->path_len.p, pref};
  DBuf<PartRec> rec(ctx, N);
  pa.rec = rec.p;
  {
    DR_STAGE("hash.partition", stream);
    launch_bucket_hist(pa, stream);
    launch_scan_u32(tcnt.p, toff.p, ncell, ss(pscratch), stream);
    launch_bucket_offsets(toff.p, nb, nt, boff.p, stream);
    launch_bucket_scatter(pa, stream);
  }
  // ---- K3 refinement (large replays): buckets of more than 2048 records on average are split by the
  // next key bits, so that K4 reduces each in one pass (k_bucket_split; DR_OPT_SPLIT = 0 turns it off) ----
  int sbits = 0;
  if (ctx->opt.split)
    while ((N >> (bits + sbits)) > 2048 && sbits < 6) ++sbits;
  DBuf<PartRec> rec2;
  DBuf<uint64_t> boff2;
  const PartRec* krec = rec.p;
  const uint64_t* kboff = boff.p;
  if (sbits) {
    DR_STAGE("hash.split", stream);
    rec2 = DBuf<PartRec>(ctx, N);
    boff2 = DBuf<uint64_t>(ctx, (uint64_t(nb) << sbits) + 1);
    launch_bucket_split(SplitArgs{rec.p, boff.p, bits, sbits, rec2.p, boff2.p}, nb, stream);
    krec = rec2.p;
    kboff = boff2.p;
  }
  const uint32_t knb = nb << sbits;  // K4's buckets
  const int kbits = bits + sbits;
  // ---- K4: per-bucket last-writer-wins ----
  DBuf<uint32_t> olive(ctx, N), otomb(ctx, N), lcount(ctx, knb), tcount(ctx, knb), pcount(ctx, knb), rlist(ctx, knb),
      xlist(ctx, knb);
  DBuf<uint2> opair(ctx, N);
  DBuf<unsigned long long> totals(ctx, 8), bstats(ctx, uint64_t(knb) * 5);
  totals.zero(stream);
  ReduceArgs ra{krec, kboff, knb, kbits, st->size.p, st->path_ptr.p, st->path_len.p, olive.p, otomb.p, opair.p, pref,
                lcount.p, tcount.p, pcount.p, totals.p, rlist.p, xlist.p, bstats.p, nullptr};
  // a timed replay (per-kernel mode) also counts the verifier's pairs and path bytes: its own byte
  // model beside the 69 B/action budget (bench.py "verify")
  DBuf<unsigned long long> vstats;
  if (ctx->timing && ctx->timing_only.empty()) {
    vstats = DBuf<unsigned long long>(ctx, 2 * uint64_t(knb));
    vstats.zero(stream);
    ra.vstats = vstats.p;
  }
  std::unique_ptr<StageRange> reduce_range(new StageRange("reduce", stream));
  auto upload_list = [&](const std::vector<uint32_t>& v) {
    DBuf<uint32_t> d(ctx, v.size());
    HIP_OK(hipMemcpyAsync(d.p, v.data(), v.size() * 4, hipMemcpyHostToDevice, stream));
    return d;
  };
  if (flags & (DR_FLAG_EXACT_REDUCE | DR_FLAG_REDUCE64)) {  // test hooks: force the fallback reducers
    std::vector<uint32_t> all(knb);
    for (uint32_t b = 0; b < knb; ++b) all[b] = b;
    DBuf<uint32_t> d = upload_list(all);
    if (flags & DR_FLAG_EXACT_REDUCE) {
      launch_bucket_exact(ra, d.p, knb, stream);
    } else {
      launch_bucket_reduce64(ra, d.p, knb, stream);
      launch_bucket_exact(ra, xlist.p, knb, stream, totals.p + 4);
    }
  } else {
    launch_bucket_reduce(ra, stream);
    launch_bucket_verify(ra, stream);  // byte verification of every merged pair
    // the fallbacks read their bucket lists' lengths on the device (no host round trip)
    launch_bucket_reduce64(ra, rlist.p, knb, stream, totals.p + 3);
    launch_bucket_exact(ra, xlist.p, knb, stream, totals.p + 4);
    if (std::getenv("DR_REDUCE_DEBUG")) {
      const std::vector<unsigned long long> t = d2h(totals.p, 8, stream);
      std::vector<uint64_t> bo = d2h(kboff, knb + 1, stream);
      std::vector<uint32_t> rl = d2h(rlist.p, size_t(std::min<unsigned long long>(t[3], knb)), stream);
      std::fprintf(stderr, "reduce: %u buckets (%d split bits), %llu to the 64-bit reducer, %llu to the exact one; sizes:",
                   knb, sbits, t[3], t[4]);
      for (uint32_t b : rl) std::fprintf(stderr, " %llu", (unsigned long long)(bo[b + 1] - bo[b]));
      std::fprintf(stderr, "\n");
    }
  }
  reduce_range.reset();
  DR_STAGE("compact", stream);
  // ---- compaction (survivor lists sized to the bound; the counts come back once, at the end) ----
  DBuf<uint64_t> loff(ctx, knb + 1), tmoff(ctx, knb + 1);
  if (knb > 16384) {
    // a split replay's 2^16+ buckets: one workgroup walking 64+ buckets per thread took 0.23 ms on
    // config 4; the grid-wide scans and a separate sum instead
    DBuf<uint8_t> sscr(ctx, scan_scratch_for(knb));
    launch_scan_u32(lcount.p, loff.p, knb, ss(sscr), stream);
    launch_scan_u32(tcount.p, tmoff.p, knb, ss(sscr), stream);
    launch_sum_stats(ra, stream);
  } else {
    launch_survivor_scan(lcount.p, tcount.p, knb, loff.p, tmoff.p, stream, bstats.p, totals.p);  // + the sums
  }
  st->live = DBuf<uint32_t>(ctx, N);
  st->tomb = DBuf<uint32_t>(ctx, N);
  launch_compact2(CompactArgs{olive.p, kboff, lcount.p, loff.p, knb, st->live.p},
                  CompactArgs{otomb.p, kboff, tcount.p, tmoff.p, knb, st->tomb.p}, stream);
  HIP_OK(hipMemcpyAsync(totals.p + 7, boff.p + nb, 8, hipMemcpyDeviceToDevice, stream));
  ReducePending rp;
  rp.totals = std::move(totals);
  rp.vstats = std::move(vstats);
  return rp;
}

static size_t reduce_queue_readback(dr_ctx* ctx, ReducePending& rp, size_t at) {
  rp.pin_at = at;
  HIP_OK(hipMemcpyAsync(ctx->pinned() + at, rp.totals.p, 8 * sizeof(uint64_t), hipMemcpyDeviceToHost, ctx->stream));
  return at + 8;
}

// After the stream has drained: the survivor counts and computedState counters.
static void reduce_finish(dr_ctx* ctx, dr_state* st, const ReducePending& rp) {
  if (rp.vstats.p) {  // (timed replays) reported with the kernel times: "stat.verify_pairs", "stat.verify_path_bytes"
    const std::vector<unsigned long long> v = d2h(rp.vstats.p, rp.vstats.n, ctx->stream);
    double pairs = 0, bytes = 0;
    for (size_t k = 0; k + 1 < v.size(); k += 2) {
      pairs += double(v[k]);
      bytes += double(v[k + 1]);
    }
    ctx->stats.emplace_back("stat.verify_pairs", pairs);
    ctx->stats.emplace_back("stat.verify_path_bytes", bytes);
  }
  const uint64_t* tot = ctx->pinned() + rp.pin_at;
  const uint64_t N = st->n_actions;
  const uint64_t n_file_actions = tot[7];
  st->n_live = tot[0];
  st->n_tomb = tot[2];
  st->counts.num_files = int64_t(tot[0]);
  st->counts.size_in_bytes = int64_t(tot[1]);
  st->counts.num_removes = int64_t(tot[2]);
  st->counts.live_key_sum = tot[5];
  st->counts.tomb_key_sum = tot[6];
  st->counts.num_actions = int64_t(N);
  st->counts.num_file_actions = int64_t(n_file_actions);
}

static void reduce_actions(dr_ctx* ctx, dr_state* st, int64_t cutoff, uint32_t flags = 0) {
  ReducePending rp = reduce_launch(ctx, st, cutoff, flags);
  reduce_queue_readback(ctx, rp, 0);
  HIP_OK(hipStreamSynchronize(ctx->stream));
  reduce_finish(ctx, st, rp);
}

static dr_state* new_state(dr_ctx* ctx, const std::shared_ptr<StagedData>& sp) {
  auto st = std::make_unique<dr_state>();
  st->ctx = ctx;
  st->staged = sp;
  if (sp) st->sources.push_back(sp);
  st->counts.version = sp ? sp->version : -1;
  return st.release();
}

// ---------------------------------------------------------------------------------------------------
// incremental tail apply (the reference rebuilds the state from the last
// checkpoint instead, D/SnapshotManagement.scala:286-330)
// ---------------------------------------------------------------------------------------------------
static IndexArgs ix_args(IncChain& c) {
  IndexArgs a{};
  a.kind = c.kind.p;
  a.flags = c.flags.p;
  a.key = c.key.p;
  a.path_ptr = c.path_ptr.p;
  a.path_len = c.path_len.p;
  a.size = c.size.p;
  a.delts = c.delts.p;
  a.keys = c.keys.p;
  a.vals = c.vals.p;
  a.mask = c.tcap - 1;
  a.ctr = c.ctr.p;
  a.tomb_list = c.tomb_list.p;
  a.tomb_cap = c.tomb_cap;
  return a;
}

template <typename T>
static void grow_copy(dr_ctx* ctx, DBuf<T>& b, uint64_t keep, uint64_t cap) {
  DBuf<T> nb(ctx, cap);
  if (keep) HIP_OK(hipMemcpyAsync(nb.p, b.p, keep * sizeof(T), hipMemcpyDeviceToDevice, ctx->stream));
  b = std::move(nb);
}

// store capacity for `need` actions (growth by half: amortised O(1) per appended action)
static void chain_reserve(IncChain& c, uint64_t need) {
  if (need <= c.cap) return;
  const uint64_t cap = std::max<uint64_t>({need, c.cap + c.cap / 2, uint64_t(1) << 16});
  if (cap >= (uint64_t(1) << 32) - 1) fail(DR_E_REBUILD, "apply chain store is full: rebuild the snapshot");
  grow_copy(c.ctx, c.kind, c.n, cap);
  grow_copy(c.ctx, c.flags, c.n, cap);
  grow_copy(c.ctx, c.key, c.n, cap);
  grow_copy(c.ctx, c.path_ptr, c.n, cap);
  grow_copy(c.ctx, c.src_off, c.n, cap);
  grow_copy(c.ctx, c.path_len, c.n, cap);
  grow_copy(c.ctx, c.src_len, c.n, cap);
  grow_copy(c.ctx, c.size, c.n, cap);
  grow_copy(c.ctx, c.delts, c.n, cap);
  grow_copy(c.ctx, c.src_id, c.n, cap);
  c.cap = cap;
}

// table room for `add` more keys at load <= 1/2 (rehash into twice the needed size)
static void chain_table_reserve(IncChain& c, uint64_t add) {
  if ((c.used + add) * 2 <= c.tcap) return;
  uint64_t cap = 1024;
  while (cap < (c.used + add) * 4) cap <<= 1;
  DBuf<unsigned long long> nk(c.ctx, cap);
  DBuf<uint32_t> nv(c.ctx, cap);
  nk.zero(c.ctx->stream);
  nv.zero(c.ctx->stream);
  launch_ix_rehash(c.keys.p, c.vals.p, c.tcap, nk.p, nv.p, cap - 1, c.ctx->stream);
  c.keys = std::move(nk);
  c.vals = std::move(nv);
  c.tcap = cap;
}

static void chain_tomb_reserve(IncChain& c, uint64_t add) {
  if (c.tomb_n + add <= c.tomb_cap) return;
  const uint64_t cap = std::max<uint64_t>({c.tomb_n + add, c.tomb_cap * 2, 4096});
  grow_copy(c.ctx, c.tomb_list, c.tomb_n, cap);
  c.tomb_cap = cap;
}

// Copies the survivors of `base` (live files, then tombstones: distinct paths) into dst[0, M).
struct ActionDst {
  uint8_t *kind, *flags;
  uint64_t *key, *path_ptr, *src_off;
  uint32_t *path_len, *src_len;
  int64_t *size, *delts;
  uint16_t* src_id;
};
static void ensure_ready(dr_state& st);
static void gather_survivors(dr_ctx* ctx, dr_state& base, const ActionDst& d) {
  hipStream_t stream = ctx->stream;
  // base's lists in action order first: the store then keeps the log's order within each side, so an
  // applied state lists its rows as a full replay of its segment does (order_lists)
  ensure_ready(base);
  const uint64_t M = base.n_live + base.n_tomb;
  if (!M) return;
  DBuf<uint32_t> sidx(ctx, M);
  if (base.n_live) HIP_OK(hipMemcpyAsync(sidx.p, base.live.p, base.n_live * 4, hipMemcpyDeviceToDevice, stream));
  if (base.n_tomb)
    HIP_OK(hipMemcpyAsync(sidx.p + base.n_live, base.tomb.p, base.n_tomb * 4, hipMemcpyDeviceToDevice, stream));
  launch_gather_u8(base.kind.p, sidx.p, M, d.kind, stream);
  launch_gather_u8(base.flags.p, sidx.p, M, d.flags, stream);
  launch_gather_u64(base.key.p, sidx.p, M, d.key, stream);
  launch_gather_u64(base.path_ptr.p, sidx.p, M, d.path_ptr, stream);
  launch_gather_u32(base.path_len.p, sidx.p, M, d.path_len, stream);
  launch_gather_u64(reinterpret_cast<const uint64_t*>(base.size.p), sidx.p, M, reinterpret_cast<uint64_t*>(d.size),
                    stream);
  launch_gather_u64(reinterpret_cast<const uint64_t*>(base.delts.p), sidx.p, M,
                    reinterpret_cast<uint64_t*>(d.delts), stream);
  launch_gather_u64(base.src_off.p, sidx.p, M, d.src_off, stream);
  launch_gather_u32(base.src_len.p, sidx.p, M, d.src_len, stream);
  if (base.src_id.p) launch_gather_u16(base.src_id.p, sidx.p, M, d.src_id, stream);
  else HIP_OK(hipMemsetD16Async(reinterpret_cast<hipDeviceptr_t>(d.src_id), 0, M, stream));
}

// Appends src's T actions at dst offset `at`, all from source `sid` (one launch); with `ctr`, the
// same launch sets the index counters (AppendArgs).
static AppendArgs append_args(const ActionDst& d, uint64_t at, dr_state& src, uint16_t sid, unsigned long long* ctr,
                              uint32_t ctr_at, unsigned long long ctr_val);
static void append_actions(dr_ctx* ctx, const ActionDst& d, uint64_t at, dr_state& src, uint16_t sid,
                           unsigned long long* ctr = nullptr, uint32_t ctr_at = 0, unsigned long long ctr_val = 0) {
  if (!src.n_actions && !ctr) return;
  launch_append_actions(append_args(d, at, src, sid, ctr, ctr_at, ctr_val), ctx->stream);
}
static AppendArgs append_args(const ActionDst& d, uint64_t at, dr_state& src, uint16_t sid, unsigned long long* ctr,
                              uint32_t ctr_at, unsigned long long ctr_val) {
  const uint64_t T = src.n_actions;
  AppendArgs a{};
  a.ctr = ctr;
  a.nctr = IX_C_N;
  a.ctr_at = ctr_at;
  a.ctr_val = ctr_val;
  a.src = ActionArrays{src.kind.p, src.flags.p, src.key.p, src.path_ptr.p, src.path_len.p, src.size.p, src.delts.p,
                       src.src_off.p, src.src_len.p};
  a.dst = ActionArrays{d.kind + at, d.flags + at, d.key + at, d.path_ptr + at, d.path_len + at, d.size + at,
                       d.delts + at, d.src_off + at, d.src_len + at};
  a.src_id = d.src_id + at;
  a.n = T;
  a.sid = sid;
  return a;
}

static ActionDst chain_dst(IncChain& c) {
  return ActionDst{c.kind.p, c.flags.p, c.key.p, c.path_ptr.p, c.src_off.p, c.path_len.p, c.src_len.p,
                   c.size.p, c.delts.p, c.src_id.p};
}

static void materialize(dr_state& st);

// r06: every consumer sees the survivor lists in action order -- the order of the winning actions in
// the segment (checkpoint rows, then commits line by line; for a chain state, its store's order), so
// a state's rows, row ranges and their boundaries are a function of the log alone, not of the
// reducer's atomics. A replay on another GPU of the same segment lists the same rows in the same
// order (what an RDD partition recomputed off its executor needs: INTEGRATION.md §1). Sorted once, on
// first use, off the replay's own time.
static void order_lists(dr_state& st) {
  if (st.ordered) return;
  dr_ctx* ctx = st.ctx;
  hipStream_t stream = ctx->stream;
  const uint64_t N = st.n_actions, W = (N + 31) / 32;
  DBuf<uint32_t> bm, cnt;
  DBuf<uint64_t> off;
  DBuf<uint8_t> scratch;
  for (int which = 0; which < 2; ++which) {
    uint32_t* list = which == 0 ? st.live.p : st.tomb.p;
    const uint64_t n = which == 0 ? st.n_live : st.n_tomb;
    if (n < 2) continue;
    if (!bm.p) {
      bm = DBuf<uint32_t>(ctx, W);
      cnt = DBuf<uint32_t>(ctx, W);
      off = DBuf<uint64_t>(ctx, W + 1);
      scratch = DBuf<uint8_t>(ctx, scan_scratch_for(W));
    }
    bm.zero(stream);
    launch_bits_mark(list, n, N, bm.p, stream);
    launch_bits_popc(bm.p, W, cnt.p, stream);
    launch_scan_u32(cnt.p, off.p, W, ss(scratch), stream);
    launch_bits_emit(bm.p, W, off.p, list, stream);
    // distinct entries below N, or the list would lose rows: a replay invariant, checked here
    const uint64_t got = d2h_one(off.p + W, stream);
    if (got != n)
      fail(DR_E_INTERNAL, fmt("survivor list %d: %llu distinct indices of %llu", which, (unsigned long long)got,
                              (unsigned long long)n));
  }
  st.ordered = true;
}

// Chain states read the store through views (refreshed on every use: a later apply may have grown
// the store) and build their survivor lists from the index on first use. Every state's lists are
// put in action order on first use.
static void ensure_ready(dr_state& st) {
  if (!st.chain) {
    order_lists(st);
    return;
  }
  IncChain& c = *st.chain;
  const uint64_t n = st.n_actions;
  st.kind.view(c.kind, n);
  st.flags.view(c.flags, n);
  st.key.view(c.key, n);
  st.path_ptr.view(c.path_ptr, n);
  st.src_off.view(c.src_off, n);
  st.path_len.view(c.path_len, n);
  st.src_len.view(c.src_len, n);
  st.size.view(c.size, n);
  st.delts.view(c.delts, n);
  st.src_id.view(c.src_id, n);
  if (st.sources.size() != st.nsrc) {
    st.sources.assign(c.sources.begin(), c.sources.begin() + st.nsrc);
    st.staged = c.sources[0];
  }
  if (!st.lists_ready) {
    materialize(st);
    st.arenas = c.arenas;
    st.lists_ready = true;
  }
  order_lists(st);
}

// Survivor lists of a chain state: the head's index values -- an older state's after its later
// applies are undone on a copy -- classified at the state's cutoff and compacted in slot order.
static void materialize(dr_state& st) {
  IncChain& c = *st.chain;
  dr_ctx* ctx = st.ctx;
  hipStream_t stream = ctx->stream;
  IndexArgs a = ix_args(c);
  const uint32_t* vals = c.vals.p;
  DBuf<uint32_t> tmp;
  if (st.gen != c.head) {
    tmp = DBuf<uint32_t>(ctx, c.tcap);
    HIP_OK(hipMemcpyAsync(tmp.p, c.vals.p, c.tcap * 4, hipMemcpyDeviceToDevice, stream));
    for (uint32_t g = c.head; g > st.gen; --g) launch_ix_undo(a, tmp.p, c.undo[g - 1].e.p, c.undo[g - 1].n, stream);
    vals = tmp.p;
  }
  const uint64_t C = c.tcap;
  DBuf<uint32_t> lf(ctx, C), tf(ctx, C);
  DBuf<uint64_t> lp(ctx, C + 1), tp(ctx, C + 1);
  DBuf<uint8_t> scratch(ctx, scan_scratch_for(C));
  launch_ix_classify(a, vals, C, st.cutoff, lf.p, tf.p, stream);
  launch_scan_u32(lf.p, lp.p, C, ss(scratch), stream);
  launch_scan_u32(tf.p, tp.p, C, ss(scratch), stream);
  const uint64_t nl = d2h_one(lp.p + C, stream), nt = d2h_one(tp.p + C, stream);
  if (int64_t(nl) != st.counts.num_files || int64_t(nt) != st.counts.num_removes)
    fail(DR_E_INTERNAL, fmt("apply chain index disagrees with its counters (%llu/%lld files, %llu/%lld tombstones)",
                            (unsigned long long)nl, (long long)st.counts.num_files, (unsigned long long)nt,
                            (long long)st.counts.num_removes));
  st.live = DBuf<uint32_t>(ctx, nl);
  st.tomb = DBuf<uint32_t>(ctx, nt);
  launch_ix_emit(vals, C, lf.p, lp.p, tf.p, tp.p, st.live.p, st.tomb.p, stream);
  st.n_live = nl;
  st.n_tomb = nt;
}

// A chain's first image: the base's survivors and their index. nullptr when two survivors share a
// 64-bit path key (the full reduction handles that exactly).
static std::shared_ptr<IncChain> chain_from(dr_ctx* ctx, dr_state& base, uint64_t room) {
  hipStream_t stream = ctx->stream;
  auto ch = std::make_shared<IncChain>();
  IncChain& c = *ch;
  c.ctx = ctx;
  const uint64_t M = base.n_live + base.n_tomb;
  chain_reserve(c, M + room);
  gather_survivors(ctx, base, chain_dst(c));
  c.n = M;
  c.ctr = DBuf<unsigned long long>(ctx, IX_C_N);
  c.ctr.zero(stream);
  chain_table_reserve(c, M + room);
  chain_tomb_reserve(c, base.n_tomb + room);
  IndexArgs a = ix_args(c);
  a.lo = 0;
  a.hi = M;
  launch_ix_build(a, stream);
  const std::vector<unsigned long long> ctr = d2h(c.ctr.p, IX_C_N, stream);
  if (ctr[IX_C_COLLIDE]) return nullptr;
  c.used = ctr[IX_C_NEW_SLOTS];
  c.tomb_n = ctr[IX_C_TOMB_FILL];
  c.sources = base.sources;
  c.arenas = base.arenas;
  return ch;
}

// Applies the parsed tail `t` to the head of chain `ch` (base is the head's state). O(tail): the
// tail's actions are appended to the store and only their keys are probed. nullptr (the index
// restored) when a 64-bit key collision needs the full reduction.
static dr_state* apply_incremental(dr_ctx* ctx, dr_state& base, const std::shared_ptr<IncChain>& ch, dr_state& t,
                                   const std::shared_ptr<StagedData>& tail, int64_t cutoff, int64_t version,
                                   ParsePending& pp, std::vector<NonFileAction>& nf) {
  DR_STAGE("apply", ctx->stream);
  hipStream_t stream = ctx->stream;
  IncChain& c = *ch;
  const uint64_t T = t.n_actions, lo = c.n;
  chain_reserve(c, lo + T);
  chain_table_reserve(c, T);
  chain_tomb_reserve(c, T);
  DBuf<uint32_t> tslot(ctx, T), tprev(ctx, T);
  IncChain::Undo u;
  u.e = DBuf<uint2>(ctx, T);
  IndexArgs a = ix_args(c);
  a.lo = lo;
  a.hi = lo + T;
  a.t_slot = tslot.p;
  a.t_prev = tprev.p;
  a.old_cut = base.cutoff;
  a.new_cut = cutoff;
  a.undo = u.e.p;
  // the index counters start at zero but for the tombstone list's fill (set by the append launch)
  const AppendArgs ap = append_args(chain_dst(c), lo, t, uint16_t(c.sources.size()), c.ctr.p, IX_C_TOMB_FILL, c.tomb_n);
  // one round trip: the tail's parse counters and non-file lines with the index counters, written
  // into the pinned words by the apply's last launch (the one-launch apply itself, the expiry's last
  // workgroup, or a readback launch of their own)
  ReadbackArgs rb{};
  int nrb = 0;
  const size_t at = parse_queue_readback(ctx, pp, 0, &rb, &nrb);
  rb.src[nrb] = reinterpret_cast<const uint64_t*>(c.ctr.p), rb.dst[nrb] = ctx->pinned_dev() + at, rb.n[nrb++] = IX_C_N;
  rb.flag = ctx->pinned_dev() + dr_ctx::kPinFlag;
  rb.seq = ++ctx->pin_seq;
  const bool expire = cutoff > base.cutoff && c.tomb_n;
  bool read_back = false;
  if (T && T <= APPLY_SMALL_MAX) {  // a streamed commit: post-parse, append and both index passes in one launch
    if (pp.parse_deferred) {
      // r06: a short candidate list's expiry and the readback in the same launch (one launch per
      // commit instead of two; the second launch's dispatch sat in every commit's latency)
      const bool fuse = !expire || c.tomb_n <= APPLY_FUSED_EXPIRY_MAX;
      launch_apply_commit(pp.tail_ja, pp.tail_cg, ap, a, stream, fuse && expire ? c.tomb_n : 0, fuse ? &rb : nullptr);
      read_back = fuse;
    } else {
      launch_apply_small(pp.tail_deferred ? &pp.tail_ja : nullptr, pp.tail_cg, ap, a, stream);
    }
    pp.tail_deferred = pp.parse_deferred = false;
  } else {
    parse_flush_tail(ctx, pp);
    launch_append_actions(ap, stream);
    launch_ix_touch(a, stream);
    launch_ix_delta(a, stream);
  }
  if (!read_back) {
    if (expire) launch_ix_expire(a, c.tomb_n, stream, &rb);
    else launch_readback(rb, stream);
  }
  ctx->wait_readback(rb.seq);
  std::vector<unsigned long long> ctr(ctx->pinned() + at, ctx->pinned() + at + IX_C_N);
  if (!parse_finish(ctx, tail, &t, pp, nf)) fail(DR_E_INTERNAL, "applied tail: canonicalisation arena too small");
  c.used += ctr[IX_C_NEW_SLOTS];
  // (DR_IX_TEST_COLLIDE: test hook for the rollback)
  if (ctr[IX_C_COLLIDE] || std::getenv("DR_IX_TEST_COLLIDE")) {  // undo this apply's first touches: the head is the base again
    launch_ix_undo(a, c.vals.p, u.e.p, ctr[IX_C_UNDO_FILL], stream);
    HIP_OK(hipStreamSynchronize(stream));
    return nullptr;
  }
  c.n = lo + T;
  c.tomb_n = ctr[IX_C_TOMB_FILL];
  u.n = ctr[IX_C_UNDO_FILL];
  c.undo.push_back(std::move(u));
  c.head += 1;
  c.sources.push_back(tail);
  c.arenas.insert(c.arenas.end(), t.arenas.begin(), t.arenas.end());
  std::unique_ptr<dr_state> st(new_state(ctx, nullptr));
  st->chain = ch;
  st->gen = c.head;
  st->nsrc = uint32_t(c.sources.size());
  st->n_actions = c.n;
  st->lists_ready = false;
  st->cutoff = cutoff;
  dr_counts& k = st->counts;
  k = base.counts;
  k.num_files += int64_t(ctr[IX_C_FILES]);
  k.size_in_bytes += int64_t(ctr[IX_C_SIZE]);
  k.num_removes += int64_t(ctr[IX_C_REMOVES]);
  k.live_key_sum += ctr[IX_C_LKS];
  k.tomb_key_sum += ctr[IX_C_TKS];
  k.num_actions = base.counts.num_actions + int64_t(T);
  k.num_file_actions = base.counts.num_file_actions + int64_t(ctr[IX_C_FILE_ACTIONS]);
  k.malformed_lines = base.counts.malformed_lines + t.counts.malformed_lines;
  k.version = version;
  // the head's tombstone candidates, compacted once they are mostly stale
  if (c.tomb_n > 2 * uint64_t(k.num_removes) + (uint64_t(1) << 16)) {
    DBuf<ulonglong2> nl(ctx, c.tomb_cap);
    HIP_OK(hipMemsetAsync(c.ctr.p + IX_C_TOMB_FILL, 0, 8, stream));
    IndexArgs b = ix_args(c);
    b.new_cut = cutoff;
    launch_ix_tomb_compact(b, c.tomb_list.p, c.tomb_n, nl.p, stream);
    c.tomb_n = d2h_one(c.ctr.p + IX_C_TOMB_FILL, stream);
    c.tomb_list = std::move(nl);
  }
  return st.release();
}

// Validates a tail against its base: JSON commits only, contiguous versions, a cutoff that does
// not move backwards. Returns the new version.
static int64_t check_tail(dr_state& base, const std::shared_ptr<StagedData>& tail, int64_t cutoff) {
  if (!tail->parts.empty()) fail(DR_E_INVALID_ARG, "an applied tail holds commit (JSON) files only");
  if (base.sources.empty() && !base.chain) fail(DR_E_INVALID_ARG, "base state has no staged segment");
  if (base.sharded) fail(DR_E_UNSUPPORTED, "a sharded replay's part cannot take a tail on its own: shard the tail too");
  const uint64_t nsrc = base.chain ? base.nsrc : base.sources.size();
  if (nsrc >= 65535) fail(DR_E_REBUILD, "too many applied tails on one state: rebuild the snapshot");
  // the base kept only tombstones with delTimestamp > base.cutoff: an earlier cutoff (a longer
  // delta.deletedFileRetentionDuration, a clock moved back) would need the ones it dropped
  if (cutoff < base.cutoff)
    fail(DR_E_REBUILD, fmt("retention cutoff %lld is earlier than the base state's %lld: rebuild the snapshot",
                           (long long)cutoff, (long long)base.cutoff));
  std::vector<int64_t> vers;
  for (const JsonFileRec& j : tail->jfiles) vers.push_back(j.version);
  std::sort(vers.begin(), vers.end());
  bool contiguous = true;
  for (size_t k = 0; k < vers.size(); ++k) contiguous &= vers[k] == base.counts.version + 1 + int64_t(k);
  if (!contiguous) {  // verifyDeltaVersions' message (D/SnapshotManagement.scala:365-372)
    std::string v = std::to_string(base.counts.version);
    for (int64_t x : vers) v += ", " + std::to_string(x);
    fail(DR_E_NONCONTIGUOUS, "Versions (Vector(" + v + ")) are not contiguous.");
  }
  return vers.empty() ? base.counts.version : vers.back();
}

// Tail apply. The head of an apply chain (or a full replay, which starts a chain) takes the O(tail)
// index path; any other base -- an older state of a chain, a forced reducer, a key collision --
// takes the full path: the base's survivors (distinct paths, so their relative order is free) are
// the replay prefix, the tail's lines follow in file order, and K3/K4 run over the concatenation
// with the new cutoff, the same result as replaying the whole segment (tombstones the base dropped
// stay dropped, so the cutoff must not move backwards). Nothing of the base is re-parsed either way.
static dr_state* apply_tail(dr_ctx* ctx, dr_state& base, const std::shared_ptr<StagedData>& tail, int64_t cutoff,
                            uint32_t flags) {
  DR_STAGE("apply", ctx->stream);
  const int64_t version = check_tail(base, tail, cutoff);
  std::unique_ptr<dr_state> t(new_state(ctx, tail));
  std::vector<NonFileAction> nf;
  // the tail's parse is queued; the incremental path reads its counters back with the index's
  ParsePending pp = parse_launch(ctx, tail, t.get(), true, /*defer_tail=*/true);
  bool parsed = false;
  // protocol / metaData / txn: the base's winners first, then the tail's actions in order
  auto all_nonfile = [&] {
    std::vector<NonFileAction> all = base.nonfile;
    for (size_t k = 0; k < all.size(); ++k) all[k].order = k;
    for (NonFileAction& a : nf) {
      a.order += all.size();
      all.push_back(a);
    }
    return all;
  };
  const bool forced = (flags & (DR_FLAG_EXACT_REDUCE | DR_FLAG_REDUCE64)) || ctx->opt.apply_full;
  if (!forced) {
    std::shared_ptr<IncChain> ch;
    if (base.chain && base.gen == base.chain->head) ch = base.chain;
    else if (!base.chain) ch = chain_from(ctx, base, std::max<uint64_t>(t->n_actions, 1024));
    if (ch) {
      dr_state* r0 = apply_incremental(ctx, base, ch, *t, tail, cutoff, version, pp, nf);
      parsed = true;
      if (r0) {
        std::unique_ptr<dr_state> r(r0);
        std::vector<NonFileAction> all = all_nonfile();
        reduce_nonfile(*r, all, !(flags & DR_FLAG_NO_VALIDATION));
        return r.release();
      }
    }
  }
  if (!parsed) {
    parse_flush_tail(ctx, pp);
    parse_queue_readback(ctx, pp, 0);
    HIP_OK(hipStreamSynchronize(ctx->stream));
    if (!parse_finish(ctx, tail, t.get(), pp, nf)) fail(DR_E_INTERNAL, "applied tail: canonicalisation arena too small");
  }
  std::vector<NonFileAction> all = all_nonfile();
  ensure_ready(base);
  hipStream_t stream = ctx->stream;
  const uint64_t M = base.n_live + base.n_tomb, T = t->n_actions, N = M + T;
  if (N >= (uint64_t(1) << 30)) fail(DR_E_UNSUPPORTED, "more than 2^30 actions in one replay");
  std::unique_ptr<dr_state> st(new_state(ctx, nullptr));
  st->staged = base.staged;
  st->sources = base.sources;
  st->sources.push_back(tail);
  st->arenas = base.arenas;
  st->arenas.insert(st->arenas.end(), t->arenas.begin(), t->arenas.end());
  st->counts.version = version;
  st->n_actions = N;
  st->kind = DBuf<uint8_t>(ctx, N);
  st->flags = DBuf<uint8_t>(ctx, N);
  st->key = DBuf<uint64_t>(ctx, N);
  st->path_ptr = DBuf<uint64_t>(ctx, N);
  st->path_len = DBuf<uint32_t>(ctx, N);
  st->size = DBuf<int64_t>(ctx, N);
  st->delts = DBuf<int64_t>(ctx, N);
  st->src_off = DBuf<uint64_t>(ctx, N);
  st->src_len = DBuf<uint32_t>(ctx, N);
  st->src_id = DBuf<uint16_t>(ctx, N);
  const ActionDst d{st->kind.p, st->flags.p, st->key.p, st->path_ptr.p, st->src_off.p, st->path_len.p,
                    st->src_len.p, st->size.p, st->delts.p, st->src_id.p};
  gather_survivors(ctx, base, d);
  append_actions(ctx, d, M, *t, uint16_t(st->sources.size() - 1));
  (void)stream;
  reduce_actions(ctx, st.get(), cutoff, flags);
  st->cutoff = cutoff;
  // a full replay of the segment would count every action of the base's segment plus the tail's
  st->counts.num_file_actions = base.counts.num_file_actions + (st->counts.num_file_actions - int64_t(M));
  st->counts.num_actions = base.counts.num_actions + int64_t(T);
  st->counts.malformed_lines = base.counts.malformed_lines + t->counts.malformed_lines;
  reduce_nonfile(*st, all, !(flags & DR_FLAG_NO_VALIDATION));
  return st.release();
}

// A full replay is queued end to end (K1, K2, k_canon, K3, K4, compaction) and read back once: the
// counters, error codes and non-file line list of the parse and the reducer's totals land in the
// pinned words with one stream sync. The host's protocol / metaData / txn reduction follows.
static dr_state* replay(dr_ctx* ctx, const std::shared_ptr<StagedData>& sp, int64_t cutoff, uint32_t flags) {
  DR_STAGE("delta.stateReconstruction", ctx->stream);
  std::unique_ptr<dr_state> st(new_state(ctx, sp));
  ctx->mark("start");
  std::vector<NonFileAction> nf;
  static const bool dbg = std::getenv("DR_HOST_DEBUG") != nullptr;  // host phase times per replay
  const double t0 = dbg ? now_s() : 0;
  double t1 = 0, t2 = 0;
  for (;;) {
    ParsePending pp = parse_launch(ctx, sp, st.get(), true);
    ReducePending rp = reduce_launch(ctx, st.get(), cutoff, flags);
    reduce_queue_readback(ctx, rp, parse_queue_readback(ctx, pp, 0));
    if (dbg) t1 = now_s();
    HIP_OK(hipStreamSynchronize(ctx->stream));
    if (dbg) t2 = now_s();
    if (parse_finish(ctx, sp, st.get(), pp, nf)) {
      reduce_finish(ctx, st.get(), rp);
      break;
    }
    // the arena hint was too small: redo with the exact size (parse_finish stored it)
    st.reset(new_state(ctx, sp));
  }
  st->cutoff = cutoff;
  reduce_nonfile(*st, nf, !(flags & DR_FLAG_NO_VALIDATION));
  if (dbg)
    std::fprintf(stderr, "replay host: queue %.1f us, wait %.1f us, finish %.1f us (%zu non-file actions)\n",
                 (t1 - t0) * 1e6, (t2 - t1) * 1e6, (now_s() - t2) * 1e6, nf.size());
  ctx->mark("end");
  return st.release();
}

// ---------------------------------------------------------------------------------------------------
// export (records materialised on the host from the resident state)
// ---------------------------------------------------------------------------------------------------
template <typename T>
static DBuf<T> upload(dr_ctx* ctx, const T* src, size_t n) {
  DBuf<T> d(ctx, n);
  if (n) HIP_OK(hipMemcpyAsync(d.p, src, n * sizeof(T), hipMemcpyHostToDevice, ctx->stream));
  return d;
}

// Export of one side, built on the device (k_export): the canonical paths and the replay's
// size / deletionTimestamp from the action arrays, every other field from the survivor's JSON line
// or from the checkpoint's leaves of that side (decoded on first export, K2's page decoder), then one
// copy of the columns to the host.
struct ExpDecoded {
  DBuf<uint8_t> def[8], rep[8];
  DBuf<int64_t> ival[8];
  DBuf<uint64_t> sptr[8], row_start[2];
  DBuf<uint32_t> slen[8];
  ExpFlat flat[4]{};
  ExpMap map[2]{};
};

static const char* kExpLeaf[8] = {"size", "modificationTime", "extendedFileMetadata", "stats",
                                  "partitionValues.key_value.key", "partitionValues.key_value.value",
                                  "tags.key_value.key", "tags.key_value.value"};

static void decode_export_side(dr_state& st, int which, ExpDecoded& D) {
  dr_ctx* ctx = st.ctx;
  hipStream_t stream = ctx->stream;
  StagedData& s = *st.sources[0];
  const uint64_t R = s.ck_rows;
  if (!R) return;
  const std::string pre = which == DR_LIVE ? "add." : "remove.";
  {
    std::lock_guard<std::mutex> g(s.pv_mu);
    if (!s.exp[which]) {
      auto P = std::make_unique<PagePlan>();
      for (const char* leaf : kExpLeaf) P->paths.push_back(pre + leaf);
      plan_pages(s, *P);
      s.exp[which] = std::move(P);
    }
  }
  PagePlan& P = *s.exp[which];
  ParquetArgs pa{};
  pa.ncols = 8;
  for (int c = 0; c < 8; ++c) {
    if (!P.present[c]) continue;
    const uint64_t L = P.levels[c];
    D.def[c] = DBuf<uint8_t>(ctx, L);
    D.def[c].zero(stream);
    const bool str = c == 3 || c >= 4;
    if (c >= 4) D.rep[c] = DBuf<uint8_t>(ctx, L);
    if (str) {
      D.sptr[c] = DBuf<uint64_t>(ctx, L);
      D.slen[c] = DBuf<uint32_t>(ctx, L);
    } else {
      D.ival[c] = DBuf<int64_t>(ctx, L);
    }
    pa.cols[c] = FlatColumn{D.def[c].p, D.rep[c].p, D.ival[c].p, D.sptr[c].p, D.slen[c].p};
  }
  DBuf<uint64_t> dict_ptr;
  DBuf<uint32_t> dict_len, pq_err(ctx, 1);
  pq_err.zero(stream);
  decode_pages(ctx, P, pa, dict_ptr, dict_len, pq_err, nullptr);
  if (d2h_one(pq_err.p, stream) != 0)
    fail(DR_E_PARQUET, fmt("device decode of the %sexport columns failed (code %u)", pre.c_str(), d2h_one(pq_err.p, stream)));
  for (int c = 0; c < 4; ++c) {
    if (!P.present[c]) continue;
    if (P.levels[c] != R) fail(DR_E_PARQUET, pre + kExpLeaf[c] + ": one value per checkpoint row expected");
    D.flat[c] = ExpFlat{D.def[c].p, D.ival[c].p, D.sptr[c].p, D.slen[c].p, P.max_def[c]};
  }
  for (int m = 0; m < 2; ++m) {
    const int kc = 4 + 2 * m, vc = kc + 1;
    if (!P.present[kc] || !P.present[vc]) continue;
    const uint64_t E = P.levels[kc];
    if (P.levels[vc] != E) fail(DR_E_PARQUET, pre + kExpLeaf[kc] + ": key/value columns disagree");
    const pq::Leaf* leaf = s.parts[0].meta.leaf(pre + kExpLeaf[kc]);
    if (!leaf || leaf->def_of.size() < 3) fail(DR_E_PARQUET, pre + kExpLeaf[kc] + ": unexpected map layout");
    DBuf<uint32_t> rflag(ctx, E);
    DBuf<uint64_t> rpos(ctx, E + 1);
    DBuf<uint8_t> scratch(ctx, scan_scratch_for(E));
    launch_rep0_flags(D.rep[kc].p, E, rflag.p, stream);
    launch_scan_u32(rflag.p, rpos.p, E, ss(scratch), stream);
    if (d2h_one(rpos.p + E, stream) != R) fail(DR_E_PARQUET, pre + kExpLeaf[kc] + ": one map per checkpoint row expected");
    D.row_start[m] = DBuf<uint64_t>(ctx, R + 1);
    launch_row_starts(D.rep[kc].p, E, rpos.p, D.row_start[m].p, stream);
    HIP_OK(hipMemcpyAsync(D.row_start[m].p + R, &E, 8, hipMemcpyHostToDevice, stream));
    D.map[m] = ExpMap{D.row_start[m].p, D.def[kc].p, D.sptr[kc].p, D.slen[kc].p, D.def[vc].p, D.sptr[vc].p,
                      D.slen[vc].p, leaf->def_of[1], leaf->def_of[2], P.max_def[vc]};
  }
}


// One side's export columns in HBM (k_export's output; the checkpoint encoder reads them there).
struct DevExport {
  uint64_t n = 0;
  DBuf<uint64_t> path_ptr, path_off, delts;  // path_off: exclusive scan of the lengths (n + 1)
  DBuf<uint32_t> path_len;
  DBuf<uint8_t> path_bytes, flags;
  DBuf<int64_t> size, mtime;
  DBuf<uint8_t> efm, stats_null, pv_null, tags_null;
  DBuf<uint64_t> off[EXC_N];                 // exclusive scans of the per-record counts (n + 1)
  uint64_t tot[EXC_N] = {};
  uint64_t path_nb = 0;                      // path bytes
  DBuf<uint8_t> stats_bytes, pv_key_bytes, pv_val_bytes, tags_key_bytes, tags_val_bytes, pv_val_null, tags_val_null;
  DBuf<int64_t> pv_key_off, pv_val_off, tags_key_off, tags_val_off;  // per entry (entries + 1)
};

// Records [lo, hi) of the side (export order); the whole side by default. `at` (may be null) is
// called with 0 once the paths, flags and deletion timestamps are enqueued, 1 once pass 1's scalars
// and offsets are (before the host waits for their totals), 2 once every column is: a streamed
// export queues each group's copy to the host there.
static void export_device(dr_state& st, int which, DevExport& X, uint64_t lo = 0, uint64_t hi = UINT64_MAX,
                          const std::function<void(int)>* at = nullptr) {
  DR_STAGE("export", st.ctx->stream);
  ensure_ready(st);
  dr_ctx* ctx = st.ctx;
  hipStream_t stream = ctx->stream;
  StagedData& s = *st.sources[0];
  const uint64_t total = which == DR_LIVE ? st.n_live : st.n_tomb;
  hi = std::min(hi, total);
  lo = std::min(lo, hi);
  const uint64_t n = hi - lo;
  const uint32_t* didx = (which == DR_LIVE ? st.live.p : st.tomb.p) + lo;
  X.n = n;
  // canonical paths, deletionTimestamp and flags from the action arrays
  X.path_ptr = DBuf<uint64_t>(ctx, n);
  X.path_off = DBuf<uint64_t>(ctx, n + 1);
  X.delts = DBuf<uint64_t>(ctx, n);
  X.path_len = DBuf<uint32_t>(ctx, n);
  X.flags = DBuf<uint8_t>(ctx, n);
  DBuf<uint8_t> scratch(ctx, scan_scratch_for(n));
  launch_gather_u64(st.path_ptr.p, didx, n, X.path_ptr.p, stream);
  launch_gather_u32(st.path_len.p, didx, n, X.path_len.p, stream);
  launch_gather_u64(reinterpret_cast<const uint64_t*>(st.delts.p), didx, n, X.delts.p, stream);
  launch_gather_u8(st.flags.p, didx, n, X.flags.p, stream);
  launch_scan_u32(X.path_len.p, X.path_off.p, n, ss(scratch), stream);
  if (!n) HIP_OK(hipMemsetAsync(X.path_off.p, 0, 8, stream));
  const uint64_t nb = n ? d2h_one(X.path_off.p + n, stream) : 0;
  X.path_bytes = DBuf<uint8_t>(ctx, nb + 16);  // +16: whole-word loads of the record hash
  X.path_nb = nb;
  launch_gather_bytes(X.path_ptr.p, X.path_len.p, X.path_off.p, n, X.path_bytes.p, stream);
  if (at) (*at)(0);
  if (!st.exp_dec[which]) {
    auto d = std::make_shared<ExpDecoded>();
    decode_export_side(st, which, *d);
    st.exp_dec[which] = d;
  }
  const ExpDecoded& D = *st.exp_dec[which];
  ExportArgs a{};
  a.idx = didx;
  a.n = n;

  a.side = which == DR_LIVE ? 0 : 1;
  a.json = s.d_json.p;
  a.ck_rows = s.ck_rows;
  a.src_off = st.src_off.p;
  a.src_len = st.src_len.p;
  a.act_size = st.size.p;
  DBuf<uint64_t> json_bases;
  if (st.src_id.p) {
    std::vector<uint64_t> bases;
    for (auto& src : st.sources) bases.push_back(reinterpret_cast<uint64_t>(src->d_json.p));
    json_bases = upload(ctx, bases.data(), bases.size());
    a.act_flags = st.flags.p;
    a.src_id = st.src_id.p;
    a.json_bases = json_bases.p;
  }
  a.ck_size = D.flat[0];
  a.ck_mtime = D.flat[1];
  a.ck_efm = D.flat[2];
  a.ck_stats = D.flat[3];
  a.ck_pv = D.map[0];
  a.ck_tags = D.map[1];
  X.size = DBuf<int64_t>(ctx, n);
  X.mtime = DBuf<int64_t>(ctx, n);
  X.efm = DBuf<uint8_t>(ctx, n);
  X.stats_null = DBuf<uint8_t>(ctx, n);
  X.pv_null = DBuf<uint8_t>(ctx, n);
  X.tags_null = DBuf<uint8_t>(ctx, n);
  DBuf<uint32_t> cnt[EXC_N];
  DBuf<uint32_t> err(ctx, 1);
  err.zero(stream);
  a.size = X.size.p;
  a.mtime = X.mtime.p;
  a.efm = X.efm.p;
  a.stats_null = X.stats_null.p;
  a.pv_null = X.pv_null.p;
  a.tags_null = X.tags_null.p;
  a.error = err.p;
  for (int k = 0; k < EXC_N; ++k) {
    cnt[k] = DBuf<uint32_t>(ctx, n);
    X.off[k] = DBuf<uint64_t>(ctx, n + 1);
    a.cnt[k] = cnt[k].p;
  }
  DBuf<uint64_t> stats_src(ctx, n);
  DBuf<uint32_t> stats_srclen(ctx, n);
  a.stats_src = stats_src.p;
  a.stats_srclen = stats_srclen.p;
  // pass 1: scalars + counts, the checkpoint rows and the JSON lines in launches of their own (the
  // survivors mix them; the JSON walk needs the line stage, which costs the checkpoint rows occupancy)
  {
    DBuf<uint32_t> jf(ctx, n), jpos(ctx, n), cpos(ctx, n);
    DBuf<uint64_t> js(ctx, n + 1);
    launch_export_flags(a, jf.p, stream);
    launch_scan_u32(jf.p, js.p, n, ss(scratch), stream);
    const uint64_t nj = n ? d2h_one(js.p + n, stream) : 0;
    launch_export_split(jf.p, js.p, n, jpos.p, cpos.p, stream);
    a.pos = cpos.p;
    a.npos = n - nj;
    launch_export(a, false, stream);
    a.pos = jpos.p;
    a.npos = nj;
    launch_export(a, true, stream);
    a.pos = nullptr;
    a.npos = n;
  }
  for (int k = 0; k < EXC_N; ++k) {
    launch_scan_u32(cnt[k].p, X.off[k].p, n, ss(scratch), stream);
    if (!n) HIP_OK(hipMemsetAsync(X.off[k].p, 0, 8, stream));
    a.off[k] = X.off[k].p;
  }
  if (at) (*at)(1);
  for (int k = 0; k < EXC_N && n; ++k) X.tot[k] = d2h_one(X.off[k].p + n, stream);
  if (d2h_one(err.p, stream)) fail(DR_E_PARSE, "malformed survivor line at export");
  X.stats_bytes = DBuf<uint8_t>(ctx, X.tot[EXC_STATS] + 16);
  X.pv_key_bytes = DBuf<uint8_t>(ctx, X.tot[EXC_PV_KB] + 16);
  X.pv_val_bytes = DBuf<uint8_t>(ctx, X.tot[EXC_PV_VB] + 16);
  X.tags_key_bytes = DBuf<uint8_t>(ctx, X.tot[EXC_TAGS_KB] + 16);
  X.tags_val_bytes = DBuf<uint8_t>(ctx, X.tot[EXC_TAGS_VB] + 16);
  X.pv_val_null = DBuf<uint8_t>(ctx, X.tot[EXC_PV_N] + 1);
  X.tags_val_null = DBuf<uint8_t>(ctx, X.tot[EXC_TAGS_N] + 1);
  X.pv_key_off = DBuf<int64_t>(ctx, X.tot[EXC_PV_N] + 1);
  X.pv_val_off = DBuf<int64_t>(ctx, X.tot[EXC_PV_N] + 1);
  X.tags_key_off = DBuf<int64_t>(ctx, X.tot[EXC_TAGS_N] + 1);
  X.tags_val_off = DBuf<int64_t>(ctx, X.tot[EXC_TAGS_N] + 1);
  for (DBuf<int64_t>* o : {&X.pv_key_off, &X.pv_val_off, &X.tags_key_off, &X.tags_val_off})
    HIP_OK(hipMemsetAsync(o->p, 0, 8, stream));
  a.write = 1;
  a.stats_bytes = X.stats_bytes.p;
  a.pv_key_off = X.pv_key_off.p;
  a.pv_val_off = X.pv_val_off.p;
  a.pv_val_null = X.pv_val_null.p;
  a.pv_key_bytes = X.pv_key_bytes.p;
  a.pv_val_bytes = X.pv_val_bytes.p;
  a.tags_key_off = X.tags_key_off.p;
  a.tags_val_off = X.tags_val_off.p;
  a.tags_val_null = X.tags_val_null.p;
  a.tags_key_bytes = X.tags_key_bytes.p;
  a.tags_val_bytes = X.tags_val_bytes.p;
  // checkpoint rows' map entries: their sources, gathered after pass 2 (JSON entries keep length 0)
  DBuf<uint64_t> ent_src[4];
  DBuf<uint32_t> ent_len[4];
  const uint64_t ent_n[4] = {X.tot[EXC_PV_N], X.tot[EXC_PV_N], X.tot[EXC_TAGS_N], X.tot[EXC_TAGS_N]};
  for (int q = 0; q < 4; ++q) {
    ent_src[q] = DBuf<uint64_t>(ctx, ent_n[q] + 1);
    ent_len[q] = DBuf<uint32_t>(ctx, ent_n[q] + 1);
    ent_len[q].zero(stream);
  }
  a.pv_ksrc = ent_src[0].p;
  a.pv_vsrc = ent_src[1].p;
  a.tags_ksrc = ent_src[2].p;
  a.tags_vsrc = ent_src[3].p;
  a.pv_klen = ent_len[0].p;
  a.pv_vlen = ent_len[1].p;
  a.tags_klen = ent_len[2].p;
  a.tags_vlen = ent_len[3].p;
  launch_export(a, true, stream);  // pass 2: bytes and entries
  launch_gather_bytes(ent_src[0].p, ent_len[0].p, reinterpret_cast<const uint64_t*>(X.pv_key_off.p), ent_n[0],
                      X.pv_key_bytes.p, stream);
  launch_gather_bytes(ent_src[1].p, ent_len[1].p, reinterpret_cast<const uint64_t*>(X.pv_val_off.p), ent_n[1],
                      X.pv_val_bytes.p, stream);
  launch_gather_bytes(ent_src[2].p, ent_len[2].p, reinterpret_cast<const uint64_t*>(X.tags_key_off.p), ent_n[2],
                      X.tags_key_bytes.p, stream);
  launch_gather_bytes(ent_src[3].p, ent_len[3].p, reinterpret_cast<const uint64_t*>(X.tags_val_off.p), ent_n[3],
                      X.tags_val_bytes.p, stream);
  // a checkpoint record's stats are one contiguous decoded string: copied whole, several lanes each
  launch_gather_bytes(stats_src.p, stats_srclen.p, X.off[EXC_STATS].p, n, X.stats_bytes.p, stream);
  if (at) (*at)(2);
}

// Both sides' device export columns, built once per state and kept until its release.
static const DevExport& materialize(dr_state& st, int which) {
  if (!st.dexp[which]) {
    auto X = std::make_shared<DevExport>();
    export_device(st, which, *X);
    st.dexp[which] = X;
  }
  return *st.dexp[which];
}

// Order-free full-record checksum of one side (dr_state_record_sums): k_record_hash over the
// side's device export columns.
static uint64_t record_sum(dr_state& st, int which, uint64_t* hashes = nullptr) {
  dr_ctx* ctx = st.ctx;
  hipStream_t stream = ctx->stream;
  const DevExport& X = materialize(st, which);
  DBuf<unsigned long long> sum(ctx, 1);
  sum.zero(stream);
  RecordHashArgs a{};
  a.n = X.n;
  a.side = which == DR_LIVE ? 0 : 1;
  a.path_bytes = X.path_bytes.p;
  a.path_off = X.path_off.p;
  a.size = X.size.p;
  a.mtime = X.mtime.p;
  a.delts = X.delts.p;
  a.flags = X.flags.p;
  a.efm = X.efm.p;
  a.stats_null = X.stats_null.p;
  a.stats_off = X.off[EXC_STATS].p;
  a.stats_bytes = X.stats_bytes.p;
  a.pv_null = X.pv_null.p;
  a.pv_entry = X.off[EXC_PV_N].p;
  a.pv_key_off = X.pv_key_off.p;
  a.pv_key_bytes = X.pv_key_bytes.p;
  a.pv_val_off = X.pv_val_off.p;
  a.pv_val_bytes = X.pv_val_bytes.p;
  a.pv_val_null = X.pv_val_null.p;
  a.tags_null = X.tags_null.p;
  a.tags_entry = X.off[EXC_TAGS_N].p;
  a.tags_key_off = X.tags_key_off.p;
  a.tags_key_bytes = X.tags_key_bytes.p;
  a.tags_val_off = X.tags_val_off.p;
  a.tags_val_bytes = X.tags_val_bytes.p;
  a.tags_val_null = X.tags_val_null.p;
  a.sum = sum.p;
  DBuf<uint64_t> each;
  if (hashes) {
    each = DBuf<uint64_t>(ctx, X.n);
    a.out = each.p;
  }
  if (const char* m = std::getenv("DR_RECORD_FIELDS")) a.field_mask = uint32_t(std::strtoul(m, nullptr, 0));  // diagnostics
  launch_record_hash(a, stream);
  if (hashes && X.n) HIP_OK(hipMemcpyAsync(hashes, each.p, X.n * 8, hipMemcpyDeviceToHost, stream));
  return uint64_t(d2h_one(sum.p, stream));
}

// The host columns of dr_export in three groups, each ready at one point of export_device:
// 0 paths and deletion timestamps, 1 pass 1's scalars and offsets, 2 the bytes and map entries.
struct ExportCol {
  void** dst;
  const void* src;
  uint64_t bytes;
};
static std::vector<ExportCol> export_group(ExportCols& ex, const DevExport& X, int g, const uint8_t* dvalid,
                                           const int64_t* ddelts) {
  const uint64_t n = X.n;
  if (g == 0)
    return {{(void**)&ex.path_off, X.path_off.p, 8 * (n + 1)},
            {(void**)&ex.path_bytes, X.path_bytes.p, X.path_nb},
            {(void**)&ex.delts, ddelts, 8 * n},
            {(void**)&ex.delts_valid, dvalid, n}};
  if (g == 1)
    return {{(void**)&ex.size, X.size.p, 8 * n},
            {(void**)&ex.mtime, X.mtime.p, 8 * n},
            {(void**)&ex.efm, X.efm.p, n},
            {(void**)&ex.stats_null, X.stats_null.p, n},
            {(void**)&ex.pv_null, X.pv_null.p, n},
            {(void**)&ex.tags_null, X.tags_null.p, n},
            {(void**)&ex.stats_off, X.off[EXC_STATS].p, 8 * (n + 1)},
            {(void**)&ex.pv_entry_off, X.off[EXC_PV_N].p, 8 * (n + 1)},
            {(void**)&ex.tags_entry_off, X.off[EXC_TAGS_N].p, 8 * (n + 1)}};
  return {{(void**)&ex.stats_bytes, X.stats_bytes.p, X.tot[EXC_STATS]},
          {(void**)&ex.pv_key_off, X.pv_key_off.p, 8 * (X.tot[EXC_PV_N] + 1)},
          {(void**)&ex.pv_val_off, X.pv_val_off.p, 8 * (X.tot[EXC_PV_N] + 1)},
          {(void**)&ex.pv_val_null, X.pv_val_null.p, X.tot[EXC_PV_N]},
          {(void**)&ex.pv_key_bytes, X.pv_key_bytes.p, X.tot[EXC_PV_KB]},
          {(void**)&ex.pv_val_bytes, X.pv_val_bytes.p, X.tot[EXC_PV_VB]},
          {(void**)&ex.tags_key_off, X.tags_key_off.p, 8 * (X.tot[EXC_TAGS_N] + 1)},
          {(void**)&ex.tags_val_off, X.tags_val_off.p, 8 * (X.tot[EXC_TAGS_N] + 1)},
          {(void**)&ex.tags_val_null, X.tags_val_null.p, X.tot[EXC_TAGS_N]},
          {(void**)&ex.tags_key_bytes, X.tags_key_bytes.p, X.tot[EXC_TAGS_KB]},
          {(void**)&ex.tags_val_bytes, X.tags_val_bytes.p, X.tot[EXC_TAGS_VB]}};
}
static uint64_t group_bytes(const std::vector<ExportCol>& cols) {
  uint64_t t = 0;
  for (const ExportCol& c : cols) t += (c.bytes + 63) & ~uint64_t(63);
  return t;
}
// Carves the columns out of the pinned block (64-byte aligned slices) and queues their copies.
static void queue_group(const std::vector<ExportCol>& cols, void* block, hipStream_t s) {
  uint8_t* at = static_cast<uint8_t*>(block);
  for (const ExportCol& c : cols) {
    *c.dst = at;
    if (c.bytes) HIP_OK(hipMemcpyAsync(at, c.src, c.bytes, hipMemcpyDeviceToHost, s));
    at += (c.bytes + 63) & ~uint64_t(63);
  }
}

// dr_state_export: the side's resident columns into pinned host memory. A side not yet materialised
// is streamed: its column groups cross to the host on stream2 while the device still extracts the
// later groups (the paths during the checkpoint decode and pass 1, the scalars during pass 2), and
// the pinned blocks of groups 0 and 1 -- sized by the record count alone -- are taken from the
// context's cache (or pinned) on a helper thread while the device works.
static void build_export(dr_state& st, int which) {
  ensure_ready(st);
  ExportCols& ex = st.exp[which];
  if (ex.built) return;
  dr_ctx* ctx = st.ctx;
  hipStream_t stream = ctx->stream;
  ex.ctx = ctx;
  DBuf<uint8_t> dvalid;
  DBuf<int64_t> ddelts;
  auto fix_delts = [&](const DevExport& X) {  // delTs validity is F_HAS_DELTS; an absent delTs reads 0
    dvalid = DBuf<uint8_t>(ctx, X.n);
    ddelts = DBuf<int64_t>(ctx, X.n);
    launch_delts_fix(X.flags.p, reinterpret_cast<const int64_t*>(X.delts.p), X.n, dvalid.p, ddelts.p, stream);
  };
  if (st.dexp[which]) {  // materialised before: one block, every copy queued at once
    const DevExport& X = *st.dexp[which];
    ex.n = int64_t(X.n);
    fix_delts(X);
    std::vector<ExportCol> cols;
    for (int g = 0; g < 3; ++g) {
      std::vector<ExportCol> c = export_group(ex, X, g, dvalid.p, ddelts.p);
      cols.insert(cols.end(), c.begin(), c.end());
    }
    ex.blocks.push_back(ctx->host_alloc(group_bytes(cols)));
    queue_group(cols, ex.blocks.back(), stream);
    HIP_OK(hipStreamSynchronize(stream));
    ex.built = true;
    return;
  }
  auto Xp = std::make_shared<DevExport>();
  DevExport& X = *Xp;
  hipStream_t cs = ctx->stream2;
  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
  for (hipEvent_t& e : ev) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  std::thread pin;
  void* block01 = nullptr;
  std::exception_ptr pin_err;
  const std::function<void(int)> at = [&](int g) {
    if (g == 0) {
      fix_delts(X);
      HIP_OK(hipEventRecord(ev[0], stream));
      // groups 0 and 1 are sized by the record count and the path bytes (group 1's columns are not
      // allocated yet: only its sizes are read here)
      const uint64_t b0 = group_bytes(export_group(ex, X, 0, dvalid.p, ddelts.p));
      const uint64_t b1 = group_bytes(export_group(ex, X, 1, dvalid.p, ddelts.p));
      pin = std::thread([&, b0, b1] {
        try {
          HIP_OK(hipSetDevice(ctx->device));
          block01 = ctx->host_alloc(b0 + b1);
        } catch (...) {
          pin_err = std::current_exception();
        }
      });
    } else if (g == 1) {
      HIP_OK(hipEventRecord(ev[1], stream));
      pin.join();
      if (pin_err) std::rethrow_exception(pin_err);
      ex.blocks.push_back(block01);
      HIP_OK(hipStreamWaitEvent(cs, ev[0], 0));
      const std::vector<ExportCol> c0 = export_group(ex, X, 0, dvalid.p, ddelts.p);
      const std::vector<ExportCol> c1 = export_group(ex, X, 1, dvalid.p, ddelts.p);
      queue_group(c0, block01, cs);
      HIP_OK(hipStreamWaitEvent(cs, ev[1], 0));
      queue_group(c1, static_cast<uint8_t*>(block01) + group_bytes(c0), cs);
    } else {
      HIP_OK(hipEventRecord(ev[2], stream));
      std::vector<ExportCol> c2 = export_group(ex, X, 2, dvalid.p, ddelts.p);
      ex.blocks.push_back(ctx->host_alloc(group_bytes(c2)));
      HIP_OK(hipStreamWaitEvent(cs, ev[2], 0));
      queue_group(c2, ex.blocks.back(), cs);
    }
  };
  try {
    export_device(st, which, X, 0, UINT64_MAX, &at);
  } catch (...) {
    if (pin.joinable()) pin.join();
    if (block01 && (ex.blocks.empty() || ex.blocks.front() != block01)) ctx->host_release(block01);
    (void)hipStreamSynchronize(cs);
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
    throw;
  }
  ex.n = int64_t(X.n);
  HIP_OK(hipStreamSynchronize(cs));
  HIP_OK(hipStreamSynchronize(stream));
  for (hipEvent_t e : ev) HIP_OK(hipEventDestroy(e));
  st.dexp[which] = Xp;
  ex.built = true;
}

// ---------------------------------------------------------------------------------------------------
// K5: partition pruning (DeltaLog.filterFileList, D/DeltaLog.scala:500-547)
// ---------------------------------------------------------------------------------------------------
static const char* kPvKey = "add.partitionValues.key_value.key";
static const char* kPvVal = "add.partitionValues.key_value.value";

// Host validation of the postfix program: operand indices and stack discipline.
static void check_program(const dr_predicate& p) {
  if (p.ncols < 0 || uint32_t(p.ncols) > filter_max_cols())
    fail(DR_E_UNSUPPORTED, fmt("at most %u partition columns per predicate", filter_max_cols()));
  if (p.nops <= 0 || !p.ops) fail(DR_E_INVALID_ARG, "empty predicate program");
  if (p.ncols && (!p.col_names || !p.col_types)) fail(DR_E_INVALID_ARG, "missing partition columns");
  if (p.nlits && (!p.lit_types || !p.lit_i64 || !p.lit_null || !p.lit_str_off))
    fail(DR_E_INVALID_ARG, "missing literals");
  for (int32_t c = 0; c < p.ncols; ++c)
    if (p.col_types[c] < DR_T_STRING || p.col_types[c] > DR_T_BOOLEAN || !p.col_names[c])
      fail(DR_E_UNSUPPORTED, "unsupported partition column type");
  // stack discipline: every op's operands are whole subtrees (postfix -> tree)
  std::vector<int32_t> stack;
  for (int32_t k = 0; k < p.nops; ++k) {
    const int op = p.ops[k].opcode, arg = p.ops[k].arg;
    size_t pops = 0;
    switch (op) {
      case DR_OP_COL:
        if (arg < 0 || arg >= p.ncols) fail(DR_E_INVALID_ARG, "predicate column index out of range");
        break;
      case DR_OP_LIT:
        if (arg < 0 || arg >= p.nlits) fail(DR_E_INVALID_ARG, "predicate literal index out of range");
        break;
      case DR_OP_EQ: case DR_OP_NE: case DR_OP_LT: case DR_OP_LE: case DR_OP_GT: case DR_OP_GE:
      case DR_OP_NSEQ: case DR_OP_AND: case DR_OP_OR:
        pops = 2;
        break;
      case DR_OP_IN:
        if (arg < 0) fail(DR_E_INVALID_ARG, "predicate stack underflow (IN)");
        pops = size_t(arg) + 1;
        break;
      case DR_OP_ISNULL: case DR_OP_ISNOTNULL: case DR_OP_NOT:
        pops = 1;
        break;
      default: fail(DR_E_INVALID_ARG, fmt("unknown predicate opcode %d", op));
    }
    if (stack.size() < pops)
      fail(DR_E_INVALID_ARG, op == DR_OP_IN ? "predicate stack underflow (IN)" : "predicate stack underflow");
    stack.resize(stack.size() - pops);
    stack.push_back(k);
  }
  if (stack.size() != 1) fail(DR_E_INVALID_ARG, "predicate program must leave one value");
}

// Lowers the ABI program to the device form. `x e1..en IN(n)` becomes
// `x IN_START e1 IN_STEP .. en IN_STEP IN_END`, so an IN list of any length needs two stack slots
// beyond its value (In.eval semantics are unchanged: true if any element equals, else null if the
// value or any element is null, else false). Returns (opcode, arg) pairs; fails if the lowered
// program still needs more than the device stack.
static std::vector<int32_t> lower_program(const dr_predicate& p) {
  // subtree extents: start[k] = first op of the subtree rooted at op k
  std::vector<int32_t> start(size_t(p.nops)), stack;
  std::vector<std::vector<int32_t>> kids(size_t(p.nops));
  for (int32_t k = 0; k < p.nops; ++k) {
    const int op = p.ops[k].opcode;
    size_t pops = op == DR_OP_COL || op == DR_OP_LIT ? 0
                : op == DR_OP_IN ? size_t(p.ops[k].arg) + 1
                : (op == DR_OP_ISNULL || op == DR_OP_ISNOTNULL || op == DR_OP_NOT) ? 1 : 2;
    kids[size_t(k)].assign(stack.end() - ptrdiff_t(pops), stack.end());
    stack.resize(stack.size() - pops);
    start[size_t(k)] = kids[size_t(k)].empty() ? k : start[size_t(kids[size_t(k)][0])];
    stack.push_back(k);
  }
  std::vector<int32_t> out;
  int depth = 0, max_depth = 0;
  auto put = [&](int32_t op, int32_t arg, int delta) {
    out.push_back(op);
    out.push_back(arg);
    depth += delta;
    max_depth = std::max(max_depth, depth);
  };
  std::function<void(int32_t)> emit = [&](int32_t k) {
    const int op = p.ops[k].opcode, arg = p.ops[k].arg;
    const auto& ch = kids[size_t(k)];
    if (op == DR_OP_IN) {
      emit(ch[0]);
      put(FILTER_OP_IN_START, 0, +1);
      for (size_t q = 1; q < ch.size(); ++q) {
        emit(ch[q]);
        put(FILTER_OP_IN_STEP, 0, -1);
      }
      put(FILTER_OP_IN_END, 0, -1);
      return;
    }
    for (int32_t c : ch) emit(c);
    put(op, arg, 1 - int(ch.size()));
  };
  emit(p.nops - 1);
  if (uint32_t(max_depth) > filter_max_stack()) fail(DR_E_UNSUPPORTED, "predicate program too deep");
  return out;
}

// Leaf form of a program (k_filter_leaf) when every comparison is between one partition column and
// literals of its kind and the rest is AND / OR / NOT: each leaf is evaluated straight from the typed
// K5 cache, IN lists become sorted sets searched by bisection, and the boolean combination runs on
// a register stack. Returns false (generic interpreter, k_filter_typed) for anything else.
struct LeafPlan {
  std::vector<FilterLeaf> leaves;
  std::vector<int32_t> prog;
  std::vector<int64_t> i64;        // literal slots
  std::vector<std::string> str;
};
static bool leafify(const dr_predicate& p, LeafPlan& L) {
  std::vector<std::vector<int32_t>> kids(size_t(p.nops));
  std::vector<int32_t> stack;
  for (int32_t k = 0; k < p.nops; ++k) {
    const int op = p.ops[k].opcode;
    const size_t pops = op == DR_OP_COL || op == DR_OP_LIT ? 0
                      : op == DR_OP_IN ? size_t(p.ops[k].arg) + 1
                      : (op == DR_OP_ISNULL || op == DR_OP_ISNOTNULL || op == DR_OP_NOT) ? 1 : 2;
    kids[size_t(k)].assign(stack.end() - ptrdiff_t(pops), stack.end());
    stack.resize(stack.size() - pops);
    stack.push_back(k);
  }
  auto is_col = [&](int32_t k) { return p.ops[k].opcode == DR_OP_COL; };
  auto is_lit = [&](int32_t k) { return p.ops[k].opcode == DR_OP_LIT; };
  auto kind_ok = [&](int32_t col, int32_t lit) {  // string columns with string literals, others numeric
    return (p.col_types[col] == DR_T_STRING) == (p.lit_types[lit] == DR_T_STRING);
  };
  auto slot = [&](int32_t lit) {
    L.i64.push_back(p.lit_i64[lit]);
    L.str.emplace_back(reinterpret_cast<const char*>(p.lit_str_bytes) + p.lit_str_off[lit],
                       size_t(p.lit_str_off[lit + 1] - p.lit_str_off[lit]));
    return int32_t(L.i64.size() - 1);
  };
  int depth = 0, max_depth = 0;
  std::function<bool(int32_t)> emit = [&](int32_t k) -> bool {
    const int op = p.ops[k].opcode;
    const auto& ch = kids[size_t(k)];
    auto push_leaf = [&](const FilterLeaf& f) {
      L.prog.push_back(LEAF_OP_LEAF);
      L.prog.push_back(int32_t(L.leaves.size()));
      L.leaves.push_back(f);
      max_depth = std::max(max_depth, ++depth);
      return true;
    };
    switch (op) {
      case DR_OP_AND: case DR_OP_OR:
        if (!emit(ch[0]) || !emit(ch[1])) return false;
        L.prog.push_back(op == DR_OP_AND ? LEAF_OP_AND : LEAF_OP_OR);
        L.prog.push_back(0);
        --depth;
        return true;
      case DR_OP_NOT:
        if (!emit(ch[0])) return false;
        L.prog.push_back(LEAF_OP_NOT);
        L.prog.push_back(0);
        return true;
      case DR_OP_ISNULL: case DR_OP_ISNOTNULL:
        if (!is_col(ch[0])) return false;
        return push_leaf(FilterLeaf{p.ops[ch[0]].arg, op, 0, 0, 0, 0});
      case DR_OP_EQ: case DR_OP_NE: case DR_OP_LT: case DR_OP_LE: case DR_OP_GT: case DR_OP_GE: case DR_OP_NSEQ: {
        int32_t c, l, fop = op;
        if (is_col(ch[0]) && is_lit(ch[1])) {
          c = p.ops[ch[0]].arg; l = p.ops[ch[1]].arg;
        } else if (is_lit(ch[0]) && is_col(ch[1])) {
          c = p.ops[ch[1]].arg; l = p.ops[ch[0]].arg;
          fop = op == DR_OP_LT ? DR_OP_GT : op == DR_OP_GT ? DR_OP_LT : op == DR_OP_LE ? DR_OP_GE
              : op == DR_OP_GE ? DR_OP_LE : op;
        } else {
          return false;
        }
        if (!p.lit_null[l] && !kind_ok(c, l)) return false;
        return push_leaf(FilterLeaf{c, fop, slot(l), 0, p.lit_null[l] ? 1 : 0, 0});
      }
      case DR_OP_IN: {
        if (!is_col(ch[0])) return false;
        const int32_t c = p.ops[ch[0]].arg;
        const bool str = p.col_types[c] == DR_T_STRING;
        bool has_null = false;
        std::vector<int64_t> iv;
        std::vector<std::string> sv;
        for (size_t q = 1; q < ch.size(); ++q) {
          if (!is_lit(ch[q])) return false;
          const int32_t l = p.ops[ch[q]].arg;
          if (p.lit_null[l]) { has_null = true; continue; }
          if (!kind_ok(c, l)) return false;
          if (str) sv.emplace_back(reinterpret_cast<const char*>(p.lit_str_bytes) + p.lit_str_off[l],
                                   size_t(p.lit_str_off[l + 1] - p.lit_str_off[l]));
          else iv.push_back(p.lit_i64[l]);
        }
        std::sort(iv.begin(), iv.end());
        iv.erase(std::unique(iv.begin(), iv.end()), iv.end());
        std::sort(sv.begin(), sv.end());  // bytewise (std::string compares as unsigned char)
        sv.erase(std::unique(sv.begin(), sv.end()), sv.end());
        const int32_t first = int32_t(L.i64.size());
        const size_t m = str ? sv.size() : iv.size();
        // an integer set spanning < 2^16 values: a bitmap, one word read per file instead of a
        // binary search (pad = 1; literals [min, words, bits...])
        if (!str && m >= 8 && uint64_t(iv.back()) - uint64_t(iv.front()) < 65536) {
          const uint64_t span = uint64_t(iv.back()) - uint64_t(iv.front()) + 1, nw = (span + 63) / 64;
          std::vector<uint64_t> bits(nw, 0);
          for (int64_t x : iv) {
            const uint64_t d = uint64_t(x) - uint64_t(iv.front());
            bits[d >> 6] |= uint64_t(1) << (d & 63);
          }
          L.i64.push_back(iv.front());
          L.i64.push_back(int64_t(nw));
          for (uint64_t w : bits) L.i64.push_back(int64_t(w));
          L.str.resize(L.i64.size());
          return push_leaf(FilterLeaf{c, DR_OP_IN, first, int32_t(m), has_null ? 1 : 0, 1});
        }
        for (size_t q = 0; q < m; ++q) {
          L.i64.push_back(str ? 0 : iv[q]);
          L.str.push_back(str ? sv[q] : std::string());
        }
        return push_leaf(FilterLeaf{c, DR_OP_IN, first, int32_t(m), has_null ? 1 : 0, 0});
      }
      default:
        return false;
    }
  };
  return emit(p.nops - 1) && max_depth <= 32;
}

// Builds the K5 cache columns `want` (name, type) of st's live AddFiles in one k_pv_extract pass.
// Java's Double.parseDouble / Float.parseFloat for the values k_pv_extract left to the host (more
// than 19 significant digits, exponents off Clinger's fast path, hexadecimal significands): the text
// was already checked against the decimal grammar on the device; glibc's strtod / strtof round
// correctly, as Java does. Java's hexadecimal form needs a binary exponent ('p'): without one the
// cast is null.
static void fix_fp_values(dr_ctx* ctx, dr_state::PvCol& col, const DBuf<uint64_t>& hard, uint64_t nh) {
  hipStream_t stream = ctx->stream;
  const std::vector<uint64_t> h = d2h(hard.p, 3 * nh, stream);
  const bool is_float = (col.type & 0xff) == DR_T_FLOAT;
  std::vector<uint64_t> rows(nh), bits(nh);
  std::vector<uint8_t> nulls(nh, 0);
  for (uint64_t k = 0; k < nh; ++k) {
    rows[k] = h[3 * k];
    std::string t(size_t(h[3 * k + 2]), '\0');
    if (!t.empty()) HIP_OK(hipMemcpy(&t[0], reinterpret_cast<const void*>(h[3 * k + 1]), t.size(), hipMemcpyDeviceToHost));
    size_t b = 0, e = t.size();
    while (b < e && uint8_t(t[b]) <= ' ') ++b;
    while (e > b && uint8_t(t[e - 1]) <= ' ') --e;
    t = t.substr(b, e - b);
    if (!t.empty() && strchr("fFdD", t.back())) t.pop_back();
    const size_t x = t.find_first_of("xX");
    if (x != std::string::npos && t.find_first_of("pP") == std::string::npos) {
      nulls[k] = 1;
      continue;
    }
    char* end = nullptr;
    if (is_float) {
      const float f = strtof(t.c_str(), &end);
      uint32_t u;
      memcpy(&u, &f, 4);
      bits[k] = u;
    } else {
      const double d = strtod(t.c_str(), &end);
      memcpy(&bits[k], &d, 8);
    }
    if (end != t.c_str() + t.size()) nulls[k] = 1;
  }
  // one upload of the rows, values and null bytes (the host vectors outlive the synchronisation
  // below), then one scatter into the cache columns
  DBuf<uint64_t> d_rows(ctx, nh), d_bits(ctx, nh);
  DBuf<uint8_t> d_nulls(ctx, nh);
  HIP_OK(hipMemcpyAsync(d_rows.p, rows.data(), nh * 8, hipMemcpyHostToDevice, stream));
  HIP_OK(hipMemcpyAsync(d_bits.p, bits.data(), nh * 8, hipMemcpyHostToDevice, stream));
  HIP_OK(hipMemcpyAsync(d_nulls.p, nulls.data(), nh, hipMemcpyHostToDevice, stream));
  launch_scatter_fp(d_rows.p, d_bits.p, d_nulls.p, nh, is_float ? col.w32.p : nullptr, is_float ? nullptr : col.w64.p,
                    col.isnull.p, stream);
  HIP_OK(hipStreamSynchronize(stream));
}

static void build_pv_columns(dr_state& st, const std::vector<std::pair<std::string, int32_t>>& want) {
  dr_ctx* ctx = st.ctx;
  hipStream_t stream = ctx->stream;
  StagedData& s = *st.sources[0];
  const uint64_t R = s.ck_rows;
  const uint64_t n = st.n_live;
  PvExtractArgs a{};
  a.live = st.live.p;
  a.n_live = n;
  a.src_off = st.src_off.p;
  a.src_len = st.src_len.p;
  a.ck_rows = R;
  a.json = s.d_json.p;
  DBuf<uint64_t> json_bases;
  if (st.src_id.p) {
    std::vector<uint64_t> bases;
    for (auto& src : st.sources) bases.push_back(reinterpret_cast<uint64_t>(src->d_json.p));
    json_bases = upload(ctx, bases.data(), bases.size());
    a.act_flags = st.flags.p;
    a.src_id = st.src_id.p;
    a.json_bases = json_bases.p;
  }
  // checkpoint side: decode the add.partitionValues map columns (planned once per staged segment;
  // the decoded entries are freed once the typed columns are built)
  DBuf<uint8_t> kdef, krep, vdef, vrep;
  DBuf<uint64_t> kptr, vptr, row_start, dict_ptr, rpos;
  DBuf<uint32_t> klen, vlen, dict_len, pq_err(ctx, 1), rflag;
  DBuf<uint8_t> scratch(ctx, scan_scratch_for(0));
  pq_err.zero(stream);
  if (R && n) {
    {
      std::lock_guard<std::mutex> g(s.pv_mu);
      if (!s.pv) {
        auto P = std::make_unique<PagePlan>();
        P->paths = {kPvKey, kPvVal};
        plan_pages(s, *P);
        s.pv = std::move(P);
      }
    }
    PagePlan& P = *s.pv;
    if (P.present[0] && P.present[1]) {
      const uint64_t E = P.levels[0];
      if (P.levels[1] != E) fail(DR_E_PARQUET, "partitionValues key/value columns disagree");
      kdef = DBuf<uint8_t>(ctx, E); krep = DBuf<uint8_t>(ctx, E); kptr = DBuf<uint64_t>(ctx, E); klen = DBuf<uint32_t>(ctx, E);
      vdef = DBuf<uint8_t>(ctx, E); vrep = DBuf<uint8_t>(ctx, E); vptr = DBuf<uint64_t>(ctx, E); vlen = DBuf<uint32_t>(ctx, E);
      kdef.zero(stream);
      vdef.zero(stream);
      ParquetArgs pa{};
      pa.ncols = 2;
      pa.cols[0] = FlatColumn{kdef.p, krep.p, nullptr, kptr.p, klen.p};
      pa.cols[1] = FlatColumn{vdef.p, vrep.p, nullptr, vptr.p, vlen.p};
      if (scratch.n < scan_scratch_for(E)) scratch = DBuf<uint8_t>(ctx, scan_scratch_for(E));
      decode_pages(ctx, P, pa, dict_ptr, dict_len, pq_err, scratch.p);
      if (d2h_one(pq_err.p, stream) != 0)
        fail(DR_E_PARQUET, fmt("device decode of add.partitionValues failed (code %u)", d2h_one(pq_err.p, stream)));
      rflag = DBuf<uint32_t>(ctx, E);
      rpos = DBuf<uint64_t>(ctx, E + 1);
      launch_rep0_flags(krep.p, E, rflag.p, stream);
      launch_scan_u32(rflag.p, rpos.p, E, ss(scratch), stream);
      if (d2h_one(rpos.p + E, stream) != R) fail(DR_E_PARQUET, "add.partitionValues: one map per checkpoint row expected");
      row_start = DBuf<uint64_t>(ctx, R + 1);
      launch_row_starts(krep.p, E, rpos.p, row_start.p, stream);
      HIP_OK(hipMemcpyAsync(row_start.p + R, &E, 8, hipMemcpyHostToDevice, stream));
      a.has_map = 1;
      a.row_start = row_start.p;
      a.key_def = kdef.p; a.key_ptr = kptr.p; a.key_len = klen.p; a.key_max_def = P.max_def[0];
      a.val_def = vdef.p; a.val_ptr = vptr.p; a.val_len = vlen.p; a.val_max_def = P.max_def[1];
    }
  }
  std::vector<uint64_t> name_off(want.size() + 1, 0);
  std::string names;
  for (size_t c = 0; c < want.size(); ++c) {
    names += want[c].first;
    name_off[c + 1] = names.size();
  }
  DBuf<uint64_t> d_name_off = upload(ctx, name_off.data(), name_off.size());
  DBuf<uint8_t> d_names = upload(ctx, reinterpret_cast<const uint8_t*>(names.data()), names.size());
  a.ncols = int32_t(want.size());
  a.col_name_off = d_name_off.p;
  a.col_names = d_names.p;
  std::vector<std::unique_ptr<dr_state::PvCol>> made;
  for (size_t c = 0; c < want.size(); ++c) {
    auto col = std::make_unique<dr_state::PvCol>();
    col->name = want[c].first;
    col->type = want[c].second;
    col->isnull = DBuf<uint8_t>(ctx, n);
    PvColumn& pc = a.cols[c];
    pc.type = col->type;
    pc.isnull = col->isnull.p;
    const int base = col->type & 0xff;
    if (base == DR_T_STRING || base == DR_T_BINARY) {
      col->sptr = DBuf<uint64_t>(ctx, n);
      col->slen = DBuf<uint32_t>(ctx, n);
      col->s8 = DBuf<uint64_t>(ctx, n);
      pc.sptr = col->sptr.p;
      pc.slen = col->slen.p;
      pc.s8 = col->s8.p;
    } else if (base == DR_T_LONG || base == DR_T_DOUBLE || base == DR_T_TIMESTAMP || base == DR_T_DECIMAL) {
      col->w64 = DBuf<int64_t>(ctx, n);
      pc.w64 = col->w64.p;
      if (base == DR_T_DECIMAL) {
        col->w64hi = DBuf<int64_t>(ctx, n);
        pc.w64hi = col->w64hi.p;
        if (((col->type >> 8) & 0xff) <= 9) {
          col->w32 = DBuf<uint32_t>(ctx, n);
          pc.w32 = col->w32.p;
        }
      }
    } else {
      col->w32 = DBuf<uint32_t>(ctx, n);
      pc.w32 = col->w32.p;
    }
    made.push_back(std::move(col));
  }
  // counters: 0 arena fill, 1 arena need, 2.. per column: float / double values left to the host
  const size_t nc = want.size();
  DBuf<unsigned long long> ctr(ctx, 2 + nc);
  DBuf<uint32_t> ferr(ctx, 1);
  ctr.zero(stream);
  ferr.zero(stream);
  a.arena_fill = ctr.p;
  a.arena_need = ctr.p + 1;
  a.error = ferr.p;
  for (size_t c = 0; c < nc; ++c) a.cols[c].nhard = ctr.p + 2 + c;
  launch_pv_extract(a, stream);
  const std::vector<unsigned long long> cnt = d2h(ctr.p, 2 + nc, stream);
  std::vector<DBuf<uint64_t>> hard(nc);
  bool rerun = cnt[1] != 0;
  for (size_t c = 0; c < nc; ++c)
    if (cnt[2 + c]) {
      hard[c] = DBuf<uint64_t>(ctx, 3 * cnt[2 + c]);
      a.cols[c].hard = hard[c].p;
      rerun = true;
    }
  if (rerun) {
    // some partition values carry JSON escapes (unescaped into an arena) or are floating-point
    // numbers off the device's exact path (listed for the host): rerun with those buffers
    if (cnt[1]) {
      auto arena = std::make_shared<DBuf<uint8_t>>(ctx, cnt[1] + 64);
      a.arena = arena->p;
      a.arena_cap = cnt[1] + 64;
      st.pv_arenas.push_back(arena);
    }
    HIP_OK(hipMemsetAsync(ctr.p, 0, 8 * (2 + nc), stream));
    launch_pv_extract(a, stream);
  }
  const uint32_t e = d2h_one(ferr.p, stream);
  if (e & 1u) fail(DR_E_PARSE, "malformed add.partitionValues in a live AddFile's JSON line");
  if (e & 2u) fail(DR_E_INTERNAL, "partition value arena overflow");
  for (size_t c = 0; c < nc; ++c)
    if (cnt[2 + c]) fix_fp_values(ctx, *made[c], hard[c], cnt[2 + c]);
  for (auto& c : made) st.pv_cols.push_back(std::move(c));
}

// ---------------------------------------------------------------------------------------------------
// checkpoint writer on the device (Checkpoints.writeCheckpoint / buildCheckpoint,
// D/Checkpoints.scala:229-365): the state's rows -- protocol, metaData, txns, then allFiles, then the
// tombstones, every record with dataChange=false -- as one Parquet part. The file-action columns
// are encoded on the device from the device export (k_enc_*: levels + PLAIN values, bit-packed
// levels); the handful of protocol / metaData / txn rows and the footer are written on the host.
// The device columns' pages are SNAPPY-compressed on the device with DR_CKPT_SNAPPY (Spark's default
// codec; k_snap_compress), else written UNCOMPRESSED; the host-encoded head-row pages are
// uncompressed. The schema is the reference's checkpoint schema, nullable throughout.
// ---------------------------------------------------------------------------------------------------
struct ThriftW {  // Thrift compact protocol
  std::vector<uint8_t> b;
  std::vector<int> last{0};
  void varint(uint64_t v) {
    while (v >= 0x80) { b.push_back(uint8_t(v) | 0x80); v >>= 7; }
    b.push_back(uint8_t(v));
  }
  static uint64_t zz(int64_t v) { return (uint64_t(v) << 1) ^ uint64_t(v >> 63); }
  void field(int id, uint8_t type) {
    const int d = id - last.back();
    if (d > 0 && d <= 15) b.push_back(uint8_t(d << 4) | type);
    else { b.push_back(type); varint(zz(id)); }
    last.back() = id;
  }
  void i32(int id, int32_t v) { field(id, 5); varint(zz(v)); }
  void i64(int id, int64_t v) { field(id, 6); varint(zz(v)); }
  void str(int id, const std::string& s) { field(id, 8); varint(s.size()); b.insert(b.end(), s.begin(), s.end()); }
  void begin_struct(int id) { field(id, 12); last.push_back(0); }
  void end_struct() { b.push_back(0); last.pop_back(); }
  void begin_list(int id, uint8_t etype, size_t n) {
    field(id, 9);
    if (n < 15) b.push_back(uint8_t(n << 4) | etype);
    else { b.push_back(0xF0 | etype); varint(n); }
  }
  void elem_begin() { last.push_back(0); }  // a struct element of a list: no field header
  void elem_end() { b.push_back(0); last.pop_back(); }
  void elem_i32(int32_t v) { varint(zz(v)); }
  void elem_str(const std::string& s) { varint(s.size()); b.insert(b.end(), s.begin(), s.end()); }
};

enum PqType { PQ_BOOLEAN = 0, PQ_INT32 = 1, PQ_INT64 = 2, PQ_INT96 = 3, PQ_FLOAT = 4, PQ_DOUBLE = 5, PQ_BYTE_ARRAY = 6,
              PQ_FLBA = 7 };
enum PqConv { PC_UTF8 = 0, PC_MAP = 1, PC_LIST = 3, PC_DECIMAL = 5, PC_DATE = 6, PC_INT_8 = 15, PC_INT_16 = 16 };
enum PqRep { PR_REQUIRED = 0, PR_OPTIONAL = 1, PR_REPEATED = 2 };

struct SElem {
  std::string name;
  int type = -1, rep = -1, nkids = -1, conv = -1;
  int type_length = -1, scale = -1, precision = -1;  // FIXED_LEN_BYTE_ARRAY / DECIMAL
};

// One leaf of the checkpoint schema and how its column is produced.
struct CkLeafW {
  std::vector<std::string> path;
  int phys = 0, max_def = 0, max_rep = 0;
  int side = -1;             // 0 adds, 1 removes (device), -1 protocol / metaData / txn rows (host)
  EncLeaf enc{};             // device source (side leaves)
  // host leaves: per head row, its levels and PLAIN values
  std::vector<std::vector<uint8_t>> hdef, hrep, hval;
};

template <typename V>
static void put_u32le(V& b, uint32_t v) {
  for (int k = 0; k < 4; ++k) b.push_back(uint8_t(v >> (8 * k)));
}
template <typename V>
static void put_varint(V& b, uint64_t v) {
  while (v >= 0x80) { b.push_back(uint8_t(v) | 0x80); v >>= 7; }
  b.push_back(uint8_t(v));
}
static int level_width(int max_level) {
  int w = 0;
  while ((1 << w) <= max_level) ++w;
  return w;
}
// RLE runs of `lv` then `zeros` zero levels (the RLE/bit-packing hybrid, RLE runs only)
static void rle_levels(std::vector<uint8_t>& out, const std::vector<uint8_t>& lv, uint64_t zeros, int width) {
  const int vb = (width + 7) / 8;
  size_t i = 0;
  while (i < lv.size()) {
    size_t j = i;
    while (j < lv.size() && lv[j] == lv[i]) ++j;
    uint64_t run = j - i;
    if (j == lv.size() && lv[i] == 0) { run += zeros; zeros = 0; }
    put_varint(out, run << 1);
    for (int k = 0; k < vb; ++k) out.push_back(uint8_t(lv[i] >> (8 * k)));
    i = j;
  }
  if (zeros) {
    put_varint(out, zeros << 1);
    for (int k = 0; k < vb; ++k) out.push_back(0);
  }
}

// Levels and PLAIN values of one head row for a host leaf (the action's JSON as the checkpoint
// writer's row: a missing field is null; txn.version and the protocol versions default to 0).
static void head_row_levels(const CkLeafW& L, int top_kind, const NonFileAction* a, std::vector<uint8_t>& def,
                            std::vector<uint8_t>& rep, std::vector<uint8_t>& val) {
  static const char* kTop[3] = {"txn", "metaData", "protocol"};
  const int mine = L.path[0] == kTop[0] ? 4 : L.path[0] == kTop[1] ? 3 : 5;
  if (!a || a->kind != mine) {
    def.push_back(0);
    if (L.max_rep) rep.push_back(0);
    return;
  }
  (void)top_kind;
  auto put_value = [&](const JVal& v) {
    if (L.phys == PQ_BYTE_ARRAY) {
      const std::string s = v.t == JVal::STR ? v.s : json_dump(v);
      put_u32le(val, uint32_t(s.size()));
      val.insert(val.end(), s.begin(), s.end());
    } else if (L.phys == PQ_INT64) {
      const uint64_t x = uint64_t(v.as_int());
      for (int k = 0; k < 8; ++k) val.push_back(uint8_t(x >> (8 * k)));
    } else {
      put_u32le(val, uint32_t(int32_t(v.as_int())));
    }
  };
  const JVal* cur = a->val.get();
  int d = 1;  // the top-level struct is defined
  const bool map_key = L.path.size() >= 2 && L.path[L.path.size() - 2] == "key_value" && L.path.back() == "key";
  const bool map_val = L.path.size() >= 2 && L.path[L.path.size() - 2] == "key_value" && L.path.back() == "value";
  const bool list_el = L.path.size() >= 2 && L.path[L.path.size() - 2] == "list";
  const size_t nfields = L.path.size() - 1 - ((map_key || map_val || list_el) ? 2 : 0);
  static const JVal kEmptyObj = [] {
    JVal o;
    o.t = JVal::OBJ;
    return o;
  }();
  for (size_t f = 1; f <= nfields; ++f) {
    const JVal* v = cur->get(L.path[f]);
    // the checkpoint writer's metaData row: a missing format / options / configuration is empty
    if ((!v || v->t == JVal::NUL) && L.path[0] == "metaData" &&
        (L.path[f] == "format" || L.path[f] == "options" || L.path[f] == "configuration"))
      v = &kEmptyObj;
    const bool last = f == nfields && !(map_key || map_val || list_el);
    const bool dflt = last && ((L.path[0] == "txn" && L.path[1] == "version") || L.path[0] == "protocol");
    if (!v || v->t == JVal::NUL || (last && L.phys != PQ_BYTE_ARRAY && !v->is_int())) {
      if (dflt) {
        JVal zero;
        zero.t = JVal::NUM;
        zero.s = "0";
        def.push_back(uint8_t(L.max_def));
        put_value(zero);
      } else {
        def.push_back(uint8_t(d));
      }
      if (L.max_rep) rep.push_back(0);
      return;
    }
    ++d;
    cur = v;
  }
  if (!(map_key || map_val || list_el)) {
    def.push_back(uint8_t(d));
    put_value(*cur);
    return;
  }
  // a map (object) or a list (array): defined at d; empty -> one level at d
  std::vector<const JVal*> keys_v;
  std::vector<std::string> keys;
  std::vector<const JVal*> vals;
  if (list_el && cur->t == JVal::ARR) {
    for (const JVal& x : cur->a) vals.push_back(&x);
  } else if (!list_el && cur->t == JVal::OBJ) {
    for (auto& kv : cur->o) {  // first position, last value per key (LinkedHashMap)
      size_t k = 0;
      while (k < keys.size() && keys[k] != kv.first) ++k;
      if (k == keys.size()) { keys.push_back(kv.first); vals.push_back(&kv.second); }
      else vals[k] = &kv.second;
    }
  }
  if (vals.empty()) {
    def.push_back(uint8_t(d));
    rep.push_back(0);
    return;
  }
  for (size_t e = 0; e < vals.size(); ++e) {
    rep.push_back(e ? 1 : 0);
    if (map_key) {
      def.push_back(uint8_t(d + 1));
      put_u32le(val, uint32_t(keys[e].size()));
      val.insert(val.end(), keys[e].begin(), keys[e].end());
    } else if (vals[e]->t == JVal::NUL) {
      def.push_back(uint8_t(d + 1));
    } else {
      def.push_back(uint8_t(d + 2));
      put_value(*vals[e]);
    }
  }
}

// A partition column's Spark type name (the schemaString's) -> dr_pred_type (decimal(p,s): the
// precision and scale ride in bits 8..23 of the code); -1 when the cast is not supported.
static int32_t spark_type_code(const std::string& t) {
  if (t == "string") return DR_T_STRING;
  if (t == "byte") return DR_T_BYTE;
  if (t == "short") return DR_T_SHORT;
  if (t == "integer") return DR_T_INT;
  if (t == "long") return DR_T_LONG;
  if (t == "date") return DR_T_DATE;
  if (t == "boolean") return DR_T_BOOLEAN;
  if (t == "float") return DR_T_FLOAT;
  if (t == "double") return DR_T_DOUBLE;
  if (t == "timestamp") return DR_T_TIMESTAMP;
  if (t == "binary") return DR_T_BINARY;
  int p = 0, sc = 0;
  char close = 0;
  if (t == "decimal") return DR_T_DECIMAL | (10 << 8);  // DecimalType.USER_DEFAULT: decimal(10,0)
  if (std::sscanf(t.c_str(), "decimal(%d,%d%c", &p, &sc, &close) == 3 && close == ')' && p >= 1 && p <= 38 &&
      sc >= 0 && sc <= p)
    return DR_T_DECIMAL | (p << 8) | (sc << 16);
  return -1;
}

// Bytes of a FIXED_LEN_BYTE_ARRAY decimal of this precision (Spark's Decimal.minBytesForPrecision).
static int decimal_bytes(int precision) {
  int n = 1;
  while (std::pow(2.0, 8.0 * n - 1) < std::pow(10.0, precision)) ++n;
  return n;
}

// The part file as it is built: host-encoded bytes (page headers, head-row leaves, the footer) and
// device page bodies, each at its file offset. The device bodies stay in HBM until the file is
// complete; then one pinned block of the exact size takes every segment (the bodies by D2H copies
// queued back to back, one stream sync) and is handed to the caller (dr_free returns it to the
// context's pinned pool): no pageable D2H, no realloc growth, no second host copy.
struct PartFile {
  struct Seg {
    uint64_t off = 0;
    std::vector<uint8_t> h;
    DBuf<uint8_t> d;
    uint64_t dn = 0;
  };
  std::vector<Seg> segs;
  uint64_t size = 0;
  std::vector<uint8_t>& tail() {  // the host segment at the end of the file
    if (segs.empty() || segs.back().dn) {
      segs.emplace_back();
      segs.back().off = size;
    }
    return segs.back().h;
  }
  template <typename It>
  void host(It a, It b) {
    std::vector<uint8_t>& t = tail();
    const size_t k = size_t(std::distance(a, b));
    t.insert(t.end(), a, b);
    size += k;
  }
  void host(std::initializer_list<uint8_t> l) { host(l.begin(), l.end()); }
  void push_back(uint8_t x) {  // (put_u32le / put_varint)
    tail().push_back(x);
    ++size;
  }
  void dev(DBuf<uint8_t>&& b, uint64_t n) {
    if (!n) return;
    segs.emplace_back();
    segs.back().off = size;
    segs.back().d = std::move(b);
    segs.back().dn = n;
    size += n;
  }
};

// Pinned part files handed out by dr_state_write_checkpoint, by address: dr_free returns one to its
// context's pinned pool (or frees it when the context is gone).
static std::mutex g_pinned_out_mu;
static std::unordered_map<void*, dr_ctx*> g_pinned_out;

// A range outlives its state and its context: live ranges are registered in g_ranges, and
// dr_ctx_destroy detaches those of its context (their blocks are then unpinned by dr_range_release
// itself instead of returning to the context's cache).
struct dr_range {
  dr_ctx* ctx = nullptr;
  void* block = nullptr;
  dr_range() = default;
  dr_range(const dr_range&) = delete;
  dr_range& operator=(const dr_range&) = delete;
  ~dr_range() {
    if (!block) return;
    if (ctx) ctx->host_release(block);
    else (void)hipHostFree(block);
  }
};
static std::mutex g_ranges_mu;
static std::unordered_set<dr_range*> g_ranges;

struct CkPartOut {
  uint8_t* data = nullptr;  // pinned (dr_ctx::host_alloc), registered in g_pinned_out
  uint64_t len = 0;
  int64_t rows = 0;
  int64_t add_rows = 0;  // add rows encoded (Checkpoints.scala:325-328's accumulator)
};

static void write_checkpoint_part(dr_state& st, int32_t part, int32_t parts, uint32_t opts, uint64_t rg_rows,
                                  CkPartOut& out) {
  DR_STAGE("checkpoint.write", st.ctx->stream);
  dr_ctx* ctx = st.ctx;
  ctx->begin_call();
  ensure_ready(st);
  hipStream_t stream = ctx->stream;
  // A sharded replay's state writes its own part: all of its survivors (hash-clustered, PROTOCOL.md's
  // parts may split the rows any way), the protocol / metaData / txn rows in part 1 only.
  // DR_CKPT_DEBUG=1: wall time per phase on stderr (device work synchronised at each mark)
  const bool dbg = std::getenv("DR_CKPT_DEBUG") != nullptr;
  auto t_last = std::chrono::steady_clock::now();
  std::map<std::string, double> t_acc;
  auto tmark = [&](const char* what) {
    if (!dbg) return;
    HIP_OK(hipStreamSynchronize(stream));
    const auto now = std::chrono::steady_clock::now();
    t_acc[what] += std::chrono::duration<double, std::milli>(now - t_last).count();
    t_last = now;
  };
  // head rows: protocol, metaData, txns (the checkpoint writer's order)
  std::vector<const NonFileAction*> head;
  const NonFileAction* md = nullptr;
  for (const NonFileAction& a : st.nonfile) if (a.kind == 5) head.push_back(&a);
  for (const NonFileAction& a : st.nonfile) if (a.kind == 3) { head.push_back(&a); md = &a; }
  for (const NonFileAction& a : st.nonfile) if (a.kind == 4) head.push_back(&a);
  if (st.sharded && part != 1) head.clear();
  const uint64_t H = head.size(), NA = st.n_live, NR = st.n_tomb, ROWS = H + NA + NR;
  const uint64_t step = parts > 1 && !st.sharded ? (ROWS + uint64_t(parts) - 1) / uint64_t(parts) : ROWS;
  const uint64_t p0 = st.sharded ? 0 : std::min<uint64_t>(ROWS, uint64_t(part - 1) * step);
  const uint64_t p1 = std::min<uint64_t>(ROWS, p0 + step);
  out.rows = int64_t(p1 - p0);
  // partitionValues_parsed: the metadata's partition schema (D/Checkpoints.scala:372-389)
  std::vector<std::pair<std::string, int32_t>> parsed;
  if ((opts & DR_CKPT_PARSED) && md) {
    const JVal* pc = md->val->get("partitionColumns");
    const JVal* ss = md->val->get("schemaString");
    JVal schema;
    if (pc && pc->t == JVal::ARR && !pc->a.empty() && ss && ss->t == JVal::STR &&
        json_parse(ss->s.data(), ss->s.size(), &schema)) {
      const JVal* fields = schema.get("fields");
      for (const JVal& c : pc->a) {
        int32_t code = -1;
        if (fields && fields->t == JVal::ARR)
          for (const JVal& f : fields->a) {
            const JVal* nm = f.get("name");
            const JVal* ty = f.get("type");
            if (nm && nm->t == JVal::STR && nm->s == c.s && ty && ty->t == JVal::STR) code = spark_type_code(ty->s);
          }
        if (code < 0) fail(DR_E_UNSUPPORTED, "partitionValues_parsed of partition column " + c.s + ": unsupported type");
        parsed.push_back({c.s, code});
      }
    }
  }
  if (!parsed.empty()) {
    std::vector<std::pair<std::string, int32_t>> want;
    for (auto& pc : parsed) {
      bool have = false;
      for (auto& c : st.pv_cols) have |= c->name == pc.first && c->type == pc.second;
      if (!have) want.push_back(pc);
    }
    if (!want.empty() && st.n_live) build_pv_columns(st, want);
  }
  // only the records of this part: adds [a0, a1), removes [b0, b1) (side-relative)
  const uint64_t a0 = std::min(NA, p0 > H ? p0 - H : 0), a1 = std::min(NA, p1 > H ? p1 - H : 0);
  const uint64_t b0 = std::min(NR, p0 > H + NA ? p0 - H - NA : 0), b1 = std::min(NR, p1 > H + NA ? p1 - H - NA : 0);
  tmark("setup");
  DevExport X[2];
  export_device(st, DR_LIVE, X[0], a0, a1);
  export_device(st, DR_TOMBSTONES, X[1], b0, b1);
  out.add_rows = int64_t(X[0].n);
  tmark("export");
  // ---- schema (DFS) and leaves ----
  std::vector<SElem> schema;
  std::vector<CkLeafW> leaves;
  std::vector<std::string> at;  // current group path
  auto group = [&](const std::string& name, int rep, int nkids, int conv = -1) {
    schema.push_back(SElem{name, -1, rep, nkids, conv});
  };
  auto leaf = [&](const std::string& name, int rep, int phys, int conv, int max_def, int max_rep, int side,
                  EncLeaf enc = EncLeaf{}) {
    schema.push_back(SElem{name, phys, rep, -1, conv});
    CkLeafW L;
    L.path = at;
    L.path.push_back(name);
    L.phys = phys;
    L.max_def = max_def;
    L.max_rep = max_rep;
    L.side = side;
    L.enc = enc;
    leaves.push_back(std::move(L));
  };
  auto str_map = [&](const std::string& name, int base, int side, EncLeaf k, EncLeaf v) {
    group(name, PR_OPTIONAL, 1, PC_MAP);
    at.push_back(name);
    group("key_value", PR_REPEATED, 2);
    at.push_back("key_value");
    leaf("key", PR_REQUIRED, PQ_BYTE_ARRAY, PC_UTF8, base + 2, 1, side, k);
    leaf("value", PR_OPTIONAL, PQ_BYTE_ARRAY, PC_UTF8, base + 3, 1, side, v);
    at.pop_back();
    at.pop_back();
  };
  auto side_map = [&](const DevExport& x, bool pv) {
    EncLeaf k{}, v{};
    k.kind = ENC_MAP_KEY;
    v.kind = ENC_MAP_VAL;
    k.null = v.null = pv ? x.pv_null.p : x.tags_null.p;
    k.entry_off = v.entry_off = pv ? x.off[EXC_PV_N].p : x.off[EXC_TAGS_N].p;
    k.eoff = pv ? x.pv_key_off.p : x.tags_key_off.p;
    k.ebytes = pv ? x.pv_key_bytes.p : x.tags_key_bytes.p;
    v.eoff = pv ? x.pv_val_off.p : x.tags_val_off.p;
    v.ebytes = pv ? x.pv_val_bytes.p : x.tags_val_bytes.p;
    v.enull = pv ? x.pv_val_null.p : x.tags_val_null.p;
    k.def_null = v.def_null = 1;
    k.def_present = 3;
    v.def_present = 4;
    return std::make_pair(k, v);
  };
  auto flat = [&](int kind, int dn, int dp) {
    EncLeaf e{};
    e.kind = kind;
    e.def_null = dn;
    e.def_present = dp;
    return e;
  };
  const bool stats = (opts & DR_CKPT_STATS) != 0;
  group("schema", -1, 5);
  // txn
  group("txn", PR_OPTIONAL, 3);
  at = {"txn"};
  leaf("appId", PR_OPTIONAL, PQ_BYTE_ARRAY, PC_UTF8, 2, 0, -1);
  leaf("version", PR_OPTIONAL, PQ_INT64, -1, 2, 0, -1);
  leaf("lastUpdated", PR_OPTIONAL, PQ_INT64, -1, 2, 0, -1);
  // add
  group("add", PR_OPTIONAL, 6 + (stats ? 1 : 0) + (parsed.empty() ? 0 : 1));
  at = {"add"};
  {
    const DevExport& x = X[0];
    EncLeaf e = flat(ENC_STR_OFF, 1, 2);
    e.off = x.path_off.p;
    e.bytes = x.path_bytes.p;
    leaf("path", PR_OPTIONAL, PQ_BYTE_ARRAY, PC_UTF8, 2, 0, 0, e);
    auto pv = side_map(x, true);
    str_map("partitionValues", 1, 0, pv.first, pv.second);
    e = flat(ENC_I64, 1, 2);
    e.i64 = x.size.p;
    leaf("size", PR_OPTIONAL, PQ_INT64, -1, 2, 0, 0, e);
    e = flat(ENC_I64, 1, 2);
    e.i64 = x.mtime.p;
    leaf("modificationTime", PR_OPTIONAL, PQ_INT64, -1, 2, 0, 0, e);
    leaf("dataChange", PR_OPTIONAL, PQ_BOOLEAN, -1, 2, 0, 0, flat(ENC_BOOL, 1, 2));
    auto tg = side_map(x, false);
    str_map("tags", 1, 0, tg.first, tg.second);
    if (stats) {
      e = flat(ENC_STR_OFF, 1, 2);
      e.off = x.off[EXC_STATS].p;
      e.bytes = x.stats_bytes.p;
      e.null = x.stats_null.p;
      leaf("stats", PR_OPTIONAL, PQ_BYTE_ARRAY, PC_UTF8, 2, 0, 0, e);
    }
    if (!parsed.empty()) {
      group("partitionValues_parsed", PR_OPTIONAL, int(parsed.size()));
      at.push_back("partitionValues_parsed");
      for (auto& pc : parsed) {
        const dr_state::PvCol* col = nullptr;
        for (auto& c : st.pv_cols) if (c->name == pc.first && c->type == pc.second) col = c.get();
        EncLeaf f{};
        f.def_null = 2;
        f.def_present = 3;
        if (col) f.null = col->isnull.p + a0;
        int phys = PQ_INT32, conv = -1, tlen = -1;
        const int prec = (pc.second >> 8) & 0xff, scale = (pc.second >> 16) & 0xff;
        switch (pc.second & 0xff) {
          case DR_T_STRING:
          case DR_T_BINARY:  // Cast(string AS binary): the UTF-8 bytes, no UTF8 annotation
            f.kind = ENC_STR_PTR;
            if (col) { f.sptr = col->sptr.p + a0; f.slen = col->slen.p + a0; }
            phys = PQ_BYTE_ARRAY;
            conv = (pc.second & 0xff) == DR_T_STRING ? PC_UTF8 : -1;
            break;
          case DR_T_LONG: f.kind = ENC_I64; if (col) f.i64 = col->w64.p + a0; phys = PQ_INT64; break;
          case DR_T_DOUBLE: f.kind = ENC_I64; if (col) f.i64 = col->w64.p + a0; phys = PQ_DOUBLE; break;
          case DR_T_FLOAT: f.kind = ENC_I32; if (col) f.i32 = col->w32.p + a0; phys = PQ_FLOAT; break;
          case DR_T_TIMESTAMP:  // spark.sql.parquet.outputTimestampType's default, INT96
            f.kind = ENC_INT96;
            if (col) f.i64 = col->w64.p + a0;
            phys = PQ_INT96;
            break;
          case DR_T_DECIMAL:  // Spark's non-legacy decimal layout: INT32 / INT64 / FIXED_LEN_BYTE_ARRAY
            conv = PC_DECIMAL;
            if (prec <= 9) {
              f.kind = ENC_I32;
              if (col) f.i32 = col->w32.p + a0;
            } else if (prec <= 18) {
              f.kind = ENC_I64;
              if (col) f.i64 = col->w64.p + a0;
              phys = PQ_INT64;
            } else {
              f.kind = ENC_FLBA_BE;
              if (col) { f.i64 = col->w64.p + a0; f.i64hi = col->w64hi.p + a0; }
              f.width = uint32_t(decimal_bytes(prec));
              tlen = int(f.width);
              phys = PQ_FLBA;
            }
            break;
          case DR_T_BOOLEAN: f.kind = ENC_BOOL; if (col) f.i32 = col->w32.p + a0; phys = PQ_BOOLEAN; break;
          default:
            f.kind = ENC_I32;
            if (col) f.i32 = col->w32.p + a0;
            conv = pc.second == DR_T_DATE ? PC_DATE : pc.second == DR_T_BYTE ? PC_INT_8 : pc.second == DR_T_SHORT ? PC_INT_16 : -1;
        }
        leaf(pc.first, PR_OPTIONAL, phys, conv, 3, 0, 0, f);
        if ((pc.second & 0xff) == DR_T_DECIMAL) {
          schema.back().scale = scale;
          schema.back().precision = prec;
          schema.back().type_length = tlen;
        }
      }
      at.pop_back();
    }
  }
  // remove
  group("remove", PR_OPTIONAL, 7);
  at = {"remove"};
  {
    const DevExport& x = X[1];
    EncLeaf e = flat(ENC_STR_OFF, 1, 2);
    e.off = x.path_off.p;
    e.bytes = x.path_bytes.p;
    leaf("path", PR_OPTIONAL, PQ_BYTE_ARRAY, PC_UTF8, 2, 0, 1, e);
    e = flat(ENC_I64, 1, 2);
    e.i64 = reinterpret_cast<const int64_t*>(x.delts.p);
    e.vflags = x.flags.p;
    e.vbit = 1;  // F_HAS_DELTS
    leaf("deletionTimestamp", PR_OPTIONAL, PQ_INT64, -1, 2, 0, 1, e);
    leaf("dataChange", PR_OPTIONAL, PQ_BOOLEAN, -1, 2, 0, 1, flat(ENC_BOOL, 1, 2));
    e = flat(ENC_BOOL, 1, 2);
    e.b8 = x.efm.p;
    leaf("extendedFileMetadata", PR_OPTIONAL, PQ_BOOLEAN, -1, 2, 0, 1, e);
    auto pv = side_map(x, true);
    str_map("partitionValues", 1, 1, pv.first, pv.second);
    e = flat(ENC_I64, 1, 2);
    e.i64 = x.size.p;
    leaf("size", PR_OPTIONAL, PQ_INT64, -1, 2, 0, 1, e);
    auto tg = side_map(x, false);
    str_map("tags", 1, 1, tg.first, tg.second);
  }
  // metaData
  group("metaData", PR_OPTIONAL, 8);
  at = {"metaData"};
  leaf("id", PR_OPTIONAL, PQ_BYTE_ARRAY, PC_UTF8, 2, 0, -1);
  leaf("name", PR_OPTIONAL, PQ_BYTE_ARRAY, PC_UTF8, 2, 0, -1);
  leaf("description", PR_OPTIONAL, PQ_BYTE_ARRAY, PC_UTF8, 2, 0, -1);
  group("format", PR_OPTIONAL, 2);
  at = {"metaData", "format"};
  leaf("provider", PR_OPTIONAL, PQ_BYTE_ARRAY, PC_UTF8, 3, 0, -1);
  str_map("options", 2, -1, EncLeaf{}, EncLeaf{});
  at = {"metaData"};
  leaf("schemaString", PR_OPTIONAL, PQ_BYTE_ARRAY, PC_UTF8, 2, 0, -1);
  group("partitionColumns", PR_OPTIONAL, 1, PC_LIST);
  at = {"metaData", "partitionColumns"};
  group("list", PR_REPEATED, 1);
  at.push_back("list");
  leaf("element", PR_OPTIONAL, PQ_BYTE_ARRAY, PC_UTF8, 4, 1, -1);
  at = {"metaData"};
  str_map("configuration", 1, -1, EncLeaf{}, EncLeaf{});
  leaf("createdTime", PR_OPTIONAL, PQ_INT64, -1, 2, 0, -1);
  // protocol
  group("protocol", PR_OPTIONAL, 2);
  at = {"protocol"};
  leaf("minReaderVersion", PR_OPTIONAL, PQ_INT32, -1, 2, 0, -1);
  leaf("minWriterVersion", PR_OPTIONAL, PQ_INT32, -1, 2, 0, -1);
  // host leaves: their levels / values per head row
  for (CkLeafW& L : leaves) {
    if (L.side >= 0) continue;
    L.hdef.resize(H);
    L.hrep.resize(H);
    L.hval.resize(H);
    for (uint64_t h = 0; h < H; ++h) head_row_levels(L, 0, head[h], L.hdef[h], L.hrep[h], L.hval[h]);
  }
  // ---- pages ----
  PartFile f;
  f.host({'P', 'A', 'R', '1'});
  struct ChunkMeta { int64_t off, size, usize, nval; int codec; };
  struct RG { std::vector<ChunkMeta> cols; int64_t rows, bytes; };
  std::vector<RG> rgs;
  const uint64_t rgn = rg_rows ? rg_rows : (uint64_t(1) << 20);
  DBuf<uint8_t> scratch(ctx, scan_scratch_for(std::min<uint64_t>(rgn, p1 - p0) + 1));
  for (uint64_t r0 = p0; r0 < p1; r0 += rgn) {
    const uint64_t r1 = std::min(p1, r0 + rgn);
    RG rg;
    rg.rows = int64_t(r1 - r0);
    rg.bytes = 0;
    for (CkLeafW& L : leaves) {
      std::vector<uint8_t> rep, def, vals, dev_prefix;
      DBuf<uint8_t> dev_out;  // a device leaf's page body (after dev_prefix), compressed or not
      uint64_t nlev = 0, dev_body_raw = 0, dev_out_len = 0;
      int dev_codec = 0;
      const int dw = level_width(L.max_def), rw = level_width(L.max_rep);
      const uint64_t side_lo = L.side == 0 ? H + a0 : H + NA + b0, side_n = L.side == 0 ? a1 - a0 : b1 - b0;
      const bool dev = L.side >= 0 && r0 < side_lo + side_n && r1 > side_lo;
      if (!dev) {
        std::vector<uint8_t> hd, hr;
        for (uint64_t g = r0; g < std::min<uint64_t>(r1, H); ++g) {
          if (L.side >= 0) { hd.push_back(0); if (L.max_rep) hr.push_back(0); continue; }
          hd.insert(hd.end(), L.hdef[g].begin(), L.hdef[g].end());
          hr.insert(hr.end(), L.hrep[g].begin(), L.hrep[g].end());
          vals.insert(vals.end(), L.hval[g].begin(), L.hval[g].end());
        }
        const uint64_t zeros = r1 - std::max<uint64_t>(r0, std::min<uint64_t>(r1, H));
        nlev = hd.size() + zeros;
        if (L.max_rep) rle_levels(rep, hr, zeros, rw);
        rle_levels(def, hd, zeros, dw);
      } else {
        const uint64_t R = r1 - r0;
        DBuf<uint32_t> nl(ctx, R), vb(ctx, R);
        DBuf<uint64_t> lo(ctx, R + 1), vo(ctx, R + 1);
        EncArgs a{};
        a.L = L.enc;
        a.r0 = r0;
        a.r1 = r1;
        a.side_lo = side_lo;
        a.n = side_n;
        a.nlev = nl.p;
        a.vbytes = vb.p;
        tmark("host_leaves");
        launch_enc_count(a, stream);
        launch_scan_u32(nl.p, lo.p, R, ss(scratch), stream);
        launch_scan_u32(vb.p, vo.p, R, ss(scratch), stream);
        nlev = d2h_one(lo.p + R, stream);
        const uint64_t nvb = d2h_one(vo.p + R, stream);
        DBuf<uint8_t> dl(ctx, nlev + 8), rl(ctx, L.max_rep ? nlev + 8 : 1), vv(ctx, nvb + 8);
        a.lev_off = lo.p;
        a.val_off = vo.p;
        a.def = dl.p;
        a.rep = rl.p;
        a.vals = vv.p;
        launch_enc_fill(a, stream);
        const uint64_t groups = (nlev + 7) / 8;
        DBuf<uint8_t> rpk(ctx, L.max_rep ? groups * uint64_t(rw) + 1 : 1), dpk(ctx, groups * uint64_t(dw) + 1),
            bpk(ctx, L.phys == PQ_BOOLEAN ? (nvb + 7) / 8 + 1 : 1);
        if (L.max_rep) launch_enc_pack(rl.p, nlev, rw, rpk.p, stream);
        launch_enc_pack(dl.p, nlev, dw, dpk.p, stream);
        if (L.phys == PQ_BOOLEAN) launch_enc_pack(vv.p, nvb, 1, bpk.p, stream);
        const uint64_t vbytes = L.phys == PQ_BOOLEAN ? (nvb + 7) / 8 : nvb;
        const uint8_t* vsrc = L.phys == PQ_BOOLEAN ? bpk.p : vv.p;
        // the page body on the device: [u32 + rep levels] [u32 + def levels] values
        std::vector<uint8_t> rh, dh;
        put_varint(rh, (groups << 1) | 1);
        put_varint(dh, (groups << 1) | 1);
        const uint64_t rsec = L.max_rep ? rh.size() + groups * uint64_t(rw) : 0, dsec = dh.size() + groups * uint64_t(dw);
        const uint64_t bsize = (L.max_rep ? 4 + rsec : 0) + 4 + dsec + vbytes;
        std::vector<uint8_t> hdr_r, hdr_d;
        if (L.max_rep) { put_u32le(hdr_r, uint32_t(rsec)); hdr_r.insert(hdr_r.end(), rh.begin(), rh.end()); }
        put_u32le(hdr_d, uint32_t(dsec));
        hdr_d.insert(hdr_d.end(), dh.begin(), dh.end());
        DBuf<uint8_t> bodyd(ctx, bsize + 64);  // the compressor reads up to 16 bytes past the end
        uint64_t at = 0;
        auto h2d_at = [&](const std::vector<uint8_t>& h) {
          if (!h.empty()) HIP_OK(hipMemcpyAsync(bodyd.p + at, h.data(), h.size(), hipMemcpyHostToDevice, stream));
          at += h.size();
        };
        auto d2d_at = [&](const uint8_t* src, uint64_t nb) {
          if (nb) HIP_OK(hipMemcpyAsync(bodyd.p + at, src, nb, hipMemcpyDeviceToDevice, stream));
          at += nb;
        };
        if (L.max_rep) { h2d_at(hdr_r); d2d_at(rpk.p, groups * uint64_t(rw)); }
        h2d_at(hdr_d);
        d2d_at(dpk.p, groups * uint64_t(dw));
        d2d_at(vsrc, vbytes);
        dev_body_raw = bsize;
        tmark("encode");
        if (opts & DR_CKPT_SNAPPY) {
          // one workgroup per 8 KiB fragment, then the fragments compacted into one stream on the
          // device: only the compressed bytes cross to the host, once, into the file
          const uint64_t frag = snap_compress_frag(), nfrag = (bsize + frag - 1) / frag, slot = snap_compress_slot();
          DBuf<uint8_t> cz(ctx, nfrag * slot + 16);
          DBuf<uint32_t> czl(ctx, nfrag + 1);
          DBuf<uint64_t> czo(ctx, nfrag + 1);
          launch_snap_compress(bodyd.p, bsize, cz.p, czl.p, stream);
          launch_scan_u32(czl.p, czo.p, nfrag, ss(scratch), stream);
          dev_out_len = d2h_one(czo.p + nfrag, stream);
          dev_out = DBuf<uint8_t>(ctx, dev_out_len + 1);
          launch_snap_gather(cz.p, czl.p, czo.p, uint32_t(nfrag), dev_out.p, stream);
          put_varint(dev_prefix, bsize);  // the snappy preamble: uncompressed length
          dev_codec = 1;
          tmark("compress");
        } else {
          dev_out_len = bsize;
          dev_out = std::move(bodyd);
        }
      }
      if (L.phys == PQ_BOOLEAN && !dev) {  // host BOOLEAN values are bytes until packed (none are written)
        vals.clear();
      }
      std::vector<uint8_t> body;  // a host leaf's page body
      uint64_t raw, blen;
      int codec = 0;
      if (dev) {
        raw = dev_body_raw;
        blen = dev_prefix.size() + dev_out_len;
        codec = dev_codec;
      } else {
        if (L.max_rep) { put_u32le(body, uint32_t(rep.size())); body.insert(body.end(), rep.begin(), rep.end()); }
        put_u32le(body, uint32_t(def.size()));
        body.insert(body.end(), def.begin(), def.end());
        body.insert(body.end(), vals.begin(), vals.end());
        raw = blen = body.size();
      }
      if (raw > uint64_t(INT32_MAX)) fail(DR_E_UNSUPPORTED, "checkpoint page over 2 GiB: use smaller row groups");
      ThriftW ph;
      ph.i32(1, 0);  // DATA_PAGE
      ph.i32(2, int32_t(raw));
      ph.i32(3, int32_t(blen));
      ph.begin_struct(5);
      ph.i32(1, int32_t(nlev));
      ph.i32(2, 0);  // PLAIN
      ph.i32(3, 3);  // RLE
      ph.i32(4, 3);  // RLE
      ph.end_struct();
      ph.b.push_back(0);
      const int64_t off = int64_t(f.size);
      f.host(ph.b.begin(), ph.b.end());
      if (dev) {
        f.host(dev_prefix.begin(), dev_prefix.end());
        f.dev(std::move(dev_out), dev_out_len);  // copied out with the rest of the file below
      } else {
        f.host(body.begin(), body.end());
      }
      rg.cols.push_back(ChunkMeta{off, int64_t(ph.b.size() + blen), int64_t(ph.b.size() + raw), int64_t(nlev), codec});
      tmark("file");
      rg.bytes += int64_t(ph.b.size() + blen);
    }
    rgs.push_back(std::move(rg));
  }
  // ---- footer ----
  ThriftW fm;
  fm.i32(1, 1);
  fm.begin_list(2, 12, schema.size());
  for (const SElem& e : schema) {
    fm.elem_begin();
    if (e.type >= 0) fm.i32(1, e.type);
    if (e.type_length >= 0) fm.i32(2, e.type_length);
    if (e.rep >= 0) fm.i32(3, e.rep);
    fm.str(4, e.name);
    if (e.nkids >= 0) fm.i32(5, e.nkids);
    if (e.conv >= 0) fm.i32(6, e.conv);
    if (e.scale >= 0) fm.i32(7, e.scale);
    if (e.precision >= 0) fm.i32(8, e.precision);
    fm.elem_end();
  }
  fm.i64(3, int64_t(p1 - p0));
  fm.begin_list(4, 12, rgs.size());
  for (const RG& rg : rgs) {
    fm.elem_begin();
    fm.begin_list(1, 12, rg.cols.size());
    for (size_t c = 0; c < rg.cols.size(); ++c) {
      const CkLeafW& L = leaves[c];
      const ChunkMeta& m = rg.cols[c];
      fm.elem_begin();
      fm.i64(2, m.off);
      fm.begin_struct(3);
      fm.i32(1, L.phys);
      fm.begin_list(2, 5, 2);
      fm.elem_i32(0);  // PLAIN
      fm.elem_i32(3);  // RLE
      fm.begin_list(3, 8, L.path.size());
      for (const std::string& s : L.path) fm.elem_str(s);
      fm.i32(4, m.codec);  // UNCOMPRESSED / SNAPPY
      fm.i64(5, m.nval);
      fm.i64(6, m.usize);
      fm.i64(7, m.size);
      fm.i64(9, m.off);
      fm.end_struct();
      fm.elem_end();
    }
    fm.i64(2, rg.bytes);
    fm.i64(3, rg.rows);
    fm.elem_end();
  }
  fm.str(6, "libdeltareplay (MI355X checkpoint writer)");
  fm.b.push_back(0);
  f.host(fm.b.begin(), fm.b.end());
  put_u32le(f, uint32_t(fm.b.size()));
  f.host({'P', 'A', 'R', '1'});
  tmark("footer");
  // ---- the file into one pinned block: host segments copied, device bodies DMA'd, one sync ----
  uint8_t* host = static_cast<uint8_t*>(ctx->host_alloc(f.size));
  try {
    for (PartFile::Seg& g : f.segs) {
      if (g.dn) HIP_OK(hipMemcpyAsync(host + g.off, g.d.p, g.dn, hipMemcpyDeviceToHost, stream));
      else if (!g.h.empty()) std::memcpy(host + g.off, g.h.data(), g.h.size());
    }
    HIP_OK(hipStreamSynchronize(stream));
  } catch (...) {
    (void)hipStreamSynchronize(stream);
    ctx->host_release(host);
    throw;
  }
  {
    std::lock_guard<std::mutex> g(g_pinned_out_mu);
    g_pinned_out[host] = ctx;
  }
  out.data = host;
  out.len = f.size;
  tmark("d2h");
  if (dbg)
    for (auto& kv : t_acc) fprintf(stderr, "[ckpt] %-12s %9.3f ms\n", kv.first.c_str(), kv.second);
  ctx->collect_timings();
}

static std::vector<int64_t> select_flags(dr_state& st, DBuf<uint32_t>& flag);

static PvColumn pv_column(const dr_state::PvCol& c) {
  PvColumn p{};
  p.type = c.type;
  p.w32 = c.w32.p;
  p.w64 = c.w64.p;
  p.sptr = c.sptr.p;
  p.slen = c.slen.p;
  p.isnull = c.isnull.p;
  p.s8 = c.s8.p;
  p.w64hi = c.w64hi.p;
  return p;
}

// Dictionary-encodes a typed partition column (k_dict_*): abandoned (dict = 0) past DICT_MAX - 1
// distinct values, for DECIMAL (two-word values) and on a string hash collision.
static void build_dict(dr_state& st, dr_state::PvCol& col) {
  if (col.dict >= 0) return;
  col.dict = 0;
  const int base = col.type & 0xff;
  if (base == DR_T_DECIMAL || !st.n_live) return;
  dr_ctx* ctx = st.ctx;
  hipStream_t stream = ctx->stream;
  const uint64_t n = st.n_live;
  DBuf<uint64_t> keys(ctx, DICT_SLOTS), scan(ctx, DICT_SLOTS + 1);
  DBuf<uint32_t> tags(ctx, DICT_SLOTS), slot_code(ctx, DICT_SLOTS), occ(ctx, DICT_SLOTS);
  DBuf<unsigned long long> ctr(ctx, 2);
  DBuf<uint8_t> scratch(ctx, scan_scratch_for(DICT_SLOTS));
  tags.zero(stream);
  ctr.zero(stream);
  PvDictArgs a{};
  a.n = n;
  a.col = pv_column(col);
  a.key_tab = keys.p;
  a.tag_tab = tags.p;
  a.slot_code = slot_code.p;
  a.ctr = ctr.p;
  launch_dict_insert(a, stream);
  launch_dict_occupied(a, occ.p, stream);
  launch_scan_u32(occ.p, scan.p, DICT_SLOTS, ss(scratch), stream);
  const uint64_t distinct = d2h_one(scan.p + DICT_SLOTS, stream);
  if (d2h_one(ctr.p + 1, stream) || distinct + 1 >= DICT_MAX) return;
  DBuf<uint32_t> rep(ctx, DICT_MAX + 1);
  DBuf<uint16_t> code(ctx, n);
  a.rep = rep.p;
  a.code = code.p;
  launch_dict_number(a, scan.p, stream);
  launch_dict_code(a, stream);
  if (d2h_one(ctr.p + 1, stream)) return;  // a string hash collision
  col.code = std::move(code);
  col.rep = std::move(rep);
  col.ncode = uint32_t(distinct + 1);
  col.dict = 1;
}

static std::vector<int64_t> filter_state(dr_state& st, const dr_predicate& pred) {
  DR_STAGE("filter", st.ctx->stream);
  check_program(pred);
  dr_ctx* ctx = st.ctx;
  ctx->begin_call();
  ensure_ready(st);
  hipStream_t stream = ctx->stream;
  if (st.sources.empty()) fail(DR_E_INVALID_ARG, "state has no staged segment");
  // the predicate's columns in the K5 cache (built for the ones not there yet)
  auto find = [&](const std::string& name, int32_t type) -> dr_state::PvCol* {
    for (auto& c : st.pv_cols)
      if (c->name == name && c->type == type) return c.get();
    return nullptr;
  };
  std::vector<std::pair<std::string, int32_t>> want;
  for (int32_t c = 0; c < pred.ncols; ++c) {
    std::pair<std::string, int32_t> k{pred.col_names[c], pred.col_types[c]};
    if (!find(k.first, k.second) && std::find(want.begin(), want.end(), k) == want.end()) want.push_back(k);
  }
  if (!want.empty() && st.n_live) build_pv_columns(st, want);
  FilterTypedArgs fa{};
  fa.n_live = st.n_live;
  fa.ncols = pred.ncols;
  for (int32_t c = 0; c < pred.ncols; ++c) {
    dr_state::PvCol* col = find(pred.col_names[c], pred.col_types[c]);
    if (!col) {  // no live files: nothing was built
      fa.cols[c].type = pred.col_types[c];
      continue;
    }
    fa.cols[c] = pv_column(*col);
  }
  LeafPlan lp;
  const bool force_generic = ctx->opt.filter_eval == 2;  // DR_OPT_FILTER_EVAL: k_filter_typed
  if (!force_generic && leafify(pred, lp) && lp.prog.size() / 2 <= filter_leaf_max_prog() &&
      lp.leaves.size() <= filter_leaf_max_leaves() && lp.i64.size() <= filter_leaf_max_i64() &&
      lp.str.size() <= filter_leaf_max_str()) {
    FilterLeafArgs la{};
    la.n_live = st.n_live;
    for (int32_t c = 0; c < pred.ncols; ++c) la.cols[c] = fa.cols[c];
    std::vector<uint64_t> soff(lp.str.size() + 1, 0), s8(lp.str.size() + 1, 0);
    std::string sbytes;
    for (size_t q = 0; q < lp.str.size(); ++q) {
      sbytes += lp.str[q];
      soff[q + 1] = sbytes.size();
      for (size_t k = 0; k < 8; ++k) s8[q] = (s8[q] << 8) | (k < lp.str[q].size() ? uint8_t(lp.str[q][k]) : 0u);
    }
    la.nprog = int32_t(lp.prog.size() / 2);
    la.n_i64 = int32_t(lp.i64.size());
    la.n_str = int32_t(lp.str.size());
    la.nleaves = int32_t(lp.leaves.size());
    std::vector<int32_t> ucol;
    for (const FilterLeaf& f : lp.leaves)
      if (std::find(ucol.begin(), ucol.end(), f.col) == ucol.end()) ucol.push_back(f.col);
    la.nucol = ucol.size() <= size_t(FL_UCOLS) ? int32_t(ucol.size()) : 0;
    for (int32_t u = 0; u < la.nucol; ++u) la.ucol[u] = ucol[size_t(u)];
    for (FilterLeaf& f : lp.leaves) {
      f.slot = -1;
      for (int32_t u = 0; u < la.nucol; ++u)
        if (la.ucol[u] == f.col) f.slot = u;
      f.ctype = la.cols[f.col].type;
    }
    const uint64_t ng = filter_leaf_groups(st.n_live);
    DBuf<uint64_t> mask(ctx, uint64_t(filter_leaf_mask_words()) * ng), wg_off(ctx, ng + 1);
    DBuf<uint32_t> wg_count(ctx, ng);
    DBuf<uint8_t> scratch(ctx, scan_scratch_for(ng));
    wg_count.zero(stream);
    la.mask = mask.p;
    la.wg_count = wg_count.p;
    // the dictionary path when every column the leaves read has a dictionary and the leaf tables fit
    std::vector<dr_state::PvCol*> ucols;
    for (int32_t u = 0; u < la.nucol; ++u) ucols.push_back(find(pred.col_names[la.ucol[u]], pred.col_types[la.ucol[u]]));
    bool use_dict = la.nucol > 0 && st.n_live && ctx->opt.filter_eval == 0;  // DR_OPT_FILTER_EVAL
    for (dr_state::PvCol* c : ucols) {
      if (!use_dict || !c) { use_dict = false; break; }
      build_dict(st, *c);
      use_dict = c->dict == 1;
    }
    std::vector<uint32_t> tab_off(lp.leaves.size() + 1, 0);
    if (use_dict) {
      for (size_t l = 0; l < lp.leaves.size(); ++l) tab_off[l + 1] = tab_off[l] + ucols[size_t(lp.leaves[l].slot)]->ncode;
      use_dict = tab_off.back() <= filter_dict_max_tab();
    }
    // the program, leaves and literals in one upload (each pageable upload is a staged copy of its own)
    std::vector<uint8_t> blob;
    auto put = [&](const void* src, size_t bytes) -> size_t {
      const size_t at = (blob.size() + 15) & ~size_t(15);
      blob.resize(at + bytes);
      if (bytes) std::memcpy(blob.data() + at, src, bytes);
      return at;
    };
    const size_t o_s8 = put(s8.data(), 8 * s8.size()), o_soff = put(soff.data(), 8 * soff.size());
    const size_t o_prog = put(lp.prog.data(), 4 * lp.prog.size()), o_i64 = put(lp.i64.data(), 8 * lp.i64.size());
    const size_t o_leaves = put(lp.leaves.data(), sizeof(FilterLeaf) * lp.leaves.size());
    const size_t o_toff = put(tab_off.data(), 4 * tab_off.size()), o_sb = put(sbytes.data(), sbytes.size());
    DBuf<uint8_t> d_blob = upload(ctx, blob.data(), blob.size());
    la.lit_s8 = reinterpret_cast<const uint64_t*>(d_blob.p + o_s8);
    la.lit_str_off = reinterpret_cast<const uint64_t*>(d_blob.p + o_soff);
    la.prog = reinterpret_cast<const int32_t*>(d_blob.p + o_prog);
    la.lit_i64 = reinterpret_cast<const int64_t*>(d_blob.p + o_i64);
    la.leaves = reinterpret_cast<const FilterLeaf*>(d_blob.p + o_leaves);
    la.lit_str = d_blob.p + o_sb;
    const uint32_t* d_toff = reinterpret_cast<const uint32_t*>(d_blob.p + o_toff);
    DBuf<uint8_t> d_tab;
    if (use_dict) {
      d_tab = DBuf<uint8_t>(ctx, tab_off.back());
      DictLeafArgs d{};
      d.leaves = la.leaves;
      d.nleaves = la.nleaves;
      for (int32_t c = 0; c < pred.ncols; ++c) d.cols[c] = la.cols[c];
      for (int32_t u = 0; u < la.nucol; ++u) {
        d.rep[la.ucol[u]] = ucols[size_t(u)]->rep.p;
        d.ncode[la.ucol[u]] = ucols[size_t(u)]->ncode;
      }
      d.tab_off = d_toff;
      d.tab = d_tab.p;
      d.lit_i64 = la.lit_i64;
      d.lit_s8 = la.lit_s8;
      d.lit_str_off = la.lit_str_off;
      d.lit_str = la.lit_str;
      d.n_live = st.n_live;
      launch_dict_leaf(d, tab_off.back(), stream);
      FilterDictArgs f{};
      f.n_live = st.n_live;
      for (int32_t u = 0; u < la.nucol; ++u) f.code[u] = ucols[size_t(u)]->code.p;
      f.nslot = la.nucol;
      f.leaves = la.leaves;
      f.nleaves = la.nleaves;
      f.prog = la.prog;
      f.nprog = la.nprog;
      f.tab_off = d_toff;
      f.tab = d_tab.p;
      f.tab_bytes = tab_off.back();
      f.mask = mask.p;
      f.wg_count = wg_count.p;
      launch_filter_dict(f, stream);
    } else {
      launch_filter_leaf(la, stream);
    }
    launch_scan_u32(wg_count.p, wg_off.p, ng, ss(scratch), stream);
    const uint64_t nsel = ng ? d2h_one(wg_off.p + ng, stream) : 0;
    DBuf<int64_t> sel(ctx, nsel);
    if (nsel) launch_select_bits(mask.p, wg_off.p, st.n_live, sel.p, stream);
    std::vector<int64_t> out = d2h(sel.p, nsel, stream);
    ctx->collect_timings();
    return out;
  }
  const std::vector<int32_t> ops = lower_program(pred);
  std::vector<uint64_t> lit_off(size_t(pred.nlits) + 1, 0);
  for (int32_t k = 0; k <= pred.nlits && pred.nlits; ++k) lit_off[size_t(k)] = uint64_t(pred.lit_str_off[k]);
  const uint64_t lit_bytes = pred.nlits ? lit_off[size_t(pred.nlits)] : 0;
  DBuf<int32_t> d_ops = upload(ctx, ops.data(), ops.size());
  DBuf<int32_t> d_lt = upload(ctx, pred.lit_types, size_t(pred.nlits));
  DBuf<int64_t> d_li = upload(ctx, pred.lit_i64, size_t(pred.nlits));
  DBuf<uint8_t> d_ln = upload(ctx, pred.lit_null, size_t(pred.nlits));
  DBuf<uint64_t> d_lo = upload(ctx, lit_off.data(), lit_off.size());
  DBuf<uint8_t> d_ls = upload(ctx, pred.lit_str_bytes, size_t(lit_bytes));
  fa.nops = int32_t(ops.size() / 2);
  fa.ops = d_ops.p;
  fa.lit_types = d_lt.p;
  fa.lit_i64 = d_li.p;
  fa.lit_null = d_ln.p;
  fa.lit_str_off = d_lo.p;
  fa.lit_str = d_ls.p;
  DBuf<uint32_t> flag(ctx, st.n_live);
  fa.flag = flag.p;
  launch_filter_typed(fa, stream);
  return select_flags(st, flag);
}

// Selected live-file ordinals from per-file flags (scan + compaction), then the call's timings.
// ---------------------------------------------------------------------------------------------------
// scan-side consumers: DeltaSourceSnapshot's (modificationTime, path) order and
// TahoeFileIndex.listFiles' partition groups, computed over the resident state.
// ---------------------------------------------------------------------------------------------------
static std::vector<int64_t> to_host_positions(const DBuf<uint32_t>& keys, uint64_t n, hipStream_t stream) {
  const std::vector<uint32_t> k = d2h(keys.p, n, stream);
  return std::vector<int64_t>(k.begin(), k.end());
}

// DeltaSourceSnapshot.initialFiles (D/files/DeltaSourceSnapshot.scala:53-95):
// allFiles.sort("modificationTime", "path"): live export positions in that order.
static std::vector<int64_t> scan_order(dr_state& st) {
  dr_ctx* ctx = st.ctx;
  ctx->begin_call();
  ensure_ready(st);
  hipStream_t stream = ctx->stream;
  if (st.sources.empty()) fail(DR_E_INVALID_ARG, "state has no staged segment");
  StagedData& s = *st.sources[0];
  const uint64_t n = st.n_live, R = s.ck_rows;
  if (!n) return {};
  MtimeArgs a{};
  a.live = st.live.p;
  a.n_live = n;
  a.src_off = st.src_off.p;
  a.src_len = st.src_len.p;
  a.ck_rows = R;
  a.json = s.d_json.p;
  DBuf<uint64_t> json_bases;
  if (st.src_id.p) {
    std::vector<uint64_t> bases;
    for (auto& src : st.sources) bases.push_back(reinterpret_cast<uint64_t>(src->d_json.p));
    json_bases = upload(ctx, bases.data(), bases.size());
    a.act_flags = st.flags.p;
    a.src_id = st.src_id.p;
    a.json_bases = json_bases.p;
  }
  DBuf<uint8_t> cdef;
  DBuf<int64_t> cval;
  DBuf<uint64_t> dict_ptr;
  DBuf<uint32_t> dict_len, pq_err(ctx, 1);
  pq_err.zero(stream);
  if (R) {
    {
      std::lock_guard<std::mutex> g(s.pv_mu);
      if (!s.mt) {
        auto P = std::make_unique<PagePlan>();
        P->paths = {"add.modificationTime"};
        plan_pages(s, *P);
        s.mt = std::move(P);
      }
    }
    PagePlan& P = *s.mt;
    if (P.present[0]) {
      if (P.levels[0] != R) fail(DR_E_PARQUET, "add.modificationTime: one value per checkpoint row expected");
      cdef = DBuf<uint8_t>(ctx, R);
      cval = DBuf<int64_t>(ctx, R);
      cdef.zero(stream);
      ParquetArgs pa{};
      pa.ncols = 1;
      pa.cols[0] = FlatColumn{cdef.p, nullptr, cval.p, nullptr, nullptr};
      decode_pages(ctx, P, pa, dict_ptr, dict_len, pq_err, nullptr);
      if (d2h_one(pq_err.p, stream) != 0)
        fail(DR_E_PARQUET, fmt("device decode of add.modificationTime failed (code %u)", d2h_one(pq_err.p, stream)));
      a.ck_def = cdef.p;
      a.ck_val = cval.p;
      a.ck_max_def = P.max_def[0];
    }
  }
  DBuf<int64_t> mt(ctx, n);
  DBuf<uint32_t> err(ctx, 1);
  err.zero(stream);
  a.out = mt.p;
  a.error = err.p;
  launch_mtime_extract(a, stream);
  if (d2h_one(err.p, stream)) fail(DR_E_PARSE, "malformed add object in a live AddFile's JSON line");
  DBuf<uint64_t> pp(ctx, n);
  DBuf<uint32_t> pl(ctx, n), keys(ctx, n);
  launch_gather_u64(st.path_ptr.p, st.live.p, n, pp.p, stream);
  launch_gather_u32(st.path_len.p, st.live.p, n, pl.p, stream);
  launch_iota_u32(keys.p, n, stream);
  size_t tb = 0;
  launch_sort_scan_order(nullptr, &tb, keys.p, n, mt.p, pp.p, pl.p, stream);
  DBuf<uint8_t> temp(ctx, tb);
  launch_sort_scan_order(temp.p, &tb, keys.p, n, mt.p, pp.p, pl.p, stream);
  ctx->collect_timings();
  return to_host_positions(keys, n, stream);
}

// TahoeFileIndex.listFiles (D/files/TahoeFileIndex.scala:58-81): `rows` (live export positions, e.g. a
// dr_filter result; null = all) grouped by the values of the table's partition columns (the
// metadata's partitionColumns, raw strings, null distinct from every string). Returns the rows in
// group order (groups ordered by their values, nulls first; rows ascending within a group) and the
// groups' start offsets (+ the end).
static void partition_groups(dr_state& st, const int64_t* rows, int64_t nrows, std::vector<int64_t>& order,
                             std::vector<int64_t>& off) {
  dr_ctx* ctx = st.ctx;
  ctx->begin_call();
  ensure_ready(st);
  hipStream_t stream = ctx->stream;
  std::vector<std::string> cols;
  for (const NonFileAction& a : st.nonfile) {
    if (a.kind != 3) continue;
    const JVal* pc = a.val->get("partitionColumns");
    if (pc && pc->t == JVal::ARR)
      for (const JVal& c : pc->a)
        if (c.t == JVal::STR) cols.push_back(c.s);
  }
  if (cols.size() > PV_MAXC) fail(DR_E_UNSUPPORTED, fmt("more than %d partition columns", PV_MAXC));
  const uint64_t n = rows ? uint64_t(nrows) : st.n_live;
  order.clear();
  off.assign(1, 0);
  if (!n) return;
  for (uint64_t i = 0; rows && i < n; ++i)
    if (rows[i] < 0 || uint64_t(rows[i]) >= st.n_live) fail(DR_E_INVALID_ARG, "row out of range");
  if (cols.empty()) {  // an unpartitioned table: one group
    for (uint64_t i = 0; i < n; ++i) order.push_back(rows ? rows[i] : int64_t(i));
    std::sort(order.begin(), order.end());
    off.push_back(int64_t(n));
    return;
  }
  std::vector<std::pair<std::string, int32_t>> want;
  for (const std::string& c : cols) {
    bool have = false;
    for (auto& pc : st.pv_cols) have |= pc->name == c && pc->type == DR_T_STRING;
    if (!have) want.push_back({c, DR_T_STRING});
  }
  if (!want.empty()) build_pv_columns(st, want);
  GroupCols g{};
  g.ncols = int32_t(cols.size());
  for (size_t c = 0; c < cols.size(); ++c)
    for (auto& pc : st.pv_cols)
      if (pc->name == cols[c] && pc->type == DR_T_STRING) {
        g.sptr[c] = pc->sptr.p;
        g.slen[c] = pc->slen.p;
        g.isnull[c] = pc->isnull.p;
      }
  DBuf<uint32_t> keys(ctx, n);
  if (rows) {
    std::vector<uint32_t> r(rows, rows + n);
    std::sort(r.begin(), r.end());
    HIP_OK(hipMemcpyAsync(keys.p, r.data(), n * 4, hipMemcpyHostToDevice, stream));
  } else {
    launch_iota_u32(keys.p, n, stream);
  }
  size_t tb = 0;
  launch_sort_groups(nullptr, &tb, keys.p, n, g, stream);
  DBuf<uint8_t> temp(ctx, tb);
  launch_sort_groups(temp.p, &tb, keys.p, n, g, stream);
  DBuf<uint32_t> flag(ctx, n);
  DBuf<uint64_t> pos(ctx, n + 1);
  DBuf<uint8_t> scratch(ctx, scan_scratch_for(n));
  launch_group_flags(keys.p, n, g, flag.p, stream);
  launch_scan_u32(flag.p, pos.p, n, ss(scratch), stream);
  const uint64_t ng = d2h_one(pos.p + n, stream);
  DBuf<int64_t> starts(ctx, ng);
  launch_select(flag.p, pos.p, n, starts.p, stream);
  ctx->collect_timings();
  order = to_host_positions(keys, n, stream);
  off = d2h(starts.p, ng, stream);
  off.push_back(int64_t(n));
}

static std::vector<int64_t> select_flags(dr_state& st, DBuf<uint32_t>& flag) {
  dr_ctx* ctx = st.ctx;
  hipStream_t stream = ctx->stream;
  DBuf<uint8_t> scratch(ctx, scan_scratch_for(st.n_live));
  DBuf<uint64_t> pos(ctx, st.n_live + 1);
  launch_scan_u32(flag.p, pos.p, st.n_live, ss(scratch), stream);
  const uint64_t nsel = st.n_live ? d2h_one(pos.p + st.n_live, stream) : 0;
  DBuf<int64_t> sel(ctx, nsel);
  launch_select(flag.p, pos.p, st.n_live, sel.p, stream);
  std::vector<int64_t> out = d2h(sel.p, nsel, stream);
  ctx->collect_timings();
  return out;
}

// ---------------------------------------------------------------------------------------------------
// multi-GPU shards: contiguous slices of the replay order, then path-hash exchange
// ---------------------------------------------------------------------------------------------------
struct ShardUnit {
  SegFile f;
  int32_t rg_lo = 0, rg_hi = -1;   // checkpoint row groups [rg_lo, rg_hi); JSON: 0, -1
  uint64_t weight = 0;
};

// Relative device cost of the units: JSON bytes are parsed once (weight 1/byte); checkpoint row
// groups are weighted by the compressed bytes of the decoded columns (inflate + decode ~4x the
// per-byte cost of JSON, measured) plus the per-row assembly.
static std::vector<ShardUnit> shard_units(const std::string& log_path, const LogSegmentInfo& seg) {
  std::vector<ShardUnit> units;
  for (const SegFile& f : seg.checkpoint) {
    const std::string p = log_path + "/" + f.name;
    std::vector<uint8_t> tail = read_tail(p, 8);
    if (tail.size() < 8 || memcmp(tail.data() + 4, "PAR1", 4)) fail(DR_E_PARQUET, fmt("%s is not a parquet file", f.name.c_str()));
    uint32_t flen;
    memcpy(&flen, tail.data(), 4);
    std::vector<uint8_t> foot = read_tail(p, uint64_t(flen) + 8);
    std::vector<uint8_t> buf(4 + foot.size());
    memcpy(buf.data(), "PAR1", 4);
    memcpy(buf.data() + 4, foot.data(), foot.size());
    pq::FileMeta m = pq::parse_footer(buf.data(), buf.size());
    if (m.row_groups.empty()) {
      ShardUnit u;
      u.f = f;
      u.weight = 1;
      units.push_back(u);
      continue;
    }
    for (size_t g = 0; g < m.row_groups.size(); ++g) {
      ShardUnit u;
      u.f = f;
      u.rg_lo = int32_t(g);
      u.rg_hi = int32_t(g + 1);
      uint64_t hot = 0;
      for (auto& c : m.row_groups[g].cols)
        for (int h = 0; h < HC_N; ++h)
          if (c.path == kHotPath[h]) hot += uint64_t(c.total_compressed);
      u.weight = 4 * hot + 16 * uint64_t(m.row_groups[g].num_rows) + 1;
      units.push_back(u);
    }
  }
  for (const SegFile& f : seg.deltas) {
    ShardUnit u;
    u.f = f;
    u.weight = file_size(log_path + "/" + f.name) + 1;
    units.push_back(u);
  }
  return units;
}

// Contiguous split of the units by weight: unit k goes to the rank whose share contains the
// midpoint of its weight interval (deterministic: every rank computes the same plan).
static std::vector<int32_t> shard_assign(const std::vector<ShardUnit>& units, int32_t world) {
  uint64_t total = 0;
  for (auto& u : units) total += u.weight;
  std::vector<int32_t> owner(units.size(), 0);
  uint64_t before = 0;
  for (size_t k = 0; k < units.size(); ++k) {
    const long double mid = (long double)before + (long double)units[k].weight / 2;
    int32_t r = int32_t(mid * world / (long double)std::max<uint64_t>(total, 1));
    owner[k] = std::min(std::max(r, 0), world - 1);
    before += units[k].weight;
  }
  return owner;
}

static std::shared_ptr<StagedData> stage_shard(dr_ctx* ctx, const std::string& log_path, int64_t version,
                                               int32_t world, int32_t rank) {
  LogSegmentInfo seg = get_log_segment(log_path, version);
  std::vector<ShardUnit> units = shard_units(log_path, seg);
  std::vector<int32_t> owner = shard_assign(units, world);
  // this rank's units: merge consecutive row groups of one checkpoint part
  std::vector<ShardUnit> mine;
  for (size_t k = 0; k < units.size(); ++k) {
    if (owner[k] != rank) continue;
    const ShardUnit& u = units[k];
    if (!mine.empty() && mine.back().f.name == u.f.name && u.f.kind == DR_FILE_CHECKPOINT &&
        mine.back().rg_hi == u.rg_lo) {
      mine.back().rg_hi = u.rg_hi;
      continue;
    }
    mine.push_back(u);
  }
  std::vector<StageSrc> src;
  for (auto& u : mine) {
    StageSrc x;
    x.version = u.f.version;
    x.kind = u.f.kind;
    x.part = u.f.part;
    x.path = log_path + "/" + u.f.name;
    x.rg_lo = u.rg_lo;
    x.rg_hi = u.rg_hi;
    src.push_back(std::move(x));
  }
  auto s = stage_sources(ctx, src);
  s->version = seg.version;
  return s;
}

struct dr_shard {
  dr_ctx* ctx = nullptr;
  std::shared_ptr<StagedData> staged;
  std::unique_ptr<dr_state> st;
  std::vector<NonFileAction> nf;
  uint32_t world = 1;
  uint64_t nsend = 0, send_path_bytes = 0;
  DBuf<uint32_t> send_idx, send_plen;
  DBuf<uint64_t> send_poff;
  bool reduced = false;
  bool owner_read = false;        // the owner side's counters are on the host (sh.owner)
  dr_counts owner{};
  ParsePending parse;             // the sender side's parse; its counters come back in shard_finish
  std::unique_ptr<dr_state> own;  // the owner side's reduced shard (alive until the verdicts are set)
  ReducePending red;
};

// Sender side, step 1: parse this rank's slice, count its file actions and their canonical path
// bytes per owner and lay out the send order (stable per owner). One round trip: the per-owner
// record and byte counts the caller needs to size the exchange.
static void shard_begin(dr_shard& sh, uint64_t* send_counts, uint64_t* send_bytes) {
  dr_ctx* ctx = sh.ctx;
  hipStream_t stream = ctx->stream;
  sh.st.reset(new_state(ctx, sh.staged));
  ctx->mark("start");
  sh.parse = parse_launch(ctx, sh.staged, sh.st.get(), true);
  dr_state& st = *sh.st;
  const uint64_t N = st.n_actions;
  const uint32_t W = sh.world;
  const uint64_t nt = shard_tiles(N);
  const uint64_t nc = uint64_t(W) * nt;
  DBuf<uint32_t> bcnt(ctx, nc), bbytes(ctx, nc);
  DBuf<uint64_t> boff(ctx, nc + 1), byoff(ctx, nc + 1), sizes(ctx, 2 * uint64_t(W) + 1);
  DBuf<uint8_t> scratch(ctx, scan_scratch_for(nc));
  ShardArgs a{st.kind.p, st.flags.p, st.key.p, st.size.p, st.delts.p, st.path_len.p, N, W, nt,
              bcnt.p, boff.p, nullptr, 0, bbytes.p};
  launch_shard_count(a, stream);
  launch_scan_u32(bcnt.p, boff.p, nc, ss(scratch), stream);
  launch_scan_u32(bbytes.p, byoff.p, nc, ss(scratch), stream);
  launch_shard_sizes(bbytes.p, boff.p, byoff.p, W, nt, sizes.p, stream);
  const std::vector<uint64_t> z = d2h(sizes.p, 2 * uint64_t(W) + 1, stream);
  if (z[2 * W]) fail(DR_E_UNSUPPORTED, "more than 4 GiB of canonical paths in one shard tile");
  sh.nsend = 0;
  sh.send_path_bytes = 0;
  for (uint32_t d = 0; d < W; ++d) {
    send_counts[d] = z[d];
    send_bytes[d] = z[W + d];
    sh.nsend += z[d];
    sh.send_path_bytes += z[W + d];
  }
  sh.send_idx = DBuf<uint32_t>(ctx, sh.nsend);
  a.send_idx = sh.send_idx.p;
  a.nsend = sh.nsend;
  launch_shard_scatter(a, stream);
  // path byte offsets of the send order (their per-owner totals are send_bytes)
  sh.send_plen = DBuf<uint32_t>(ctx, sh.nsend);
  sh.send_poff = DBuf<uint64_t>(ctx, sh.nsend + 1);
  launch_gather_u32(st.path_len.p, sh.send_idx.p, sh.nsend, sh.send_plen.p, stream);
  DBuf<uint8_t> scratch2(ctx, scan_scratch_for(sh.nsend));
  launch_scan_u32(sh.send_plen.p, sh.send_poff.p, sh.nsend, ss(scratch2), stream);
}

// Sender side, step 2: the 32 B records and the path bytes in send order. `sync`: return only when
// the buffers are written (a caller exchanging them on another stream); the library's own RCCL
// exchange runs on the same stream and needs no sync.
static void shard_pack(dr_shard& sh, void* send_rec, void* send_path, bool sync = true) {
  dr_ctx* ctx = sh.ctx;
  hipStream_t stream = ctx->stream;
  dr_state& st = *sh.st;
  ShardArgs a{st.kind.p, st.flags.p, st.key.p, st.size.p, st.delts.p, st.path_len.p, st.n_actions, sh.world,
              0, nullptr, nullptr, sh.send_idx.p, sh.nsend, nullptr};
  launch_shard_pack(a, static_cast<ShardRec*>(send_rec), sh.send_plen.p, stream);
  DBuf<uint64_t> ptrs(ctx, sh.nsend);
  launch_gather_u64(st.path_ptr.p, sh.send_idx.p, sh.nsend, ptrs.p, stream);
  launch_gather_bytes(ptrs.p, sh.send_plen.p, sh.send_poff.p, sh.nsend, static_cast<uint8_t*>(send_path), stream);
  if (sync) HIP_OK(hipStreamSynchronize(stream));
}

// Owner side: K3/K4 over the received records (in rank order = replay order) and one verdict byte
// per record (1 live, 2 kept tombstone, 0 dropped), the survivor lists' lengths read on the device.
static void shard_reduce(dr_shard& sh, const void* recv_rec, uint64_t n, const void* recv_path, int64_t cutoff,
                         uint8_t* verdict, bool sync = true) {
  dr_ctx* ctx = sh.ctx;
  hipStream_t stream = ctx->stream;
  std::unique_ptr<dr_state> own(new_state(ctx, nullptr));
  own->n_actions = n;
  own->kind = DBuf<uint8_t>(ctx, n);
  own->flags = DBuf<uint8_t>(ctx, n);
  own->key = DBuf<uint64_t>(ctx, n);
  own->path_ptr = DBuf<uint64_t>(ctx, n);
  own->path_len = DBuf<uint32_t>(ctx, n);
  own->size = DBuf<int64_t>(ctx, n);
  own->delts = DBuf<int64_t>(ctx, n);
  own->src_off = DBuf<uint64_t>(ctx, n);
  own->src_len = DBuf<uint32_t>(ctx, n);
  const ShardRec* rec = static_cast<const ShardRec*>(recv_rec);
  DBuf<uint64_t> poff(ctx, n + 1);
  DBuf<uint8_t> scratch(ctx, scan_scratch_for(n));
  launch_shard_plen(rec, n, own->path_len.p, stream);
  launch_scan_u32(own->path_len.p, poff.p, n, ss(scratch), stream);
  ActionArrays act{own->kind.p, own->flags.p, own->key.p, own->path_ptr.p, own->path_len.p, own->size.p,
                   own->delts.p, own->src_off.p, own->src_len.p};
  launch_shard_unpack(rec, n, static_cast<const uint8_t*>(recv_path), poff.p, act, stream);
  sh.red = reduce_launch(ctx, own.get(), cutoff);
  if (n) HIP_OK(hipMemsetAsync(verdict, 0, n, stream));
  // the reducer's totals: [0] live survivors, [2] kept tombstones (the compacted lists' lengths)
  launch_verdict_set(own->live.p, n, sh.red.totals.p + 0, 1, verdict, stream);
  launch_verdict_set(own->tomb.p, n, sh.red.totals.p + 2, 2, verdict, stream);
  sh.own = std::move(own);
  if (sync) {
    reduce_queue_readback(ctx, sh.red, 0);
    HIP_OK(hipStreamSynchronize(stream));
    reduce_finish(ctx, sh.own.get(), sh.red);
    sh.owner = sh.own->counts;
    sh.owner_read = true;
  }
  sh.reduced = true;
}

// Sender side, last step: the returned verdicts select this rank's survivors (its share of allFiles
// / tombstones). One round trip reads the parse's counters and non-file lines, the survivor counts,
// the owner side's counters (when shard_reduce did not) and, for the library's RCCL replay, the
// all-reduced table-wide counters (`sums_dev`, 8 words, copied to `sums`).
static dr_state* shard_finish(dr_shard& sh, const uint8_t* verdict_back, const int64_t* sums_dev = nullptr,
                              int64_t* sums = nullptr) {
  dr_ctx* ctx = sh.ctx;
  hipStream_t stream = ctx->stream;
  dr_state& st = *sh.st;
  const uint64_t n = sh.nsend;
  DBuf<uint32_t> fl(ctx, n), ft(ctx, n);
  DBuf<uint64_t> pl(ctx, n + 1), pt(ctx, n + 1);
  DBuf<uint8_t> scratch(ctx, scan_scratch_for(n));
  launch_verdict_flags(verdict_back, n, fl.p, ft.p, stream);
  launch_scan_u32(fl.p, pl.p, n, ss(scratch), stream);
  launch_scan_u32(ft.p, pt.p, n, ss(scratch), stream);
  st.live = DBuf<uint32_t>(ctx, n);  // bounded by the records sent; the counts come back below
  st.tomb = DBuf<uint32_t>(ctx, n);
  launch_verdict_collect(verdict_back, sh.send_idx.p, n, 1, pl.p, st.live.p, stream);
  launch_verdict_collect(verdict_back, sh.send_idx.p, n, 2, pt.p, st.tomb.p, stream);
  size_t at = parse_queue_readback(ctx, sh.parse, 0);
  uint64_t* h = ctx->pinned();
  const size_t at_n = at;
  HIP_OK(hipMemcpyAsync(h + at_n, pl.p + n, 8, hipMemcpyDeviceToHost, stream));
  HIP_OK(hipMemcpyAsync(h + at_n + 1, pt.p + n, 8, hipMemcpyDeviceToHost, stream));
  at += 2;
  if (!sh.owner_read && sh.own) at = reduce_queue_readback(ctx, sh.red, at);
  const size_t at_sums = at;
  if (sums_dev) HIP_OK(hipMemcpyAsync(h + at_sums, sums_dev, 8 * sizeof(int64_t), hipMemcpyDeviceToHost, stream));
  HIP_OK(hipStreamSynchronize(stream));
  if (!parse_finish(ctx, sh.staged, &st, sh.parse, sh.nf))
    fail(DR_E_INTERNAL, "sharded replay: the canonicalisation arena hint of this segment was too small");
  st.n_live = h[at_n];
  st.n_tomb = h[at_n + 1];
  if (!sh.owner_read && sh.own) {
    reduce_finish(ctx, sh.own.get(), sh.red);
    sh.owner = sh.own->counts;
    sh.owner_read = true;
  }
  if (sums) std::memcpy(sums, h + at_sums, 8 * sizeof(int64_t));
  sh.own.reset();
  // counters: the owner-side partial sums (their sum over ranks is the table's computedState)
  st.counts.num_files = sh.owner.num_files;
  st.counts.size_in_bytes = sh.owner.size_in_bytes;
  st.counts.num_removes = sh.owner.num_removes;
  st.counts.live_key_sum = sh.owner.live_key_sum;
  st.counts.tomb_key_sum = sh.owner.tomb_key_sum;
  st.counts.num_file_actions = sh.owner.num_file_actions;
  st.counts.num_actions = int64_t(st.n_actions);
  st.sharded = true;
  reduce_nonfile(st, sh.nf, false);
  ctx->mark("end");
  return sh.st.release();
}

// ---------------------------------------------------------------------------------------------------
// the sharded replay inside the library: RCCL over xGMI, no host framework. The
// communicator is the caller's (one per process and device); librccl is loaded on first use, so a
// single-GPU host needs none. Collectives run on the context's stream, ordered with the kernels.
// ---------------------------------------------------------------------------------------------------
struct Rccl {
  void* h = nullptr;
  std::string why;
  ncclResult_t (*get_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  const char* (*err)(ncclResult_t) = nullptr;
};

static Rccl& rccl() {
  static Rccl r = [] {
    Rccl x;
    x.h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!x.h) x.h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!x.h) {
      const char* e = dlerror();
      x.why = e ? e : "dlopen failed";
      return x;
    }
    auto sym = [&](auto& fn, const char* name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(x.h, name));
      if (!fn && x.why.empty()) x.why = std::string("missing symbol ") + name;
    };
    sym(x.get_id, "ncclGetUniqueId");
    sym(x.init_rank, "ncclCommInitRank");
    sym(x.destroy, "ncclCommDestroy");
    sym(x.send, "ncclSend");
    sym(x.recv, "ncclRecv");
    sym(x.group_start, "ncclGroupStart");
    sym(x.group_end, "ncclGroupEnd");
    sym(x.all_reduce, "ncclAllReduce");
    sym(x.all_gather, "ncclAllGather");
    sym(x.err, "ncclGetErrorString");
    return x;
  }();
  if (!r.why.empty()) fail(DR_E_UNSUPPORTED, "librccl is not usable: " + r.why);
  return r;
}

#define RC_OK(x)                                                                          \
  do {                                                                                    \
    const ncclResult_t rc_ = (x);                                                         \
    if (rc_ != ncclSuccess) fail(DR_E_DEVICE, std::string("RCCL: ") + rccl().err(rc_) + " (" #x ")"); \
  } while (0)

// In-process stand-in for an RCCL communicator (test hook, dr_comm_loopback_id): the ranks are threads
// of this process, each with its own dr_ctx. Every collective publishes this rank's device buffers,
// meets the others at a barrier, copies what it receives from the peers' buffers on its own stream
// and meets them again before anyone may reuse a buffer -- so replay_sharded_rccl's own control flow
// (count matrix, byte all-to-alls, verdict return, counter all-reduce, non-file all-gather) runs at
// W > 1 on one GPU. A rank that fails aborts the group: the others fail instead of waiting.
struct LoopGroup {
  int32_t world = 0;
  std::mutex mu;
  std::condition_variable cv;
  int32_t arrived = 0;
  uint64_t gen = 0;
  bool aborted = false;
  std::vector<const uint8_t*> ptr;             // each rank's published send buffer
  std::vector<const uint64_t*> cnt;            // each rank's per-peer byte counts (all-to-all)
  void barrier() {
    std::unique_lock<std::mutex> g(mu);
    if (aborted) fail(DR_E_INTERNAL, "loopback communicator aborted by another rank");
    const uint64_t my = gen;
    if (++arrived == world) {
      arrived = 0;
      ++gen;
      cv.notify_all();
      return;
    }
    if (!cv.wait_for(g, std::chrono::seconds(120), [&] { return gen != my || aborted; }))
      fail(DR_E_INTERNAL, "loopback communicator: a rank did not arrive within 120 s");
    if (aborted) fail(DR_E_INTERNAL, "loopback communicator aborted by another rank");
  }
  void abort() {
    std::lock_guard<std::mutex> g(mu);
    aborted = true;
    cv.notify_all();
  }
};

static std::mutex g_loop_mu;
static std::map<uint64_t, std::weak_ptr<LoopGroup>> g_loop_groups;
static const char kLoopMagic[8] = {'D', 'R', 'L', 'O', 'O', 'P', 'B', 'K'};

struct dr_comm {
  dr_ctx* ctx = nullptr;
  ncclComm_t comm = nullptr;
  std::shared_ptr<LoopGroup> loop;  // set: loopback transport instead of RCCL
  int32_t world = 1, rank = 0;
};

// The collectives replay_sharded_rccl needs, over RCCL or the loopback group.
static void comm_all_gather(dr_comm& c, const void* send, void* recv, uint64_t bytes) {
  hipStream_t stream = c.ctx->stream;
  if (!c.loop) {
    RC_OK(rccl().all_gather(send, recv, bytes, ncclUint8, c.comm, stream));
    return;
  }
  LoopGroup& g = *c.loop;
  HIP_OK(hipStreamSynchronize(stream));
  g.ptr[c.rank] = static_cast<const uint8_t*>(send);
  g.barrier();
  for (int32_t p = 0; p < c.world; ++p)
    if (bytes) HIP_OK(hipMemcpyAsync(static_cast<uint8_t*>(recv) + uint64_t(p) * bytes, g.ptr[p], bytes,
                                     hipMemcpyDeviceToDevice, stream));
  HIP_OK(hipStreamSynchronize(stream));
  g.barrier();
}

static void comm_all_reduce_sum_i64(dr_comm& c, int64_t* buf, uint64_t n) {
  hipStream_t stream = c.ctx->stream;
  if (!c.loop) {
    RC_OK(rccl().all_reduce(buf, buf, n, ncclInt64, ncclSum, c.comm, stream));
    return;
  }
  LoopGroup& g = *c.loop;
  const std::vector<int64_t> mine = d2h(buf, n, stream);
  g.ptr[c.rank] = reinterpret_cast<const uint8_t*>(mine.data());  // host vectors: summed on the host
  g.barrier();
  std::vector<uint64_t> tot(n, 0);
  for (int32_t p = 0; p < c.world; ++p)
    for (uint64_t i = 0; i < n; ++i) tot[i] += uint64_t(reinterpret_cast<const int64_t*>(g.ptr[p])[i]);
  g.barrier();
  HIP_OK(hipMemcpyAsync(buf, tot.data(), n * 8, hipMemcpyHostToDevice, stream));
  HIP_OK(hipStreamSynchronize(stream));
}

// All-to-all of byte ranges: send[so_p, so_p + scnt[p]) to each peer p, recv rcnt[p] bytes from each
// peer in rank order (grouped point-to-point: the xGMI links are peer-to-peer).
static void rccl_all_to_all(dr_comm& c, const uint8_t* send, const std::vector<uint64_t>& scnt, uint8_t* recv,
                            const std::vector<uint64_t>& rcnt) {
  hipStream_t stream = c.ctx->stream;
  if (c.loop) {
    LoopGroup& g = *c.loop;
    HIP_OK(hipStreamSynchronize(stream));
    g.ptr[c.rank] = send;
    g.cnt[c.rank] = scnt.data();
    g.barrier();
    uint64_t ro = 0;
    for (int32_t p = 0; p < c.world; ++p) {
      uint64_t so = 0;
      for (int32_t q = 0; q < c.rank; ++q) so += g.cnt[p][q];
      if (g.cnt[p][c.rank] != rcnt[p])
        fail(DR_E_INTERNAL, fmt("loopback all-to-all: rank %d sends %llu bytes to rank %d, which expects %llu", p,
                                (unsigned long long)g.cnt[p][c.rank], c.rank, (unsigned long long)rcnt[p]));
      if (rcnt[p]) HIP_OK(hipMemcpyAsync(recv + ro, g.ptr[p] + so, rcnt[p], hipMemcpyDeviceToDevice, stream));
      ro += rcnt[p];
    }
    HIP_OK(hipStreamSynchronize(stream));
    g.barrier();
    return;
  }
  Rccl& R = rccl();
  RC_OK(R.group_start());
  uint64_t so = 0, ro = 0;
  for (int32_t p = 0; p < c.world; ++p) {
    if (scnt[p]) RC_OK(R.send(send + so, scnt[p], ncclUint8, p, c.comm, stream));
    if (rcnt[p]) RC_OK(R.recv(recv + ro, rcnt[p], ncclUint8, p, c.comm, stream));
    so += scnt[p];
    ro += rcnt[p];
  }
  RC_OK(R.group_end());
}

// Every rank's text, in rank order: one all-gather of fixed slots (length word + bytes) and one
// read-back; a text longer than the slot costs a second, exactly sized round (every rank sees the
// same lengths, so all take it together).
static std::vector<std::string> rccl_all_gather_text(dr_comm& c, const std::string& mine) {
  dr_ctx* ctx = c.ctx;
  hipStream_t stream = ctx->stream;
  uint64_t slot = uint64_t(16) << 10;
  for (int round = 0;; ++round) {
    std::vector<uint8_t> buf(slot, 0);
    const uint64_t n = mine.size();
    std::memcpy(buf.data(), &n, 8);
    std::memcpy(buf.data() + 8, mine.data(), std::min<uint64_t>(n, slot - 8));
    DBuf<uint8_t> d(ctx, slot), all(ctx, slot * c.world);
    HIP_OK(hipMemcpyAsync(d.p, buf.data(), slot, hipMemcpyHostToDevice, stream));
    comm_all_gather(c, d.p, all.p, slot);
    const std::vector<uint8_t> h = d2h(all.p, slot * c.world, stream);
    std::vector<std::string> out;
    uint64_t mx = 0;
    for (int32_t p = 0; p < c.world; ++p) {
      uint64_t L = 0;
      std::memcpy(&L, h.data() + uint64_t(p) * slot, 8);
      mx = std::max(mx, L);
      if (L <= slot - 8) out.emplace_back(reinterpret_cast<const char*>(h.data() + uint64_t(p) * slot + 8), L);
    }
    if (mx <= slot - 8) return out;
    if (round) fail(DR_E_INTERNAL, "non-file text all-gather: lengths changed between rounds");
    slot = mx + 8;
  }
}

// One rank's part of the sharded replay (collective over the communicator; every rank stages its
// own slice with dr_stage_log_shard). The returned state holds this rank's surviving records (its
// export is its share of allFiles / tombstones) and the table-wide counters and non-file winners.
// The table-wide non-file winners of a sharded replay from every rank's local winners, one JSON
// action per line in rank order (= replay order: the slices are contiguous); InMemoryLogReplay's
// rule over them, as the single `null` partition (D/Snapshot.scala:103).
static void set_nonfile_lines(dr_state& st, const std::string& lines, bool validate) {
  std::vector<NonFileAction> merged;
  size_t b = 0;
  while (b < lines.size()) {
    size_t e = lines.find('\n', b);
    if (e == std::string::npos) e = lines.size();
    JVal v;
    if (e > b && json_parse(lines.data() + b, e - b, &v) && v.t == JVal::OBJ && !v.o.empty()) {
      NonFileAction a;
      const std::string& key = v.o[0].first;
      a.kind = key == "metaData" ? 3 : key == "txn" ? 4 : 5;
      a.order = merged.size();
      a.val = std::make_shared<const JVal>(v.o[0].second);
      a.json = lines.substr(b, e - b);
      merged.push_back(std::move(a));
    }
    b = e + 1;
  }
  reduce_nonfile(st, merged, validate);
}

static dr_state* replay_sharded_rccl(dr_comm& c, const std::shared_ptr<StagedData>& staged, int64_t cutoff,
                                     uint32_t flags) {
  dr_ctx* ctx = c.ctx;
  hipStream_t stream = ctx->stream;
  const uint32_t W = uint32_t(c.world);
  dr_shard sh;
  sh.ctx = ctx;
  sh.staged = staged;
  sh.world = W;
  // round trip 1: this rank's per-owner record and byte counts (the parse is queued before them)
  std::vector<uint64_t> sc(W), sb(W);
  shard_begin(sh, sc.data(), sb.data());
  // every rank's send counts and bytes: recv counts are this rank's column (round trip 2)
  DBuf<uint64_t> mine(ctx, 2 * W), all(ctx, 2 * uint64_t(W) * W);
  std::vector<uint64_t> m(sc);
  m.insert(m.end(), sb.begin(), sb.end());
  HIP_OK(hipMemcpyAsync(mine.p, m.data(), 16 * W, hipMemcpyHostToDevice, stream));
  comm_all_gather(c, mine.p, all.p, 16 * uint64_t(W));
  const std::vector<uint64_t> M = d2h(all.p, 2 * uint64_t(W) * W, stream);
  std::vector<uint64_t> rc(W), rb(W), scb(W), rcb(W);
  uint64_t nrecv = 0, nrecv_b = 0, nsend = 0, nsend_b = 0;
  for (uint32_t p = 0; p < W; ++p) {
    rc[p] = M[uint64_t(p) * 2 * W + c.rank];
    rb[p] = M[uint64_t(p) * 2 * W + W + c.rank];
    scb[p] = sc[p] * sizeof(ShardRec);
    rcb[p] = rc[p] * sizeof(ShardRec);
    nrecv += rc[p];
    nrecv_b += rb[p];
    nsend += sc[p];
    nsend_b += sb[p];
  }
  DBuf<uint8_t> send_rec(ctx, std::max<uint64_t>(nsend, 1) * sizeof(ShardRec)), send_path(ctx, nsend_b + 1),
      recv_rec(ctx, std::max<uint64_t>(nrecv, 1) * sizeof(ShardRec)), recv_path(ctx, nrecv_b + 1),
      verdict(ctx, nrecv + 1), back(ctx, nsend + 1);
  // pack, exchange, reduce, return the verdicts and all-reduce the counters: all queued on the
  // context's stream (RCCL is stream-ordered), no host round trip
  shard_pack(sh, send_rec.p, send_path.p, /*sync=*/false);
  {
    DR_STAGE("exchange", c.ctx->stream);
    rccl_all_to_all(c, send_rec.p, scb, recv_rec.p, rcb);
    rccl_all_to_all(c, send_path.p, sb, recv_path.p, rb);
  }
  shard_reduce(sh, recv_rec.p, nrecv, recv_path.p, cutoff, verdict.p, /*sync=*/false);
  rccl_all_to_all(c, verdict.p, rc, back.p, sc);
  DBuf<int64_t> sums(ctx, 8);
  launch_shard_partials(sh.red.totals.p, sh.parse.counters.p, int64_t(sh.st->n_actions), sums.p, stream);
  comm_all_reduce_sum_i64(c, sums.p, 8);
  // round trip 3: survivors, parse counters, table-wide counters
  int64_t t[8];
  std::unique_ptr<dr_state> st(shard_finish(sh, back.p, sums.p, t));
  st->local_counts = st->counts;
  st->has_local_counts = true;
  dr_counts& k = st->counts;
  k.num_files = t[0];
  k.size_in_bytes = t[1];
  k.num_removes = t[2];
  k.num_actions = t[3];
  k.num_file_actions = t[4];
  k.malformed_lines = t[5];
  k.live_key_sum = uint64_t(t[6]);
  k.tomb_key_sum = uint64_t(t[7]);
  // non-file winners: every rank's, in rank order (= replay order: slices are contiguous); round trip 4
  std::string text;
  for (const NonFileAction& a : st->nonfile) text += a.json + "\n";
  std::string lines;
  for (const std::string& part_text : rccl_all_gather_text(c, text)) lines += part_text;
  set_nonfile_lines(*st, lines, !(flags & DR_FLAG_NO_VALIDATION));
  return st.release();
}

// ---------------------------------------------------------------------------------------------------
// per-line commit decode (getChanges' Action.fromJson hot fields; K1 only)
// ---------------------------------------------------------------------------------------------------
struct dr_parsed {
  std::shared_ptr<StagedData> staged;
  std::vector<int64_t> version, size, delts;
  std::vector<uint64_t> line_off, path_off;
  std::vector<uint32_t> line_len, path_len;
  std::vector<uint8_t> kind, flags;
};

static void parse_commits(dr_ctx* ctx, const std::shared_ptr<StagedData>& sp, dr_parsed& out) {
  if (!sp->parts.empty()) fail(DR_E_INVALID_ARG, "dr_parse_commits takes commit (JSON) files only");
  hipStream_t stream = ctx->stream;
  std::unique_ptr<dr_state> st(new_state(ctx, sp));
  std::vector<NonFileAction> nf;
  parse_actions(ctx, sp, st.get(), nf, /*canonicalize=*/false);
  const uint64_t n = st->n_actions;
  out.staged = sp;
  out.kind = d2h(st->kind.p, n, stream);
  out.flags = d2h(st->flags.p, n, stream);
  out.size = d2h(st->size.p, n, stream);
  out.delts = d2h(st->delts.p, n, stream);
  out.line_off = d2h(st->src_off.p, n, stream);
  out.line_len = d2h(st->src_len.p, n, stream);
  out.path_len = d2h(st->path_len.p, n, stream);
  std::vector<uint64_t> pp = d2h(st->path_ptr.p, n, stream);
  const uint64_t base = reinterpret_cast<uint64_t>(sp->d_json.p);
  out.path_off.resize(n);
  out.version.resize(n);
  size_t f = 0;
  for (uint64_t i = 0; i < n; ++i) {
    out.flags[i] &= uint8_t(~2u);  // F_SPECIAL_PATH is internal
    out.path_off[i] = pp[i] ? pp[i] - base : 0;
    while (f + 1 < sp->jfiles.size() && out.line_off[i] >= sp->jfiles[f + 1].off) ++f;
    out.version[i] = sp->jfiles.empty() ? -1 : sp->jfiles[f].version;
  }
}

// ---------------------------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------------------------
namespace {
template <typename F>
int guard(dr_ctx* ctx, F&& f) {
  // one call at a time per context (dr_ctx::api_mu): the context's streams, scratch, timing vectors and
  // error text, and its states' lazily built members (materialize, the K5 cache), are shared
  std::unique_lock<std::recursive_mutex> lk;
  if (ctx) lk = std::unique_lock<std::recursive_mutex>(ctx->api_mu);
  try {
    f();
    if (ctx && dr_ctx::poison()) {
      const std::string bad = ctx->check_quarantine();
      if (!bad.empty()) fail(DR_E_INTERNAL, "DR_POISON: " + bad);
    }
    if (ctx) ctx->err.clear();
    return DR_OK;
  } catch (const Error& e) {
    if (ctx) ctx->err = e.what();
    return e.status;
  } catch (const std::bad_alloc&) {
    if (ctx) ctx->err = "host allocation failed";
    return DR_E_OOM;
  } catch (const std::exception& e) {
    if (ctx) ctx->err = e.what();
    return DR_E_INTERNAL;
  }
}
}  // namespace

extern "C" {

int dr_abi_version(void) { return DR_ABI_VERSION; }

int dr_ctx_create(int device, dr_ctx** out) {
  if (!out) return DR_E_INVALID_ARG;
  *out = nullptr;
  auto c = std::make_unique<dr_ctx>();
  c->device = device;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) {
    (void)hipGetLastError();
    return DR_E_DEVICE;
  }
  if (hipSetDevice(device) != hipSuccess) return DR_E_DEVICE;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return DR_E_DEVICE;
  if (hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking) != hipSuccess) return DR_E_DEVICE;
  *out = c.release();
  return DR_OK;
}

void dr_ctx_destroy(dr_ctx* ctx) {
  if (!ctx) return;
  {  // a call still running on another thread finishes first
    std::lock_guard<std::recursive_mutex> g(ctx->api_mu);
  }
  {  // row ranges still held by the caller unpin their blocks on their own (dr_range_release)
    std::lock_guard<std::mutex> g(g_ranges_mu);
    for (dr_range* r : g_ranges)
      if (r->ctx == ctx) r->ctx = nullptr;
  }
  (void)hipStreamSynchronize(ctx->stream);
  (void)hipStreamSynchronize(ctx->stream2);
  ctx->trim();
  ctx->host_trim();
  {  // part files still held by the caller are freed by dr_free on their own
    std::lock_guard<std::mutex> g(g_pinned_out_mu);
    for (auto& kv : g_pinned_out)
      if (kv.second == ctx) kv.second = nullptr;
  }
  for (uint8_t* p : ctx->bounce) (void)hipHostFree(p);
  for (hipEvent_t e : ctx->bounce_ev) (void)hipEventDestroy(e);
  if (ctx->hpin) (void)hipHostFree(ctx->hpin);
  ctx->drop_timings();
  for (hipEvent_t e : ctx->ev_pool) (void)hipEventDestroy(e);
  (void)hipStreamDestroy(ctx->stream);
  (void)hipStreamDestroy(ctx->stream2);
  delete ctx;
}

static int64_t* option_slot(dr_ctx* ctx, int32_t option) {
  dr_ctx::Options& o = ctx->opt;
  switch (option) {
    case DR_OPT_OVERLAP: return &o.overlap;
    case DR_OPT_SPLIT: return &o.split;
    case DR_OPT_BUCKET_BITS: return &o.bucket_bits;
    case DR_OPT_FILTER_EVAL: return &o.filter_eval;
    case DR_OPT_APPLY_FULL: return &o.apply_full;
    case DR_OPT_CANON_HINT: return &o.canon_hint;
    case DR_OPT_JSON_STAGED: return &o.json_staged;
    case DR_OPT_HOST_CACHE_BYTES: return &o.host_cache_bytes;
    default: return nullptr;
  }
}

int dr_ctx_set_option(dr_ctx* ctx, int32_t option, int64_t value) {
  if (!ctx) return DR_E_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(ctx->api_mu);
  int64_t* v = option_slot(ctx, option);
  bool ok = v != nullptr;
  switch (option) {  // the accepted values (include/deltareplay.h)
    case DR_OPT_OVERLAP: case DR_OPT_SPLIT: case DR_OPT_APPLY_FULL: case DR_OPT_JSON_STAGED:
      ok = value == 0 || value == 1;
      break;
    case DR_OPT_BUCKET_BITS: ok = value >= -1 && value <= 32; break;
    case DR_OPT_FILTER_EVAL: ok = value >= 0 && value <= 2; break;
    case DR_OPT_CANON_HINT: ok = value >= -1; break;
    case DR_OPT_HOST_CACHE_BYTES: ok = value >= 0; break;
    default: break;
  }
  if (!ok) {
    ctx->err = fmt("option %d: value %lld not accepted", int(option), (long long)value);
    return DR_E_INVALID_ARG;
  }
  *v = value;
  return DR_OK;
}

int dr_ctx_get_option(dr_ctx* ctx, int32_t option, int64_t* value) {
  if (!ctx || !value) return DR_E_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(ctx->api_mu);
  const int64_t* v = option_slot(ctx, option);
  if (!v) {
    ctx->err = fmt("unknown option %d", int(option));
    return DR_E_INVALID_ARG;
  }
  *value = *v;
  return DR_OK;
}

const char* dr_last_error(const dr_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }
const char* dr_state_last_error(const dr_state* state) {
  return state ? dr_last_error(state->ctx) : "null state";
}
const char* dr_comm_last_error(const dr_comm* comm) { return comm ? dr_last_error(comm->ctx) : "null communicator"; }

int dr_log_segment(dr_ctx* ctx, const char* log_path, int64_t version_to_load, char* buf, uint64_t buf_len,
                   uint64_t* needed, int64_t* version_out) {
  return guard(ctx, [&] {
    if (!log_path) fail(DR_E_INVALID_ARG, "null log path");
    LogSegmentInfo seg = get_log_segment(log_path, version_to_load);
    std::string s;
    for (auto& f : seg.checkpoint) s += fmt("%d %lld %d %s\n", f.kind, (long long)f.version, f.part, f.name.c_str());
    for (auto& f : seg.deltas) s += fmt("%d %lld %d %s\n", f.kind, (long long)f.version, f.part, f.name.c_str());
    if (needed) *needed = s.size() + 1;
    if (version_out) *version_out = seg.version;
    if (buf && buf_len) {
      size_t n = std::min<size_t>(s.size(), buf_len - 1);
      memcpy(buf, s.data(), n);
      buf[n] = 0;
    }
  });
}

int dr_stage(dr_ctx* ctx, const dr_file* files, int32_t nfiles, dr_staged** out) {
  if (!ctx || !out || (nfiles && !files)) return DR_E_INVALID_ARG;
  return guard(ctx, [&] {
    HIP_OK(hipSetDevice(ctx->device));
    auto s = std::make_unique<dr_staged>();
    s->d = stage_files(ctx, files, nfiles);
    *out = s.release();
  });
}

// Hadoop Path of a path or URI string, for equality: scheme (a bare path is "file"), authority, and
// the path with repeated and trailing '/' removed (org.apache.hadoop.fs.Path normalisation).
struct HPath {
  std::string scheme, authority, path;
  bool operator==(const HPath& o) const { return scheme == o.scheme && authority == o.authority && path == o.path; }
};
static HPath hpath(const std::string& s) {
  HPath h;
  size_t i = 0;
  const size_t colon = s.find(':');
  if (colon != std::string::npos && colon > 0 && s.find('/') > colon) {
    bool ok = std::isalpha(static_cast<unsigned char>(s[0])) != 0;
    for (size_t k = 1; k < colon; ++k) {
      const char c = s[k];
      ok &= std::isalnum(static_cast<unsigned char>(c)) || c == '+' || c == '-' || c == '.';
    }
    if (ok) {
      h.scheme = s.substr(0, colon);
      i = colon + 1;
    }
  }
  if (h.scheme.empty()) h.scheme = "file";
  if (s.compare(i, 2, "//") == 0) {
    const size_t e = s.find('/', i + 2);
    h.authority = s.substr(i + 2, e == std::string::npos ? std::string::npos : e - i - 2);
    i = e == std::string::npos ? s.size() : e;
  }
  for (; i < s.size(); ++i) {
    if (s[i] == '/' && !h.path.empty() && h.path.back() == '/') continue;
    h.path += s[i];
  }
  if (h.path.size() > 1 && h.path.back() == '/') h.path.pop_back();
  return h;
}

static void check_named_files(const char* log_path, const dr_file* files, const char* const* names, int32_t n) {
  const HPath base = hpath(log_path);
  for (int32_t k = 0; k < n; ++k) {
    const std::string name = names && names[k] ? names[k] : "";
    if (name.empty()) continue;  // an unnamed (cached) input, as the reference accepts ""
    HPath parent = hpath(name);
    const size_t slash = parent.path.rfind('/');
    const std::string leaf = slash == std::string::npos ? parent.path : parent.path.substr(slash + 1);
    parent.path = slash == std::string::npos ? std::string() : slash == 0 ? std::string("/") : parent.path.substr(0, slash);
    if (!(parent == base))
      fail(DR_E_FOREIGN_FILE, "File (" + name + ") doesn't belong in the transaction log at " + log_path +
                                  ". Please contact Databricks Support.");
    const dr_file& f = files[k];
    const bool ok = f.kind == DR_FILE_JSON
                        ? is_delta_file(leaf) && file_version(leaf) == f.version
                        : is_checkpoint_file(leaf) && file_version(leaf) == f.version && checkpoint_part(leaf) == f.part;
    if (!ok)
      fail(DR_E_INVALID_ARG, fmt("file name %s does not name a %s of version %lld (part %d)", leaf.c_str(),
                                 f.kind == DR_FILE_JSON ? "delta file" : "checkpoint", (long long)f.version, f.part));
  }
}

int dr_stage_named(dr_ctx* ctx, const char* log_path, const dr_file* files, const char* const* names, int32_t nfiles,
                   dr_staged** out) {
  if (!ctx || !out || !log_path || (nfiles && !files)) return DR_E_INVALID_ARG;
  return guard(ctx, [&] {
    check_named_files(log_path, files, names, nfiles);
    HIP_OK(hipSetDevice(ctx->device));
    auto s = std::make_unique<dr_staged>();
    s->d = stage_files(ctx, files, nfiles);
    *out = s.release();
  });
}

int dr_stage_log(dr_ctx* ctx, const char* log_path, int64_t version_to_load, dr_staged** out) {
  if (!ctx || !out || !log_path) return DR_E_INVALID_ARG;
  return guard(ctx, [&] {
    HIP_OK(hipSetDevice(ctx->device));
    LogSegmentInfo seg = get_log_segment(log_path, version_to_load);
    std::vector<StageSrc> src;
    for (auto* list : {&seg.checkpoint, &seg.deltas})
      for (auto& f : *list) {
        StageSrc x;
        x.version = f.version;
        x.kind = f.kind;
        x.part = f.part;
        x.path = std::string(log_path) + "/" + f.name;
        src.push_back(std::move(x));
      }
    auto s = std::make_unique<dr_staged>();
    s->d = stage_sources(ctx, src);
    s->d->version = seg.version;
    *out = s.release();
  });
}

int dr_staged_release(dr_staged* staged) {
  delete staged;
  return DR_OK;
}

int dr_staged_bytes(const dr_staged* staged, uint64_t* json_bytes, uint64_t* checkpoint_bytes) {
  if (!staged) return DR_E_INVALID_ARG;
  if (json_bytes) *json_bytes = staged->d->h_json.size();
  if (checkpoint_bytes) {
    uint64_t n = 0;
    for (auto& p : staged->d->parts) n += p.len;
    *checkpoint_bytes = n;
  }
  return DR_OK;
}

int dr_staged_plan(const dr_staged* staged, uint64_t* out, int32_t cap, int32_t* n) {
  if (!staged || !out || !n) return DR_E_INVALID_ARG;
  const StagedData& s = *staged->d;
  uint64_t ck = 0, cs = 0, us = 0;
  for (auto& p : s.parts) ck += p.len;
  for (auto& p : s.hot.pages) { cs += p.csize; us += p.usize; }
  const PagePlan& h = s.hot;
  const uint64_t v[14] = {s.h_json.size(), ck, s.ck_rows, s.hot.pages.size(), cs, us, s.hot.dict_entries,
                          h.snap_in_bytes, h.snap_out_bytes, h.nchunks, h.block_page.size(), h.snap_elements,
                          h.copy_bytes, s.json_lines};
  int32_t k = 0;
  for (; k < cap && k < 14; ++k) out[k] = v[k];
  *n = k;
  return DR_OK;
}

int dr_replay_staged(dr_ctx* ctx, const dr_staged* staged, int64_t cutoff, uint32_t flags, dr_state** out) {
  if (!ctx || !staged || !out) return DR_E_INVALID_ARG;
  *out = nullptr;
  int rc = guard(ctx, [&] {
    HIP_OK(hipSetDevice(ctx->device));
    ctx->begin_call();
    *out = replay(ctx, staged->d, cutoff, flags);
    ctx->collect_timings();
  });
  if (rc != DR_OK) ctx->drop_timings();
  return rc;
}

int dr_replay(dr_ctx* ctx, const dr_file* files, int32_t nfiles, int64_t cutoff, uint32_t flags, dr_state** out) {
  dr_staged* s = nullptr;
  int rc = dr_stage(ctx, files, nfiles, &s);
  if (rc != DR_OK) return rc;
  rc = dr_replay_staged(ctx, s, cutoff, flags, out);
  dr_staged_release(s);
  return rc;
}

int dr_state_release(dr_state* state) {
  if (!state) return DR_OK;
  std::lock_guard<std::recursive_mutex> g(state->ctx->api_mu);  // after any call using it on another thread
  (void)hipStreamSynchronize(state->ctx->stream);
  delete state;
  return DR_OK;
}

int dr_state_apply(dr_ctx* ctx, dr_state* base, const dr_staged* tail, int64_t min_file_retention_timestamp,
                   uint32_t flags, dr_state** out) {
  if (!ctx || !base || !tail || !out) return DR_E_INVALID_ARG;
  *out = nullptr;
  int rc = guard(ctx, [&] {
    HIP_OK(hipSetDevice(ctx->device));
    ctx->begin_call();
    ctx->mark("start");
    *out = apply_tail(ctx, *base, tail->d, min_file_retention_timestamp, flags);
    ctx->mark("end");
    ctx->collect_timings();
  });
  if (rc != DR_OK) ctx->drop_timings();
  return rc;
}

int dr_state_counts(dr_state* state, dr_counts* out) {
  if (!state || !out) return DR_E_INVALID_ARG;
  *out = state->counts;
  return DR_OK;
}

int dr_state_local_counts(dr_state* state, dr_counts* out) {
  if (!state || !out) return DR_E_INVALID_ARG;
  *out = state->has_local_counts ? state->local_counts : state->counts;
  return DR_OK;
}

// ValidateChecksum.checkMismatch (D/Checksum.scala:178-191) against ReadChecksum's parse of the
// version's .crc first line (D/Checksum.scala:101-148, JsonUtils.mapper: unknown fields ignored).
// A Long field that is absent or null reads as 0; a number with a fraction is truncated and a
// numeric string is coerced (Jackson's defaults); anything else is a parse failure.
static bool crc_long(const JVal& o, const char* name, int64_t* out) {
  const JVal* v = o.get(name);
  *out = 0;
  if (!v || v->t == JVal::NUL) return true;
  std::string t;
  if (v->t == JVal::NUM) t = v->s;
  else if (v->t == JVal::STR) t = v->s;
  else return false;
  errno = 0;
  char* end = nullptr;
  const long long x = std::strtoll(t.c_str(), &end, 10);
  if (end == t.c_str() || errno) return false;
  if (*end == '.' || *end == 'e' || *end == 'E') {  // ACCEPT_FLOAT_AS_INT: truncate
    const double d = std::strtod(t.c_str(), &end);
    if (*end || d != d || d >= 9.3e18 || d <= -9.3e18) return false;
    *out = int64_t(d);
    return true;
  }
  if (*end) return false;
  *out = int64_t(x);
  return true;
}

int dr_state_check_checksum(dr_state* state, const char* crc, uint64_t crc_len, char* msg, uint64_t msg_cap,
                            uint64_t* msg_len) {
  if (!state || (!crc && crc_len) || !msg_len) return DR_E_INVALID_ARG;
  *msg_len = 0;
  if (!crc_len) return DR_E_NO_CHECKSUM;  // delta.checksum.error.empty
  JVal v;
  if (!json_parse(crc, crc_len, &v) || v.t != JVal::OBJ) return DR_E_NO_CHECKSUM;  // error.parsing
  int64_t tsb, nf, nm, np, nt;
  if (!crc_long(v, "tableSizeBytes", &tsb) || !crc_long(v, "numFiles", &nf) || !crc_long(v, "numMetadata", &nm) ||
      !crc_long(v, "numProtocol", &np) || !crc_long(v, "numTransactions", &nt))
    return DR_E_NO_CHECKSUM;
  const dr_counts& c = state->counts;
  std::string out;
  auto cmp = [&](int64_t expected, int64_t found, const char* title) {
    if (expected == found) return;
    if (!out.empty()) out += "\n";
    out += fmt("%s - Expected: %lld Computed: %lld", title, (long long)expected, (long long)found);
  };
  cmp(tsb, c.size_in_bytes, "Table size (bytes)");
  cmp(nf, c.num_files, "Number of files");
  cmp(nm, c.num_metadata, "Metadata updates");
  cmp(np, c.num_protocol, "Protocol updates");
  cmp(nt, c.num_set_transactions, "Transactions");
  if (out.empty()) return DR_OK;
  *msg_len = out.size();
  if (msg && msg_cap) {
    const size_t k = std::min<size_t>(out.size(), msg_cap - 1);
    memcpy(msg, out.data(), k);
    msg[k] = 0;
  }
  return DR_E_CHECKSUM;
}

int dr_state_nonfile_json(dr_state* state, const char** json, uint64_t* len) {
  if (!state || !json || !len) return DR_E_INVALID_ARG;
  *json = state->nonfile_json.c_str();
  *len = state->nonfile_json.size();
  return DR_OK;
}

int dr_state_export(dr_state* state, int32_t which, dr_export* out) {
  if (!state || !out || (which != DR_LIVE && which != DR_TOMBSTONES)) return DR_E_INVALID_ARG;
  return guard(state->ctx, [&] {
    build_export(*state, which);
    ExportCols& e = state->exp[which];
    *out = dr_export{};
    out->n = e.n;
    out->path_off = e.path_off; out->path_bytes = e.path_bytes;
    out->size = e.size; out->modification_time = e.mtime;
    out->deletion_timestamp = e.delts; out->deletion_timestamp_valid = e.delts_valid;
    out->extended_file_metadata = e.efm;
    out->stats_off = e.stats_off; out->stats_bytes = e.stats_bytes; out->stats_null = e.stats_null;
    out->pv_entry_off = e.pv_entry_off; out->pv_null = e.pv_null;
    out->pv_key_off = e.pv_key_off; out->pv_key_bytes = e.pv_key_bytes;
    out->pv_val_off = e.pv_val_off; out->pv_val_bytes = e.pv_val_bytes; out->pv_val_null = e.pv_val_null;
    out->tags_entry_off = e.tags_entry_off; out->tags_null = e.tags_null;
    out->tags_key_off = e.tags_key_off; out->tags_key_bytes = e.tags_key_bytes;
    out->tags_val_off = e.tags_val_off; out->tags_val_bytes = e.tags_val_bytes;
    out->tags_val_null = e.tags_val_null;
  });
}

static int64_t* malloc_copy(const std::vector<int64_t>& v);

// ---- row-range export (ABI 3) ------------------------------------------------------------------
// A host copy of rows [lo, hi) of one side's resident export columns, every offset array rebased to
// the range (so no column of a range is larger than the caller planned: a JVM direct buffer holds
// at most 2^31 - 1 bytes). One pinned block from the context's cache, returned by dr_range_release.

// The eight row-level and eight entry-level offsets that bound rows [lo, hi) of X.
struct RangeBounds {
  uint64_t path[2], stats[2], pvn[2], tgn[2], pvk[2], pvv[2], tgk[2], tgv[2];
};
static RangeBounds range_bounds(const DevExport& X, uint64_t lo, uint64_t hi, hipStream_t stream) {
  RangeBounds b;
  const uint64_t r[2] = {lo, hi};
  for (int k = 0; k < 2; ++k) {
    b.path[k] = d2h_one(X.path_off.p + r[k], stream);
    b.stats[k] = d2h_one(X.off[EXC_STATS].p + r[k], stream);
    b.pvn[k] = d2h_one(X.off[EXC_PV_N].p + r[k], stream);
    b.tgn[k] = d2h_one(X.off[EXC_TAGS_N].p + r[k], stream);
  }
  for (int k = 0; k < 2; ++k) {
    b.pvk[k] = uint64_t(d2h_one(X.pv_key_off.p + b.pvn[k], stream));
    b.pvv[k] = uint64_t(d2h_one(X.pv_val_off.p + b.pvn[k], stream));
    b.tgk[k] = uint64_t(d2h_one(X.tags_key_off.p + b.tgn[k], stream));
    b.tgv[k] = uint64_t(d2h_one(X.tags_val_off.p + b.tgn[k], stream));
  }
  return b;
}

static void export_range(dr_state& st, int which, uint64_t lo, uint64_t hi, dr_range& R, dr_export* out) {
  dr_ctx* ctx = st.ctx;
  hipStream_t stream = ctx->stream;
  const DevExport& X = materialize(st, which);
  hi = std::min<uint64_t>(hi, X.n);
  lo = std::min(lo, hi);
  const uint64_t n = hi - lo;
  const RangeBounds b = range_bounds(X, lo, hi, stream);
  const uint64_t npv = b.pvn[1] - b.pvn[0], ntg = b.tgn[1] - b.tgn[0];
  DBuf<uint8_t> dvalid(ctx, n + 1);
  DBuf<int64_t> ddelts(ctx, n + 1);
  launch_delts_fix(X.flags.p + lo, reinterpret_cast<const int64_t*>(X.delts.p) + lo, n, dvalid.p, ddelts.p, stream);
  // the eight offset columns rebased to the range on the device, then copied (a host loop over them
  // took ~30 ms per 1M-row range of config 4, whose 4 partition columns give 8M map offsets per range)
  const uint64_t roff[8] = {0, n + 1, 2 * (n + 1), 3 * (n + 1), 4 * (n + 1), 4 * (n + 1) + npv + 1,
                            4 * (n + 1) + 2 * (npv + 1), 4 * (n + 1) + 2 * (npv + 1) + ntg + 1};
  DBuf<int64_t> reb(ctx, 4 * (n + 1) + 2 * (npv + 1) + 2 * (ntg + 1));
  {
    const int64_t* src[8] = {reinterpret_cast<const int64_t*>(X.path_off.p + lo),
                             reinterpret_cast<const int64_t*>(X.off[EXC_STATS].p + lo),
                             reinterpret_cast<const int64_t*>(X.off[EXC_PV_N].p + lo),
                             reinterpret_cast<const int64_t*>(X.off[EXC_TAGS_N].p + lo),
                             X.pv_key_off.p + b.pvn[0], X.pv_val_off.p + b.pvn[0], X.tags_key_off.p + b.tgn[0],
                             X.tags_val_off.p + b.tgn[0]};
    const uint64_t cnt[8] = {n + 1, n + 1, n + 1, n + 1, npv + 1, npv + 1, ntg + 1, ntg + 1};
    const uint64_t base[8] = {b.path[0], b.stats[0], b.pvn[0], b.tgn[0], b.pvk[0], b.pvv[0], b.tgk[0], b.tgv[0]};
    for (int k = 0; k < 8; ++k) launch_rebase_i64(src[k], cnt[k], int64_t(base[k]), reb.p + roff[k], stream);
  }
  ExportCols ex;  // only its pointer fields: the columns are carved from R.block
  auto u8 = [](const void* p, uint64_t k) { return static_cast<const uint8_t*>(p) + k; };
  const std::vector<ExportCol> cols = {
      {(void**)&ex.path_off, reb.p + roff[0], 8 * (n + 1)},
      {(void**)&ex.path_bytes, u8(X.path_bytes.p, b.path[0]), b.path[1] - b.path[0]},
      {(void**)&ex.delts, ddelts.p, 8 * n},
      {(void**)&ex.delts_valid, dvalid.p, n},
      {(void**)&ex.size, X.size.p + lo, 8 * n},
      {(void**)&ex.mtime, X.mtime.p + lo, 8 * n},
      {(void**)&ex.efm, X.efm.p + lo, n},
      {(void**)&ex.stats_null, X.stats_null.p + lo, n},
      {(void**)&ex.pv_null, X.pv_null.p + lo, n},
      {(void**)&ex.tags_null, X.tags_null.p + lo, n},
      {(void**)&ex.stats_off, reb.p + roff[1], 8 * (n + 1)},
      {(void**)&ex.pv_entry_off, reb.p + roff[2], 8 * (n + 1)},
      {(void**)&ex.tags_entry_off, reb.p + roff[3], 8 * (n + 1)},
      {(void**)&ex.stats_bytes, u8(X.stats_bytes.p, b.stats[0]), b.stats[1] - b.stats[0]},
      {(void**)&ex.pv_key_off, reb.p + roff[4], 8 * (npv + 1)},
      {(void**)&ex.pv_val_off, reb.p + roff[5], 8 * (npv + 1)},
      {(void**)&ex.pv_val_null, X.pv_val_null.p + b.pvn[0], npv},
      {(void**)&ex.pv_key_bytes, u8(X.pv_key_bytes.p, b.pvk[0]), b.pvk[1] - b.pvk[0]},
      {(void**)&ex.pv_val_bytes, u8(X.pv_val_bytes.p, b.pvv[0]), b.pvv[1] - b.pvv[0]},
      {(void**)&ex.tags_key_off, reb.p + roff[6], 8 * (ntg + 1)},
      {(void**)&ex.tags_val_off, reb.p + roff[7], 8 * (ntg + 1)},
      {(void**)&ex.tags_val_null, X.tags_val_null.p + b.tgn[0], ntg},
      {(void**)&ex.tags_key_bytes, u8(X.tags_key_bytes.p, b.tgk[0]), b.tgk[1] - b.tgk[0]},
      {(void**)&ex.tags_val_bytes, u8(X.tags_val_bytes.p, b.tgv[0]), b.tgv[1] - b.tgv[0]}};
  R.ctx = ctx;
  R.block = ctx->host_alloc(group_bytes(cols));
  queue_group(cols, R.block, stream);
  HIP_OK(hipStreamSynchronize(stream));
  *out = dr_export{};
  out->n = int64_t(n);
  out->path_off = ex.path_off; out->path_bytes = ex.path_bytes;
  out->size = ex.size; out->modification_time = ex.mtime;
  out->deletion_timestamp = ex.delts; out->deletion_timestamp_valid = ex.delts_valid;
  out->extended_file_metadata = ex.efm;
  out->stats_off = ex.stats_off; out->stats_bytes = ex.stats_bytes; out->stats_null = ex.stats_null;
  out->pv_entry_off = ex.pv_entry_off; out->pv_null = ex.pv_null;
  out->pv_key_off = ex.pv_key_off; out->pv_key_bytes = ex.pv_key_bytes;
  out->pv_val_off = ex.pv_val_off; out->pv_val_bytes = ex.pv_val_bytes; out->pv_val_null = ex.pv_val_null;
  out->tags_entry_off = ex.tags_entry_off; out->tags_null = ex.tags_null;
  out->tags_key_off = ex.tags_key_off; out->tags_key_bytes = ex.tags_key_bytes;
  out->tags_val_off = ex.tags_val_off; out->tags_val_bytes = ex.tags_val_bytes;
  out->tags_val_null = ex.tags_val_null;
}

// The offsets of the row-level columns at sample rows, and of the entry-level columns at the
// samples' entries: the byte size of every column of a range between two samples, without copying
// the columns (dr_state_export_plan).
struct RangeSampler {
  const DevExport& X;
  dr_ctx* ctx;
  std::vector<uint64_t> rows, po, so, pe, te, pk, pv, tk, tv;
  void sample(std::vector<uint64_t> r) {
    rows = std::move(r);
    hipStream_t stream = ctx->stream;
    auto gather = [&](const uint64_t* src, const std::vector<uint64_t>& idx, std::vector<uint64_t>& dst) {
      std::vector<uint32_t> i32(idx.size());
      for (size_t k = 0; k < idx.size(); ++k) {
        if (idx[k] > 0xffffffffull) fail(DR_E_UNSUPPORTED, "export plan: more than 2^32 map entries in a side");
        i32[k] = uint32_t(idx[k]);
      }
      DBuf<uint32_t> di = upload(ctx, i32.data(), i32.size());
      DBuf<uint64_t> dd(ctx, idx.size());
      launch_gather_u64(src, di.p, idx.size(), dd.p, stream);
      dst = d2h(dd.p, idx.size(), stream);
    };
    gather(X.path_off.p, rows, po);
    gather(X.off[EXC_STATS].p, rows, so);
    gather(X.off[EXC_PV_N].p, rows, pe);
    gather(X.off[EXC_TAGS_N].p, rows, te);
    gather(reinterpret_cast<const uint64_t*>(X.pv_key_off.p), pe, pk);
    gather(reinterpret_cast<const uint64_t*>(X.pv_val_off.p), pe, pv);
    gather(reinterpret_cast<const uint64_t*>(X.tags_key_off.p), te, tk);
    gather(reinterpret_cast<const uint64_t*>(X.tags_val_off.p), te, tv);
  }
  // the largest column (bytes) of the range between samples i < j
  uint64_t cost(size_t i, size_t j) const {
    const uint64_t n = rows[j] - rows[i], npv = pe[j] - pe[i], ntg = te[j] - te[i];
    uint64_t m = 8 * (n + 1);
    for (uint64_t v : {po[j] - po[i], so[j] - so[i], 8 * (npv + 1), pk[j] - pk[i], pv[j] - pv[i], 8 * (ntg + 1),
                       tk[j] - tk[i], tv[j] - tv[i]})
      m = std::max(m, v);
    return m;
  }
};

// Greedy row ranges of [lo, hi): as many rows as fit max_rows and max_bytes per column, sampled every
// `step` rows; a sample interval that alone exceeds max_bytes is split row by row.
static void plan_ranges(const DevExport& X, dr_ctx* ctx, uint64_t lo, uint64_t hi, uint64_t step, uint64_t max_rows,
                        uint64_t max_bytes, std::vector<int64_t>& bounds) {
  std::vector<uint64_t> r;
  for (uint64_t x = lo; x < hi; x += step) r.push_back(x);
  r.push_back(hi);
  RangeSampler S{X, ctx};
  S.sample(std::move(r));
  size_t i = 0;
  while (S.rows[i] < hi) {
    size_t j = i + 1;
    if (S.cost(i, j) > max_bytes) {
      if (step == 1) fail(DR_E_UNSUPPORTED, fmt("export plan: row %llu alone holds a column over %llu bytes",
                                                (unsigned long long)S.rows[i], (unsigned long long)max_bytes));
      plan_ranges(X, ctx, S.rows[i], S.rows[j], 1, max_rows, max_bytes, bounds);
      i = j;
      continue;
    }
    while (j + 1 < S.rows.size() && S.rows[j + 1] - S.rows[i] <= max_rows && S.cost(i, j + 1) <= max_bytes) ++j;
    if (S.rows[j] - S.rows[i] > max_rows) {  // a sample interval longer than max_rows: split it evenly
      for (uint64_t x = S.rows[i] + max_rows; x < S.rows[j]; x += max_rows) bounds.push_back(int64_t(x));
    }
    bounds.push_back(int64_t(S.rows[j]));
    i = j;
  }
}

int dr_state_export_plan(dr_state* state, int32_t which, int64_t max_rows, uint64_t max_bytes, int64_t** bounds,
                         int64_t* nranges) {
  if (!state || !bounds || !nranges || (which != DR_LIVE && which != DR_TOMBSTONES) || max_rows <= 0 ||
      max_bytes < 64)
    return DR_E_INVALID_ARG;
  *bounds = nullptr;
  *nranges = 0;
  return guard(state->ctx, [&] {
    HIP_OK(hipSetDevice(state->ctx->device));
    const DevExport& X = materialize(*state, which);
    std::vector<int64_t> b{0};
    if (X.n) {
      const uint64_t step = std::max<uint64_t>(1, std::min<uint64_t>(4096, uint64_t(max_rows)));
      plan_ranges(X, state->ctx, 0, X.n, step, uint64_t(max_rows), max_bytes, b);
    }
    *bounds = malloc_copy(b);
    *nranges = int64_t(b.size()) - 1;
  });
}

int dr_state_export_range(dr_state* state, int32_t which, int64_t row_begin, int64_t row_end, dr_range** range,
                          dr_export* out) {
  if (!state || !range || !out || (which != DR_LIVE && which != DR_TOMBSTONES) || row_begin < 0 ||
      row_end < row_begin)
    return DR_E_INVALID_ARG;
  *range = nullptr;
  return guard(state->ctx, [&] {
    HIP_OK(hipSetDevice(state->ctx->device));
    auto R = std::make_unique<dr_range>();
    export_range(*state, which, uint64_t(row_begin), uint64_t(row_end), *R, out);
    std::lock_guard<std::mutex> g(g_ranges_mu);
    g_ranges.insert(R.get());
    *range = R.release();
  });
}

int dr_range_release(dr_range* range) {
  if (!range) return DR_OK;
  // the registry lock is held while the block returns to its context, so dr_ctx_destroy cannot free
  // the context in between (it detaches ranges under the same lock)
  std::lock_guard<std::mutex> g(g_ranges_mu);
  if (!g_ranges.erase(range)) return DR_E_INVALID_ARG;  // not a live range (released twice)
  delete range;
  return DR_OK;
}

int dr_state_materialize(dr_state* state, uint64_t* bytes) {
  if (!state) return DR_E_INVALID_ARG;
  return guard(state->ctx, [&] {
    HIP_OK(hipSetDevice(state->ctx->device));
    uint64_t b = 0;
    for (int w = 0; w < 2; ++w) {
      const DevExport& X = materialize(*state, w);
      const uint64_t n = X.n;
      b += n * (8 + 4 + 8 + 8 + 1 + 8 + 8 + 4 * 1) + 3 * 8 * (n + 1) + X.path_bytes.n;
      b += X.tot[EXC_STATS] + X.tot[EXC_PV_KB] + X.tot[EXC_PV_VB] + X.tot[EXC_TAGS_KB] + X.tot[EXC_TAGS_VB];
      b += 17 * (X.tot[EXC_PV_N] + X.tot[EXC_TAGS_N]);
    }
    HIP_OK(hipStreamSynchronize(state->ctx->stream));
    if (bytes) *bytes = b;
  });
}

int dr_state_record_sums(dr_state* state, uint64_t* live_sum, uint64_t* tomb_sum) {
  if (!state || !live_sum || !tomb_sum) return DR_E_INVALID_ARG;
  return guard(state->ctx, [&] {
    HIP_OK(hipSetDevice(state->ctx->device));
    *live_sum = record_sum(*state, DR_LIVE);
    *tomb_sum = record_sum(*state, DR_TOMBSTONES);
  });
}

int dr_state_record_hashes(dr_state* state, int32_t which, uint64_t* out, int64_t n) {
  if (!state || (which != DR_LIVE && which != DR_TOMBSTONES) || n < 0 || (n && !out)) return DR_E_INVALID_ARG;
  return guard(state->ctx, [&] {
    HIP_OK(hipSetDevice(state->ctx->device));
    const int64_t rows = int64_t(which == DR_LIVE ? state->n_live : state->n_tomb);
    if (n != rows) fail(DR_E_INVALID_ARG, fmt("record hashes: the side holds %lld rows, the buffer %lld",
                                             (long long)rows, (long long)n));
    (void)record_sum(*state, which, out);
  });
}

int dr_filter(dr_state* state, const dr_predicate* pred, int64_t** selected, int64_t* nselected) {
  if (!state || !pred || !selected || !nselected) return DR_E_INVALID_ARG;
  *selected = nullptr;
  *nselected = 0;
  return guard(state->ctx, [&] {
    HIP_OK(hipSetDevice(state->ctx->device));
    std::vector<int64_t> v = filter_state(*state, *pred);
    int64_t* out = static_cast<int64_t*>(malloc(std::max<size_t>(v.size(), 1) * sizeof(int64_t)));
    if (!out) throw std::bad_alloc();
    if (!v.empty()) memcpy(out, v.data(), v.size() * sizeof(int64_t));
    *selected = out;
    *nselected = int64_t(v.size());
  });
}

static int64_t* malloc_copy(const std::vector<int64_t>& v) {
  int64_t* out = static_cast<int64_t*>(malloc(std::max<size_t>(v.size(), 1) * sizeof(int64_t)));
  if (!out) throw std::bad_alloc();
  if (!v.empty()) memcpy(out, v.data(), v.size() * sizeof(int64_t));
  return out;
}

int dr_state_scan_order(dr_state* state, int64_t** order, int64_t* n) {
  if (!state || !order || !n) return DR_E_INVALID_ARG;
  *order = nullptr;
  *n = 0;
  return guard(state->ctx, [&] {
    HIP_OK(hipSetDevice(state->ctx->device));
    std::vector<int64_t> v = scan_order(*state);
    *order = malloc_copy(v);
    *n = int64_t(v.size());
  });
}

int dr_state_partition_groups(dr_state* state, const int64_t* rows, int64_t nrows, int64_t** order,
                              int64_t** group_off, int64_t* ngroups) {
  if (!state || !order || !group_off || !ngroups || (rows && nrows < 0)) return DR_E_INVALID_ARG;
  *order = nullptr;
  *group_off = nullptr;
  *ngroups = 0;
  return guard(state->ctx, [&] {
    HIP_OK(hipSetDevice(state->ctx->device));
    std::vector<int64_t> o, g;
    partition_groups(*state, rows, nrows, o, g);
    *order = malloc_copy(o);
    *group_off = malloc_copy(g);
    *ngroups = int64_t(g.size()) - 1;
  });
}

int dr_state_write_checkpoint(dr_state* state, int32_t part, int32_t parts, uint32_t opts, uint64_t row_group_rows,
                              uint8_t** bytes, uint64_t* len, int64_t* rows, int64_t* add_rows) {
  if (!state || !bytes || !len || parts < 1 || part < 1 || part > parts) return DR_E_INVALID_ARG;
  *bytes = nullptr;
  *len = 0;
  return guard(state->ctx, [&] {
    HIP_OK(hipSetDevice(state->ctx->device));
    CkPartOut o;
    write_checkpoint_part(*state, part, parts, opts, row_group_rows, o);
    *len = o.len;
    *bytes = o.data;  // pinned: the caller frees it with dr_free
    if (rows) *rows = o.rows;
    if (add_rows) *add_rows = o.add_rows;
  });
}

void dr_free(void* p) {
  if (!p) return;
  {
    std::unique_lock<std::mutex> g(g_pinned_out_mu);
    auto it = g_pinned_out.find(p);
    if (it != g_pinned_out.end()) {
      dr_ctx* ctx = it->second;
      g_pinned_out.erase(it);
      // (still under the lock: dr_ctx_destroy detaches its blocks under it before freeing the context)
      if (ctx) ctx->host_release(p);  // back to the context's pool
      else (void)hipHostFree(p);      // its context is gone
      return;
    }
  }
  free(p);
}

int dr_state_set_nonfile_json(dr_state* state, const char* lines, uint64_t len, uint32_t flags) {
  if (!state || (!lines && len)) return DR_E_INVALID_ARG;
  return guard(state->ctx, [&] {
    if (!state->sharded) fail(DR_E_INVALID_ARG, "dr_state_set_nonfile_json takes a sharded replay's state");
    set_nonfile_lines(*state, std::string(lines ? lines : "", len), !(flags & DR_FLAG_NO_VALIDATION));
  });
}

int dr_set_timing_only(dr_ctx* ctx, const char* kernel) {
  if (!ctx) return DR_E_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(ctx->api_mu);
  ctx->timing_only = kernel ? kernel : "";
  return DR_OK;
}

int dr_set_timing(dr_ctx* ctx, int32_t on) {
  if (!ctx) return DR_E_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(ctx->api_mu);
  ctx->timing = on != 0;
  return DR_OK;
}

int dr_last_timings(dr_ctx* ctx, char* names, uint64_t names_len, float* ms, int32_t cap, int32_t* n) {
  if (!ctx || !n) return DR_E_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(ctx->api_mu);
  std::string all;
  int32_t k = 0;
  for (auto& t : ctx->timings) {
    if (k < cap && ms) ms[k] = t.second;
    all += t.first;
    all.push_back('\0');
    ++k;
  }
  *n = k;
  if (names && names_len) {
    size_t c = std::min<size_t>(all.size(), names_len);
    memcpy(names, all.data(), c);
  }
  return DR_OK;
}

/* ---- multi-GPU shards ---- */
int dr_shard_plan(dr_ctx* ctx, const char* log_path, int64_t version_to_load, int32_t world, char* buf,
                  uint64_t buf_len, uint64_t* needed) {
  if (!log_path || world < 1) return DR_E_INVALID_ARG;  // host only: ctx may be NULL
  return guard(ctx, [&] {
    LogSegmentInfo seg = get_log_segment(log_path, version_to_load);
    std::vector<ShardUnit> units = shard_units(log_path, seg);
    std::vector<int32_t> owner = shard_assign(units, world);
    std::string s;
    for (size_t k = 0; k < units.size(); ++k)
      s += fmt("%d %d %lld %d %d %d %llu %s\n", owner[k], units[k].f.kind, (long long)units[k].f.version, units[k].f.part,
               units[k].rg_lo, units[k].rg_hi, (unsigned long long)units[k].weight, units[k].f.name.c_str());
    if (needed) *needed = s.size() + 1;
    if (buf && buf_len) {
      size_t n = std::min<size_t>(s.size(), buf_len - 1);
      memcpy(buf, s.data(), n);
      buf[n] = 0;
    }
  });
}

int dr_stage_log_shard(dr_ctx* ctx, const char* log_path, int64_t version_to_load, int32_t world, int32_t rank,
                       dr_staged** out) {
  if (!ctx || !out || !log_path || world < 1 || rank < 0 || rank >= world) return DR_E_INVALID_ARG;
  return guard(ctx, [&] {
    HIP_OK(hipSetDevice(ctx->device));
    auto s = std::make_unique<dr_staged>();
    s->d = stage_shard(ctx, log_path, version_to_load, world, rank);
    *out = s.release();
  });
}

int dr_shard_begin(dr_ctx* ctx, const dr_staged* staged, int32_t world, dr_shard** out, uint64_t* send_counts,
                   uint64_t* send_bytes) {
  if (!ctx || !staged || !out || !send_counts || !send_bytes || world < 1 || uint32_t(world) > shard_max_world())
    return DR_E_INVALID_ARG;
  *out = nullptr;
  return guard(ctx, [&] {
    HIP_OK(hipSetDevice(ctx->device));
    auto sh = std::make_unique<dr_shard>();
    sh->ctx = ctx;
    sh->staged = staged->d;
    sh->world = uint32_t(world);
    ctx->begin_call();
    shard_begin(*sh, send_counts, send_bytes);
    *out = sh.release();
  });
}

int dr_shard_pack(dr_shard* shard, void* send_rec, void* send_path) {
  if (!shard || !shard->st || (shard->nsend && (!send_rec || (shard->send_path_bytes && !send_path))))
    return DR_E_INVALID_ARG;
  return guard(shard->ctx, [&] { shard_pack(*shard, send_rec, send_path); });
}

int dr_shard_reduce(dr_shard* shard, const void* recv_rec, uint64_t n_recv, const void* recv_path,
                    uint64_t recv_path_bytes, int64_t min_file_retention_timestamp, uint8_t* verdict) {
  if (!shard || !shard->st || (n_recv && (!recv_rec || !verdict)) || (recv_path_bytes && !recv_path))
    return DR_E_INVALID_ARG;
  return guard(shard->ctx, [&] { shard_reduce(*shard, recv_rec, n_recv, recv_path, min_file_retention_timestamp, verdict); });
}

int dr_shard_finish(dr_shard* shard, const uint8_t* verdict_back, dr_state** out) {
  if (!shard || !shard->st || !out || (shard->nsend && !verdict_back)) return DR_E_INVALID_ARG;
  *out = nullptr;
  dr_ctx* ctx = shard->ctx;
  int rc = guard(ctx, [&] {
    if (!shard->reduced) fail(DR_E_INVALID_ARG, "dr_shard_finish before dr_shard_reduce");
    *out = shard_finish(*shard, verdict_back);
    ctx->collect_timings();
  });
  if (rc != DR_OK) ctx->drop_timings();
  return rc;
}

int dr_parse_commits(dr_ctx* ctx, const dr_staged* staged, dr_parsed** out, dr_lines* lines) {
  if (!ctx || !staged || !out || !lines) return DR_E_INVALID_ARG;
  *out = nullptr;
  return guard(ctx, [&] {
    HIP_OK(hipSetDevice(ctx->device));
    auto p = std::make_unique<dr_parsed>();
    ctx->begin_call();
    parse_commits(ctx, staged->d, *p);
    ctx->collect_timings();
    *lines = dr_lines{};
    lines->n = int64_t(p->kind.size());
    lines->version = p->version.data();
    lines->line_off = p->line_off.data();
    lines->line_len = p->line_len.data();
    lines->kind = p->kind.data();
    lines->flags = p->flags.data();
    lines->path_off = p->path_off.data();
    lines->path_len = p->path_len.data();
    lines->size = p->size.data();
    lines->deletion_timestamp = p->delts.data();
    lines->bytes = p->staged->h_json.data();
    lines->nbytes = p->staged->h_json.size();
    *out = p.release();
  });
}

int dr_comm_unique_id(uint8_t* id) {
  if (!id) return DR_E_INVALID_ARG;
  try {
    ncclUniqueId u;
    if (rccl().get_id(&u) != ncclSuccess) return DR_E_DEVICE;
    memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
    return DR_OK;
  } catch (const Error& e) {
    return e.status;
  } catch (...) {
    return DR_E_INTERNAL;
  }
}

int dr_comm_loopback_id(uint8_t* id) {
  if (!id) return DR_E_INVALID_ARG;
  static std::atomic<uint64_t> next{1};
  memset(id, 0, 128);
  memcpy(id, kLoopMagic, 8);
  const uint64_t g = next.fetch_add(1);
  memcpy(id + 8, &g, 8);
  return DR_OK;
}

int dr_comm_create(dr_ctx* ctx, const uint8_t* id, int32_t world, int32_t rank, dr_comm** out) {
  if (!ctx || !id || !out || world < 1 || rank < 0 || rank >= world || uint32_t(world) > shard_max_world())
    return DR_E_INVALID_ARG;
  *out = nullptr;
  return guard(ctx, [&] {
    HIP_OK(hipSetDevice(ctx->device));
    auto c = std::make_unique<dr_comm>();
    c->ctx = ctx;
    c->world = world;
    c->rank = rank;
    if (memcmp(id, kLoopMagic, 8) == 0) {
      uint64_t gid;
      memcpy(&gid, id + 8, 8);
      std::lock_guard<std::mutex> g(g_loop_mu);
      std::shared_ptr<LoopGroup> grp = g_loop_groups[gid].lock();
      if (!grp) {
        grp = std::make_shared<LoopGroup>();
        grp->world = world;
        grp->ptr.assign(size_t(world), nullptr);
        grp->cnt.assign(size_t(world), nullptr);
        g_loop_groups[gid] = grp;
      }
      if (grp->world != world) fail(DR_E_INVALID_ARG, "loopback communicator joined with a different world size");
      c->loop = grp;
    } else {
      ncclUniqueId u;
      memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
      RC_OK(rccl().init_rank(&c->comm, world, u, rank));
    }
    *out = c.release();
  });
}

int dr_comm_release(dr_comm* comm) {
  if (!comm) return DR_E_INVALID_ARG;
  if (comm->comm) (void)rccl().destroy(comm->comm);
  delete comm;
  return DR_OK;
}

int dr_replay_sharded(dr_comm* comm, const dr_staged* staged, int64_t min_file_retention_timestamp, uint32_t flags,
                      dr_state** out) {
  if (!comm || !staged || !out) return DR_E_INVALID_ARG;
  *out = nullptr;
  dr_ctx* ctx = comm->ctx;
  const int rc = guard(ctx, [&] {
    HIP_OK(hipSetDevice(ctx->device));
    ctx->begin_call();
    *out = replay_sharded_rccl(*comm, staged->d, min_file_retention_timestamp, flags);
    ctx->collect_timings();
  });
  if (rc != DR_OK && comm->loop) comm->loop->abort();  // the other ranks fail instead of waiting
  return rc;
}

int dr_parsed_release(dr_parsed* parsed) {
  delete parsed;
  return DR_OK;
}

int dr_shard_release(dr_shard* shard) {
  if (!shard) return DR_OK;
  std::lock_guard<std::recursive_mutex> g(shard->ctx->api_mu);
  (void)hipStreamSynchronize(shard->ctx->stream);
  delete shard;
  return DR_OK;
}

}  // extern "C"

