// Multi-threaded native ingest of a Molly output directory:
// faultinjectors/molly.go:15-163 (LoadOutput: per-run provenance files, clock
// times from labels, run_<iteration>_<cond>_ ID prefixes) fused with the
// interning that replaces loadProv's per-element CREATE/MERGE round trips
// (graphing/pre-post-prov.go:25-213), producing the nemo_corpus arrays.
//
// Graphs are parsed in parallel (one file per task); strings are interned per
// graph in first-appearance order and merged into the global table/label ids
// in graph order, so the result is identical to the sequential interning of
// nemo_amd/corpus.py (tests/test_ingest.py checks it array for array).
// Host code only; no device work.
#include <emmintrin.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/nemohip.h"

namespace {

struct Str {
  uint32_t off, len;
};

// Live mappings of the process: every graph keeps its file mapped while it
// lives (its strings are views), so a one-shot ingest of many runs would pass
// the kernel's vm.max_map_count (65530 by default) and mmap would fail.  Past
// a limit (half the kernel's, or NEMO_INGEST_MAP_LIMIT) a file is read into a
// heap buffer instead; the parse is the same either way.
std::atomic<int64_t> g_live_maps{0};
int64_t map_limit() {
  static const int64_t lim = [] {
    if (const char *e = getenv("NEMO_INGEST_MAP_LIMIT")) return (int64_t)atoll(e);
    int64_t k = 65530;
    if (FILE *f = fopen("/proc/sys/vm/max_map_count", "r")) {
      long long v;
      if (fscanf(f, "%lld", &v) == 1 && v > 0) k = v;
      fclose(f);
    }
    return k / 2;
  }();
  return lim;
}

// a provenance file mapped read-only (page-cache pages, no copy), or read
// into a heap buffer past the mapping limit; released with its graph
struct FileMap {
  void *p = nullptr;
  size_t n = 0;
  std::unique_ptr<char[]> heap;  // the read() fallback (p points into it)
  FileMap() = default;
  FileMap(const FileMap &) = delete;
  FileMap &operator=(const FileMap &) = delete;
  FileMap(FileMap &&o) noexcept : p(o.p), n(o.n), heap(std::move(o.heap)) { o.p = nullptr, o.n = 0; }
  FileMap &operator=(FileMap &&o) noexcept {
    if (this != &o) reset(), p = o.p, n = o.n, heap = std::move(o.heap), o.p = nullptr, o.n = 0;
    return *this;
  }
  ~FileMap() { reset(); }
  void reset() {
    if (p && !heap) {
      munmap(p, n);
      g_live_maps.fetch_sub(1, std::memory_order_relaxed);
    }
    heap.reset();
    p = nullptr, n = 0;
  }
  bool mapped() const { return p && !heap; }
  // false: the file cannot be opened or read
  bool open(const char *path) {
    reset();
    const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) return false;
    struct stat st;
    bool ok = fstat(fd, &st) == 0 && S_ISREG(st.st_mode);
    if (ok && st.st_size > 0) {
      const size_t sz = (size_t)st.st_size;
      void *m = MAP_FAILED;
      if (g_live_maps.fetch_add(1, std::memory_order_relaxed) < map_limit())
        m = mmap(nullptr, sz, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
      if (m != MAP_FAILED) {
        p = m, n = sz;
      } else {  // over the limit, or the kernel refused (ENOMEM at vm.max_map_count)
        g_live_maps.fetch_sub(1, std::memory_order_relaxed);
        heap.reset(new char[sz + 64]);
        size_t got = 0;
        while (got < sz) {
          const ssize_t r = ::read(fd, heap.get() + got, sz - got);
          if (r <= 0) break;
          got += (size_t)r;
        }
        if (got != sz) {
          heap.reset();
          ok = false;
        } else {
          memset(heap.get() + sz, 0, 64);
          p = heap.get(), n = sz;
        }
      }
    }
    close(fd);
    return ok;
  }
};

// an array written in full after each resize (the output arrays, a graph's
// per-node fields): resize neither keeps nor initialises the contents, so
// nothing is zero-filled and the output pages are first touched by the
// parallel fill
template <class T>
struct RawBuf {
  std::unique_ptr<T[]> p;
  size_t n = 0, cap = 0;
  void resize(size_t m) {
    if (m > cap) p.reset(new T[m]), cap = m;
    n = m;
  }
  T *data() const { return p.get(); }
  size_t size() const { return n; }
  T *begin() const { return p.get(); }
  T &operator[](size_t i) { return p[i]; }
  const T &operator[](size_t i) const { return p[i]; }
  void clear() { n = 0; }
};

struct Graph {
  // Str offsets below flen are bytes of the mapped file (strings without
  // escapes), at and above it the arena (decoded strings, clock times)
  FileMap file;
  const char *fb = "";
  uint32_t flen = 0;
  std::vector<char> arena;
  // per node, written in full by parse_graph: the ID, and a goal's time or a
  // rule's type (the strings nemo_ingest_string hands out)
  RawBuf<Str> id, tt;
  uint32_t n_goals = 0;
  std::vector<uint32_t> src, dst, rank;
  RawBuf<uint32_t> ltab, llab;
  RawBuf<uint8_t> tclass;
  std::vector<Str> tabs, labs;  // local first-appearance order
  std::vector<uint64_t> labh;   // hash_sv of each of labs (the global interning's shard and slot)
  std::string err;
  std::string_view sv(Str s) const {
    return std::string_view(s.off < flen ? fb + s.off : arena.data() + (s.off - flen), s.len);
  }
  // empty again, keeping the vectors' memory (a stream reuses its graphs chunk after chunk:
  // no fresh pages to fault in)
  void reset() {
    file.reset();
    fb = "";
    flen = 0;
    n_goals = 0;
    id.clear(), tt.clear();
    tabs.clear(), labs.clear();
    for (auto *v : {&src, &dst, &rank}) v->clear();
    ltab.clear(), llab.clear();
    arena.clear(), tclass.clear(), labh.clear(), err.clear();
  }
};
struct Rec {  // a goal's or rule's fields: id, label, table, time / type
  Str f[4];
};

// ---- open-addressing tables (the per-graph maps are hot: one lookup per node and edge) ----
// Keys of more than 8 bytes are hashed from whole 8-byte loads inside the key.
inline uint64_t load8(const char *p) {
  uint64_t w;
  memcpy(&w, p, 8);
  return w;
}
// a == b with short keys compared inline (no memcmp call): up to 16 bytes as two
// overlapping loads each way, exact bytes only
inline bool sveq(std::string_view a, std::string_view b) {
  const size_t n = a.size();
  if (n != b.size()) return false;
  const char *x = a.data(), *y = b.data();
  if (n >= 8) {
    if (n > 16) return !memcmp(x, y, n);
    return load8(x) == load8(y) && load8(x + n - 8) == load8(y + n - 8);
  }
  if (n >= 4) {
    uint32_t x0, x1, y0, y1;
    memcpy(&x0, x, 4), memcpy(&x1, x + n - 4, 4), memcpy(&y0, y, 4), memcpy(&y1, y + n - 4, 4);
    return x0 == y0 && x1 == y1;
  }
  for (size_t i = 0; i < n; i++)
    if (x[i] != y[i]) return false;
  return true;
}
inline uint64_t hash_sv(std::string_view s) {
  const size_t n = s.size();
  const char *p = s.data();
  uint64_t h = 0x9E3779B97F4A7C15ull ^ n;
  if (n <= 8) {  // exact bytes (a short key may end a buffer): for a given n these words tell every key apart
    uint64_t w = 0;
    if (n >= 4) {
      uint32_t a, b;
      memcpy(&a, p, 4);
      memcpy(&b, p + n - 4, 4);
      w = (uint64_t)a | (uint64_t)b << 32;
    } else if (n) {
      w = (uint64_t)(uint8_t)p[0] | (uint64_t)(uint8_t)p[n / 2] << 8 | (uint64_t)(uint8_t)p[n - 1] << 16;
    }
    h = (h ^ w) * 0xff51afd7ed558ccdull;
  } else if (n <= 16) {
    h = (h ^ load8(p)) * 0xff51afd7ed558ccdull;
    h = (h ^ (h >> 32) ^ load8(p + n - 8)) * 0xc4ceb9fe1a85ec53ull;
  } else {
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
      h = (h ^ load8(p + i)) * 0xff51afd7ed558ccdull;
      h ^= h >> 32;
    }
    h = (h ^ load8(p + n - 8)) * 0xc4ceb9fe1a85ec53ull;
  }
  h ^= h >> 33;  // fmix64: every key bit reaches the low (slot) bits
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ull;
  return h ^ (h >> 33);
}

// string_view -> u32 with hash-tagged slots, reused from graph to graph by one
// thread: a slot is live only in the epoch that wrote it, so no clearing
struct FlatMap {
  struct Slot {  // the key's view in the slot: one cache line per probe
    const char *kp;
    uint32_t klen, tag, val, epoch;
  };
  std::vector<Slot> slot;
  size_t mask = 0;
  uint32_t epoch = 0;
  void init(size_t n) {
    size_t cap = 16;
    while (cap < 2 * n + 16) cap <<= 1;
    if (cap > slot.size() || ++epoch == 0) {
      slot.assign(std::max(cap, slot.size()), Slot{nullptr, 0, 0, 0, 0});
      epoch = 1;
    }
    mask = cap - 1;
  }
  // value of k, inserting v if absent; second = inserted
  std::pair<uint32_t, bool> emplace(std::string_view k, uint32_t v) { return emplace_h(k, hash_sv(k), v); }
  std::pair<uint32_t, bool> emplace_h(std::string_view k, uint64_t h, uint32_t v) {
    const uint32_t tag = (uint32_t)(h >> 32);
    for (size_t i = h & mask;; i = (i + 1) & mask) {
      Slot &sl = slot[i];
      if (sl.epoch != epoch) {
        sl = Slot{k.data(), (uint32_t)k.size(), tag, v, epoch};
        return {v, true};
      }
      if (sl.tag == tag && sveq(std::string_view(sl.kp, sl.klen), k)) return {sl.val, false};
    }
  }
  uint32_t find(std::string_view k) const {
    const uint64_t h = hash_sv(k);
    const uint32_t tag = (uint32_t)(h >> 32);
    for (size_t i = h & mask;; i = (i + 1) & mask) {
      const Slot &sl = slot[i];
      if (sl.epoch != epoch) return ~0u;
      if (sl.tag == tag && sveq(std::string_view(sl.kp, sl.klen), k)) return sl.val;
    }
  }
};

// u64 keys whose bits 28-31 and 60-63 are clear (two u28 node indices), reused
// like FlatMap: the slot's epoch sits in those bits (8-byte slots)
struct FlatSet64 {
  std::vector<uint64_t> slot;
  size_t mask = 0;
  uint32_t epoch = 0;  // 1..255
  static uint64_t tagged(uint64_t k, uint32_t e) { return k | (uint64_t)(e & 0xFu) << 28 | (uint64_t)(e >> 4) << 60; }
  void init(size_t n) {
    size_t cap = 16;
    while (cap < 2 * n + 16) cap <<= 1;
    if (cap > slot.size() || ++epoch == 256) {
      slot.assign(std::max(cap, slot.size()), 0);  // epoch 0: empty
      epoch = 1;
    }
    mask = cap - 1;
  }
  bool insert(uint64_t k) {
    const uint64_t t = tagged(k, epoch), em = tagged(0, 0xFFu);
    for (size_t h = ((k * 0x9E3779B97F4A7C15ull) >> 20) & mask;; h = (h + 1) & mask) {
      const uint64_t x = slot[h];
      if ((x & em) != (t & em)) return slot[h] = t, true;
      if (x == t) return false;
    }
  }
};

// The global interning: string -> id, in first-appearance order, keys viewing
// storage that outlives the map (the graphs' arenas, or the stream's tables).
struct InternMap {
  struct Slot {
    uint32_t tag, val;  // val ~0u = empty
  };
  std::vector<Slot> slot;
  std::vector<std::string_view> key;
  size_t mask = 0, n = 0;
  void grow() {
    const size_t cap = std::max<size_t>(64, 2 * slot.size());
    std::vector<Slot> os(cap, Slot{0, ~0u});
    std::vector<std::string_view> ok(cap);
    os.swap(slot);
    ok.swap(key);
    mask = cap - 1;
    for (size_t i = 0; i < os.size(); i++) {
      if (os[i].val == ~0u) continue;
      size_t j = hash_sv(ok[i]) & mask;
      while (slot[j].val != ~0u) j = (j + 1) & mask;
      slot[j] = os[i];
      key[j] = ok[i];
    }
  }
  // the id of k; absent: make(k) stores it and returns (its id, a view of the stored copy)
  template <class F>
  uint32_t intern(std::string_view k, F &&make) {
    if (2 * (n + 1) > slot.size()) grow();
    const uint64_t h = hash_sv(k);
    const uint32_t tag = (uint32_t)(h >> 32);
    for (size_t i = h & mask;; i = (i + 1) & mask) {
      if (slot[i].val == ~0u) {
        const std::pair<uint32_t, std::string_view> m = make(k);
        slot[i] = Slot{tag, m.first};
        key[i] = m.second;
        n++;
        return m.first;
      }
      if (slot[i].tag == tag && sveq(key[i], k)) return slot[i].val;
    }
  }
};

// n persistent workers (a stream's, so that their per-thread maps and lists
// stay allocated from chunk to chunk); run(f) runs f once on every worker
class WorkerPool {
 public:
  explicit WorkerPool(int n) {
    for (int i = 0; i < n; i++) th_.emplace_back([this] { loop(); });
  }
  ~WorkerPool() {
    {
      std::lock_guard<std::mutex> l(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : th_) t.join();
  }
  void run(const std::function<void()> &f) {
    std::unique_lock<std::mutex> l(m_);
    job_ = &f;
    left_ = (int)th_.size();
    gen_++;
    cv_.notify_all();
    done_.wait(l, [this] { return left_ == 0; });
    job_ = nullptr;
  }

 private:
  void loop() {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> l(m_);
    for (;;) {
      cv_.wait(l, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      const std::function<void()> *f = job_;
      l.unlock();
      (*f)();
      l.lock();
      if (--left_ == 0) done_.notify_one();
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<void()> *job_ = nullptr;
  uint64_t gen_ = 0;
  int left_ = 0;
  bool stop_ = false;
};

// f on nt threads: the pool's workers, or nt - 1 new threads and the caller
using Runner = std::function<void(const std::function<void()> &)>;
inline Runner make_runner(WorkerPool *pool, int nt) {
  if (pool) return [pool](const std::function<void()> &f) { pool->run(f); };
  return [nt](const std::function<void()> &f) {
    std::vector<std::thread> th;
    for (int i = 1; i < nt; i++) th.emplace_back(f);
    f();
    for (auto &t : th) t.join();
  };
}

// The global label interning, sharded by hash so that threads intern in
// parallel with the sequential result.  A label's shard is fixed by its hash;
// each shard is filled by one thread walking the graphs in order, so an entry
// is created at the label's first appearance (graph, local index), which is
// flagged.  One serial pass over the local labels in graph order then numbers
// the flagged ones: global ids in first-appearance order, as one map would give.
struct ShardIntern {
  static constexpr uint32_t NEW = 1u << 31, SH = 25;  // lre entry: NEW | shard << SH | shard index
  struct Shard {
    // open-addressing slots: hash tag, shard index (~0u empty), and keys of up
    // to 16 bytes inline (a lookup touches one slot; longer keys compare
    // against `key`)
    struct Slot {
      uint32_t tag, val, len, pad;
      char b[16];
    };
    std::vector<Slot> slot;
    size_t mask = 0;
    std::vector<std::string_view> key;
    std::vector<uint64_t> hash;
    std::vector<uint32_t> gid;        // by shard index: the global id
    static void put(Slot &sl, uint32_t t, uint32_t v, std::string_view k) {
      sl.tag = t, sl.val = v, sl.len = (uint32_t)std::min<size_t>(k.size(), 0xFFFFFFFFu);
      if (k.size() <= 16) memcpy(sl.b, k.data(), k.size());
    }
    void grow() {
      const size_t cap = std::max<size_t>(64, 2 * slot.size());
      slot.assign(cap, Slot{0, ~0u, 0, 0, {}});
      mask = cap - 1;
      for (uint32_t x = 0; x < key.size(); x++) {
        size_t i = hash[x] & mask;
        while (slot[i].val != ~0u) i = (i + 1) & mask;
        put(slot[i], (uint32_t)(hash[x] >> 32), x, key[x]);
      }
    }
    // the shard index of k, and whether it is new
    std::pair<uint32_t, bool> intern(std::string_view k, uint64_t h) {
      if (2 * (key.size() + 1) > slot.size()) grow();
      const uint32_t t = (uint32_t)(h >> 32);
      for (size_t i = h & mask;; i = (i + 1) & mask) {
        Slot &sl = slot[i];
        if (sl.val == ~0u) {
          put(sl, t, (uint32_t)key.size(), k);
          key.push_back(k);
          hash.push_back(h);
          gid.push_back(~0u);
          return {sl.val, true};
        }
        if (sl.tag == t && sl.len == k.size() &&
            (k.size() <= 16 ? sveq(std::string_view(sl.b, k.size()), k) : sveq(key[sl.val], k)))
          return {sl.val, false};
      }
    }
  };
  std::vector<Shard> sh;  // one per thread of the first merge (fixed from then on)
  uint64_t count = 0;     // labels numbered so far
  std::vector<std::vector<uint32_t>> bli;  // per graph: its local labels grouped by shard
  std::vector<uint32_t> boff;              // per graph: S + 1 group bounds in bli
  uint32_t shard_of(uint64_t h) const { return (uint32_t)(((h >> 40) * sh.size()) >> 24); }

  // lre[g][li] = global id of graph g's local label li.  add(view) stores a
  // new label's name (its index is the global id) and returns the view the
  // shard keeps from then on (the graphs' arenas may not outlive the call).
  template <class Add>
  bool merge(std::vector<Graph> &gs, uint32_t G, int nt, const Runner &run, std::vector<std::vector<uint32_t>> &lre,
             Add &&add) {
    if (sh.empty()) sh.resize((size_t)std::min(64, std::max(1, nt)));
    const uint32_t S = (uint32_t)sh.size();
    if (bli.size() < G) bli.resize(G);
    boff.resize((size_t)G * (S + 1));
    // each graph's labels grouped by shard (in parallel by graph), so that a
    // shard's thread reads its own labels only
    std::atomic<uint32_t> nextb{0};
    auto phase_0 = [&] {
      uint32_t cur[65];
      for (uint32_t g; (g = nextb.fetch_add(1)) < G;) {
        const Graph &gr = gs[g];
        const uint32_t L = (uint32_t)gr.labh.size();
        uint32_t *off = &boff[(size_t)g * (S + 1)];
        std::fill(off, off + S + 1, 0u);
        for (uint32_t li = 0; li < L; li++) off[shard_of(gr.labh[li]) + 1]++;
        for (uint32_t k = 0; k < S; k++) off[k + 1] += off[k];
        std::copy(off, off + S, cur);
        bli[g].resize(L);
        for (uint32_t li = 0; li < L; li++) bli[g][cur[shard_of(gr.labh[li])]++] = li;
        lre[g].resize(L);  // every entry is written by its shard below
      }
    };
    run(phase_0);
    std::atomic<uint32_t> nexts{0};
    std::atomic<bool> over{false};  // a shard index past SH bits would spill into the shard field
    auto phase_a = [&] {
      for (uint32_t k; (k = nexts.fetch_add(1)) < S;) {
        Shard &d = sh[k];
        for (uint32_t g = 0; g < G; g++) {
          const Graph &gr = gs[g];
          const uint32_t *off = &boff[(size_t)g * (S + 1)];
          for (uint32_t x = off[k]; x < off[k + 1]; x++) {
            const uint32_t li = bli[g][x];
            const auto r = d.intern(gr.sv(gr.labs[li]), gr.labh[li]);
            if (r.first >= (1u << SH)) {
              over.store(true, std::memory_order_relaxed);
              return;
            }
            lre[g][li] = (r.second ? NEW : 0u) | (k << SH) | r.first;
          }
        }
      }
    };
    run(phase_a);
    if (over.load()) return false;
    for (uint32_t g = 0; g < G; g++)  // first appearances in graph order
      for (uint32_t &x : lre[g])
        if (x & NEW) {
          x &= ~NEW;
          Shard &d = sh[x >> SH];
          const uint32_t si = x & ((1u << SH) - 1u);
          if (count >= 0xFFFFFFFFull || d.key.size() >= (1u << SH)) return false;
          d.gid[si] = (uint32_t)count++;
          d.key[si] = add(d.key[si]);
        }
    std::atomic<uint32_t> nextg{0};
    auto phase_c = [&] {
      for (uint32_t g; (g = nextg.fetch_add(1)) < G;)
        for (uint32_t &x : lre[g]) x = sh[x >> SH].gid[x & ((1u << SH) - 1u)];
    };
    run(phase_c);
    return true;
  }
};

// Molly's node IDs are "goal<n>" / "rule<n>" with n decimal.  When every ID
// of a kind in a graph has that shape, n is below a bound and no two of them
// share n, the ID -> node map of that kind is an array indexed by n; an entry
// keeps the digit count too, so that "goal07" does not find "goal7".  Anything
// else takes the hash maps (the results are the same).
struct NumMap {
  std::vector<uint32_t> v;     // n -> node | digits << 28 (~0u: none)
  std::vector<uint32_t> used;  // the n set for this graph (cleared after it)
  uint32_t nd0 = 0, nmax = 0;  // the first ID's digit count, the largest n
  bool uniform = true;         // every ID has nd0 digits: n order is the IDs' string order
  void clear() {
    for (uint32_t n : used) v[n] = ~0u;
    used.clear();
    nd0 = nmax = 0;
    uniform = true;
  }
};
// n and digit count of "<pfx><digits>" (4-byte prefix, 1..9 digits)
inline bool id_num(std::string_view s, const char *pfx, uint32_t &n, uint32_t &nd) {
  if (s.size() < 5 || s.size() > 13 || memcmp(s.data(), pfx, 4)) return false;
  if (s.size() == 12) {  // eight digits (zero-padded IDs) at once: all in '0'..'9', then combined in pairs
    uint64_t v;
    memcpy(&v, s.data() + 4, 8);
    if ((v & 0xF0F0F0F0F0F0F0F0ull) != 0x3030303030303030ull ||
        ((v + 0x0606060606060606ull) & 0xF0F0F0F0F0F0F0F0ull) != 0x3030303030303030ull)
      return false;
    v &= 0x0F0F0F0F0F0F0F0Full;
    v = (v * 2561) >> 8;
    v = ((v & 0x00FF00FF00FF00FFull) * 6553601) >> 16;
    v = ((v & 0x0000FFFF0000FFFFull) * 42949672960001ull) >> 32;
    n = (uint32_t)v;
    nd = 8;
    return true;
  }
  uint32_t x = 0;
  for (size_t i = 4; i < s.size(); i++) {
    const uint32_t d = (uint32_t)(unsigned char)s[i] - '0';
    if (d > 9) return false;
    x = x * 10 + d;
  }
  n = x;
  nd = (uint32_t)s.size() - 4;
  return true;
}

// per-thread maps and lists of parse_graph, reused from graph to graph
struct ParseMaps {
  std::vector<Rec> goals, rules;
  std::vector<std::pair<Str, Str>> edges;
  NumMap gnum, rnum;
  FlatMap gidx, ridx, tabs, labs;
  FlatSet64 seen;
  std::vector<std::pair<uint64_t, uint32_t>> keys;
};
thread_local ParseMaps t_maps;

// ---- a schema-directed JSON reader (encoding/json semantics for the fields used) ----
struct Json {
  const char *p, *e;
  bool ok = true;
  int depth = 0;  // nesting of skip(): untrusted input cannot grow the ingest thread's stack unboundedly
  static constexpr int kMaxDepth = 512;
  std::vector<char> key;  // scratch for object keys (capacity reused)

  __attribute__((always_inline)) void ws() {
    if (p < e && (unsigned char)*p > ' ') return;  // the common case: no white space
    if (e - p >= 2 && *p == ' ' && (unsigned char)p[1] > ' ') {  // one space (json.dump's separators)
      p++;
      return;
    }
    while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) p++;
  }
  __attribute__((always_inline)) bool lit(const char *s) {
    if (p >= e || *p != *s) return false;
    const size_t n = strlen(s);
    if ((size_t)(e - p) >= n && !memcmp(p, s, n)) {
      p += n;
      return true;
    }
    return false;
  }
  static int hex(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }
  static void utf8(std::vector<char> &o, uint32_t cp) {
    if (cp < 0x80) {
      o.push_back((char)cp);
    } else if (cp < 0x800) {
      o.push_back((char)(0xC0 | (cp >> 6)));
      o.push_back((char)(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      o.push_back((char)(0xE0 | (cp >> 12)));
      o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      o.push_back((char)(0x80 | (cp & 0x3F)));
    } else {
      o.push_back((char)(0xF0 | (cp >> 18)));
      o.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
      o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      o.push_back((char)(0x80 | (cp & 0x3F)));
    }
  }
  uint32_t u4() {
    if (e - p < 4) return ok = false, 0;
    uint32_t v = 0;
    for (int i = 0; i < 4; i++) {
      int h = hex(p[i]);
      if (h < 0) return ok = false, 0;
      v = v * 16 + h;
    }
    p += 4;
    return v;
  }
  // the first '"' or '\\' at or after q (e if none), 16 bytes at a time
  __attribute__((always_inline)) const char *scan(const char *q) const {
    const __m128i quote = _mm_set1_epi8('"'), bslash = _mm_set1_epi8('\\');
    while (e - q >= 16) {
      const __m128i x = _mm_loadu_si128((const __m128i *)q);
      const int m = _mm_movemask_epi8(_mm_or_si128(_mm_cmpeq_epi8(x, quote), _mm_cmpeq_epi8(x, bslash)));
      if (m) return q + __builtin_ctz((unsigned)m);
      q += 16;
    }
    while (q < e && *q != '"' && *q != '\\') q++;
    return q;
  }
  // a string as a view: in place when it has no escapes (offset from base, the
  // buffer the reader walks), else decoded and appended to `o` (offset bias + its place in o)
  __attribute__((always_inline)) bool sview(std::vector<char> &o, const char *base, uint32_t bias, Str &out) {
    ws();
    if (p >= e || *p != '"') return ok = false;
    const char *q = scan(p + 1);
    if (q < e && *q == '"') {
      out = Str{(uint32_t)(p + 1 - base), (uint32_t)(q - p - 1)};
      p = q + 1;
      return true;
    }
    const size_t o0 = o.size();
    if (!str(o)) return false;
    out = Str{(uint32_t)(bias + o0), (uint32_t)(o.size() - o0)};
    return true;
  }
  // string into `o` (appended); returns false on error
  bool str(std::vector<char> &o) {
    ws();
    if (p >= e || *p != '"') return ok = false;
    p++;
    while (p < e) {
      const char *q = scan(p);
      o.insert(o.end(), p, q);
      p = q;
      if (p >= e) break;
      if (*p == '"') {
        p++;
        return true;
      }
      p++;  // backslash
      if (p >= e) break;
      char c = *p++;
      switch (c) {
        case '"': o.push_back('"'); break;
        case '\\': o.push_back('\\'); break;
        case '/': o.push_back('/'); break;
        case 'b': o.push_back('\b'); break;
        case 'f': o.push_back('\f'); break;
        case 'n': o.push_back('\n'); break;
        case 'r': o.push_back('\r'); break;
        case 't': o.push_back('\t'); break;
        case 'u': {
          uint32_t cp = u4();
          if (cp >= 0xD800 && cp < 0xDC00 && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
            const char *save = p;
            p += 2;
            uint32_t lo = u4();
            if (lo >= 0xDC00 && lo < 0xE000) cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            else p = save, cp = 0xFFFD;
          } else if (cp >= 0xD800 && cp < 0xE000) {
            cp = 0xFFFD;  // lone surrogate: encoding/json substitutes U+FFFD
          }
          utf8(o, cp);
          break;
        }
        default: return ok = false;
      }
    }
    return ok = false;
  }
  void skip() {
    ws();
    if (p >= e) {
      ok = false;
      return;
    }
    char c = *p;
    if (c == '"') {
      std::vector<char> tmp;
      str(tmp);
    } else if (c == '{' || c == '[') {
      if (depth >= kMaxDepth) {
        ok = false;
        return;
      }
      struct Nest {
        int &d;
        explicit Nest(int &x) : d(x) { d++; }
        ~Nest() { d--; }
      } nest(depth);
      char close = c == '{' ? '}' : ']';
      p++;
      ws();
      if (p < e && *p == close) {
        p++;
        return;
      }
      while (ok) {
        if (c == '{') {
          std::vector<char> k;
          if (!str(k)) return;
          ws();
          if (p >= e || *p != ':') {
            ok = false;
            return;
          }
          p++;
        }
        skip();
        ws();
        if (p < e && *p == ',') {
          p++;
          continue;
        }
        if (p < e && *p == close) {
          p++;
          return;
        }
        ok = false;
      }
    } else if (lit("true") || lit("false") || lit("null")) {
    } else {
      const char *q = p;
      auto numch = [](char x) { return (x >= '0' && x <= '9') || x == '+' || x == '-' || x == '.' || x == 'e' || x == 'E'; };
      while (p < e && numch(*p)) p++;
      if (p == q) ok = false;
    }
  }
};

// ", <digits>, __WILDCARD__)" and ", <digits>, <digits>)" (molly.go:74-89):
// the leftmost match's group 1 as [*d0, *d0 + *dn) of s
bool clock_time(std::string_view s, bool wild, size_t *d0, size_t *dn) {
  for (size_t i = 0; i + 2 <= s.size(); i++) {
    if (s[i] != ',' || s[i + 1] != ' ') continue;
    size_t j = i + 2, a = j;
    while (j < s.size() && isdigit((unsigned char)s[j])) j++;
    if (j == a || j + 2 > s.size() || s[j] != ',' || s[j + 1] != ' ') continue;
    size_t k = j + 2;
    if (wild) {
      if (s.substr(k, 13) != "__WILDCARD__)") continue;
    } else {
      size_t k0 = k;
      while (k < s.size() && isdigit((unsigned char)s[k])) k++;
      if (k == k0 || k >= s.size() || s[k] != ')') continue;
    }
    *d0 = a, *dn = j - a;
    return true;
  }
  return false;
}

uint8_t type_class(std::string_view t) {
  return t == "next" ? NEMO_TYPE_NEXT : t == "async" ? NEMO_TYPE_ASYNC : NEMO_TYPE_OTHER;
}

// a key's bytes and closing quote as a little-endian word (the in-place key match of parse_graph)
#define KEY3(a, b) ((uint64_t)(a) | (uint64_t)(b) << 8 | (uint64_t)'"' << 16)
#define KEY5(a, b, c, d) \
  ((uint64_t)(a) | (uint64_t)(b) << 8 | (uint64_t)(c) << 16 | (uint64_t)(d) << 24 | (uint64_t)'"' << 32)
#define KEY6(a, b, c, d, e)                                                                              \
  ((uint64_t)(a) | (uint64_t)(b) << 8 | (uint64_t)(c) << 16 | (uint64_t)(d) << 24 | (uint64_t)(e) << 32 | \
   (uint64_t)'"' << 40)

// key k (a view into the arena) equals the lower-case keyword s, case-insensitively
// (encoding/json matches keys case-insensitively): the exact spelling first
inline bool keyis(std::string_view k, const char *s, size_t n) {
  if (k.size() != n) return false;
  if (!memcmp(k.data(), s, n)) return true;
  for (size_t i = 0; i < n; i++)
    if (tolower((unsigned char)k[i]) != s[i]) return false;
  return true;
}

// the keys of goals (0), rules (1) and edges (2) in the order Molly and json.dump
// write them, as the in-place match's (mask, word, advance)
constexpr uint64_t kPredM[3][4] = {{0xFFFFFFull, 0xFFFFFFFFFFFFull, 0xFFFFFFFFFFFFull, 0xFFFFFFFFFFull},
                                   {0xFFFFFFull, 0xFFFFFFFFFFFFull, 0xFFFFFFFFFFFFull, 0xFFFFFFFFFFull},
                                   {0xFFFFFFFFFFull, 0xFFFFFFull, 0, 0}};
constexpr uint64_t kPredK[3][4] = {
    {KEY3('i', 'd'), KEY6('l', 'a', 'b', 'e', 'l'), KEY6('t', 'a', 'b', 'l', 'e'), KEY5('t', 'i', 'm', 'e')},
    {KEY3('i', 'd'), KEY6('l', 'a', 'b', 'e', 'l'), KEY6('t', 'a', 'b', 'l', 'e'), KEY5('t', 'y', 'p', 'e')},
    {KEY5('f', 'r', 'o', 'm'), KEY3('t', 'o'), 1, 1}};
constexpr uint32_t kPredA[3][4] = {{4, 7, 7, 6}, {4, 7, 7, 6}, {6, 4, 0, 0}};

void parse_graph(const std::string &path, uint32_t iteration, const char *cond, Graph &g) {
  // the file is mapped: strings without escapes are views of it, decoded ones
  // and clock times go to the arena (reserved: no reallocation, the maps hold views)
  if (!g.file.open(path.c_str()) || g.file.n >= 0xF0000000u) {
    g.err = "Failed reading " + std::string(cond == std::string("pre") ? "antecedent" : "consequent") +
            " provenance of file '" + path + "'";
    return;
  }
  const size_t fsz = g.file.n;
  if (fsz) g.fb = (const char *)g.file.p;
  g.flen = (uint32_t)fsz;
  g.arena.reserve(2 * fsz + 64);
  const char *base = g.fb;
  const uint32_t bias = g.flen;
  Json j{base, base + fsz};
  ParseMaps &M = t_maps;
  std::vector<Rec> &goals = M.goals, &rules = M.rules;
  std::vector<std::pair<Str, Str>> &edges = M.edges;
  goals.clear(), rules.clear(), edges.clear();
  j.ws();
  if (j.lit("null")) {
  } else if (j.p < j.e && *j.p == '{') {
    j.p++;
    j.ws();
    if (j.p < j.e && *j.p == '}') j.p++;
    else
      while (j.ok) {
        Str ks;
        if (!j.sview(g.arena, base, bias, ks)) break;
        const std::string_view key = g.sv(ks);
        j.ws();
        if (j.p >= j.e || *j.p != ':') {
          j.ok = false;
          break;
        }
        j.p++;
        const int which = keyis(key, "goals", 5) ? 0 : keyis(key, "rules", 5) ? 1 : keyis(key, "edges", 5) ? 2 : -1;
        j.ws();
        if (which < 0 || j.lit("null")) {
          if (which < 0) j.skip();
        } else if (j.p < j.e && *j.p == '[') {
          j.p++;
          j.ws();
          if (j.p < j.e && *j.p == ']') j.p++;
          else
            while (j.ok) {
              j.ws();
              if (j.p >= j.e || *j.p != '{') {
                j.ok = false;
                break;
              }
              j.p++;
              Rec r{};
              std::pair<Str, Str> ed{};
              int nf = 0;  // the field expected next
              j.ws();
              if (j.p < j.e && *j.p == '}') j.p++;
              else
                while (j.ok) {
                  int f = -1;
                  j.ws();  // after ", " (json.dump's separators)
                  // the exact lower-case keys, matched in place (the closing quote included)
                  if (j.e - j.p >= 9 && *j.p == '"') {
                    const uint64_t w = load8(j.p + 1);
                    uint32_t adv = 0;
                    if (nf < (which == 2 ? 2 : 4) && (w & kPredM[which][nf]) == kPredK[which][nf]) {
                      f = nf, adv = kPredA[which][nf];  // the field after the last one (the writers' order)
                    } else if (which == 2) {
                      if ((w & 0xFFFFFFFFFFull) == KEY5('f', 'r', 'o', 'm')) f = 0, adv = 6;
                      else if ((w & 0xFFFFFFull) == KEY3('t', 'o')) f = 1, adv = 4;
                    } else if ((w & 0xFFFFFFull) == KEY3('i', 'd')) {
                      f = 0, adv = 4;
                    } else if ((w & 0xFFFFFFFFFFFFull) == KEY6('l', 'a', 'b', 'e', 'l')) {
                      f = 1, adv = 7;
                    } else if ((w & 0xFFFFFFFFFFFFull) == KEY6('t', 'a', 'b', 'l', 'e')) {
                      f = 2, adv = 7;
                    } else if ((w & 0xFFFFFFFFFFull) ==
                               (which == 0 ? KEY5('t', 'i', 'm', 'e') : KEY5('t', 'y', 'p', 'e'))) {
                      f = 3, adv = 6;
                    }
                    j.p += adv;
                  }
                  if (f < 0) {  // any other spelling or key (encoding/json matches keys case-insensitively)
                    Str kst;
                    if (!j.sview(g.arena, base, bias, kst)) break;
                    const std::string_view k = g.sv(kst);
                    if (which == 2) {
                      f = keyis(k, "from", 4) ? 0 : keyis(k, "to", 2) ? 1 : -1;
                    } else {
                      if (keyis(k, "id", 2)) f = 0;
                      else if (keyis(k, "label", 5)) f = 1;
                      else if (keyis(k, "table", 5)) f = 2;
                      else if (keyis(k, which == 0 ? "time" : "type", 4)) f = 3;
                    }
                  }
                  j.ws();
                  if (j.p >= j.e || *j.p != ':') {
                    j.ok = false;
                    break;
                  }
                  j.p++;
                  j.ws();
                  if (f < 0) {
                    j.skip();
                  } else if (j.lit("null")) {
                  } else {
                    Str sv;
                    if (!j.sview(g.arena, base, bias, sv)) break;
                    if (which == 2) (f == 0 ? ed.first : ed.second) = sv;
                    else r.f[f] = sv;
                  }
                  nf = f + 1;
                  j.ws();
                  if (j.p < j.e && *j.p == ',') {
                    j.p++;
                    continue;
                  }
                  if (j.p < j.e && *j.p == '}') {
                    j.p++;
                    break;
                  }
                  j.ok = false;
                }
              if (which == 0) goals.push_back(r);
              else if (which == 1) rules.push_back(r);
              else edges.push_back(ed);
              j.ws();
              if (j.p < j.e && *j.p == ',') {
                j.p++;
                continue;
              }
              if (j.p < j.e && *j.p == ']') {
                j.p++;
                break;
              }
              j.ok = false;
            }
        } else {
          j.ok = false;
        }
        j.ws();
        if (j.p < j.e && *j.p == ',') {
          j.p++;
          continue;
        }
        if (j.p < j.e && *j.p == '}') {
          j.p++;
          break;
        }
        j.ok = false;
      }
  } else {
    j.ok = false;
  }
  j.ws();
  if (!j.ok || j.p != j.e) {
    g.err = std::string("Failed to unmarshal JSON ") + (cond == std::string("pre") ? "antecedent" : "consequent") +
            " provenance data: " + path;
    return;
  }
  const size_t V = goals.size() + rules.size();
  if (V >= (1u << 28)) {  // the per-graph maps pack node indices in 28 bits (NumMap, FlatSet64)
    g.err = std::string("Too many nodes (") + std::to_string(V) + ") in " +
            (cond == std::string("pre") ? "antecedent" : "consequent") + " provenance: " + path;
    return;
  }
  g.n_goals = (uint32_t)goals.size();
  // sized once and written by index (a push_back per field and node was a
  // capacity check each)
  g.id.resize(V), g.tt.resize(V);
  g.ltab.resize(V), g.llab.resize(V), g.tclass.resize(V);
  FlatMap &gidx = M.gidx, &ridx = M.ridx, &tabs = M.tabs, &labs = M.labs;
  gidx.init(goals.size()), ridx.init(rules.size()), tabs.init(64), labs.init(V);
  auto intern = [&](FlatMap &m, std::vector<Str> &order, Str s) {
    if (order.size() * 2 + 16 > m.mask) {  // grow: rehash the distinct keys seen so far
      m.init(order.size() * 2 + 16);
      for (uint32_t i = 0; i < order.size(); i++) m.emplace(g.sv(order[i]), i);
    }
    auto it = m.emplace(g.sv(s), (uint32_t)order.size());
    if (it.second) order.push_back(s);
    return it.first;
  };
  // tables repeat in runs (a relation's facts and rules come together): the last one is checked first
  std::string_view last_tab;
  uint32_t last_tid = ~0u;
  auto intern_table = [&](Str s) {
    const std::string_view k = g.sv(s);
    if (last_tid != ~0u && sveq(k, last_tab)) return last_tid;
    last_tab = k;
    return last_tid = intern(tabs, g.tabs, s);
  };
  g.labh.reserve(V);
  auto intern_label = [&](Str s) {  // the same, keeping each distinct label's hash
    if (g.labs.size() * 2 + 16 > labs.mask) {
      labs.init(g.labs.size() * 2 + 16);
      for (uint32_t i = 0; i < g.labs.size(); i++) labs.emplace_h(g.sv(g.labs[i]), g.labh[i], i);
    }
    const std::string_view k = g.sv(s);
    const uint64_t h = hash_sv(k);
    auto it = labs.emplace_h(k, h, (uint32_t)g.labs.size());
    if (it.second) {
      g.labs.push_back(s);
      g.labh.push_back(h);
    }
    return it.first;
  };
  // the ID -> node maps, numeric when the IDs allow (NumMap), else hashed; a
  // duplicate ID is the reference's uniqueness error (pre-post-prov.go:68, :129)
  const uint32_t nbound = (uint32_t)std::min<size_t>(4 * V + 4096, 1u << 27);
  auto build_ids = [&](const std::vector<Rec> &recs, uint32_t base, const char *pfx, NumMap &nm, FlatMap &hm,
                       const char *what, const char *cons) -> int {  // 1 numeric, 0 hashed, -1 duplicate
    bool num = true;
    if (nm.v.size() < nbound) nm.v.resize(nbound, ~0u);
    for (uint32_t k = 0; k < recs.size() && num; k++) {
      uint32_t n, nd;
      if (!id_num(g.sv(recs[k].f[0]), pfx, n, nd) || n >= nbound) {
        num = false;
      } else if (nm.v[n] == ~0u) {
        nm.v[n] = (base + k) | (nd << 28);
        if (nm.used.empty()) nm.nd0 = nd;
        nm.uniform &= nd == nm.nd0;
        nm.nmax = std::max(nm.nmax, n);
        nm.used.push_back(n);
      } else if ((nm.v[n] >> 28) != nd) {
        num = false;  // "goal7" and "goal07": the hash map tells them apart
      } else {
        g.err = "Run " + std::to_string(iteration) + ": duplicate " + what + " id run_" + std::to_string(iteration) +
                "_" + cond + "_" + std::string(g.sv(recs[k].f[0])) + " (" + cons + ")";
        return -1;
      }
    }
    if (num) return 1;
    nm.clear();
    for (uint32_t k = 0; k < recs.size(); k++)
      if (!hm.emplace(g.sv(recs[k].f[0]), base + k).second) {
        g.err = "Run " + std::to_string(iteration) + ": duplicate " + what + " id run_" + std::to_string(iteration) +
                "_" + cond + "_" + std::string(g.sv(recs[k].f[0])) + " (" + cons + ")";
        return -1;
      }
    return 0;
  };
  const int gnumk = build_ids(goals, 0, "goal", M.gnum, gidx, "goal", "Goal.id IS UNIQUE, pre-post-prov.go:68");
  if (gnumk < 0) {
    M.gnum.clear();
    return;
  }
  const int rnumk = build_ids(rules, (uint32_t)goals.size(), "rule", M.rnum, ridx, "rule",
                              "Rule.id IS UNIQUE, pre-post-prov.go:129");
  if (rnumk < 0) {
    M.gnum.clear(), M.rnum.clear();
    return;
  }
  for (uint32_t i = 0; i < goals.size(); i++) {
    const Rec &r = goals[i];
    Str t = r.f[3];
    if (g.sv(r.f[2]) == "clock") {  // molly.go:74-89: the two-number match wins over the wildcard one
      // the time is a substring of the label: a view at the label's offset
      // (a label is contiguous in the file or in the arena)
      const std::string_view lab = g.sv(r.f[1]);
      size_t d0, dn;
      if (clock_time(lab, false, &d0, &dn) || clock_time(lab, true, &d0, &dn))
        t = Str{r.f[1].off + (uint32_t)d0, (uint32_t)dn};
    }
    g.id[i] = r.f[0], g.tt[i] = t;
    g.ltab[i] = intern_table(r.f[2]);
    g.llab[i] = intern_label(r.f[1]);
    g.tclass[i] = 0;
  }
  for (uint32_t k = 0; k < rules.size(); k++) {
    const Rec &r = rules[k];
    const size_t i = goals.size() + k;
    g.id[i] = r.f[0], g.tt[i] = r.f[3];
    g.ltab[i] = intern_table(r.f[2]);
    g.llab[i] = intern_label(r.f[1]);
    g.tclass[i] = type_class(g.sv(r.f[3]));
  }
  if (gnumk == 1 && rnumk == 1 && M.gnum.uniform && M.rnum.uniform) {
    // "goal<n>" / "rule<n>" with one digit count per kind: string order is
    // every goal ("g" < "r"), then every rule, each by n -- the arrays in order
    g.rank.assign(V, 0);
    uint32_t pos = 0;
    for (const NumMap *nm : {&M.gnum, &M.rnum})
      for (uint32_t n = 0; n <= nm->nmax && !nm->used.empty(); n++)
        if (nm->v[n] != ~0u) g.rank[nm->v[n] & ((1u << 28) - 1u)] = pos++;
  } else {
  // rank of each node's ID inside the graph (the prefix is common, so unprefixed order == prefixed order)
  // sorted by 8-byte big-endian keys taken at offset 0 (a shorter ID pads with
  // zero bytes, so the key order agrees with the string order); a run of equal
  // keys is sorted again by the next 8 bytes, and so on
  std::vector<std::pair<uint64_t, uint32_t>> &order = M.keys;
  order.resize(V);
  auto key_at = [&](uint32_t i, size_t o) {
    const std::string_view x = g.sv(g.id[i]);
    if (x.size() >= o + 8) return __builtin_bswap64(load8(x.data() + o));
    uint64_t k = 0;
    for (size_t b = o; b < x.size(); b++) k |= (uint64_t)(uint8_t)x[b] << (56 - 8 * (b - o));
    return k;
  };
  auto by_key = [](const std::pair<uint64_t, uint32_t> &a, const std::pair<uint64_t, uint32_t> &b) {
    return a.first != b.first ? a.first < b.first : a.second < b.second;
  };
  for (uint32_t i = 0; i < V; i++) order[i] = {key_at(i, 0), i};
  std::sort(order.begin(), order.end(), by_key);
  // runs of equal keys: (begin, end, offset of the next key)
  std::vector<std::array<uint32_t, 3>> runs;
  for (uint32_t i = 0; i < V;) {
    uint32_t j = i + 1;
    while (j < V && order[j].first == order[i].first) j++;
    if (j - i > 1) runs.push_back({i, j, 8});
    i = j;
  }
  while (!runs.empty()) {
    const auto r = runs.back();
    runs.pop_back();
    bool longer = false;  // some ID of the run goes past the keys read so far
    for (uint32_t i = r[0]; i < r[1]; i++) {
      longer |= g.id[order[i].second].len > r[2];
      order[i].first = key_at(order[i].second, r[2]);
    }
    if (!longer) {  // keys equal to the end: IDs that differ only by embedded NUL bytes
      std::sort(order.begin() + r[0], order.begin() + r[1],
                [&](const std::pair<uint64_t, uint32_t> &x, const std::pair<uint64_t, uint32_t> &y) {
                  return g.sv(g.id[x.second]) < g.sv(g.id[y.second]);
                });
      continue;
    }
    std::sort(order.begin() + r[0], order.begin() + r[1], by_key);
    for (uint32_t i = r[0]; i < r[1];) {
      uint32_t j = i + 1;
      while (j < r[1] && order[j].first == order[i].first) j++;
      if (j - i > 1) runs.push_back({i, j, r[2] + 8});
      i = j;
    }
  }
  g.rank.assign(V, 0);
  for (uint32_t pos = 0; pos < V; pos++) g.rank[order[pos].second] = pos;
  }
  FlatSet64 &seen = M.seen;
  seen.init(edges.size());
  size_t created = 0;
  g.src.reserve(edges.size()), g.dst.reserve(edges.size());
  auto find_id = [&](std::string_view x, bool goal) -> uint32_t {
    if ((goal ? gnumk : rnumk) == 0) return (goal ? gidx : ridx).find(x);
    const NumMap &nm = goal ? M.gnum : M.rnum;
    uint32_t n, nd;
    // every ID of the kind has the numeric shape: another string is none of them
    if (!id_num(x, goal ? "goal" : "rule", n, nd) || n >= nbound) return ~0u;
    const uint32_t e = nm.v[n];
    return e != ~0u && (e >> 28) == nd ? (e & ((1u << 28) - 1u)) : ~0u;
  };
  for (auto &ed : edges) {
    std::string_view f = g.sv(ed.first), t = g.sv(ed.second);
    uint32_t u, v;
    // strings.Contains(From, "goal") (pre-post-prov.go:173); "rule<digits>" holds no "goal"
    bool from_goal;
    if (f.size() >= 4 && !memcmp(f.data(), "goal", 4)) {
      from_goal = true;
    } else if (f.size() >= 4 && !memcmp(f.data(), "rule", 4)) {
      size_t i = 4;
      while (i < f.size() && (uint32_t)(unsigned char)f[i] - '0' <= 9u) i++;
      from_goal = i < f.size() && f.find("goal", 4) != std::string_view::npos;
    } else {
      from_goal = f.find("goal") != std::string_view::npos;
    }
    if (from_goal) {
      u = find_id(f, true), v = find_id(t, false);
    } else {
      u = find_id(f, false), v = find_id(t, true);
    }
    if (u == ~0u || v == ~0u || !seen.insert(((uint64_t)u << 32) | v)) continue;
    g.src.push_back(u), g.dst.push_back(v);
    created++;
  }
  M.gnum.clear(), M.rnum.clear();
  if (created != edges.size())
    g.err = "Run " + std::to_string(iteration) + ": inserted number of edges (" + std::to_string(created) +
            ") does not equal number of antecedent provenance edges (" + std::to_string(edges.size()) + ")";
}

}  // namespace

struct nemo_ingest {
  std::vector<Graph> graphs;  // 2r = pre, 2r+1 = post
  std::vector<uint32_t> iteration;
  std::vector<uint64_t> node_off, edge_off;
  RawBuf<uint32_t> word, label, rank, src, dst;
  std::vector<std::string> tables, labels;
  uint32_t table_pre = 0, table_post = 0;
};

extern "C" int nemo_ingest_molly(const char *out_dir, const uint32_t *iterations, uint32_t n_runs, int threads,
                                 nemo_ingest **out, char *err, size_t err_cap) {
  auto fail = [&](const std::string &m) {
    if (err && err_cap) snprintf(err, err_cap, "%s", m.c_str());
    return NEMO_ERR_LOAD;
  };
  if (!out_dir || !out || (n_runs && !iterations)) return NEMO_ERR_INVALID;
  // the calling thread parses too: its per-thread maps (up to ~4V + 4096 words per kind)
  // are released on the way out, as the helper threads' are when they exit
  struct ReleaseMaps {
    ~ReleaseMaps() { t_maps = ParseMaps(); }
  } release_maps;
  auto *h = new nemo_ingest();
  h->iteration.assign(iterations, iterations + n_runs);
  const uint32_t G = 2 * n_runs;
  h->graphs.resize(G);
  int nt = threads > 0 ? threads : (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  nt = std::max(1, std::min<int>(nt, (int)std::max<uint32_t>(G, 1)));
  std::atomic<uint32_t> next{0};
  auto work = [&] {
    for (uint32_t g; (g = next.fetch_add(1)) < G;) {
      const uint32_t r = g / 2;
      const char *cond = g % 2 ? "post" : "pre";
      // file name by index, ID prefix by iteration (molly.go:59-60 vs :92)
      std::string path = std::string(out_dir) + "/run_" + std::to_string(r) + "_" + cond + "_provenance.json";
      parse_graph(path, h->iteration[r], cond, h->graphs[g]);
    }
  };
  const Runner run = make_runner(nullptr, nt);
  run(work);
  for (uint32_t g = 0; g < G; g++)
    if (!h->graphs[g].err.empty()) {
      std::string m = h->graphs[g].err;
      delete h;
      return fail(m);
    }
  // global interning in graph order (== the sequential first-appearance order)
  // (keys view the graphs' arenas, alive until the ingest is freed)
  InternMap tmap;
  ShardIntern lmap;
  std::vector<std::vector<uint32_t>> tre(G), lre(G);
  h->node_off.assign(G + 1, 0);
  h->edge_off.assign(G + 1, 0);
  auto add = [](std::vector<std::string> &names) {
    return [&names](std::string_view k) {
      names.emplace_back(k);
      return std::pair<uint32_t, std::string_view>((uint32_t)names.size() - 1, k);
    };
  };
  for (uint32_t g = 0; g < G; g++) {
    Graph &gr = h->graphs[g];
    tre[g].reserve(gr.tabs.size());
    lre[g].reserve(gr.labs.size());
    for (Str s : gr.tabs) tre[g].push_back(tmap.intern(gr.sv(s), add(h->tables)));
    h->node_off[g + 1] = h->node_off[g] + gr.id.size();
    h->edge_off[g + 1] = h->edge_off[g] + gr.src.size();
  }
  if (!lmap.merge(h->graphs, G, nt, run, lre, [&](std::string_view k) {
        h->labels.emplace_back(k);
        return k;  // the arenas live as long as the ingest
      })) {
    delete h;
    return fail("too many distinct labels");
  }
  static const char *kPrePost[2] = {"pre", "post"};
  for (int k = 0; k < 2; k++)
    (k == 0 ? h->table_pre : h->table_post) = tmap.intern(kPrePost[k], add(h->tables));
  if (h->tables.size() > NEMO_MAX_TABLES) {
    delete h;
    return fail("more than NEMO_MAX_TABLES distinct tables");
  }
  const uint64_t V = h->node_off[G], E = h->edge_off[G];
  h->word.resize(V), h->label.resize(V), h->rank.resize(V), h->src.resize(E), h->dst.resize(E);
  next = 0;
  auto fill = [&] {
    for (uint32_t g; (g = next.fetch_add(1)) < G;) {
      const Graph &gr = h->graphs[g];
      const uint64_t n0 = h->node_off[g], e0 = h->edge_off[g];
      for (size_t i = 0; i < gr.id.size(); i++) {
        h->word[n0 + i] = NEMO_WORD(i >= gr.n_goals, gr.tclass[i], tre[g][gr.ltab[i]]);
        h->label[n0 + i] = lre[g][gr.llab[i]];
        h->rank[n0 + i] = gr.rank[i];
      }
      std::copy(gr.src.begin(), gr.src.end(), h->src.begin() + e0);
      std::copy(gr.dst.begin(), gr.dst.end(), h->dst.begin() + e0);
    }
  };
  run(fill);
  *out = h;
  return NEMO_OK;
}

// ---- streaming ingest: chunk i is analysed on the device
// while chunk i+1 is being parsed.  Interning is shared across chunks (ids are
// assigned in parse order), so the chunks' label and table ids agree with
// each other; the run of iteration 0
// is replicated, not owned, into every chunk after the one holding it.
struct nemo_ingest_stream {
  std::string dir;
  std::vector<uint32_t> iteration;
  std::vector<uint32_t> order;  // parse order: run 0, failedRuns[0], then runs.json order
  int threads = 1;
  uint32_t next = 0;  // next position in `order`
  InternMap tmap;        // keys view the strings of tables / labels (a deque: no relocation)
  ShardIntern lmap;
  std::deque<std::string> tables, labels;
  uint32_t table_pre = 0, table_post = 0;
  bool pre_post = false;
  int64_t run0 = -1;  // position of iteration 0 in `order` (0, or -1: absent)
  bool have_run0 = false;
  uint64_t r0_nv[2] = {0, 0}, r0_ne[2] = {0, 0};
  std::vector<uint32_t> r0_word, r0_label, r0_rank, r0_src, r0_dst;
  std::vector<Graph> gpool;                       // the chunks' graphs, reused (Graph::reset)
  std::unique_ptr<WorkerPool> workers;            // the parse / merge / fill threads, kept across chunks
  std::vector<std::vector<uint32_t>> tre, lre;    // their table / label ids
  // the chunks' arrays, double-buffered: chunk i stays valid while chunk i+1 is parsed
  struct Chunk {
    std::vector<uint32_t> it;
    RawBuf<uint32_t> word, label, rank, src, dst;
    std::vector<uint8_t> own;
    std::vector<uint64_t> node_off, edge_off;
  } buf[2];
  uint32_t calls = 0;
};

extern "C" int nemo_ingest_open(const char *out_dir, const uint32_t *iterations, uint32_t n_runs,
                                int64_t first_failed, int threads, nemo_ingest_stream **out) {
  if (!out_dir || !out || (n_runs && !iterations) || first_failed >= (int64_t)n_runs) return NEMO_ERR_INVALID;
  auto *s = new nemo_ingest_stream();
  s->dir = out_dir;
  s->iteration.assign(iterations, iterations + n_runs);
  s->threads = threads > 0 ? threads : (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  // run 0 is the good run of every diff (differential-provenance.go:26) and
  // failedRuns[0] the label source of every reference-mode diff (:22-43): both
  // are parsed first, so the first chunk holds them and every chunk that holds
  // a failed run also holds the good run
  int64_t r0 = -1;
  for (uint32_t r = 0; r < n_runs && r0 < 0; r++)
    if (iterations[r] == 0) r0 = r;
  if (r0 >= 0) {
    s->order.push_back((uint32_t)r0);
    s->run0 = 0;
  }
  if (first_failed >= 0 && first_failed != r0) s->order.push_back((uint32_t)first_failed);
  for (uint32_t r = 0; r < n_runs; r++)
    if ((int64_t)r != r0 && (int64_t)r != first_failed) s->order.push_back(r);
  *out = s;
  return NEMO_OK;
}

extern "C" int nemo_ingest_next(nemo_ingest_stream *s, uint32_t chunk, int with_run0, nemo_corpus *c, char *err,
                                size_t err_cap) {
  auto fail = [&](const std::string &m) {
    if (err && err_cap) snprintf(err, err_cap, "%s", m.c_str());
    return NEMO_ERR_LOAD;
  };
  if (!s || !c || chunk == 0) return NEMO_ERR_INVALID;
  const uint32_t R = (uint32_t)s->iteration.size();
  if (s->next >= R) return NEMO_ERR_NOTFOUND;
  const uint32_t a = s->next, b = std::min<uint32_t>(R, a + chunk), G = 2 * (b - a);
  s->next = b;
  if (s->gpool.size() < G) s->gpool.resize(G);
  std::vector<Graph> &gs = s->gpool;
  int nt = std::max(1, std::min<int>(s->threads, (int)G));
  std::atomic<uint32_t> nextg{0};
  auto work = [&] {
    for (uint32_t g; (g = nextg.fetch_add(1)) < G;) {
      const uint32_t r = s->order[a + g / 2];  // file names use the run index (molly.go:59-60)
      const char *cond = g % 2 ? "post" : "pre";
      std::string path = s->dir + "/run_" + std::to_string(r) + "_" + cond + "_provenance.json";
      gs[g].reset();
      parse_graph(path, s->iteration[r], cond, gs[g]);
    }
  };
  if (!s->workers) s->workers.reset(new WorkerPool(s->threads));
  const Runner run = make_runner(s->workers.get(), nt);
  run(work);
  for (uint32_t g = 0; g < G; g++)
    if (!gs[g].err.empty()) return fail(gs[g].err);
  if (s->tre.size() < G) s->tre.resize(G), s->lre.resize(G);
  std::vector<std::vector<uint32_t>> &tre = s->tre, &lre = s->lre;
  for (uint32_t g = 0; g < G; g++) tre[g].clear();
  auto add = [](std::deque<std::string> &names) {
    return [&names](std::string_view k) {
      names.emplace_back(k);
      return std::pair<uint32_t, std::string_view>((uint32_t)names.size() - 1, std::string_view(names.back()));
    };
  };
  for (uint32_t g = 0; g < G; g++) {
    tre[g].reserve(gs[g].tabs.size());
    for (Str x : gs[g].tabs) tre[g].push_back(s->tmap.intern(gs[g].sv(x), add(s->tables)));
  }
  if (!s->lmap.merge(gs, G, nt, run, lre, [&](std::string_view k) {
        s->labels.emplace_back(k);
        return std::string_view(s->labels.back());  // the chunk's arenas go away
      }))
    return fail("too many distinct labels");
  if (!s->pre_post) {  // fixed from the first chunk on: every chunk's corpus names the same ids
    static const char *kPrePost[2] = {"pre", "post"};
    for (int k = 0; k < 2; k++)
      (k == 0 ? s->table_pre : s->table_post) = s->tmap.intern(kPrePost[k], add(s->tables));
    s->pre_post = true;
  }
  if (s->tables.size() > NEMO_MAX_TABLES) return fail("more than NEMO_MAX_TABLES distinct tables");
  nemo_ingest_stream::Chunk &ck = s->buf[s->calls++ & 1];
  const bool rep0 = with_run0 && s->have_run0 && !(s->run0 >= a && s->run0 < b);
  const uint32_t Rc = (b - a) + (rep0 ? 1 : 0), Gc = 2 * Rc;
  ck.it.clear();
  ck.own.clear();
  ck.node_off.assign(Gc + 1, 0);
  ck.edge_off.assign(Gc + 1, 0);
  uint32_t go = 0;
  if (rep0) {
    ck.it.push_back(0);
    ck.own.push_back(0);
    for (int k = 0; k < 2; k++) {
      ck.node_off[go + 1] = ck.node_off[go] + s->r0_nv[k];
      ck.edge_off[go + 1] = ck.edge_off[go] + s->r0_ne[k];
      go++;
    }
  }
  for (uint32_t r = a; r < b; r++) {
    ck.it.push_back(s->iteration[s->order[r]]);
    ck.own.push_back(1);
    for (int k = 0; k < 2; k++) {
      const Graph &gr = gs[2 * (r - a) + k];
      ck.node_off[go + 1] = ck.node_off[go] + gr.id.size();
      ck.edge_off[go + 1] = ck.edge_off[go] + gr.src.size();
      go++;
    }
  }
  const uint64_t V = ck.node_off[Gc], E = ck.edge_off[Gc];
  ck.word.resize(V), ck.label.resize(V), ck.rank.resize(V), ck.src.resize(E), ck.dst.resize(E);
  if (rep0) {
    std::copy(s->r0_word.begin(), s->r0_word.end(), ck.word.begin());
    std::copy(s->r0_label.begin(), s->r0_label.end(), ck.label.begin());
    std::copy(s->r0_rank.begin(), s->r0_rank.end(), ck.rank.begin());
    std::copy(s->r0_src.begin(), s->r0_src.end(), ck.src.begin());
    std::copy(s->r0_dst.begin(), s->r0_dst.end(), ck.dst.begin());
  }
  const uint32_t gbase = rep0 ? 2 : 0;
  nextg = 0;
  auto fill = [&] {
    for (uint32_t g; (g = nextg.fetch_add(1)) < G;) {
      const Graph &gr = gs[g];
      const uint64_t n0 = ck.node_off[gbase + g], e0 = ck.edge_off[gbase + g];
      for (size_t i = 0; i < gr.id.size(); i++) {
        ck.word[n0 + i] = NEMO_WORD(i >= gr.n_goals, gr.tclass[i], tre[g][gr.ltab[i]]);
        ck.label[n0 + i] = lre[g][gr.llab[i]];
        ck.rank[n0 + i] = gr.rank[i];
      }
      std::copy(gr.src.begin(), gr.src.end(), ck.src.begin() + e0);
      std::copy(gr.dst.begin(), gr.dst.end(), ck.dst.begin() + e0);
    }
  };
  run(fill);
  if (s->run0 >= a && s->run0 < b) {  // keep run 0 for the chunks after this one
    const uint32_t g0 = gbase + 2 * (uint32_t)(s->run0 - a);
    const uint64_t n0 = ck.node_off[g0], n1 = ck.node_off[g0 + 2], e0 = ck.edge_off[g0], e1 = ck.edge_off[g0 + 2];
    s->r0_nv[0] = ck.node_off[g0 + 1] - n0, s->r0_nv[1] = n1 - ck.node_off[g0 + 1];
    s->r0_ne[0] = ck.edge_off[g0 + 1] - e0, s->r0_ne[1] = e1 - ck.edge_off[g0 + 1];
    s->r0_word.assign(ck.word.begin() + n0, ck.word.begin() + n1);
    s->r0_label.assign(ck.label.begin() + n0, ck.label.begin() + n1);
    s->r0_rank.assign(ck.rank.begin() + n0, ck.rank.begin() + n1);
    s->r0_src.assign(ck.src.begin() + e0, ck.src.begin() + e1);
    s->r0_dst.assign(ck.dst.begin() + e0, ck.dst.begin() + e1);
    s->have_run0 = true;
  }
  memset(c, 0, sizeof(*c));
  c->n_runs = Rc;
  c->n_tables = (uint32_t)s->tables.size();
  c->table_pre = s->table_pre;
  c->table_post = s->table_post;
  c->iteration = ck.it.data();
  c->owned = ck.own.data();
  c->node_off = ck.node_off.data();
  c->edge_off = ck.edge_off.data();
  c->node_word = ck.word.data();
  c->label = ck.label.data();
  c->id_rank = ck.rank.data();
  c->edge_src = ck.src.data();
  c->edge_dst = ck.dst.data();
  return NEMO_OK;
}

extern "C" uint64_t nemo_ingest_stream_count(const nemo_ingest_stream *s, int kind) {
  if (!s) return 0;
  return kind == NEMO_STR_TABLE ? s->tables.size() : kind == NEMO_STR_LABEL ? s->labels.size() : 0;
}

extern "C" int nemo_ingest_stream_string(const nemo_ingest_stream *s, int kind, uint64_t index, const char **str,
                                         size_t *len) {
  if (!s || !str || !len || (kind != NEMO_STR_TABLE && kind != NEMO_STR_LABEL)) return NEMO_ERR_INVALID;
  const auto &v = kind == NEMO_STR_TABLE ? s->tables : s->labels;
  if (index >= v.size()) return NEMO_ERR_INVALID;
  *str = v[index].data();
  *len = v[index].size();
  return NEMO_OK;
}

extern "C" void nemo_ingest_close(nemo_ingest_stream *s) { delete s; }

extern "C" int nemo_ingest_corpus(const nemo_ingest *h, nemo_corpus *c) {
  if (!h || !c) return NEMO_ERR_INVALID;
  memset(c, 0, sizeof(*c));
  c->n_runs = (uint32_t)h->iteration.size();
  c->n_tables = (uint32_t)h->tables.size();
  c->table_pre = h->table_pre;
  c->table_post = h->table_post;
  c->iteration = h->iteration.data();
  c->owned = nullptr;
  c->node_off = h->node_off.data();
  c->edge_off = h->edge_off.data();
  c->node_word = h->word.data();
  c->label = h->label.data();
  c->id_rank = h->rank.data();
  c->edge_src = h->src.data();
  c->edge_dst = h->dst.data();
  return NEMO_OK;
}

extern "C" uint64_t nemo_ingest_count(const nemo_ingest *h, int kind) {
  if (!h) return 0;
  if (kind == NEMO_STR_TABLE) return h->tables.size();
  if (kind == NEMO_STR_LABEL) return h->labels.size();
  return h->node_off.empty() ? 0 : h->node_off.back();
}

extern "C" int nemo_ingest_string(const nemo_ingest *h, int kind, uint64_t index, const char **s, size_t *len) {
  if (!h || !s || !len) return NEMO_ERR_INVALID;
  if (kind == NEMO_STR_TABLE || kind == NEMO_STR_LABEL) {
    const auto &v = kind == NEMO_STR_TABLE ? h->tables : h->labels;
    if (index >= v.size()) return NEMO_ERR_INVALID;
    *s = v[index].data();
    *len = v[index].size();
    return NEMO_OK;
  }
  if (h->node_off.empty() || index >= h->node_off.back()) return NEMO_ERR_INVALID;
  const uint32_t g = (uint32_t)(std::upper_bound(h->node_off.begin(), h->node_off.end(), index) - h->node_off.begin() - 1);
  const Graph &gr = h->graphs[g];
  const size_t i = index - h->node_off[g];
  const bool goal = i < gr.n_goals;
  Str st = kind == NEMO_STR_NODE_ID ? gr.id[i] : (kind == NEMO_STR_NODE_TIME) == goal ? gr.tt[i] : Str{0, 0};
  if (kind < NEMO_STR_NODE_ID || kind > NEMO_STR_NODE_TIME) return NEMO_ERR_INVALID;
  *s = gr.sv(st).data();
  *len = st.len;
  return NEMO_OK;
}

extern "C" void nemo_ingest_free(nemo_ingest *h) { delete h; }
