// node.hip — the node context: one libnemohip context per device, a corpus
// run-sharded over them, and the two cross-shard exchanges of
// the reference's analysis done in the library:
//   * prototypes: the per-shard reduction vectors [cnt[T], first[T], achvd,
//     first_nonempty, prehold, nruns] are summed with one RCCL all-reduce
//     (ncclSum: RCCL has no bitwise AND, and inter = {t : cnt[t] == achvd} is
//     the AND of prototype.go:79-109);
//   * CreateNaiveDiffProv's reference mode: every entry uses failedRuns[0]'s
//     post-goal labels (differential-provenance.go:22-43), but that run lives
//     on one shard, so its owner extracts the label set on the device and RCCL
//     broadcasts it to every shard (ncclBroadcast).
// Run 0, the good run of every diff (differential-provenance.go:26) and the
// subject of the corrections (corrections.go:210), is replicated on every
// shard and owned (counted in the reductions) by its LPT shard only.
//
// The reference caller is one Go process that constructs one Neo4J value
// (main.go:95) and calls the GraphDatabase interface serially (main.go:33-44);
// the node context keeps that contract: every entry point is synchronous for
// the caller and fans out over the shards' streams internally.  Shards on
// distinct devices reduce with RCCL (one communicator per device,
// ncclCommInitAll); shards that share a device (a test layout for one-GPU
// hosts) reduce with peer copies and a sum kernel instead, since RCCL refuses
// two ranks on one device.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "node.h"

namespace {

struct Shard {
  nemo_ctx *ctx = nullptr;
  int device = 0;
  std::vector<uint32_t> runs;  // global run index of each local run
  std::vector<uint8_t> own;    // local run is counted in the reductions
  int32_t run0_local = -1;     // local index of run 0 (owned or replica)
  uint32_t *d_lab = nullptr;   // broadcast label set [n, label...]
  uint64_t lab_cap = 0;
  std::vector<uint32_t> entries;  // global diff entry of each local entry
  // host copies of the corpus arrays handed to this shard's nemo_load_corpus
  std::vector<uint32_t> it, word, label, rank, es, ed;
  std::vector<uint64_t> no, eo;
};

// One persistent host thread per shard.  The per-shard entry points block on
// their own stream or events (a fetch waits for its kernel), so a serial loop
// over shards would serialise the devices behind those waits; the pool runs
// every shard's call at once and joins (the caller stays synchronous, as the
// reference's single goroutine expects, main.go:106-177).
class Pool {
 public:
  explicit Pool(size_t n) : slot_(n) {
    for (size_t i = 0; i < n; i++) th_.emplace_back([this, i] { loop(i); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : th_) t.join();
  }
  // run f(i) for every i on its own thread; returns when all have finished
  void run(const std::function<void(size_t)> &f) {
    std::unique_lock<std::mutex> g(m_);
    job_ = &f;
    pending_ = slot_.size();
    gen_++;
    cv_.notify_all();
    done_.wait(g, [this] { return pending_ == 0; });
    job_ = nullptr;
  }

 private:
  void loop(size_t i) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(size_t)> *f;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        f = job_;
      }
      (*f)(i);
      std::lock_guard<std::mutex> g(m_);
      if (--pending_ == 0) done_.notify_one();
    }
  }
  std::vector<char> slot_;
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<void(size_t)> *job_ = nullptr;
  size_t pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace

struct Node {
  std::vector<Shard> sh;
  Pool *pool = nullptr;  // one thread per shard (P > 1)
  bool rccl = false;
  std::vector<ncclComm_t> comms;
  // peer-copy reduction (shards sharing a device)
  uint32_t *d_tmp = nullptr;
  uint64_t tmp_cap = 0;
  std::vector<hipEvent_t> ev;
  // the global corpus
  bool loaded = false;
  uint32_t n_runs = 0, G = 0, T = 0;
  uint64_t V = 0, E = 0;
  std::vector<uint32_t> iteration;
  std::vector<uint64_t> node_off, edge_off;
  std::unordered_map<uint32_t, uint32_t> it2run;
  std::vector<uint32_t> run_shard, run_local;  // owner shard / local index of every run
  int32_t run0 = -1;
  // diff entries of the last diffprov
  uint32_t n_entries = 0;
  std::vector<uint32_t> entry_shard, entry_local;
  int pull_which = -1;
  // assembled host views
  std::vector<uint8_t> state, masks;
  std::vector<uint64_t> choff;
  std::vector<uint32_t> chht;
  bool wide = false;
};

static int fail(nemo_ctx *c, int code, const char *fmt, ...) __attribute__((format(printf, 3, 4)));
static int fail(nemo_ctx *c, int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  return ctx_fail(c, code, buf);
}

// a shard's failure, reported by the node context with the shard's message
static int sfail(nemo_ctx *c, const Shard &s, int rc) {
  std::string m = std::string("device ") + std::to_string(s.device) + ": " + nemo_last_error(s.ctx);
  return ctx_fail(c, rc, m.c_str());
}

#define SCHK(c, s, x)                  \
  do {                                 \
    int rc_ = (x);                     \
    if (rc_) return sfail((c), (s), rc_); \
  } while (0)
#define HCHK(c, x)                                                                                   \
  do {                                                                                               \
    hipError_t e_ = (x);                                                                             \
    if (e_ != hipSuccess) return fail((c), NEMO_ERR_HIP, "%s: %s", #x, hipGetErrorString(e_));        \
  } while (0)
#define NCHK(c, x)                                                                                   \
  do {                                                                                               \
    ncclResult_t r_ = (x);                                                                           \
    if (r_ != ncclSuccess) return fail((c), NEMO_ERR_HIP, "%s: %s", #x, ncclGetErrorString(r_));      \
  } while (0)

__global__ void k_sum_u32(uint32_t *acc, const uint32_t *parts, uint32_t n_parts, uint64_t len) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < len; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t s = acc[i];
    for (uint32_t p = 0; p < n_parts; p++) s += parts[p * len + i];
    acc[i] = s;
  }
}

static Node *N(const nemo_ctx *c) { return ctx_node(c); }

// f(shard, p) on every shard, one host thread per shard; the first failing
// shard's status and message are reported
static int fanout(nemo_ctx *c, Node *n, const std::function<int(Shard &, size_t)> &f) {
  const size_t P = n->sh.size();
  std::vector<int> rcs(P, 0);
  if (P == 1 || !n->pool) {
    for (size_t p = 0; p < P; p++) rcs[p] = f(n->sh[p], p);
  } else {
    n->pool->run([&](size_t p) { rcs[p] = f(n->sh[p], p); });
  }
  for (size_t p = 0; p < P; p++) SCHK(c, n->sh[p], rcs[p]);
  return NEMO_OK;
}

extern "C" int nemo_ctx_create_node(int ndev, const int *devices, nemo_ctx **out) {
  if (!out) return NEMO_ERR_INVALID;
  *out = nullptr;
  int avail = 0;
  if (hipGetDeviceCount(&avail) != hipSuccess || avail <= 0) return NEMO_ERR_NOGPU;
  if (ndev <= 0) {
    if (devices) return NEMO_ERR_INVALID;
    ndev = avail;
  }
  std::vector<int> devs(ndev);
  for (int i = 0; i < ndev; i++) {
    devs[i] = devices ? devices[i] : i;
    if (devs[i] < 0 || devs[i] >= avail) return NEMO_ERR_INVALID;
  }
  Node *n = new Node();
  n->sh.resize(ndev);
  for (int i = 0; i < ndev; i++) {
    n->sh[i].device = devs[i];
    int rc = nemo_ctx_create(devs[i], &n->sh[i].ctx);
    if (rc) {
      node_destroy(n);
      return rc;
    }
  }
  std::vector<int> sorted = devs;
  std::sort(sorted.begin(), sorted.end());
  const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
  if (distinct) {
    n->comms.resize(ndev);
    if (ncclCommInitAll(n->comms.data(), ndev, devs.data()) != ncclSuccess) {
      node_destroy(n);
      return NEMO_ERR_HIP;
    }
    n->rccl = true;
  }
  n->ev.resize(ndev, nullptr);
  for (int i = 0; i < ndev; i++) {
    hipSetDevice(devs[i]);
    hipEventCreateWithFlags(&n->ev[i], hipEventDisableTiming);
  }
  if (ndev > 1) n->pool = new Pool((size_t)ndev);
  *out = ctx_new_facade(n);
  return NEMO_OK;
}

extern "C" int nemo_node_devices(const nemo_ctx *c, int *devices, int cap) {
  const Node *n = c ? N(c) : nullptr;
  if (!n) {  // a single-device context
    if (c && devices && cap > 0) devices[0] = ctx_device(c);
    return c ? 1 : 0;
  }
  for (int i = 0; i < (int)n->sh.size() && devices && i < cap; i++) devices[i] = n->sh[i].device;
  return (int)n->sh.size();
}

void node_destroy(Node *n) {
  if (!n) return;
  delete n->pool;
  n->pool = nullptr;
  for (auto &s : n->sh) {
    if (!s.ctx) continue;
    hipSetDevice(s.device);
    nemo_synchronize(s.ctx);
    if (s.d_lab) hipFree(s.d_lab);
    nemo_ctx_destroy(s.ctx);
  }
  for (auto cm : n->comms)
    if (cm) ncclCommDestroy(cm);
  if (n->d_tmp) {
    hipSetDevice(n->sh[0].device);
    hipFree(n->d_tmp);
  }
  for (size_t i = 0; i < n->ev.size(); i++)
    if (n->ev[i]) {
      hipSetDevice(n->sh[i].device);
      hipEventDestroy(n->ev[i]);
    }
  delete n;
}

int node_set_stream(nemo_ctx *c, void *stream) {
  Node *n = N(c);
  if (n->sh.size() != 1) return fail(c, NEMO_ERR_INVALID, "a node context of several devices owns its streams");
  SCHK(c, n->sh[0], nemo_set_stream(n->sh[0].ctx, stream));
  return NEMO_OK;
}
int node_set_option(nemo_ctx *c, const char *name, int64_t value) {
  for (auto &s : N(c)->sh) SCHK(c, s, nemo_set_option(s.ctx, name, value));
  return NEMO_OK;
}
int node_set_timing(nemo_ctx *c, int enable) {
  for (auto &s : N(c)->sh) SCHK(c, s, nemo_set_timing(s.ctx, enable));
  return NEMO_OK;
}
int node_set_timing_groups(nemo_ctx *c, const char *groups) {
  for (auto &s : N(c)->sh) SCHK(c, s, nemo_set_timing_groups(s.ctx, groups));
  return NEMO_OK;
}
uint64_t node_num_nodes(const nemo_ctx *c) { return N(c)->V; }
uint64_t node_num_edges(const nemo_ctx *c) { return N(c)->E; }
size_t node_reduce_len(const nemo_ctx *c) { return 2 * (size_t)N(c)->T + 4; }

// ---- load: LPT shards, run 0 replicated --------------------------------------
static void build_shard_corpus(const nemo_corpus *in, Shard &s, nemo_corpus *out) {
  const size_t R = s.runs.size();
  s.it.resize(R);
  s.no.assign(2 * R + 1, 0);
  s.eo.assign(2 * R + 1, 0);
  for (size_t i = 0; i < R; i++) {
    const uint32_t r = s.runs[i];
    s.it[i] = in->iteration[r];
    for (int k = 0; k < 2; k++) {
      const uint32_t g = 2 * r + k;
      s.no[2 * i + k + 1] = s.no[2 * i + k] + (in->node_off[g + 1] - in->node_off[g]);
      s.eo[2 * i + k + 1] = s.eo[2 * i + k] + (in->edge_off[g + 1] - in->edge_off[g]);
    }
  }
  const uint64_t V = s.no[2 * R], E = s.eo[2 * R];
  s.word.resize(V);
  s.label.resize(V);
  s.rank.resize(in->id_rank ? V : 0);
  s.es.resize(E);
  s.ed.resize(E);
  for (size_t i = 0; i < R; i++) {
    for (int k = 0; k < 2; k++) {
      const uint32_t g = 2 * s.runs[i] + k;
      const uint64_t a = in->node_off[g], nv = in->node_off[g + 1] - a, o = s.no[2 * i + k];
      memcpy(&s.word[o], in->node_word + a, nv * 4);
      memcpy(&s.label[o], in->label + a, nv * 4);
      if (in->id_rank) memcpy(&s.rank[o], in->id_rank + a, nv * 4);
      const uint64_t b = in->edge_off[g], ne = in->edge_off[g + 1] - b, q = s.eo[2 * i + k];
      memcpy(&s.es[q], in->edge_src + b, ne * 4);
      memcpy(&s.ed[q], in->edge_dst + b, ne * 4);
    }
  }
  *out = *in;
  out->n_runs = (uint32_t)R;
  out->iteration = s.it.data();
  out->owned = s.own.data();
  out->node_off = s.no.data();
  out->edge_off = s.eo.data();
  out->node_word = s.word.data();
  out->label = s.label.data();
  out->id_rank = in->id_rank ? s.rank.data() : nullptr;
  out->edge_src = s.es.data();
  out->edge_dst = s.ed.data();
}

int node_load_corpus(nemo_ctx *c, const nemo_corpus *in) {
  Node *n = N(c);
  if (!in || !in->iteration || !in->node_off || !in->edge_off) return fail(c, NEMO_ERR_INVALID, "corpus arrays missing");
  const uint32_t R = in->n_runs, P = (uint32_t)n->sh.size();
  n->loaded = false;
  n->n_runs = R;
  n->G = 2 * R;
  n->T = in->n_tables;
  n->iteration.assign(in->iteration, in->iteration + R);
  n->node_off.assign(in->node_off, in->node_off + 2 * R + 1);
  n->edge_off.assign(in->edge_off, in->edge_off + 2 * R + 1);
  n->V = n->node_off[2 * R];
  n->E = n->edge_off[2 * R];
  n->it2run.clear();
  n->run0 = -1;
  for (uint32_t r = 0; r < R; r++) {
    if (n->it2run.count(in->iteration[r])) return fail(c, NEMO_ERR_INVALID, "duplicate run iteration %u", in->iteration[r]);
    n->it2run[in->iteration[r]] = r;
    if (in->iteration[r] == 0) n->run0 = (int32_t)r;
  }
  std::vector<uint32_t> part(R ? R : 1, 0);
  if (R && nemo_partition_runs(in, P, part.data())) return fail(c, NEMO_ERR_INVALID, "malformed corpus offsets");
  n->run_shard.assign(R, 0);
  n->run_local.assign(R, 0);
  for (auto &s : n->sh) {
    s.runs.clear();
    s.own.clear();
    s.run0_local = -1;
  }
  for (uint32_t p = 0; p < P; p++) {
    Shard &s = n->sh[p];
    for (uint32_t r = 0; r < R; r++) {
      const bool mine = part[r] == p;
      if (!mine && (int32_t)r != n->run0) continue;
      if (mine) {
        n->run_shard[r] = p;
        n->run_local[r] = (uint32_t)s.runs.size();
      }
      if ((int32_t)r == n->run0) s.run0_local = (int32_t)s.runs.size();
      s.runs.push_back(r);
      s.own.push_back(mine && (!in->owned || in->owned[r]) ? 1 : 0);
    }
  }
  // host gather + device load of every shard, one thread per device
  std::vector<int> rcs(P, 0);
  std::vector<std::thread> th;
  for (uint32_t p = 0; p < P; p++)
    th.emplace_back([&, p] {
      Shard &s = n->sh[p];
      nemo_corpus sc;
      build_shard_corpus(in, s, &sc);
      rcs[p] = nemo_load_corpus(s.ctx, &sc);
      // the host copies are not needed once the corpus is resident
      std::vector<uint32_t>().swap(s.word);
      std::vector<uint32_t>().swap(s.label);
      std::vector<uint32_t>().swap(s.rank);
      std::vector<uint32_t>().swap(s.es);
      std::vector<uint32_t>().swap(s.ed);
    });
  for (auto &t : th) t.join();
  for (uint32_t p = 0; p < P; p++) SCHK(c, n->sh[p], rcs[p]);
  n->n_entries = 0;
  n->pull_which = -1;
  n->loaded = true;
  return NEMO_OK;
}

#define NEED_LOADED(c, n) \
  if (!(n)->loaded) return fail((c), NEMO_ERR_STATE, "no corpus loaded")

int node_rebuild(nemo_ctx *c) {
  Node *n = N(c);
  NEED_LOADED(c, n);
  return fanout(c, n, [](Shard &s, size_t) { return nemo_rebuild(s.ctx); });
}
int node_mark_holds(nemo_ctx *c) {
  Node *n = N(c);
  NEED_LOADED(c, n);
  return fanout(c, n, [](Shard &s, size_t) { return nemo_mark_holds(s.ctx); });
}
int node_simplify(nemo_ctx *c) {
  Node *n = N(c);
  return fanout(c, n, [](Shard &s, size_t) { return nemo_simplify(s.ctx); });
}

// ---- cross-shard exchanges -----------------------------------------------------
// Sum the shards' reduction vectors in place on every shard.
static int allreduce_sum(nemo_ctx *c, Node *n, uint64_t len) {
  const size_t P = n->sh.size();
  if (P == 1) return NEMO_OK;
  if (n->rccl) {
    NCHK(c, ncclGroupStart());
    for (size_t p = 0; p < P; p++) {
      uint32_t *d = ctx_reduce_buf(n->sh[p].ctx);
      NCHK(c, ncclAllReduce(d, d, len, ncclUint32, ncclSum, n->comms[p], ctx_stream(n->sh[p].ctx)));
    }
    NCHK(c, ncclGroupEnd());
    return NEMO_OK;
  }
  // peer copies into shard 0, one sum kernel, copies back
  Shard &s0 = n->sh[0];
  hipStream_t st0 = ctx_stream(s0.ctx);
  HCHK(c, hipSetDevice(s0.device));
  if (n->tmp_cap < (P - 1) * len) {
    if (n->d_tmp) HCHK(c, hipFree(n->d_tmp));
    n->d_tmp = nullptr;
    HCHK(c, hipMalloc(&n->d_tmp, (P - 1) * len * 4));
    n->tmp_cap = (P - 1) * len;
  }
  for (size_t p = 1; p < P; p++) {
    HCHK(c, hipSetDevice(n->sh[p].device));
    HCHK(c, hipEventRecord(n->ev[p], ctx_stream(n->sh[p].ctx)));
    HCHK(c, hipSetDevice(s0.device));
    HCHK(c, hipStreamWaitEvent(st0, n->ev[p], 0));
    HCHK(c, hipMemcpyPeerAsync(n->d_tmp + (p - 1) * len, s0.device, ctx_reduce_buf(n->sh[p].ctx), n->sh[p].device,
                               len * 4, st0));
  }
  hipLaunchKernelGGL(k_sum_u32, dim3(16), dim3(256), 0, st0, ctx_reduce_buf(s0.ctx), n->d_tmp, (uint32_t)(P - 1), len);
  HCHK(c, hipGetLastError());
  for (size_t p = 1; p < P; p++)
    HCHK(c, hipMemcpyPeerAsync(ctx_reduce_buf(n->sh[p].ctx), n->sh[p].device, ctx_reduce_buf(s0.ctx), s0.device, len * 4,
                               st0));
  HCHK(c, hipEventRecord(n->ev[0], st0));
  for (size_t p = 1; p < P; p++) {
    HCHK(c, hipSetDevice(n->sh[p].device));
    HCHK(c, hipStreamWaitEvent(ctx_stream(n->sh[p].ctx), n->ev[0], 0));
  }
  return NEMO_OK;
}

// Broadcast `bytes` of shard `root`'s d_lab to every other shard's d_lab.
static int broadcast_labels(nemo_ctx *c, Node *n, uint32_t root, uint64_t count) {
  const size_t P = n->sh.size();
  if (P == 1) return NEMO_OK;
  if (n->rccl) {
    NCHK(c, ncclGroupStart());
    for (size_t p = 0; p < P; p++)
      NCHK(c, ncclBroadcast(n->sh[p].d_lab, n->sh[p].d_lab, count, ncclUint32, (int)root, n->comms[p],
                            ctx_stream(n->sh[p].ctx)));
    NCHK(c, ncclGroupEnd());
    return NEMO_OK;
  }
  Shard &o = n->sh[root];
  hipStream_t so = ctx_stream(o.ctx);
  // a destination's d_lab may still be read by its previous k_diff: the copy
  // waits for everything queued on that shard's stream so far
  for (size_t p = 0; p < P; p++) {
    if (p == root) continue;
    HCHK(c, hipSetDevice(n->sh[p].device));
    HCHK(c, hipEventRecord(n->ev[p], ctx_stream(n->sh[p].ctx)));
    HCHK(c, hipSetDevice(o.device));
    HCHK(c, hipStreamWaitEvent(so, n->ev[p], 0));
  }
  HCHK(c, hipSetDevice(o.device));
  for (size_t p = 0; p < P; p++)
    if (p != root) HCHK(c, hipMemcpyPeerAsync(n->sh[p].d_lab, n->sh[p].device, o.d_lab, o.device, count * 4, so));
  HCHK(c, hipEventRecord(n->ev[root], so));
  for (size_t p = 0; p < P; p++) {
    if (p == root) continue;
    HCHK(c, hipSetDevice(n->sh[p].device));
    HCHK(c, hipStreamWaitEvent(ctx_stream(n->sh[p].ctx), n->ev[root], 0));
  }
  return NEMO_OK;
}

int node_protos_partial(nemo_ctx *c, const uint32_t *success, size_t ns, uint32_t *d_red) {
  Node *n = N(c);
  NEED_LOADED(c, n);
  if (d_red && n->sh.size() > 1)
    return fail(c, NEMO_ERR_INVALID, "a node context reduces across its devices itself: pass d_reduce = NULL");
  // success iterations stay global: each shard ignores the runs it does not hold, and the first
  // one (Q-PROTO-FIRST) counts on the shard that owns it (k_reduce gates on ownership)
  const bool multi = n->sh.size() > 1;
  if (int rc = fanout(c, n, [&](Shard &s, size_t) {
        return nemo_protos_partial(s.ctx, success, ns, multi ? nullptr : d_red);
      }))
    return rc;
  return allreduce_sum(c, n, node_reduce_len(c));
}

int node_protos_finalize(nemo_ctx *c, const uint32_t *d_red, uint32_t *achieved, uint32_t *inter, uint32_t *n_inter,
                         uint32_t *uni, uint32_t *n_union, uint64_t *pre_holds, uint32_t *n_runs_total) {
  Node *n = N(c);
  if (d_red && n->sh.size() > 1) return fail(c, NEMO_ERR_INVALID, "pass d_reduce = NULL to a node context");
  SCHK(c, n->sh[0], nemo_protos_finalize(n->sh[0].ctx, d_red, achieved, inter, n_inter, uni, n_union, pre_holds,
                                          n_runs_total));
  return NEMO_OK;
}

int node_fetch_reduce(nemo_ctx *c, uint32_t *out, uint64_t cap) {
  SCHK(c, N(c)->sh[0], nemo_fetch_reduce(N(c)->sh[0].ctx, out, cap));  // every shard holds the sum
  return NEMO_OK;
}

int node_fetch_run_tables(nemo_ctx *c, int which, uint32_t *out, uint64_t cap) {
  Node *n = N(c);
  if (!out) return fail(c, NEMO_ERR_INVALID, "null output");
  const uint32_t W = (n->T + 31) / 32;
  if (cap < (uint64_t)n->n_runs * W) return fail(c, NEMO_ERR_INVALID, "capacity too small");
  return fanout(c, n, [&](Shard &s, size_t p) {
    std::vector<uint32_t> t((size_t)s.runs.size() * W + 1);
    if (int rc = nemo_fetch_run_tables(s.ctx, which, t.data(), (uint64_t)s.runs.size() * W)) return rc;
    for (size_t i = 0; i < s.runs.size(); i++)
      if (n->run_shard[s.runs[i]] == p) memcpy(out + (size_t)s.runs[i] * W, &t[i * W], W * 4);
    return NEMO_OK;
  });
}

static int owner_of_iter(nemo_ctx *c, Node *n, uint32_t it, uint32_t *run) {
  auto f = n->it2run.find(it);
  if (f == n->it2run.end()) return fail(c, NEMO_ERR_NOTFOUND, "unknown run iteration %u", it);
  *run = f->second;
  return NEMO_OK;
}

int node_missing_from(nemo_ctx *c, uint32_t failed_iter, const uint32_t *proto, uint32_t n_proto, uint32_t *out,
                      uint32_t *n_out) {
  Node *n = N(c);
  uint32_t r;
  if (int rc = owner_of_iter(c, n, failed_iter, &r)) return rc;
  Shard &s = n->sh[n->run_shard[r]];
  SCHK(c, s, nemo_missing_from(s.ctx, failed_iter, proto, n_proto, out, n_out));
  return NEMO_OK;
}

// ---- differential provenance ---------------------------------------------------
static int node_diff(nemo_ctx *c, const uint32_t *failed, size_t nf, int mode, const uint32_t *d_labels,
                     uint64_t lab_cap) {
  Node *n = N(c);
  NEED_LOADED(c, n);
  if (!failed && nf) return fail(c, NEMO_ERR_INVALID, "null failed list");
  if (mode != NEMO_DIFF_REFERENCE && mode != NEMO_DIFF_PER_RUN) return fail(c, NEMO_ERR_INVALID, "unknown diff mode %d", mode);
  const size_t P = n->sh.size();
  std::vector<std::vector<uint32_t>> lists(P);
  n->entry_shard.assign(nf, 0);
  n->entry_local.assign(nf, 0);
  for (auto &s : n->sh) s.entries.clear();
  for (size_t e = 0; e < nf; e++) {
    uint32_t r;
    if (int rc = owner_of_iter(c, n, failed[e], &r)) return rc;
    const uint32_t p = n->run_shard[r];
    n->entry_shard[e] = p;
    n->entry_local[e] = (uint32_t)lists[p].size();
    lists[p].push_back(failed[e]);
    n->sh[p].entries.push_back((uint32_t)e);
  }
  n->n_entries = n->run0 >= 0 ? (uint32_t)nf : 0;
  if (d_labels) {  // caller-provided label set (one device only)
    if (P > 1) return fail(c, NEMO_ERR_INVALID, "nemo_diffprov_labels on a node context: use nemo_diffprov");
    SCHK(c, n->sh[0], nemo_diffprov_labels(n->sh[0].ctx, lists[0].data(), lists[0].size(), d_labels, lab_cap));
    return NEMO_OK;
  }
  if (mode == NEMO_DIFF_PER_RUN || nf == 0 || P == 1 || n->run0 < 0)
    return fanout(c, n, [&](Shard &s, size_t p) { return nemo_diffprov(s.ctx, lists[p].data(), lists[p].size(), mode); });
  // reference mode over shards: failedRuns[0]'s label set from its owner, broadcast
  uint32_t r0f;
  if (int rc = owner_of_iter(c, n, failed[0], &r0f)) return rc;
  const uint32_t root = n->run_shard[r0f];
  const uint64_t cap = n->node_off[2 * r0f + 2] - n->node_off[2 * r0f + 1] + 1;
  for (auto &s : n->sh)
    if (s.lab_cap < cap) {
      HCHK(c, hipSetDevice(s.device));
      if (s.d_lab) HCHK(c, hipFree(s.d_lab));
      s.d_lab = nullptr;
      HCHK(c, hipMalloc(&s.d_lab, cap * 4));
      s.lab_cap = cap;
    }
  // every shard's stream first waits for its previous diff (on the shard's aux
  // stream), which may still read the d_lab this broadcast overwrites
  for (auto &s : n->sh) SCHK(c, s, ctx_join_aux(s.ctx));
  SCHK(c, n->sh[root], nemo_goal_labels(n->sh[root].ctx, failed[0], 1, n->sh[root].d_lab, cap));
  if (int rc = broadcast_labels(c, n, root, cap)) return rc;
  return fanout(c, n, [&](Shard &s, size_t p) {
    return nemo_diffprov_labels(s.ctx, lists[p].data(), lists[p].size(), s.d_lab, cap);
  });
}
int node_diffprov(nemo_ctx *c, const uint32_t *failed, size_t nf, int mode) {
  return node_diff(c, failed, nf, mode, nullptr, 0);
}
int node_diffprov_labels(nemo_ctx *c, const uint32_t *failed, size_t nf, const uint32_t *d_labels, uint64_t cap) {
  if (!d_labels) return fail(c, NEMO_ERR_INVALID, "no label set");
  return node_diff(c, failed, nf, NEMO_DIFF_REFERENCE, d_labels, cap);
}
int node_diffprov_host_labels(nemo_ctx *c, const uint32_t *failed, size_t nf, const uint32_t *labels, uint64_t n_labels) {
  Node *n = N(c);
  NEED_LOADED(c, n);
  // route the entries as node_diff does, every shard with the same host label set
  const size_t P = n->sh.size();
  std::vector<std::vector<uint32_t>> lists(P);
  n->entry_shard.assign(nf, 0);
  n->entry_local.assign(nf, 0);
  for (auto &s : n->sh) s.entries.clear();
  for (size_t e = 0; e < nf; e++) {
    uint32_t r;
    if (int rc = owner_of_iter(c, n, failed[e], &r)) return rc;
    const uint32_t p = n->run_shard[r];
    n->entry_shard[e] = p;
    n->entry_local[e] = (uint32_t)lists[p].size();
    lists[p].push_back(failed[e]);
    n->sh[p].entries.push_back((uint32_t)e);
  }
  n->n_entries = n->run0 >= 0 ? (uint32_t)nf : 0;
  return fanout(c, n, [&](Shard &s, size_t p) {
    return nemo_diffprov_host_labels(s.ctx, lists[p].data(), lists[p].size(), labels, n_labels);
  });
}

int node_goal_labels(nemo_ctx *c, uint32_t iteration, int cond, uint32_t *d_out, uint64_t cap) {
  Node *n = N(c);
  if (n->sh.size() > 1) return fail(c, NEMO_ERR_INVALID, "nemo_goal_labels on a node context: its diffprov broadcasts");
  SCHK(c, n->sh[0], nemo_goal_labels(n->sh[0].ctx, iteration, cond, d_out, cap));
  return NEMO_OK;
}

static uint64_t v0_of(const Node *n) {
  return n->run0 >= 0 ? n->node_off[2 * n->run0 + 2] - n->node_off[2 * n->run0 + 1] : 0;
}

int node_fetch_diff_mask(nemo_ctx *c, uint32_t entry, uint8_t *out, uint64_t cap) {
  Node *n = N(c);
  if (entry >= n->n_entries) return fail(c, NEMO_ERR_INVALID, "diff entry %u out of range", entry);
  Shard &s = n->sh[n->entry_shard[entry]];
  SCHK(c, s, nemo_fetch_diff_mask(s.ctx, n->entry_local[entry], out, cap));
  return NEMO_OK;
}
int node_fetch_diff_masks(nemo_ctx *c, uint8_t *out, uint64_t cap) {
  Node *n = N(c);
  const uint64_t V0 = v0_of(n);
  if (!out) return fail(c, NEMO_ERR_INVALID, "null output");
  if (cap < n->n_entries * V0) return fail(c, NEMO_ERR_INVALID, "capacity too small");
  return fanout(c, n, [&](Shard &s, size_t) {
    if (s.entries.empty()) return (int)NEMO_OK;
    const uint8_t *m = nullptr;
    uint64_t ne = 0, v0 = 0;
    if (int rc = nemo_diff_masks_view(s.ctx, &m, &ne, &v0)) return rc;
    for (size_t i = 0; i < s.entries.size() && m; i++) memcpy(out + s.entries[i] * V0, m + i * V0, V0);
    return (int)NEMO_OK;
  });
}
int node_diff_masks_view(nemo_ctx *c, const uint8_t **masks, uint64_t *n_entries, uint64_t *v0) {
  Node *n = N(c);
  if (!masks) return fail(c, NEMO_ERR_INVALID, "null output");
  const uint64_t V0 = v0_of(n);
  *masks = nullptr;
  if (n_entries) *n_entries = n->n_entries;
  if (v0) *v0 = V0;
  if (!n->n_entries) return NEMO_OK;
  if (n->sh.size() == 1) {
    SCHK(c, n->sh[0], nemo_diff_masks_view(n->sh[0].ctx, masks, nullptr, nullptr));
    return NEMO_OK;
  }
  n->masks.resize(n->n_entries * V0 + 1);
  if (int rc = node_fetch_diff_masks(c, n->masks.data(), n->n_entries * V0)) return rc;
  *masks = n->masks.data();
  return NEMO_OK;
}
int node_fetch_missing(nemo_ctx *c, nemo_missing *out, uint64_t cap, uint64_t *n_out) {
  Node *n = N(c);
  std::vector<std::vector<nemo_missing>> per(n->sh.size());
  if (int rc = fanout(c, n, [&](Shard &s, size_t p) {
        uint64_t k = 0;
        if (int r = nemo_fetch_missing(s.ctx, nullptr, 0, &k)) return r;
        per[p].resize(k + 1);
        if (int r = nemo_fetch_missing(s.ctx, per[p].data(), k, &k)) return r;
        per[p].resize(k);
        return (int)NEMO_OK;
      }))
    return rc;
  std::vector<nemo_missing> all;
  for (size_t p = 0; p < n->sh.size(); p++)
    for (const auto &m : per[p]) all.push_back({n->sh[p].entries[m.entry], m.rule});
  std::sort(all.begin(), all.end(), [](const nemo_missing &a, const nemo_missing &b) {
    return a.entry != b.entry ? a.entry < b.entry : a.rule < b.rule;
  });
  if (n_out) *n_out = all.size();
  if (!out) return NEMO_OK;
  if (cap < all.size()) return fail(c, NEMO_ERR_INVALID, "capacity too small");
  if (!all.empty()) memcpy(out, all.data(), all.size() * sizeof(nemo_missing));
  return NEMO_OK;
}

// ---- corrections / extensions on run 0: its owner shard ------------------------
static Shard &run0_owner(Node *n) { return n->sh[n->run0 >= 0 ? n->run_shard[n->run0] : 0]; }
int node_triggers(nemo_ctx *c) {
  Node *n = N(c);
  NEED_LOADED(c, n);
  Shard &s = run0_owner(n);
  SCHK(c, s, nemo_triggers(s.ctx));
  return NEMO_OK;
}
int node_fetch_triggers(nemo_ctx *c, uint32_t *pre, uint64_t pre_cap, uint64_t *n_pre, uint32_t *post,
                        uint64_t post_cap, uint64_t *n_post, uint32_t *async_rules, uint64_t async_cap,
                        uint64_t *n_async) {
  Shard &s = run0_owner(N(c));
  SCHK(c, s, nemo_fetch_triggers(s.ctx, pre, pre_cap, n_pre, post, post_cap, n_post, async_rules, async_cap, n_async));
  return NEMO_OK;
}

// ---- per-graph results, reassembled in global graph order ----------------------
int node_fetch_node_flags(nemo_ctx *c, uint32_t g_lo, uint32_t g_hi, uint8_t *out, uint64_t cap) {
  Node *n = N(c);
  if (!out || g_lo > g_hi || g_hi > n->G) return fail(c, NEMO_ERR_INVALID, "bad graph range");
  if (cap < n->node_off[g_hi] - n->node_off[g_lo]) return fail(c, NEMO_ERR_INVALID, "capacity too small");
  for (uint32_t g = g_lo; g < g_hi; g++) {
    const uint32_t r = g / 2;
    Shard &s = n->sh[n->run_shard[r]];
    const uint32_t lg = 2 * n->run_local[r] + (g & 1);
    const uint64_t nv = n->node_off[g + 1] - n->node_off[g];
    SCHK(c, s, nemo_fetch_node_flags(s.ctx, lg, lg + 1, out + (n->node_off[g] - n->node_off[g_lo]), nv));
  }
  return NEMO_OK;
}

static uint32_t global_graph(const Node *n, const Shard &s, uint32_t lg, bool *owned_here) {
  const uint32_t r = s.runs[lg / 2];
  *owned_here = &n->sh[n->run_shard[r]] == &s;
  return 2 * r + (lg & 1);
}

int node_fetch_chains(nemo_ctx *c, nemo_chain *out, uint64_t cap, uint64_t *n_out) {
  Node *n = N(c);
  std::vector<std::vector<nemo_chain>> per(n->sh.size());
  if (int rc = fanout(c, n, [&](Shard &s, size_t p) {
        uint64_t k = 0;
        if (int r = nemo_fetch_chains(s.ctx, nullptr, 0, &k)) return r;
        per[p].resize(k + 1);
        if (int r = nemo_fetch_chains(s.ctx, per[p].data(), k, &k)) return r;
        per[p].resize(k);
        return (int)NEMO_OK;
      }))
    return rc;
  std::vector<nemo_chain> all;
  for (size_t p = 0; p < n->sh.size(); p++)
    for (auto v : per[p]) {
      bool mine;
      const uint32_t g = global_graph(n, n->sh[p], v.graph, &mine);
      if (!mine) continue;  // run 0's replica
      v.graph = g;
      all.push_back(v);
    }
  std::sort(all.begin(), all.end(), [](const nemo_chain &a, const nemo_chain &b) {
    return a.graph != b.graph ? a.graph < b.graph : a.k < b.k;
  });
  if (n_out) *n_out = all.size();
  if (!out) return NEMO_OK;
  if (cap < all.size()) return fail(c, NEMO_ERR_INVALID, "capacity too small");
  if (!all.empty()) memcpy(out, all.data(), all.size() * sizeof(nemo_chain));
  return NEMO_OK;
}

int node_stage_simplified(nemo_ctx *c) {
  return fanout(c, N(c), [](Shard &s, size_t) { return nemo_stage_simplified(s.ctx); });
}

int node_simplified_view(nemo_ctx *c, const uint8_t **state, const uint64_t **chain_off, const uint32_t **chain_ht,
                         uint64_t *n_chains, int *wide_pairs) {
  Node *n = N(c);
  if (n->sh.size() == 1) {
    SCHK(c, n->sh[0], nemo_simplified_view(n->sh[0].ctx, state, chain_off, chain_ht, n_chains, wide_pairs));
    return NEMO_OK;
  }
  struct V {
    const uint8_t *st;
    const uint64_t *off;
    const uint32_t *ht;
    uint64_t n;
    int wide;
  };
  std::vector<V> v(n->sh.size());
  bool wide = false;
  if (int rc = fanout(c, n, [&](Shard &s, size_t p) {
        return nemo_simplified_view(s.ctx, &v[p].st, &v[p].off, &v[p].ht, &v[p].n, &v[p].wide);
      }))
    return rc;
  for (size_t p = 0; p < n->sh.size(); p++) wide |= v[p].wide != 0;
  // 2-bit node states in global node order; chain pairs in global graph order
  n->state.assign((n->V + 3) / 4 + 16, 0);
  n->choff.assign((size_t)n->G + 1, 0);
  for (uint32_t g = 0; g < n->G; g++) {
    const uint32_t r = g / 2, p = n->run_shard[r], lg = 2 * n->run_local[r] + (g & 1);
    n->choff[g + 1] = n->choff[g] + (v[p].off[lg + 1] - v[p].off[lg]);
  }
  n->chht.assign((wide ? 2 : 1) * n->choff[n->G] + 2, 0);
  for (uint32_t g = 0; g < n->G; g++) {
    const uint32_t r = g / 2, p = n->run_shard[r], lg = 2 * n->run_local[r] + (g & 1);
    const Shard &s = n->sh[p];
    // node states: shard-local node l0 + i -> global node n0 + i
    const uint64_t l0 = s.no[lg];
    const uint64_t n0 = n->node_off[g], nv = n->node_off[g + 1] - n0;
    for (uint64_t i = 0; i < nv; i++) {
      const uint64_t a = l0 + i, b = n0 + i;
      const uint32_t bits = (v[p].st[a >> 2] >> (2 * (a & 3))) & 3u;
      n->state[b >> 2] |= (uint8_t)(bits << (2 * (b & 3)));
    }
    const uint64_t k0 = v[p].off[lg], k1 = v[p].off[lg + 1], o = n->choff[g];
    for (uint64_t k = k0; k < k1; k++) {
      uint32_t h, t;
      if (v[p].wide) {
        h = v[p].ht[2 * k];
        t = v[p].ht[2 * k + 1];
      } else {
        h = v[p].ht[k] & 0xFFFFu;
        t = v[p].ht[k] >> 16;
      }
      if (wide) {
        n->chht[2 * (o + k - k0)] = h;
        n->chht[2 * (o + k - k0) + 1] = t;
      } else {
        n->chht[o + k - k0] = h | (t << 16);
      }
    }
  }
  n->wide = wide;
  if (state) *state = n->state.data();
  if (chain_off) *chain_off = n->choff.data();
  if (chain_ht) *chain_ht = n->chht.data();
  if (n_chains) *n_chains = n->choff[n->G];
  if (wide_pairs) *wide_pairs = wide ? 1 : 0;
  return NEMO_OK;
}

// ---- edge pulls ---------------------------------------------------------------------
int node_pull_edges(nemo_ctx *c, int which) {
  Node *n = N(c);
  NEED_LOADED(c, n);
  if (int rc = fanout(c, n, [&](Shard &s, size_t) { return nemo_pull_edges(s.ctx, which); })) return rc;
  n->pull_which = which;
  return NEMO_OK;
}
// global slot -> (shard, local slot)
static bool slot_of(const Node *n, uint32_t slot, uint32_t *p, uint32_t *ls) {
  if (n->pull_which == 2) {
    if (slot >= n->n_entries) return false;
    *p = n->entry_shard[slot];
    *ls = n->entry_local[slot];
    return true;
  }
  if (slot >= n->G) return false;
  *p = n->run_shard[slot / 2];
  *ls = 2 * n->run_local[slot / 2] + (slot & 1);
  return true;
}
uint64_t node_pulled_count(nemo_ctx *c, uint32_t slot) {
  Node *n = N(c);
  uint32_t p, ls;
  if (n->pull_which < 0 || !slot_of(n, slot, &p, &ls)) return 0;
  return nemo_pulled_count(n->sh[p].ctx, ls);
}
int node_fetch_pulled(nemo_ctx *c, uint32_t slot, uint32_t *src, uint32_t *dst, uint64_t cap, uint64_t *n_out) {
  Node *n = N(c);
  if (n->pull_which < 0) return fail(c, NEMO_ERR_STATE, "nothing pulled");
  uint32_t p, ls;
  if (!slot_of(n, slot, &p, &ls)) return fail(c, NEMO_ERR_INVALID, "slot %u out of range", slot);
  SCHK(c, n->sh[p], nemo_fetch_pulled(n->sh[p].ctx, ls, src, dst, cap, n_out));
  return NEMO_OK;
}
int node_fetch_pulled_all(nemo_ctx *c, uint64_t *off, uint32_t *cnt, uint32_t *src, uint32_t *dst, uint64_t cap,
                          uint64_t *n_used) {
  Node *n = N(c);
  if (n->pull_which < 0) return fail(c, NEMO_ERR_STATE, "nothing pulled");
  const uint32_t slots = n->pull_which == 2 ? n->n_entries : n->G;
  // shard p's region goes after shards 0..p-1
  std::vector<uint64_t> used(n->sh.size()), base(n->sh.size() + 1, 0);
  std::vector<std::vector<uint64_t>> so(n->sh.size());
  std::vector<std::vector<uint32_t>> sc(n->sh.size());
  if (int rc = fanout(c, n, [&](Shard &s, size_t p) {
        const uint32_t ls = n->pull_which == 2 ? (uint32_t)s.entries.size() : 2 * (uint32_t)s.runs.size();
        so[p].assign(ls + 1, 0);
        sc[p].assign(ls + 1, 0);
        return nemo_fetch_pulled_all(s.ctx, so[p].data(), sc[p].data(), nullptr, nullptr, 0, &used[p]);
      }))
    return rc;
  for (size_t p = 0; p < n->sh.size(); p++) base[p + 1] = base[p] + used[p];
  if (n_used) *n_used = base[n->sh.size()];
  for (uint32_t s = 0; s < slots; s++) {
    uint32_t p, ls;
    slot_of(n, s, &p, &ls);
    if (off) off[s] = base[p] + so[p][ls];
    if (cnt) cnt[s] = sc[p][ls];
  }
  if (!src && !dst) return NEMO_OK;
  if (cap < base[n->sh.size()]) return fail(c, NEMO_ERR_INVALID, "capacity too small");
  return fanout(c, n, [&](Shard &s, size_t p) {
    return nemo_fetch_pulled_all(s.ctx, nullptr, nullptr, src ? src + base[p] : nullptr, dst ? dst + base[p] : nullptr,
                                 used[p], &used[p]);
  });
}

int node_debug_copy(nemo_ctx *c, const char *name, void *out, uint64_t offset, uint64_t bytes) {
  SCHK(c, N(c)->sh[0], nemo_debug_copy(N(c)->sh[0].ctx, name, out, offset, bytes));
  return NEMO_OK;
}
int node_synchronize(nemo_ctx *c) {
  return fanout(c, N(c), [](Shard &s, size_t) { return nemo_synchronize(s.ctx); });
}
int node_timings(nemo_ctx *c, nemo_timing *out, uint32_t cap, uint32_t *n_out) {
  std::map<std::string, nemo_timing> acc;
  for (auto &s : N(c)->sh) {
    uint32_t k = 0;
    SCHK(c, s, nemo_timings(s.ctx, nullptr, 0, &k));
    std::vector<nemo_timing> v(k + 1);
    SCHK(c, s, nemo_timings(s.ctx, v.data(), k, &k));
    for (uint32_t i = 0; i < k; i++) {
      nemo_timing &a = acc[v[i].name];
      if (!a.name[0]) memcpy(a.name, v[i].name, sizeof a.name);
      a.launches += v[i].launches;
      a.ms += v[i].ms;
      a.bytes += v[i].bytes;
      a.edges += v[i].edges;
    }
  }
  uint32_t i = 0;
  for (auto &kv : acc) {
    if (out && i < cap) out[i] = kv.second;
    i++;
  }
  if (n_out) *n_out = i;
  return NEMO_OK;
}
int node_reset_timings(nemo_ctx *c) {
  for (auto &s : N(c)->sh) SCHK(c, s, nemo_reset_timings(s.ctx));
  return NEMO_OK;
}
