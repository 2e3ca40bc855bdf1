// api.hip — the C ABI of libnemohip (include/nemohip.h): context, device
// memory layout of a loaded corpus, phase orchestration, result fetches and
// per-kernel HIP-event timing.  No CPU fallback exists: every analysis result
// comes from the gfx950 kernels in k_*.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>
#include <thread>
#include <tuple>
#include <atomic>

#include "device.h"
#include "internal.h"
#include "node.h"

namespace {

struct Agg {
  uint64_t launches = 0;
  double ms = 0, bytes = 0, edges = 0;
};

struct PendingEv {
  std::string name;
  hipEvent_t a, b;
  double bytes, edges;
};

}  // namespace

struct nemo_ctx {
  Node *node = nullptr;  // node context: every entry point dispatches to node.hip
  int device = 0;
  hipStream_t own = nullptr, stream = nullptr;
  // uploads of a corpus of big graphs, in parts, so that the CSR build of part k overlaps the
  // upload of part k + 1 (nemo_load_corpus; option load_parts)
  hipStream_t up = nullptr;
  std::vector<hipEvent_t> ev_up;
  uint32_t load_parts = 4;
  bool load_async = false;          // option load_async: nemo_load_corpus returns once its work is queued
  bool load_check_pending = false;  // ... and the graph checks wait for the next call that reads the graphs
  std::vector<uint32_t> big_host;  // the big-graph list (DevCorpus::big) on the host
  std::string err;
  std::vector<std::string> tgroups;  // nemo_set_timing_groups: the timed groups (empty: all)
  bool timing = false;
  std::vector<PendingEv> pending;
  std::vector<hipEvent_t> ev_pool;
  std::map<std::string, Agg> agg;

  // host view of the loaded corpus
  bool loaded = false, marked = false, simplified = false, protos_done = false;
  uint32_t n_runs = 0, G = 0, T = 0, W = 0, table_pre = 0, table_post = 0;
  uint64_t V = 0, E = 0;
  std::vector<uint32_t> iteration;
  std::vector<uint8_t> owned;
  std::vector<uint64_t> node_off, edge_off;
  std::unordered_map<uint32_t, uint32_t> it2run;
  int32_t run0 = -1;
  bool has_rank = false;
  uint32_t hcap_limit = 0xFFFFFFFFu, comp_limit = 0xFFFFFFFFu, build_limit = 0xFFFFFFFFu;
  uint32_t lds_limit = 0xFFFFFFFFu;  // test knob: largest V of the LDS graph tier (0 = off)
  uint64_t glob_min_v = 65536;       // graphs with V >= this take k_chains_glob (set before load)
  uint32_t gblock_force = 0;         // global_block option (0 = by corpus shape)
  uint32_t glob_block_force = 0;     // chains_glob_block option (0 = by the number of deep graphs)
  bool glob_prep_off = false;        // chains_glob_prep option 0: k_chains_glob builds its own H* order (test knob)
  bool topo_ell_off = true;          // topo_ell option 1: deep graphs' Kahn levels by k_topo_ell (measured slower
                                     // at C5: 103 vs 84 ms per launch with its records; kept as an option, tested)
  double tierV = 0, tierE = 0;       // nodes / edges of the graphs within the tier's V/E caps
  bool diff_on_aux = true;           // diff kernels on `aux` beside the simplification (option diff_aux)
  uint32_t ms_rest = 0, pull_rest = 0;  // graphs past k_marksimp's / k_pull_lds's tiers (their global grids skipped at 0)
  double postV = 0, postE = 0;       // nodes / edges of the post graphs (k_proto's input)
  double bigV = 0, bigE = 0;         // nodes / edges of the graphs of >= NEMO_CSR_BIG nodes
  uint64_t bigVmax = 0;              // the largest of them
  uint32_t big_chunks = 1;           // k_csrb_* workgroups per big graph
  bool mark_pending = false;         // holds flags of the tier graphs not yet computed
  bool relax_off = true;             // option build_relax 1: k_build's Kahn levels by relaxation sweeps first
                                     // (measured slower at C3: k_build 2.96 -> 3.20 ms; kept as an option, tested)
  bool ms_fuse_off = true;           // option build_marksimp 1: k_build's marksimp tail (measured slower at C3:
                                     // k_build 3.00 -> 3.86 ms against k_marksimp's 0.80 ms; four workgroups
                                     // per CU by k_build's LDS image where k_marksimp runs eight waves per SIMD)
  bool ms_fused = false;             // k_build's tail wrote its graphs' final flags at the last load / rebuild,
                                     // not yet consumed by nemo_simplify (k_marksimp skips those graphs)

  DevCorpus dc{};
  uint8_t *d_owned = nullptr, *d_is_success = nullptr;
  std::vector<void *> allocs;
  std::unordered_map<void *, size_t> alloc_bytes;  // every live allocation's size (allocs and the cache)
  // blocks of the previous corpus, kept for the next load (nemo_load_corpus frees
  // what it did not reuse): reloading a corpus of the same shape allocates nothing
  std::multimap<size_t, void *> cache;
  uint32_t *d_red = nullptr;

  // diff
  uint32_t n_entries = 0, diff_cap = 0, legacy_cap = 0;
  uint32_t *d_r0lab = nullptr, *d_r0idx = nullptr, n_r0lab = 0;
  uint32_t *d_r0hkey = nullptr, *d_r0hval = nullptr, r0hmask = 0;
  uint32_t *d_r0dense = nullptr, nlab = 0;  // the dense label table of the multi-entry diff (DxArgs::r0dense)
  uint32_t *d_dsrc = nullptr, *d_miss = nullptr, *d_nmiss = nullptr;
  uint8_t *d_dbits = nullptr, *d_dmask = nullptr;
  int32_t *d_ddepth = nullptr;
  uint32_t *d_dtopo = nullptr;       // g0 in Kahn order (DiffArgs::tpos ...)
  uint64_t miss_cap = 0;
  uint64_t mrows_hint = 256, mrows_staged = 0;  // missing rows copied with the D masks (last call's count)
  // entries that share a label source share one computation: n_uniq distinct
  // sources, entry e's result is unique result dmap[e] (d_dmap on the device)
  uint32_t n_uniq = 0, *d_dmap = nullptr;
  uint8_t *d_dumask = nullptr;       // [n_uniq * V0] when n_uniq < n_entries
  std::vector<uint32_t> dmap;
  // CreateNaiveDiffProv reads only the raw run-0 graph and the label sources
  // (differential-provenance.go:22-98), so its kernels run on `aux`, beside
  // the simplification on `stream`; whatever rewrites the graphs' structure,
  // or reads the D masks on `stream`, first waits for ev_diff (join_aux)
  hipStream_t aux = nullptr;
  hipEvent_t ev_fork = nullptr;
  bool aux_pending = false;
  // the multi-entry diff (k_dx.hip): g0's Kahn-order relayout, built with the
  // CSR in every load / rebuild, and the per-call buffers (grow-only)
  nemo::DxPrep dxp{};
  nemo::DxImg dx_img[2]{};           // walk images of g0 (k_dx.hip), built for the test knob dx_img_key
  nemo::DxImgScratch dx_its{};
  int dx_img_key = -1;               // -1: not built for the current load
  bool dx_ok = false;                // relayout allocated: run 0 present, every row fits a window
  int diff_legacy = 0;               // option diff_legacy: one workgroup per entry (k_diff.hip)
  uint32_t diff_window = 0;          // option diff_window (test knob): 0 by size, 1 windowed, 2 tiny windows
  uint32_t diff_unfused = 0;         // option diff_fuse 0 (test knob): whole-graph walks hand LP rules to k_dx_lp / k_dx_emit
  uint32_t g0_maxdeg = 0;
  uint32_t dx_nu_cap = 0, dx_nch_cap = 0;
  uint32_t *d_dxpb = nullptr, *d_dxsval = nullptr, *d_dxlpl = nullptr, *d_dxfb = nullptr;
  uint64_t *d_dxw = nullptr;  // [4][nch][V0] Good / LP, B, D, leaf candidates
  bool dx_last = false;              // the last diffprov ran the multi-entry kernels

  // pulls: per-slot (offset, count) and the region cursor come back to pinned
  // memory asynchronously; the first fetch waits for them
  int pull_which = -1;
  uint32_t pull_slots = 0, pull_slot_cap = 0;
  uint32_t pull_dslots = 0;              // slots computed: diff entries sharing a label source share one
  std::vector<uint32_t> pull_map;        // which 2 with shared slots: entry -> computed slot
  uint32_t *d_pck = nullptr;          // big graphs' pull chunk table
  size_t pull_ck_cap = 0;
  uint32_t *d_pcnt = nullptr, *d_psrc = nullptr, *d_pdst = nullptr;
  uint64_t *d_poff = nullptr, pull_cap = 0;
  unsigned long long *d_pcur = nullptr;
  uint32_t *h_pcnt = nullptr;
  uint64_t *h_poff = nullptr;
  unsigned long long *h_pcur = nullptr;
  uint32_t h_pslot_cap = 0;
  hipEvent_t ev_pull = nullptr;
  bool pull_synced = true;
  uint64_t pull_hint[3] = {0, 0, 0};
  nemo::PullArgs pull_args{};

  // triggers: outputs sized at load from run 0's degrees (exact bounds), one
  // launch; the row counts come back to pinned memory asynchronously
  bool trig_done = false, trig_pending = false;
  uint32_t *d_tcounts = nullptr, *d_tpre = nullptr, *d_tpost = nullptr, *d_tasync = nullptr;
  uint32_t tcounts[3] = {0, 0, 0};
  uint64_t tcap[3] = {0, 0, 0};
  uint32_t *h_tcounts = nullptr;
  hipEvent_t ev_trig = nullptr;

  // pinned result hand-over, written by k_to_host (device -> pinned host)
  uint32_t *h_red = nullptr, *h_tab = nullptr, *h_nmiss = nullptr, *h_mrows = nullptr;
  uint8_t *h_mask = nullptr;
  uint64_t h_red_cap = 0, h_tab_cap = 0, h_nmiss_cap = 0, h_mrows_cap = 0, h_mask_cap = 0;
  uint32_t *h_tpre = nullptr, *h_tpost = nullptr, *h_tasync = nullptr;
  uint64_t h_tpre_cap = 0, h_tpost_cap = 0, h_tasync_cap = 0;
  hipEvent_t ev_protos = nullptr, ev_red = nullptr, ev_diff = nullptr, ev_misc = nullptr;
  const uint32_t *red_staged = nullptr;  // nemo_protos_stage's vector, copied into h_red behind ev_red
  // The global tiers' worklist sizes [load (k_csr/k_topo), chains (k_chains_list/_big), protos
  // (k_pg_*)] of the last full pass.  They are functions of the loaded corpus and the options
  // alone (sizes, Kahn level counts, in-degree caps, chain counts: every pass recomputes the
  // same), so once a pass's counts are known an empty tier is not launched at all (each of its
  // ~10 empty launches cost ~6 us on the analysis stream).  Reset by a load and by any option.
  uint32_t *h_tiers = nullptr;
  hipEvent_t ev_tiers = nullptr;
  bool tiers_pending = false, tiers_ok = false;
  uint32_t tiers[3] = {0, 0, 0}, tiers_run = 0;

  // pinned upload staging (success flags, diff sources): reused once the
  // previous upload from the same buffer has landed (ev_up*)
  uint32_t *d_hlab = nullptr, *h_hlab = nullptr;  // nemo_diffprov_host_labels' set [n, label...]
  uint64_t hlab_cap = 0, h_hlab_cap = 0;
  hipEvent_t ev_up_hlab = nullptr;
  uint8_t *h_succ = nullptr;
  uint32_t *h_dsrc = nullptr;
  uint64_t h_succ_cap = 0, h_dsrc_cap = 0;
  hipEvent_t ev_up_succ = nullptr, ev_up_dsrc = nullptr;

  // chain gather
  uint32_t *d_chout = nullptr;
  uint64_t *d_choff = nullptr, chout_cap = 0;

  // staged simplification results: pinned host copies made on `copy`
  hipStream_t copy = nullptr;
  hipEvent_t ev_ready = nullptr, ev_copied = nullptr;
  // the simplified pull on `aux` (option pull_aux 1; off by default: beside k_proto_lds it made
  // the C3 step 8.3 -> 9.0 ms): it waits for the end of nemo_simplify (ev_simp) only, so it runs
  // beside the protos and hand-over kernels of `stream`; anything that rewrites its inputs
  // first waits for ev_auxpull
  hipEvent_t ev_simp = nullptr, ev_auxpull = nullptr;
  // recorded by nemo_simplify once the node flags are final (after the mark / clean / delete-set
  // kernels, before the chain cover, which only reads them): the staged 2-bit node state is
  // packed and copied from there on, beside the chain cover (nemo_stage_simplified)
  hipEvent_t ev_flags = nullptr, ev_state = nullptr;
  bool flags_final = false;  // ev_flags marks the current flags (no flag-rewriting call since)
  // the hand-over kernels of nemo_stage_simplified on `aux` (option stage_aux, default on):
  // behind everything `stream` has queued so far, beside the triggers and pulls queued after
  hipEvent_t ev_stage = nullptr;
  uint32_t stage_on_aux = 1;
  hipStream_t stage_stream = nullptr;
  bool pull_aux_pending = false;
  uint32_t pull_on_aux = 0;
  bool staged = false;
  uint64_t staged_n = 0, staged_cap = 0, chht_hint = 0;
  bool pairs_wide = false;    // some graph has >= 65536 nodes: u32 pairs
  uint32_t stage_blocks = 0;  // bulk staging: 0 = runtime copies, else k_to_host on this many blocks
  bool stage_sdma = false;    // runtime copies requested as NoCU (SDMA) copies
  uint32_t stage_cus = 8;     // CUs of the copy stream (hipExtStreamCreateWithCUMask); 0 = unmasked
  uint32_t *d_state = nullptr;  // 2-bit node state (k_pack_state)
  uint32_t *d_chht = nullptr;
  uint64_t d_chht_cap = 0;
  uint8_t *h_flags = nullptr;
  uint64_t *h_choff = nullptr;
  uint32_t *h_chht = nullptr;
  uint64_t h_flags_cap = 0, h_choff_cap = 0, h_chht_cap = 0;
};

static void set_lds_tier(nemo_ctx *c);
static void set_global_block(nemo_ctx *c);
static void set_build_tier(nemo_ctx *c);
static int ensure_marked(nemo_ctx *c);

static int fail(nemo_ctx *c, int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return code;
}

#define HIPCHK(c, x)                                                                               \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) return fail((c), NEMO_ERR_HIP, "%s: %s", #x, hipGetErrorString(e_));     \
  } while (0)

// the cached blocks (nemo_ctx::cache)
static void drop_cache(nemo_ctx *c) {
  for (auto &b : c->cache) {
    c->alloc_bytes.erase(b.second);
    hipFree(b.second);
  }
  c->cache.clear();
}

template <class T>
static int dalloc(nemo_ctx *c, T **p, size_t n) {
  void *q = nullptr;
  if (n == 0) n = 1;
  // whole 16-byte chunks: stage_lds (device.h) loads aligned 16-B chunks, so
  // the chunk holding a buffer's last byte must lie inside the allocation
  const size_t bytes = (n * sizeof(T) + 15) & ~(size_t)15;
  auto it = c->cache.lower_bound(bytes);  // the smallest cached block that fits, if not much larger
  if (it != c->cache.end() && it->first <= bytes + bytes / 8 + (1u << 20)) {
    q = it->second;
    c->cache.erase(it);
  } else {
    // large blocks get headroom, so that the next corpus of about the same shape reuses them: 1/16
    // (C5's 143-run batches differ by up to 3.3 % in edges; at 1/32 a load found some block too small
    // about every other time, allocated anew (~28 ms) and the next load's drop_cache freed the unused
    // block: hipFree waits for the whole device, ~220 ms behind the other context's analysis)
    const size_t want = bytes >= (64u << 20) ? ((bytes + bytes / 16) + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1) : bytes;
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t e = hipMalloc(&q, want);
    if (getenv("NEMO_LOAD_DEBUG") && want >= (64u << 20))
      fprintf(stderr, "dalloc: new block %zu MB (%s) %.1f ms, %zu cached\n", want >> 20, e == hipSuccess ? "ok" : "failed",
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(), c->cache.size());
    if (e != hipSuccess) {
      (void)hipGetLastError();
      drop_cache(c);  // no room: the cached blocks go first, then the headroom
      e = hipMalloc(&q, bytes);
      if (e != hipSuccess) return fail(c, NEMO_ERR_HIP, "hipMalloc(%zu bytes): %s", bytes, hipGetErrorString(e));
      c->alloc_bytes[q] = bytes;
    } else {
      c->alloc_bytes[q] = want;
    }
  }
  c->allocs.push_back(q);
  *p = (T *)q;
  return NEMO_OK;
}

template <class T>
static int hgrow(nemo_ctx *c, T **p, uint64_t *cap, uint64_t n) {
  if (n <= *cap && *p) return NEMO_OK;
  if (*p) HIPCHK(c, hipHostFree(*p));
  *p = nullptr;
  *cap = 0;
  HIPCHK(c, hipHostMalloc((void **)p, (n ? n : 1) * sizeof(T), hipHostMallocDefault));
  *cap = n;
  return NEMO_OK;
}

static void dfree(nemo_ctx *c, void *p) {
  if (!p) return;
  auto it = std::find(c->allocs.begin(), c->allocs.end(), p);
  if (it != c->allocs.end()) c->allocs.erase(it);
  c->alloc_bytes.erase(p);
  hipFree(p);
}


static hipEvent_t get_event(nemo_ctx *c) {
  if (!c->ev_pool.empty()) {
    hipEvent_t e = c->ev_pool.back();
    c->ev_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  hipEventCreate(&e);
  return e;
}

// Kernels that rewrite node flags must not overtake a staged copy still in flight.
static int guard_staged(nemo_ctx *c) {
  c->flags_final = false;  // the caller is about to rewrite node flags
  if (c->staged) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_copied, 0));
  if (c->pull_aux_pending) {  // a pull on `aux` still reads the graphs, flags and chains
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_auxpull, 0));
    c->pull_aux_pending = false;
  }
  return NEMO_OK;
}

template <class F>
static int timed_on(nemo_ctx *c, hipStream_t st, const char *name, double bytes, double edges, F &&f) {
  hipEvent_t a = nullptr, b = nullptr;
  const bool timed = c->timing && (c->tgroups.empty() ||
                                   std::find(c->tgroups.begin(), c->tgroups.end(), name) != c->tgroups.end());
  if (timed) {
    a = get_event(c);
    b = get_event(c);
    hipEventRecord(a, st);
  }
  f();
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(c, NEMO_ERR_HIP, "launch %s: %s", name, hipGetErrorString(e));
  if (timed) {
    hipEventRecord(b, st);
    c->pending.push_back({name, a, b, bytes, edges});
    if (c->pending.size() > 4096) {  // bound outstanding events (they may be on two streams)
      for (auto &p : c->pending) hipEventSynchronize(p.b);
      for (auto &p : c->pending) {
        float ms = 0;
        hipEventElapsedTime(&ms, p.a, p.b);
        Agg &g = c->agg[p.name];
        g.launches++;
        g.ms += ms;
        g.bytes += p.bytes;
        g.edges += p.edges;
        c->ev_pool.push_back(p.a);
        c->ev_pool.push_back(p.b);
      }
      c->pending.clear();
    }
  }
  return NEMO_OK;
}

template <class F>
static int timed(nemo_ctx *c, const char *name, double bytes, double edges, F &&f) {
  return timed_on(c, c->stream, name, bytes, edges, f);
}

static int ensure_event(nemo_ctx *c, hipEvent_t *e) {
  if (!*e) HIPCHK(c, hipEventCreateWithFlags(e, hipEventDisableTiming));
  return NEMO_OK;
}

static void tiers_reset(nemo_ctx *c) {
  c->tiers_ok = c->tiers_pending = false;
  c->tiers_run = 0;
}
// tier k's worklist is known to be empty (no launch needed)
static bool tier_empty(nemo_ctx *c, int k) {
  if (!c->tiers_ok && c->tiers_pending && hipEventQuery(c->ev_tiers) == hipSuccess) {
    for (int i = 0; i < 3; i++) c->tiers[i] = c->h_tiers[i];
    c->tiers_ok = true;
    c->tiers_pending = false;
  }
  return c->tiers_ok && c->tiers[k] == 0;
}
// after a pass that launched all three tiers: their list counts to pinned host memory
static int tiers_capture(nemo_ctx *c, hipStream_t s) {
  if (c->tiers_ok || c->tiers_pending || c->tiers_run != 7u || !c->G) return NEMO_OK;
  if (!c->h_tiers) HIPCHK(c, hipHostMalloc((void **)&c->h_tiers, 16));
  int rc;
  if ((rc = ensure_event(c, &c->ev_tiers))) return rc;
  const size_t L = (size_t)c->G + 1;
  nemo::HostCopies hc;
  hc.add(c->h_tiers + 0, c->dc.sel + 2 * L, 4);
  hc.add(c->h_tiers + 1, c->dc.sel + L, 4);
  hc.add(c->h_tiers + 2, c->dc.sel + 3 * L, 4);
  nemo::launch_to_host_multi(hc, s);
  HIPCHK(c, hipEventRecord(c->ev_tiers, s));
  c->tiers_pending = true;
  return NEMO_OK;
}

// `stream` waits for the diff kernels queued on `aux` (see nemo_ctx::aux)
static int join_aux(nemo_ctx *c) {
  if (!c->aux_pending) return NEMO_OK;
  HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_diff, 0));
  c->aux_pending = false;
  return NEMO_OK;
}

static int run_index(nemo_ctx *c, uint32_t it, uint32_t *r) {
  auto f = c->it2run.find(it);
  if (f == c->it2run.end()) return fail(c, NEMO_ERR_NOTFOUND, "unknown run iteration %u", it);
  *r = f->second;
  return NEMO_OK;
}

template <int K>
static void sort_rows(uint32_t *rows, uint64_t n) {
  std::vector<std::array<uint32_t, K>> v(n);
  for (uint64_t i = 0; i < n; i++)
    for (int k = 0; k < K; k++) v[i][k] = rows[K * i + k];
  std::sort(v.begin(), v.end());
  for (uint64_t i = 0; i < n; i++)
    for (int k = 0; k < K; k++) rows[K * i + k] = v[i][k];
}

// ---- accessors for the node context (node.h) ----
Node *ctx_node(const nemo_ctx *c) { return c ? c->node : nullptr; }
nemo_ctx *ctx_new_facade(Node *n) {
  nemo_ctx *c = new nemo_ctx();
  c->node = n;
  return c;
}
void ctx_delete_facade(nemo_ctx *c) { delete c; }
int ctx_fail(nemo_ctx *c, int code, const char *msg) {
  if (c) c->err = msg;
  return code;
}
uint32_t *ctx_reduce_buf(nemo_ctx *c) { return c->d_red; }
hipStream_t ctx_stream(nemo_ctx *c) { return c->stream; }
int ctx_join_aux(nemo_ctx *c) { return join_aux(c); }
int ctx_device(const nemo_ctx *c) { return c->device; }

#define DISPATCH(call)              \
  do {                              \
    if (c && c->node) return call; \
  } while (0)

extern "C" {

int nemo_abi_version(void) { return NEMOHIP_ABI_VERSION; }

int nemo_host_register(const void *ptr, uint64_t bytes) {
  if (!ptr || !bytes) return NEMO_ERR_INVALID;
  return hipHostRegister(const_cast<void *>(ptr), (size_t)bytes, hipHostRegisterDefault) == hipSuccess ? NEMO_OK
                                                                                                       : NEMO_ERR_HIP;
}
int nemo_host_unregister(const void *ptr) {
  if (!ptr) return NEMO_ERR_INVALID;
  return hipHostUnregister(const_cast<void *>(ptr)) == hipSuccess ? NEMO_OK : NEMO_ERR_HIP;
}

// Run sharding: longest-processing-time-first over the runs'
// node + edge counts (both graphs), ties by run index; each run goes to the
// least-loaded part so far (ties by part index).  Deterministic, so every
// rank of a torchrun job and the in-library node context agree.
int nemo_partition_runs(const nemo_corpus *in, uint32_t n_parts, uint32_t *part_of_run) {
  if (!in || !part_of_run || n_parts == 0 || (in->n_runs && (!in->node_off || !in->edge_off))) return NEMO_ERR_INVALID;
  const uint32_t R = in->n_runs;
  std::vector<std::pair<uint64_t, uint32_t>> w(R);
  for (uint32_t r = 0; r < R; r++)
    w[r] = {in->node_off[2 * r + 2] - in->node_off[2 * r] + in->edge_off[2 * r + 2] - in->edge_off[2 * r], r};
  std::sort(w.begin(), w.end(), [](const std::pair<uint64_t, uint32_t> &a, const std::pair<uint64_t, uint32_t> &b) {
    return a.first != b.first ? a.first > b.first : a.second < b.second;
  });
  using Load = std::pair<uint64_t, uint32_t>;  // (load, part): min-heap
  std::vector<Load> heap(n_parts);
  for (uint32_t p = 0; p < n_parts; p++) heap[p] = {0, p};
  auto cmp = [](const Load &a, const Load &b) { return a > b; };
  std::make_heap(heap.begin(), heap.end(), cmp);
  for (auto &x : w) {
    std::pop_heap(heap.begin(), heap.end(), cmp);
    part_of_run[x.second] = heap.back().second;
    heap.back().first += x.first;
    std::push_heap(heap.begin(), heap.end(), cmp);
  }
  return NEMO_OK;
}

int nemo_ctx_create(int device, nemo_ctx **out) {
  if (!out) return NEMO_ERR_INVALID;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return NEMO_ERR_NOGPU;
  if (device < 0 || device >= n) return NEMO_ERR_INVALID;
  nemo_ctx *c = new nemo_ctx();
  c->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return NEMO_ERR_HIP;
  }
  c->stream = c->own;
  *out = c;
  return NEMO_OK;
}

static void release_corpus(nemo_ctx *c) {
  tiers_reset(c);
  c->flags_final = false;
  drop_cache(c);  // blocks no allocation took since the last load
  for (void *p : c->allocs) {  // kept for the next load
    auto b = c->alloc_bytes.find(p);
    if (b != c->alloc_bytes.end()) c->cache.emplace(b->second, p);
    else hipFree(p);
  }
  c->allocs.clear();
  c->dc = DevCorpus{};
  c->d_owned = c->d_is_success = nullptr;
  c->d_red = nullptr;
  c->d_r0lab = c->d_r0idx = c->d_dsrc = c->d_miss = c->d_nmiss = nullptr;
  c->d_r0hkey = c->d_r0hval = nullptr;
  c->r0hmask = 0;
  c->d_r0dense = nullptr;
  c->nlab = 0;
  c->d_dbits = c->d_dmask = nullptr;
  c->d_ddepth = nullptr;
  c->d_dtopo = nullptr;
  c->d_dmap = nullptr;
  c->d_dumask = nullptr;
  c->dxp = nemo::DxPrep{};
  for (auto &m : c->dx_img) m = nemo::DxImg{};
  c->dx_its = nemo::DxImgScratch{};
  c->dx_img_key = -1;
  c->dx_ok = false;
  c->dx_nu_cap = c->dx_nch_cap = 0;
  c->d_dxpb = c->d_dxsval = c->d_dxlpl = c->d_dxfb = nullptr;
  c->d_dxw = nullptr;
  c->n_uniq = 0;
  c->dmap.clear();
  c->aux_pending = false;
  c->n_entries = c->diff_cap = c->legacy_cap = 0;
  c->miss_cap = 0;
  c->d_pcnt = c->d_psrc = c->d_pdst = nullptr;
  c->d_poff = nullptr;
  c->d_pcur = nullptr;
  c->pull_synced = true;
  c->pull_hint[0] = c->pull_hint[1] = c->pull_hint[2] = 0;
  c->pull_cap = 0;
  c->pull_slot_cap = 0;
  c->d_pck = nullptr;
  c->pull_ck_cap = 0;
  c->pull_which = -1;
  c->d_tcounts = c->d_tpre = c->d_tpost = c->d_tasync = nullptr;
  c->d_hlab = nullptr;
  c->hlab_cap = 0;
  c->trig_pending = false;
  c->d_chout = nullptr;
  c->d_choff = nullptr;
  c->chout_cap = 0;
  c->d_chht = nullptr;
  c->d_chht_cap = 0;
  c->chht_hint = 0;
  c->d_state = nullptr;
  c->staged = false;
  c->loaded = c->marked = c->simplified = c->protos_done = c->trig_done = false;
  c->mark_pending = false;
  c->ms_fused = false;
  c->load_check_pending = false;
}

void nemo_ctx_destroy(nemo_ctx *c) {
  if (!c) return;
  if (c->node) {
    node_destroy(c->node);
    ctx_delete_facade(c);
    return;
  }
  hipSetDevice(c->device);
  hipStreamSynchronize(c->stream);
  if (c->copy) hipStreamSynchronize(c->copy);
  if (c->aux) hipStreamSynchronize(c->aux);
  release_corpus(c);
  drop_cache(c);
  for (auto &p : c->pending) {
    hipEventDestroy(p.a);
    hipEventDestroy(p.b);
  }
  for (hipEvent_t e : c->ev_pool) hipEventDestroy(e);
  if (c->copy) {
    hipStreamSynchronize(c->copy);
    hipStreamDestroy(c->copy);
  }
  if (c->ev_ready) hipEventDestroy(c->ev_ready);
  if (c->ev_copied) hipEventDestroy(c->ev_copied);
  if (c->h_flags) hipHostFree(c->h_flags);
  if (c->h_choff) hipHostFree(c->h_choff);
  if (c->h_chht) hipHostFree(c->h_chht);
  if (c->h_pcnt) hipHostFree(c->h_pcnt);
  if (c->h_poff) hipHostFree(c->h_poff);
  if (c->h_pcur) hipHostFree(c->h_pcur);
  if (c->ev_pull) hipEventDestroy(c->ev_pull);
  if (c->ev_trig) hipEventDestroy(c->ev_trig);
  if (c->ev_up_succ) hipEventDestroy(c->ev_up_succ);
  if (c->ev_up_hlab) hipEventDestroy(c->ev_up_hlab);
  if (c->h_hlab) hipHostFree(c->h_hlab);
  if (c->ev_up_dsrc) hipEventDestroy(c->ev_up_dsrc);
  if (c->h_succ) hipHostFree(c->h_succ);
  for (void *h : {(void *)c->h_red, (void *)c->h_tab, (void *)c->h_nmiss, (void *)c->h_mrows, (void *)c->h_mask,
                  (void *)c->h_tpre, (void *)c->h_tpost, (void *)c->h_tasync})
    if (h) hipHostFree(h);
  for (hipEvent_t e : {c->ev_protos, c->ev_red, c->ev_diff, c->ev_misc, c->ev_simp, c->ev_auxpull, c->ev_stage,
                       c->ev_flags, c->ev_state})
    if (e) hipEventDestroy(e);
  if (c->h_dsrc) hipHostFree(c->h_dsrc);
  if (c->h_tcounts) hipHostFree(c->h_tcounts);
  if (c->h_tiers) hipHostFree(c->h_tiers);
  if (c->ev_tiers) hipEventDestroy(c->ev_tiers);
  for (hipEvent_t e : c->ev_up) hipEventDestroy(e);
  if (c->up) {
    hipStreamSynchronize(c->up);
    hipStreamDestroy(c->up);
  }
  if (c->aux) hipStreamDestroy(c->aux);
  if (c->ev_fork) hipEventDestroy(c->ev_fork);
  if (c->own) hipStreamDestroy(c->own);
  delete c;
}

const char *nemo_last_error(const nemo_ctx *c) { return c ? c->err.c_str() : "null context"; }

int nemo_set_stream(nemo_ctx *c, void *stream) {
  DISPATCH(node_set_stream(c, stream));
  if (!c) return NEMO_ERR_INVALID;
  c->stream = stream ? (hipStream_t)stream : c->own;
  return NEMO_OK;
}

int nemo_set_option(nemo_ctx *c, const char *name, int64_t value) {
  DISPATCH(node_set_option(c, name, value));
  if (!c || !name) return NEMO_ERR_INVALID;
  tiers_reset(c);  // any option may move graphs between tiers
  c->ms_fused = false;  // ... and the fused tail's graphs were chosen under the old caps
  if (!strcmp(name, "chains_lds_max")) {
    c->hcap_limit = value < 0 ? 0xFFFFFFFFu : (uint32_t)value;
    c->dc.hcap_limit = c->hcap_limit;
    return NEMO_OK;
  }
  if (!strcmp(name, "build_lds_max")) {
    c->build_limit = value < 0 ? 0xFFFFFFFFu : (uint32_t)value;
    if (c->loaded) set_build_tier(c);
    return NEMO_OK;
  }
  if (!strcmp(name, "graph_lds_max")) {
    if (c->loaded) {
      HIPCHK(c, hipSetDevice(c->device));
      if (int rm = ensure_marked(c)) return rm;  // the deferred set depends on the tier caps
    }
    c->lds_limit = value < 0 ? 0xFFFFFFFFu : (uint32_t)value;
    if (c->loaded) set_lds_tier(c);
    return NEMO_OK;
  }
  if (!strcmp(name, "diff_legacy")) {  // 1: CreateNaiveDiffProv by the one-workgroup-per-entry kernels
    c->diff_legacy = value > 0;
    return NEMO_OK;
  }
  if (!strcmp(name, "diff_window")) {  // test knob of the multi-entry diff's walks: 0, 1 or 2
    if (value < 0 || value > 2) return fail(c, NEMO_ERR_INVALID, "diff_window: 0, 1 or 2");
    c->diff_window = (uint32_t)value;
    return NEMO_OK;
  }
  if (!strcmp(name, "stage_sdma")) {
    c->stage_sdma = value > 0;
    return NEMO_OK;
  }
  if (!strcmp(name, "stage_aux")) {  // 0: the hand-over kernels on the context's stream
    c->stage_on_aux = value != 0;
    return NEMO_OK;
  }
  if (!strcmp(name, "diff_aux")) {  // 0: the diff kernels on the context's stream, in call order
    c->diff_on_aux = value != 0;
    return NEMO_OK;
  }
  if (!strcmp(name, "pull_aux")) {  // 0: pulls on the context's stream, after everything queued before them
    c->pull_on_aux = value != 0;
    return NEMO_OK;
  }
  if (!strcmp(name, "stage_cus")) {  // takes effect when the copy stream is created (first stage)
    c->stage_cus = value < 0 ? 8u : (uint32_t)value;
    return NEMO_OK;
  }
  if (!strcmp(name, "stage_blocks")) {
    c->stage_blocks = value < 0 ? 0u : (uint32_t)value;
    return NEMO_OK;
  }
  if (!strcmp(name, "chains_glob_block")) {  // 0 (by corpus), 256 or 512; takes effect at the next load
    if (value != 0 && value != 256 && value != 512) return fail(c, NEMO_ERR_INVALID, "chains_glob_block: 0, 256 or 512");
    c->glob_block_force = (uint32_t)value;
    return NEMO_OK;
  }
  if (!strcmp(name, "chains_glob_stop")) {  // diagnostic (stamps build only; set after the load): k_chains_glob returns after phase k
    c->dc.glob_stop = value < 0 ? 0u : (uint32_t)value;
    return NEMO_OK;
  }
  if (!strcmp(name, "diff_fuse")) {  // test knob: 0 runs k_dx_lp / k_dx_emit after whole-graph walks too
    c->diff_unfused = value == 0;
    return NEMO_OK;
  }
  if (!strcmp(name, "build_relax")) {  // 1: k_build's Kahn levels by relaxation sweeps first; 0 / -1: peeling
    c->relax_off = value <= 0;
    c->dc.bld_relax = c->relax_off ? 0u : 1u;
    return NEMO_OK;
  }
  if (!strcmp(name, "build_marksimp")) {  // 1: k_build's tail; 0 / -1: k_marksimp takes every tier graph
    c->ms_fuse_off = value <= 0;
    return NEMO_OK;
  }
  if (!strcmp(name, "load_async")) {  // 1: nemo_load_corpus does not wait for its kernels (checks deferred)
    c->load_async = value > 0;
    return NEMO_OK;
  }
  if (!strcmp(name, "load_parts")) {  // big-graph corpora: uploads in this many parts (1: one upload, then the build)
    c->load_parts = value < 1 ? 4u : (uint32_t)std::min<int64_t>(value, 64);
    return NEMO_OK;
  }
  if (!strcmp(name, "topo_ell")) {  // 1: k_topo_ell for the deep graphs (child records); 0 / -1: k_topo_deep
    c->topo_ell_off = value <= 0;
    c->dc.topo_ell = c->topo_ell_off ? 0u : 1u;
    return NEMO_OK;
  }
  if (!strcmp(name, "chains_glob_prep")) {  // 0: no k_glob_prep (the per-graph front phases); takes effect at the next load
    c->glob_prep_off = value == 0;
    return NEMO_OK;
  }
  if (!strcmp(name, "chains_glob_min_v")) {  // takes effect at the next nemo_load_corpus
    c->glob_min_v = value < 0 ? ~0ull : (uint64_t)value;
    return NEMO_OK;
  }
  if (!strcmp(name, "global_block")) {  // 256, 1024, or -1 = by corpus shape (set_global_block)
    if (value != 256 && value != 1024 && value != -1) return fail(c, NEMO_ERR_INVALID, "global_block must be 256, 1024 or -1");
    c->gblock_force = value < 0 ? 0u : (uint32_t)value;
    if (c->loaded) set_global_block(c);
    return NEMO_OK;
  }
  if (!strcmp(name, "chains_comp_max")) {
    c->comp_limit = value < 0 ? 0xFFFFFFFFu : (uint32_t)value;
    c->dc.comp_limit = c->comp_limit;
    return NEMO_OK;
  }
  return fail(c, NEMO_ERR_INVALID, "unknown option %s", name);
}

int nemo_set_timing(nemo_ctx *c, int enable) {
  DISPATCH(node_set_timing(c, enable));
  if (!c) return NEMO_ERR_INVALID;
  c->timing = enable != 0;
  return NEMO_OK;
}

int nemo_set_timing_groups(nemo_ctx *c, const char *groups) {
  DISPATCH(node_set_timing_groups(c, groups));
  if (!c) return NEMO_ERR_INVALID;
  c->tgroups.clear();
  for (const char *p = groups; p && *p;) {
    const char *q = strchr(p, ',');
    const size_t n = q ? (size_t)(q - p) : strlen(p);
    if (n) c->tgroups.emplace_back(p, n);
    p = q ? q + 1 : p + n;
  }
  return NEMO_OK;
}

uint64_t nemo_num_nodes(const nemo_ctx *c) { return c ? (c->node ? node_num_nodes(c) : c->V) : 0; }
uint64_t nemo_num_edges(const nemo_ctx *c) { return c ? (c->node ? node_num_edges(c) : c->E) : 0; }

// Workgroup size of the global-tier kernels: deep corpora (at least one graph
// in eight over 64k nodes) have few graphs per CU and long per-node passes,
// so they get 1024 threads (16 waves of memory-level parallelism per graph);
// corpora of small graphs keep 256 so the early-exit workgroups of the LDS
// tier's graphs stay cheap.
static void set_global_block(nemo_ctx *c) {
  uint32_t deep = 0;
  for (uint32_t g = 0; g < c->G; g++) deep += (c->node_off[g + 1] - c->node_off[g]) >= 65536u;
  c->dc.gblock = c->gblock_force ? c->gblock_force : ((uint64_t)deep * 8u >= c->G && deep ? 1024u : NEMO_BLOCK);
}

// LDS tiers (device.h Tier): for each tiered kernel, the largest graphs,
// smallest first, whose image in that kernel's LDS layout fits LDS_TIER_BUDGET,
// i.e. two workgroups per CU.  Graphs outside a kernel's caps run its
// global-memory variant.  `graph_lds_max` caps V of every tier (test knob).
#define LDS_TIER_BUDGET (78u * 1024u)
#define NO_LEVEL_CAP 0xFFFFFFFFu
typedef uint32_t (*TierBytes)(uint32_t v, uint32_t e, uint32_t l, uint32_t words);
static Tier fit_tier(nemo_ctx *c, uint64_t vmax, uint64_t emax, uint32_t lcap, TierBytes bytes,
                     uint32_t budget = LDS_TIER_BUDGET) {
  std::vector<std::pair<uint32_t, uint32_t>> ve;
  ve.reserve(c->G);
  for (uint32_t g = 0; g < c->G; g++) {
    const uint64_t v = c->node_off[g + 1] - c->node_off[g], e = c->edge_off[g + 1] - c->edge_off[g];
    if (v <= std::min<uint64_t>(vmax, c->lds_limit) && e <= emax) ve.push_back({(uint32_t)v, (uint32_t)e});
  }
  std::sort(ve.begin(), ve.end());
  uint32_t cv = 0, ce = 0, em = 0;
  for (auto &x : ve) {
    em = std::max(em, x.second);
    const uint32_t l = std::min(x.first, lcap);
    if (bytes(x.first, em, l, c->W) > budget) break;
    cv = x.first;
    ce = em;
  }
  Tier t{0, 0, 0, 0};
  if (!cv) return t;
  t.v = cv;
  t.e = ce;
  t.l = std::min(cv, lcap);
  t.bytes = bytes(cv, ce, t.l, c->W);
  return t;
}

static void set_lds_tier(nemo_ctx *c) {
  // k_proto_lds: edges in source Kahn order + level offsets (<= 512 levels), node bytes, chains; three
  // 512-thread workgroups per CU
  const Tier tp = fit_tier(
      c, 16384, 65535, 512u,
      [](uint32_t v, uint32_t e, uint32_t l, uint32_t w) { return lds_tier_bytes(v, e, l, w); },
      160u * 1024u / 3u - 256u);
  c->dc.lds_v = tp.v;
  c->dc.lds_e = tp.e;
  c->dc.lds_l = tp.l;
  c->dc.lds_bytes = tp.bytes;
  // k_marksimp: node word + two node bytes (the edge list stays in registers / HBM); (src << 16 | dst) pairs
  c->dc.t_ms = fit_tier(c, 16384, 65535, NO_LEVEL_CAP, [](uint32_t v, uint32_t, uint32_t, uint32_t w) {
    return marksimp_bytes(v, w);
  });
  // k_diff_lds: u16 CSR both ways + rule bitmap + node bits (Kahn order and depths stay in HBM)
  c->dc.t_diff = fit_tier(c, 16384, 65535, NO_LEVEL_CAP, [](uint32_t v, uint32_t e, uint32_t l, uint32_t) {
    return diff_lds_bytes(v, e, l);
  });
  // k_pull_lds: forward u16 CSR + liveness bitmap (per-node counts in registers: 24 nodes per thread)
  c->dc.t_pull = fit_tier(c, 24u * 256u, 65535, NO_LEVEL_CAP, [](uint32_t v, uint32_t e, uint32_t, uint32_t) {
    return pull_lds_bytes(v, e);
  });
  c->tierV = c->tierE = 0;  // k_marksimp's graphs (the deferred markConditionHolds)
  c->ms_rest = c->pull_rest = 0;  // graphs the per-graph global-tier kernels must take (none: not launched)
  for (uint32_t g = 0; g < c->G; g++) {
    const uint64_t v = c->node_off[g + 1] - c->node_off[g], e = c->edge_off[g + 1] - c->edge_off[g];
    const bool ms = tier_fits(c->dc.t_ms, (uint32_t)std::min<uint64_t>(v, ~0u), (uint32_t)std::min<uint64_t>(e, ~0u), 0);
    if (ms) {
      c->tierV += (double)v;
      c->tierE += (double)e;
    } else if (v < NEMO_CSR_BIG) {
      c->ms_rest++;
    }
    if (!tier_fits(c->dc.t_pull, (uint32_t)std::min<uint64_t>(v, ~0u), (uint32_t)std::min<uint64_t>(e, ~0u), 0))
      c->pull_rest++;
  }
}

// k_build's LDS caps: the largest graphs, smallest first, whose build image
// (k_load.hip build_tier_bytes) keeps four workgroups on a CU.
#define BUILD_TIER_BUDGET (160u * 1024u / 4u - 64u)
static void set_build_tier(nemo_ctx *c) {
  std::vector<std::pair<uint32_t, uint32_t>> ve;
  ve.reserve(c->G);
  for (uint32_t g = 0; g < c->G; g++) {
    const uint64_t v = c->node_off[g + 1] - c->node_off[g], e = c->edge_off[g + 1] - c->edge_off[g];
    if (v <= std::min<uint64_t>(16384, c->build_limit) && e <= 32u * NEMO_BLOCK) ve.push_back({(uint32_t)v, (uint32_t)e});
  }
  std::sort(ve.begin(), ve.end());
  uint32_t cv = 0, ce = 0, emax = 0;
  for (auto &x : ve) {
    emax = std::max(emax, x.second);
    if (nemo::build_tier_bytes(x.first, emax) > BUILD_TIER_BUDGET) break;
    cv = x.first;
    ce = emax;
  }
  c->dc.bld_v = cv;
  c->dc.bld_e = ce;
  c->dc.bld_bytes = cv ? nemo::build_tier_bytes(cv, ce) : 0;
}

static int check_graph_errors(nemo_ctx *c) {
  std::vector<uint32_t> err(c->G), created(c->G);
  HIPCHK(c, hipMemcpyAsync(err.data(), c->dc.err, c->G * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(created.data(), c->dc.created, c->G * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (uint32_t g = 0; g < c->G; g++) {
    if (!err[g]) continue;
    const uint32_t it = c->iteration[g / 2];
    const uint64_t E = c->edge_off[g + 1] - c->edge_off[g];
    if (err[g] == NEMO_ERR_LOAD)
      return fail(c, NEMO_ERR_LOAD,
                  "Run %u: inserted number of edges (%u) does not equal number of antecedent provenance edges (%llu)",
                  it, created[g], (unsigned long long)E);
    if (err[g] == NEMO_ERR_CYCLE) return fail(c, NEMO_ERR_CYCLE, "Run %u: provenance graph is not acyclic", it);
    return fail(c, (int)err[g], "Run %u: edge references a node index out of range", it);
  }
  return NEMO_OK;
}

// Option load_async: the last load's graph checks (validations, acyclicity), before the first call
// that reads its graphs; a failed check leaves no corpus loaded, as a failed nemo_load_corpus does.
static int ensure_load_checked(nemo_ctx *c) {
  if (!c->load_check_pending) return NEMO_OK;
  c->load_check_pending = false;
  const int rc = check_graph_errors(c);
  if (rc) c->loaded = false;
  return rc;
}

// Upload parts of a corpus whose edges are mostly big graphs (nemo_load_corpus, option load_parts):
// part k = the big-list entries [b0, b1) and the edge range [e0, e1) of the graphs from big[b0] up
// to the next part's first big graph (every edge in exactly one part).
struct LoadPart {
  uint32_t b0, b1;
  uint64_t e0, e1;
};
struct LoadParts {
  std::vector<LoadPart> part;
  const uint32_t *src = nullptr, *dst = nullptr;  // the caller's edge arrays (host)
  uint32_t *es = nullptr, *ed = nullptr;          // their device copies
};

// With parts, part k's edges are copied on the upload stream and its big graphs' CSR build
// (k_csrb) is queued behind that copy alone; the host issues part k + 1's copy after queueing part
// k's kernels.  A copy from page-locked memory holds the issuing thread until it is done (~200 ms
// for a C5 batch's edges, measured), so issuing every copy first left no kernel to overlap them
// with.  The rest of the load (k_build, k_csr, the Kahn levels) runs behind the last part: the
// deep graphs' k_topo_deep is per-graph latency (~74 ms for any number of graphs), so one launch
// per part took 4 x 70 ms.
static int device_load(nemo_ctx *c, const LoadParts *lp = nullptr) {
  int rc;
  const bool split = c->dc.n_big && lp && lp->part.size() > 1;
  nemo::launch_zero(c->dc.err, c->G * sizeof(uint32_t), c->stream);
  if (split) {
    for (size_t k = 0; k < lp->part.size(); k++) {
      const LoadPart &q = lp->part[k];
      if (q.e1 > q.e0) {
        HIPCHK(c, hipMemcpyAsync(lp->es + q.e0, lp->src + q.e0, (q.e1 - q.e0) * 4, hipMemcpyHostToDevice, c->up));
        HIPCHK(c, hipMemcpyAsync(lp->ed + q.e0, lp->dst + q.e0, (q.e1 - q.e0) * 4, hipMemcpyHostToDevice, c->up));
      }
      HIPCHK(c, hipEventRecord(c->ev_up[k], c->up));
      HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_up[k], 0));
      if (q.b1 == q.b0) continue;
      DevCorpus sc = c->dc;
      sc.big = c->dc.big + q.b0;
      sc.cb_hoff = c->dc.cb_hoff + q.b0;
      sc.n_big = q.b1 - q.b0;
      const double f = (double)sc.n_big / (double)c->dc.n_big;
      if ((rc = timed(c, "k_csrb", f * (16 * c->bigE + 12 * c->bigV), f * c->bigE,
                      [&] { nemo::launch_csr_big(sc, c->big_chunks, c->stream); })))
        return rc;
    }
  }
  // graphs within k_build's LDS caps vs the global tier
  double Vb = 0, Eb = 0, Vp = 0, Ep = 0;
  for (uint32_t g = 0; g < c->G && c->dc.bld_bytes; g++) {
    const uint64_t v = c->node_off[g + 1] - c->node_off[g], e = c->edge_off[g + 1] - c->edge_off[g];
    if (v <= c->dc.bld_v && e <= c->dc.bld_e) {
      Vb += (double)v;
      Eb += (double)e;
      if (g & 1) {
        Vp += (double)v;
        Ep += (double)e;
      }
    }
  }
  const double V = (double)c->V - Vb, E = (double)c->E - Eb;
  // k_build's tail runs the deferred mark + simplification (k_marksimp's work) on the edges still
  // in its registers when every k_build graph fits the tail's LDS image
  c->dc.ms_fuse = !c->ms_fuse_off && c->dc.t_ms.bytes && c->dc.bld_bytes &&
                  marksimp_bytes(c->dc.bld_v, c->dc.words) <= c->dc.bld_bytes;
  // k_build, HBM lower bound: read the edge list (8E) and node words (4V);
  // write both column arrays (8E), both row-pointer arrays (8V), the Kahn
  // order (4V) and per-node level (4V); the level offsets are per level; post
  // graphs also their edges in source Kahn order (4E) and position offsets (4V);
  // with the tail, the node flags (1V)
  if ((rc = timed(c, "k_build", 16 * Eb + (c->dc.ms_fuse ? 21 : 20) * Vb + 4 * Ep + 4 * Vp, 2 * Eb,
                  [&] { nemo::launch_build(c->dc, c->stream); })))
    return rc;
  c->ms_fused = c->dc.ms_fuse != 0;
  // graphs past k_build: k_csr (one workgroup per graph) below NEMO_CSR_BIG nodes, k_csrb_* above
  const double Eg = std::max(0.0, E - c->bigE), Vg = std::max(0.0, V - c->bigV);
  const bool load_tier = !tier_empty(c, 0);
  if (load_tier && (rc = timed(c, "k_csr", 16 * Eg + 12 * Vg, Eg, [&] { nemo::launch_load(c->dc, c->stream); })))
    return rc;
  if (load_tier) c->tiers_run |= 1u;
  if (c->dc.n_big && !split &&
      (rc = timed(c, "k_csrb", 16 * c->bigE + 12 * c->bigV, c->bigE,
                  [&] { nemo::launch_csr_big(c->dc, c->big_chunks, c->stream); })))
    return rc;
  if ((rc = timed(c, "k_topo", 4 * E + 16 * V, E, [&] { nemo::launch_topo(c->dc, c->stream, load_tier); })))
    return rc;
  // the multi-entry diff's relayout of run 0's post graph and its walk images
  // are built by the first diffprov after a load (nemo_rebuild re-derives the
  // same graph: a relayout built from an earlier Kahn order of it stays valid)
  return NEMO_OK;
}

int nemo_load_corpus(nemo_ctx *c, const nemo_corpus *in) {
  DISPATCH(node_load_corpus(c, in));
  if (!c || !in) return NEMO_ERR_INVALID;
  const bool dbg = getenv("NEMO_LOAD_DEBUG") != nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  auto ms_since = [&] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->copy) HIPCHK(c, hipStreamSynchronize(c->copy));
  if (c->aux) HIPCHK(c, hipStreamSynchronize(c->aux));
  if (c->up) HIPCHK(c, hipStreamSynchronize(c->up));
  release_corpus(c);
  const double t_rel = ms_since();
  if (in->n_tables > NEMO_MAX_TABLES)
    return fail(c, NEMO_ERR_LIMIT, "%u tables exceed NEMO_MAX_TABLES (%u)", in->n_tables, NEMO_MAX_TABLES);
  if (!in->iteration || !in->node_off || !in->edge_off || (!in->node_word && in->n_runs))
    return fail(c, NEMO_ERR_INVALID, "corpus arrays missing");
  c->n_runs = in->n_runs;
  c->G = 2 * in->n_runs;
  c->T = in->n_tables;
  c->W = (in->n_tables + 31) / 32;
  c->table_pre = in->table_pre;
  c->table_post = in->table_post;
  c->iteration.assign(in->iteration, in->iteration + in->n_runs);
  c->owned.assign(in->n_runs, 1);
  if (in->owned)
    for (uint32_t r = 0; r < in->n_runs; r++) c->owned[r] = in->owned[r] ? 1 : 0;
  c->node_off.assign(in->node_off, in->node_off + c->G + 1);
  c->edge_off.assign(in->edge_off, in->edge_off + c->G + 1);
  c->V = c->node_off[c->G];
  c->E = c->edge_off[c->G];
  c->postV = c->postE = 0;
  for (uint32_t g = 1; g < c->G; g += 2) {
    c->postV += (double)(c->node_off[g + 1] - c->node_off[g]);
    c->postE += (double)(c->edge_off[g + 1] - c->edge_off[g]);
  }
  c->it2run.clear();
  c->run0 = -1;
  for (uint32_t r = 0; r < c->n_runs; r++) {
    if (c->it2run.count(c->iteration[r]))
      return fail(c, NEMO_ERR_INVALID, "duplicate run iteration %u", c->iteration[r]);
    c->it2run[c->iteration[r]] = r;
    if (c->iteration[r] == 0) c->run0 = (int32_t)r;
  }
  for (uint32_t g = 0; g < c->G; g++) {
    if (c->node_off[g + 1] < c->node_off[g] || c->edge_off[g + 1] < c->edge_off[g])
      return fail(c, NEMO_ERR_INVALID, "offsets not monotone at graph %u", g);
    if (c->node_off[g + 1] - c->node_off[g] >= 0xFFFFFFF0ull || c->edge_off[g + 1] - c->edge_off[g] >= 0xFFFFFFF0ull)
      return fail(c, NEMO_ERR_LIMIT, "graph %u exceeds 2^32 nodes/edges", g);
  }
  if (c->node_off[0] != 0 || c->edge_off[0] != 0) return fail(c, NEMO_ERR_INVALID, "offsets must start at 0");
  c->has_rank = in->id_rank != nullptr;
  c->pairs_wide = false;
  for (uint32_t g = 0; g < c->G; g++) c->pairs_wide |= c->node_off[g + 1] - c->node_off[g] >= 65536;
  const size_t V = c->V, E = c->E, G = c->G, R = c->n_runs;
  DevCorpus &d = c->dc;
  int rc = 0;
  uint64_t *no, *eo;
  uint32_t *word, *label, *rank = nullptr, *es, *ed;
#define A(p, n) \
  if ((rc = dalloc(c, &(p), (n)))) return rc
  A(no, G + 1);
  A(eo, G + 1);
  A(word, V);
  A(label, V);
  if (c->has_rank) A(rank, V);
  A(es, E);
  A(ed, E);
  A(d.fp, V + G);
  A(d.rp, V + G);
  A(d.fc, E);
  A(d.rc, E);
  A(d.topo, V);
  A(d.lvl, V + G);
  A(d.nlv, V);
  A(d.e2, E);
  A(d.posoff, V);
  A(d.nlev, G);
  A(d.flags, V);
  A(d.sb, V);
  A(d.s_a, V + G);
  A(d.s_b, V + G);
  A(d.s_c, V + G);
  A(d.s_d, V);
  A(d.s_e, V);
  A(d.s_f, V + G);
  A(d.s_g, V + G);
  A(d.err, G);
  A(d.created, G);
  A(d.prehold, G);
  A(d.holdany, G);
  A(d.redo, G);
  {
    // deep graphs (V >= glob_min_v): k_chains_glob's per-graph scratch regions
    std::vector<uint64_t> off(G, ~0ull);
    uint64_t words = 0;
    for (uint32_t g = 0; g < G; g++) {
      const uint64_t v = c->node_off[g + 1] - c->node_off[g], e = c->edge_off[g + 1] - c->edge_off[g];
      if (v >= c->glob_min_v && v > 0) {
        off[g] = words;
        words += (nemo::glob_words(v, e) + 63) & ~63ull;
      }
    }
    uint64_t *goff;
    A(goff, G);
    HIPCHK(c, hipMemcpy(goff, off.data(), G * 8, hipMemcpyHostToDevice));
    d.gs_off = goff;
    // a few deep graphs: 512 threads each (their parallel phases go faster); many (more
    // than two per CU): 256, so that up to four share a CU
    uint32_t n_deep = 0;
    for (uint32_t g = 0; g < G; g++) n_deep += off[g] != ~0ull;
    d.glob_block = c->glob_block_force ? c->glob_block_force : (n_deep > 512 ? 256u : 512u);
    d.gscratch = nullptr;
    if (words) A(d.gscratch, words);
    // k_glob_prep's graph list and team scratch (identity ranks only)
    std::vector<uint32_t> gl;
    for (uint32_t g = 0; g < G; g++)
      if (off[g] != ~0ull) gl.push_back(g);
    uint32_t *dgl = nullptr;
    A(dgl, gl.size());
    if (!gl.empty()) HIPCHK(c, hipMemcpy(dgl, gl.data(), gl.size() * 4, hipMemcpyHostToDevice));
    d.glob_list = dgl;
    d.n_glob = (uint32_t)gl.size();
    d.glob_prep = !gl.empty() && !c->has_rank && !c->glob_prep_off;
    d.topo_ell = c->topo_ell_off ? 0u : 1u;
    d.bld_relax = c->relax_off ? 0u : 1u;
    d.team = nullptr;
    A(d.team, nemo::glob_team_words());
    int ncu = 0;
    HIPCHK(c, hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device));
    d.n_cu = (uint32_t)std::max(ncu, 8);
  }
  A(d.chain, 5 * V);
  {
    // k_chains' per-graph scratch (5 words per node), for the graphs k_chains_glob
    // does not take (those keep theirs in the glob scratch)
    std::vector<uint64_t> off(G, 0);
    uint64_t words = 0;
    for (uint32_t g = 0; g < G; g++) {
      const uint64_t v = c->node_off[g + 1] - c->node_off[g];
      off[g] = words;
      if (!(v >= c->glob_min_v && v > 0)) words += 5 * v;
    }
    uint64_t *toff;
    A(toff, G);
    HIPCHK(c, hipMemcpy(toff, off.data(), G * 8, hipMemcpyHostToDevice));
    d.tmp_off = toff;
    A(d.chain_tmp, words);
  }
  A(d.nch, G);
  A(d.sel, 4 * ((size_t)G + 1));
  {
    // graphs of NEMO_CSR_BIG nodes or more: the multi-workgroup CSR build's list
    std::vector<uint32_t> big;
    uint64_t emax = 0;
    c->bigV = c->bigE = 0;
    c->bigVmax = 0;
    for (uint32_t g = 0; g < G; g++) {
      const uint64_t v = c->node_off[g + 1] - c->node_off[g], e = c->edge_off[g + 1] - c->edge_off[g];
      if (v < NEMO_CSR_BIG) continue;
      big.push_back(g);
      emax = std::max(emax, e);
      c->bigV += (double)v;
      c->bigVmax = std::max<uint64_t>(c->bigVmax, v);
      c->bigE += (double)e;
    }
    uint32_t *db = nullptr;
    A(db, big.size());
    if (!big.empty()) HIPCHK(c, hipMemcpy(db, big.data(), big.size() * 4, hipMemcpyHostToDevice));
    d.big = db;
    d.n_big = (uint32_t)big.size();
    c->big_host = big;
    // the bucketed build's (bucket, chunk) count tables and (key, value) edge scratch
    d.cb_hist = d.cb_key = d.cb_val = nullptr;
    d.cb_hoff = nullptr;
    d.cb_maxbk = d.cb_maxck = 0;
    std::vector<uint64_t> hoff(big.size() + 1, 0);
    bool fits = !big.empty();
    for (size_t b = 0; b < big.size(); b++) {
      const uint32_t g = big[b];
      const uint64_t v = c->node_off[g + 1] - c->node_off[g], e = c->edge_off[g + 1] - c->edge_off[g];
      const uint64_t nbk = (v + CB_NB - 1) / CB_NB, nck = (e + CB_CHUNK - 1) / CB_CHUNK;
      fits &= nbk <= CB_MAXB;
      hoff[b + 1] = hoff[b] + std::max<uint64_t>(nbk * nck, 1);
      d.cb_maxbk = std::max<uint32_t>(d.cb_maxbk, (uint32_t)nbk);
      d.cb_maxck = std::max<uint32_t>(d.cb_maxck, (uint32_t)std::max<uint64_t>(nck, 1));
    }
    if (fits) {
      uint64_t *dh = nullptr;
      A(dh, hoff.size());
      HIPCHK(c, hipMemcpy(dh, hoff.data(), hoff.size() * 8, hipMemcpyHostToDevice));
      d.cb_hoff = dh;
      A(d.cb_hist, hoff.back());
      // keys: e2's slots (k_build writes e2 only for the graphs it builds, the
      // bucketed build takes only the others: disjoint edge ranges)
      d.cb_key = d.e2;
      A(d.cb_val, E);
    }
    c->big_chunks = (uint32_t)std::min<uint64_t>(128, std::max<uint64_t>(1, (emax + 16383) / 16384));
    uint64_t vpost = 0;  // k_pg_* chunks: the largest post graph
    for (uint32_t g = 1; g < G; g += 2) vpost = std::max<uint64_t>(vpost, c->node_off[g + 1] - c->node_off[g]);
    d.pg_chunks = (uint32_t)std::min<uint64_t>(64, std::max<uint64_t>(1, vpost / 16384));
  }
  A(d.cl_first, V);
  A(d.cl_next, V);
  A(d.proto_bits, R * c->W);
  A(d.graph_tables, R * c->W);
  A(d.gate, R);
  A(c->d_owned, R);
  A(c->d_is_success, R);
  A(c->d_red, 2 * (size_t)c->T + 4);
#ifdef NEMO_STAMPS
  A(d.stamps, 16 * G);
  HIPCHK(c, hipMemsetAsync(d.stamps, 0, 16 * G * 8, c->stream));
#endif
#undef A
  hipStream_t s = c->stream;
  HIPCHK(c, hipMemcpyAsync(no, in->node_off, (G + 1) * 8, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemcpyAsync(eo, in->edge_off, (G + 1) * 8, hipMemcpyHostToDevice, s));
  if (V) {
    HIPCHK(c, hipMemcpyAsync(word, in->node_word, V * 4, hipMemcpyHostToDevice, s));
    HIPCHK(c, hipMemcpyAsync(label, in->label, V * 4, hipMemcpyHostToDevice, s));
    if (rank) HIPCHK(c, hipMemcpyAsync(rank, in->id_rank, V * 4, hipMemcpyHostToDevice, s));
  }
  // a corpus whose edges are mostly in big graphs outside k_build's caps (the deep configs) uploads
  // them in parts from device_load, each part's CSR build and Kahn levels behind its own copy
  d.G = c->G;
  set_build_tier(c);
  LoadParts lp;
  {
    const uint32_t P = c->load_parts;
    bool ok = E && d.cb_hist && P > 1 && d.n_big >= 2 * P && c->topo_ell_off && c->bigE >= 0.5 * (double)E;
    for (uint32_t b = 0; b < d.n_big && ok; b++) {  // no big graph of k_build's (its redo flag comes later)
      const uint32_t g = c->big_host[b];
      const uint64_t v = c->node_off[g + 1] - c->node_off[g], e = c->edge_off[g + 1] - c->edge_off[g];
      ok = !(d.bld_bytes && v <= d.bld_v && e <= d.bld_e);
    }
    if (ok) {
      if (!c->up) HIPCHK(c, hipStreamCreateWithFlags(&c->up, hipStreamNonBlocking));
      while (c->ev_up.size() < P) {
        hipEvent_t e = nullptr;
        HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        c->ev_up.push_back(e);
      }
      for (uint32_t k = 0; k < P; k++) {
        LoadPart q;
        q.b0 = (uint32_t)((uint64_t)d.n_big * k / P);
        q.b1 = (uint32_t)((uint64_t)d.n_big * (k + 1) / P);
        q.e0 = k ? c->edge_off[c->big_host[q.b0]] : 0;
        q.e1 = k + 1 < P ? c->edge_off[c->big_host[q.b1]] : E;
        lp.part.push_back(q);
      }
      lp.src = in->edge_src;
      lp.dst = in->edge_dst;
      lp.es = es;
      lp.ed = ed;
    }
  }
  if (lp.part.empty() && E) {
    HIPCHK(c, hipMemcpyAsync(es, in->edge_src, E * 4, hipMemcpyHostToDevice, s));
    HIPCHK(c, hipMemcpyAsync(ed, in->edge_dst, E * 4, hipMemcpyHostToDevice, s));
  }
  if (dbg)
    fprintf(stderr, "nemo_load_corpus: E %zu n_big %u G %zu cb_hist %d load_parts %u -> %zu parts; sync+release %.1f ms, +alloc %.1f ms\n",
            E, d.n_big, G, d.cb_hist != nullptr, c->load_parts, lp.part.size(), t_rel, ms_since());
  HIPCHK(c, hipMemcpyAsync(c->d_owned, c->owned.data(), R, hipMemcpyHostToDevice, s));
  HIPCHK(c, hipMemsetAsync(d.nch, 0, G * 4, s));
  HIPCHK(c, hipMemsetAsync(d.prehold, 0, G * 4, s));
  d.hcap_limit = c->hcap_limit;
  d.comp_limit = c->comp_limit;
  set_lds_tier(c);
  set_global_block(c);
  d.n_runs = c->n_runs;
  d.n_tables = c->T;
  d.words = c->W;
  d.table_pre = c->table_pre;
  d.table_post = c->table_post;
  d.node_off = no;
  d.edge_off = eo;
  d.word = word;
  d.label = label;
  d.rank = rank;
  d.esrc = es;
  d.edst = ed;
  // run 0's post goal labels, sorted, for the diff's failGoals lookup
  if (c->run0 >= 0) {
    const uint32_t g0 = 2 * c->run0 + 1;
    std::vector<std::pair<uint32_t, uint32_t>> lab;
    for (uint64_t v = c->node_off[g0]; v < c->node_off[g0 + 1]; v++)
      if (!(in->node_word[v] & NEMO_NODE_RULE)) lab.push_back({in->label[v], (uint32_t)(v - c->node_off[g0])});
    std::sort(lab.begin(), lab.end());
    std::vector<uint32_t> l(lab.size()), ix(lab.size());
    for (size_t i = 0; i < lab.size(); i++) {
      l[i] = lab[i].first;
      ix[i] = lab[i].second;
    }
    c->n_r0lab = (uint32_t)lab.size();
    // label -> first sorted entry, open-addressed at load factor <= 1/2, so a
    // lookup is one or two independent probes instead of a binary search
    uint32_t hcap = 16;
    while (hcap < 2 * lab.size()) hcap <<= 1;
    std::vector<uint32_t> hkey(hcap, 0u), hval(hcap, 0u);
    for (size_t i = 0; i < l.size(); i++) {
      if (i && l[i] == l[i - 1]) continue;
      uint32_t h = hash_label(l[i]) & (hcap - 1);
      while (hkey[h]) h = (h + 1) & (hcap - 1);
      hkey[h] = l[i] + 1u;
      hval[h] = (uint32_t)i;
    }
    c->r0hmask = hcap - 1;
    if ((rc = dalloc(c, &c->d_r0lab, l.size()))) return rc;
    if ((rc = dalloc(c, &c->d_r0idx, l.size()))) return rc;
    if ((rc = dalloc(c, &c->d_r0hkey, hcap))) return rc;
    if ((rc = dalloc(c, &c->d_r0hval, hcap))) return rc;
    HIPCHK(c, hipMemcpyAsync(c->d_r0hkey, hkey.data(), hcap * 4, hipMemcpyHostToDevice, s));
    HIPCHK(c, hipMemcpyAsync(c->d_r0hval, hval.data(), hcap * 4, hipMemcpyHostToDevice, s));
    // the same as a dense table over the label ids up to run 0's largest goal label (a source label
    // past it is no run-0 goal label), when that is at most 256M entries: one load per source goal
    // instead of a probe sequence
    const uint64_t nlab = l.empty() ? 0 : (uint64_t)l.back() + 1;  // l: run 0's goal labels, sorted
    std::vector<uint32_t> dense;
    if (nlab && nlab <= (1ull << 28)) {
      dense.assign(nlab, NEMO_NONE);
      for (size_t i = 0; i < l.size();) {
        size_t j = i;
        while (j < l.size() && l[j] == l[i]) j++;
        dense[l[i]] = (uint32_t)(i << 4) | (uint32_t)std::min<size_t>(j - i, 15);
        i = j;
      }
      if ((rc = dalloc(c, &c->d_r0dense, nlab))) return rc;
      HIPCHK(c, hipMemcpyAsync(c->d_r0dense, dense.data(), nlab * 4, hipMemcpyHostToDevice, s));
      c->nlab = (uint32_t)nlab;
    }
    if (!l.empty()) {
      HIPCHK(c, hipMemcpyAsync(c->d_r0lab, l.data(), l.size() * 4, hipMemcpyHostToDevice, s));
      HIPCHK(c, hipMemcpyAsync(c->d_r0idx, ix.data(), ix.size() * 4, hipMemcpyHostToDevice, s));
    }
    HIPCHK(c, hipStreamSynchronize(s));  // host vectors go out of scope
    // the multi-entry diff's relayout of g0: every row must fit one walk window
    const uint64_t n0 = c->node_off[g0], nv = c->node_off[g0 + 1] - n0;
    const uint64_t e0 = c->edge_off[g0], ne = c->edge_off[g0 + 1] - e0;
    std::vector<uint32_t> din(nv, 0), dout(nv, 0);
    uint32_t maxdeg = 0;
    for (uint64_t e = e0; e < e0 + ne; e++) {
      if (in->edge_src[e] < nv) maxdeg = std::max(maxdeg, ++dout[in->edge_src[e]]);
      if (in->edge_dst[e] < nv) maxdeg = std::max(maxdeg, ++din[in->edge_dst[e]]);
    }
    c->dx_ok = nv > 0 && nv < 0xFFFFFFFFull && maxdeg <= nemo::dx_max_row();
    c->g0_maxdeg = maxdeg;
    if (c->dx_ok) {
      nemo::DxPrep &p = c->dxp;
      p.g0 = g0;
      p.V0 = (uint32_t)nv;
      p.E0 = (uint32_t)ne;
      p.r0idx = c->d_r0idx;
      p.n_r0lab = c->n_r0lab;
      p.err0 = nullptr;  // set at the first diffprov (the error flags are allocated with the corpus)
      p.r0lab = c->d_r0lab;
      p.r0dense = nv < (1ull << 28) ? c->d_r0dense : nullptr;  // positions << 4 must fit
      if ((rc = dalloc(c, &p.tpos, nv)) || (rc = dalloc(c, &p.pnode, nv)) || (rc = dalloc(c, &p.info, nv)) || (rc = dalloc(c, &p.lbeg, nv)) ||
          (rc = dalloc(c, &p.lend, nv)) || (rc = dalloc(c, &p.rp, nv + 1)) || (rc = dalloc(c, &p.fp, nv + 1)) ||
          (rc = dalloc(c, &p.rc, ne + 4)) || (rc = dalloc(c, &p.fc, ne + 4)) || (rc = dalloc(c, &p.r0pos, l.size())))
        return rc;
      for (nemo::DxImg &m : c->dx_img)
        if ((rc = dalloc(c, &m.nw, 1)) || (rc = dalloc(c, &m.wb, nv + 2)) || (rc = dalloc(c, &m.stepb, nv + 2)) ||
            (rc = dalloc(c, &m.steps, 2 * nv + ne / 256 + 4)) || (rc = dalloc(c, &m.rec, ne + 4)) ||
            (rc = dalloc(c, &m.moff, nv + 1)) || (rc = dalloc(c, &m.mx, ne + 1)))
          return rc;
      nemo::DxImgScratch &t = c->dx_its;
      if ((rc = dalloc(c, &t.fseg, nv + 1)) || (rc = dalloc(c, &t.segpos, nv + 2)) ||
          (rc = dalloc(c, &t.fstep, nv + 1)) ||
          (rc = dalloc(c, &t.tsum, nemo::dx_scan_tiles((uint32_t)std::max(nv, ne) + 1))))
        return rc;
    }
  }
  // trigger outputs of run 0: pre rows (a, g, r) <= sum over goals of in*out
  // degree, post rows (g, r) <= edges, async rules <= nodes (corrections.go:30-34,121-125)
  c->tcap[0] = c->tcap[1] = c->tcap[2] = 0;
  if (c->run0 >= 0) {
    const uint32_t gp = 2 * c->run0, gq = gp + 1;
    const uint64_t v0 = c->node_off[gp], nv = c->node_off[gp + 1] - v0;
    std::vector<uint32_t> din(nv, 0), dout(nv, 0);
    for (uint64_t e = c->edge_off[gp]; e < c->edge_off[gp + 1]; e++) {
      if (in->edge_src[e] < nv) dout[in->edge_src[e]]++;
      if (in->edge_dst[e] < nv) din[in->edge_dst[e]]++;
    }
    for (uint64_t v = 0; v < nv; v++) c->tcap[0] += (uint64_t)din[v] * dout[v];
    c->tcap[1] = c->edge_off[gq + 1] - c->edge_off[gq];
    c->tcap[2] = nv;
    if ((rc = dalloc(c, &c->d_tpre, 3 * c->tcap[0] + 3))) return rc;
    if ((rc = dalloc(c, &c->d_tpost, 2 * c->tcap[1] + 2))) return rc;
    if ((rc = dalloc(c, &c->d_tasync, c->tcap[2] + 1))) return rc;
  }
  if (dbg) fprintf(stderr, "nemo_load_corpus: host part done %.1f ms\n", ms_since());
  if ((rc = device_load(c, lp.part.empty() ? nullptr : &lp))) return rc;
  if (c->load_async) {
    c->load_check_pending = true;  // the checks wait on `stream` at the next call that reads the graphs
  } else if ((rc = check_graph_errors(c))) {
    return rc;
  }
  if (dbg) fprintf(stderr, "nemo_load_corpus: done %.1f ms\n", ms_since());
  c->loaded = true;
  return NEMO_OK;
}

int nemo_rebuild(nemo_ctx *c) {
  DISPATCH(node_rebuild(c));
  if (!c) return NEMO_ERR_INVALID;
  if (!c->loaded) return fail(c, NEMO_ERR_STATE, "no corpus loaded");
  HIPCHK(c, hipSetDevice(c->device));
  int rc = ensure_load_checked(c);
  if (rc) return rc;
  rc = guard_staged(c);
  if (rc) return rc;
  if ((rc = join_aux(c))) return rc;  // the diff kernels read the graphs rebuilt here
  rc = device_load(c);
  if (rc) return rc;
  c->marked = c->simplified = c->protos_done = c->trig_done = false;
  c->mark_pending = false;
  return NEMO_OK;
}

// markConditionHolds is deferred for the LDS-tier graphs: nemo_simplify runs
// it fused with the simplification (k_marksimp).  Anything that reads the
// holds flags before that materialises it first (ensure_marked).
static int ensure_marked(nemo_ctx *c) {
  if (!c->mark_pending) return NEMO_OK;
  const double V = c->tierV, E = c->tierE;
  int rc = timed(c, "k_mark", 8 * E + 13 * V, 2 * E, [&] { nemo::launch_mark(c->dc, false, c->stream); });
  if (rc) return rc;
  c->mark_pending = false;
  c->ms_fused = false;  // k_mark rewrote every graph's flags (holds only)
  return NEMO_OK;
}

int nemo_mark_holds(nemo_ctx *c) {
  DISPATCH(node_mark_holds(c));
  if (!c) return NEMO_ERR_INVALID;
  if (!c->loaded) return fail(c, NEMO_ERR_STATE, "nemo_mark_holds before nemo_load_corpus");
  HIPCHK(c, hipSetDevice(c->device));
  if (int rl = ensure_load_checked(c)) return rl;
  const double V = (double)c->V - c->tierV, E = (double)c->E - c->tierE;
  int rc = guard_staged(c);
  if (rc) return rc;
  const bool defer = c->dc.t_ms.bytes != 0;
  rc = timed(c, "k_mark", 8 * E + 13 * V, 2 * E,
             [&] { nemo::launch_mark(c->dc, defer, c->stream, !defer || c->ms_rest); });
  if (rc) return rc;
  c->mark_pending = defer;
  c->marked = true;
  c->simplified = c->protos_done = c->trig_done = false;
  return NEMO_OK;
}

int nemo_simplify(nemo_ctx *c) {
  DISPATCH(node_simplify(c));
  if (!c) return NEMO_ERR_INVALID;
  if (!c->marked) return fail(c, NEMO_ERR_STATE, "nemo_simplify before nemo_mark_holds");
  HIPCHK(c, hipSetDevice(c->device));
  int rc = guard_staged(c);
  if (rc) return rc;
  if (c->mark_pending) {
    const double V = c->tierV, E = c->tierE, Vg = (double)c->V - V, Eg = (double)c->E - E;
    // k_build's tail did its graphs (ms_fused); an empty load tier means it took every graph
    // (none past its caps or handed back), so nothing is left for k_marksimp
    const bool skip_built = c->ms_fused;
    if (!(skip_built && tier_empty(c, 0)) &&
        (rc = timed(c, "k_marksimp", 8 * E + 5 * V, 5 * E,
                    [&] { nemo::launch_marksimp(c->dc, c->stream, skip_built); })))
      return rc;
    rc = timed(c, "k_simplify", 8 * Eg + 14 * Vg, 2 * Eg,
               [&] { nemo::launch_simplify(c->dc, true, c->stream, c->ms_rest != 0); });
    if (rc) return rc;
    c->mark_pending = false;
  } else {
    const double V = (double)c->V, E = (double)c->E;
    rc = timed(c, "k_simplify", 8 * E + 14 * V, 2 * E, [&] { nemo::launch_simplify(c->dc, false, c->stream); });
    if (rc) return rc;
  }
  c->ms_fused = false;  // consumed: the chain cover marks the flags, a later simplification recomputes them
  if ((rc = ensure_event(c, &c->ev_flags))) return rc;
  HIPCHK(c, hipEventRecord(c->ev_flags, c->stream));  // the flags are final (the chain cover reads them)
  c->flags_final = true;
  const double V = (double)c->V, E = (double)c->E;
  // reads: flags 1 + Kahn level 4 + node word 4 (+ ID rank 4) per node, the edge list 8 per edge
  const bool chain_tiers = !tier_empty(c, 1);
  rc = timed(c, "k_chains", (c->has_rank ? 13 : 9) * V + 8 * E, 0,
             [&] { nemo::launch_chains(c->dc, c->stream, chain_tiers); });
  if (rc) return rc;
  if (chain_tiers) c->tiers_run |= 2u;
  if ((rc = ensure_event(c, &c->ev_simp))) return rc;
  HIPCHK(c, hipEventRecord(c->ev_simp, c->stream));  // a simplified pull on `aux` starts here
  c->simplified = true;
  c->protos_done = false;
  return NEMO_OK;
}

size_t nemo_reduce_len(const nemo_ctx *c) { return c ? (c->node ? node_reduce_len(c) : 2 * (size_t)c->T + 4) : 0; }

int nemo_protos_partial(nemo_ctx *c, const uint32_t *success_iters, size_t n_success, uint32_t *d_red) {
  DISPATCH(node_protos_partial(c, success_iters, n_success, d_red));
  if (!c || (!success_iters && n_success)) return NEMO_ERR_INVALID;
  if (!c->simplified) return fail(c, NEMO_ERR_STATE, "nemo_protos_partial before nemo_simplify");
  if (!d_red) d_red = c->d_red;  // single-process callers use the context's own vector
  HIPCHK(c, hipSetDevice(c->device));
  if (c->red_staged) {  // a staged copy of an older vector: wait for it, then forget it
    HIPCHK(c, hipEventSynchronize(c->ev_red));
    c->red_staged = nullptr;
  }
  if (!c->ev_up_succ) HIPCHK(c, hipEventCreateWithFlags(&c->ev_up_succ, hipEventDisableTiming));
  else HIPCHK(c, hipEventSynchronize(c->ev_up_succ));  // the previous upload has landed
  int rg = hgrow(c, &c->h_succ, &c->h_succ_cap, std::max<uint64_t>(c->n_runs, 1));
  if (rg) return rg;
  uint8_t *succ = c->h_succ;
  memset(succ, 0, c->n_runs);
  uint32_t first = NEMO_NONE;
  for (size_t i = 0; i < n_success; i++) {
    auto f = c->it2run.find(success_iters[i]);
    if (f == c->it2run.end()) continue;  // another rank's run
    succ[f->second] = 1;
    if (i == 0) first = f->second;
  }
  hipStream_t s = c->stream;
  // k_proto first: it is what the analysis stream has ready when a bulk
  // staging copy starts beside it (a kernel queued behind the copy's start
  // waits for the copy's blit to drain); the reduction's inputs follow it
  // post graphs only (HBM lower bound): edges in source Kahn order 4E, node word 4V, flags 1V
  const double V = c->postV, E = c->postE;
  const bool proto_tier = !tier_empty(c, 2);
  int rc = timed(c, "k_proto", 4 * E + 5 * V, 2 * E, [&] { nemo::launch_proto(c->dc, s, proto_tier); });
  if (rc) return rc;
  if (proto_tier) c->tiers_run |= 4u;
  if ((rc = tiers_capture(c, s))) return rc;
  nemo::launch_to_host(c->d_is_success, succ, c->n_runs, s);  // pinned -> device by a copy kernel (no blit queue)
  HIPCHK(c, hipEventRecord(c->ev_up_succ, s));
  nemo::launch_zero(d_red, nemo_reduce_len(c) * 4, s);
  rc = timed(c, "k_reduce", (double)c->n_runs * (c->W * 8 + 8), 0,
             [&] { nemo::launch_reduce(c->dc, c->d_is_success, c->d_owned, first, d_red, s); });
  if (rc) return rc;
  // per-run table bitsets -> pinned host (nemo_fetch_run_tables)
  const uint64_t rw = (uint64_t)c->n_runs * c->W;
  if ((rc = ensure_event(c, &c->ev_protos))) return rc;
  if ((rc = hgrow(c, &c->h_tab, &c->h_tab_cap, 2 * rw + 1))) return rc;
  nemo::HostCopies hc;
  hc.add(c->h_tab, c->dc.proto_bits, rw * 4);
  hc.add(c->h_tab + rw, c->dc.graph_tables, rw * 4);
  nemo::launch_to_host_multi(hc, s);
  HIPCHK(c, hipEventRecord(c->ev_protos, s));
  c->protos_done = true;
  return NEMO_OK;
}

int nemo_reduce_interpret(const uint32_t *red, uint32_t T, uint32_t table_post, uint32_t *achieved, uint32_t *inter,
                          uint32_t *n_inter, uint32_t *uni, uint32_t *n_union) {
  if (!red) return NEMO_ERR_INVALID;
  uint32_t ni = 0, nu = 0;
  if (red[2 * T + 1]) {  // `longest` is only set inside the loop over list0 (prototype.go:80-103)
    for (uint32_t t = 0; t < T; t++) {
      if (t == table_post) continue;  // != condition (prototype.go:106,120)
      if (red[T + t] && red[t] == red[2 * T]) {  // foundIn == achvdCond (prototype.go:106)
        if (inter) inter[ni] = t;
        ni++;
      }
      if (red[t] > 0) {
        if (uni) uni[nu] = t;
        nu++;
      }
    }
  }
  if (achieved) *achieved = red[2 * T];
  if (n_inter) *n_inter = ni;
  if (n_union) *n_union = nu;
  return NEMO_OK;
}

static int protos_stage(nemo_ctx *c, const uint32_t *d_red) {
  int rc;
  if ((rc = ensure_event(c, &c->ev_red))) return rc;
  if (c->red_staged) HIPCHK(c, hipEventSynchronize(c->ev_red));  // h_red may be in flight
  if ((rc = hgrow(c, &c->h_red, &c->h_red_cap, 2 * (uint64_t)c->T + 4))) return rc;
  nemo::launch_to_host(c->h_red, d_red, (2 * (uint64_t)c->T + 4) * 4, c->stream);
  HIPCHK(c, hipEventRecord(c->ev_red, c->stream));
  c->red_staged = d_red;
  return NEMO_OK;
}

int nemo_protos_stage(nemo_ctx *c, const uint32_t *d_red) {
  if (!c) return NEMO_ERR_INVALID;
  if (c->node) return NEMO_OK;  // the node context reduces inside nemo_protos_finalize
  if (!d_red) d_red = c->d_red;
  if (!d_red) return fail(c, NEMO_ERR_STATE, "nemo_protos_stage before nemo_load_corpus");
  if (!c->protos_done) return fail(c, NEMO_ERR_STATE, "nemo_protos_stage before nemo_protos_partial");
  HIPCHK(c, hipSetDevice(c->device));
  return protos_stage(c, d_red);
}

int nemo_protos_finalize(nemo_ctx *c, const uint32_t *d_red, uint32_t *achieved, uint32_t *inter,
                         uint32_t *n_inter, uint32_t *uni, uint32_t *n_union, uint64_t *pre_holds,
                         uint32_t *n_runs_total) {
  DISPATCH(node_protos_finalize(c, d_red, achieved, inter, n_inter, uni, n_union, pre_holds, n_runs_total));
  if (!c) return NEMO_ERR_INVALID;
  if (!d_red) d_red = c->d_red;
  if (!d_red) return fail(c, NEMO_ERR_STATE, "nemo_protos_finalize before nemo_load_corpus");
  HIPCHK(c, hipSetDevice(c->device));
  const uint32_t T = c->T;
  int rc;
  if (c->red_staged != d_red && (rc = protos_stage(c, d_red))) return rc;
  HIPCHK(c, hipEventSynchronize(c->ev_red));
  c->red_staged = nullptr;  // consumed: the next finalize copies again unless staged again
  const uint32_t *red = c->h_red;
  if (pre_holds) *pre_holds = red[2 * T + 2];
  if (n_runs_total) *n_runs_total = red[2 * T + 3];
  return nemo_reduce_interpret(red, T, c->table_post, achieved, inter, n_inter, uni, n_union);
}

int nemo_fetch_reduce(nemo_ctx *c, uint32_t *out, uint64_t cap) {
  DISPATCH(node_fetch_reduce(c, out, cap));
  if (!c || !out) return NEMO_ERR_INVALID;
  if (!c->protos_done) return fail(c, NEMO_ERR_STATE, "nemo_fetch_reduce before nemo_protos_partial");
  const uint64_t n = 2 * (uint64_t)c->T + 4;
  if (cap < n) return fail(c, NEMO_ERR_INVALID, "capacity %llu < %llu", (unsigned long long)cap, (unsigned long long)n);
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipMemcpyAsync(out, c->d_red, n * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return NEMO_OK;
}

int nemo_prototypes(nemo_ctx *c, const uint32_t *success_iters, size_t n_success, uint32_t *achieved,
                    uint32_t *inter, uint32_t *n_inter, uint32_t *uni, uint32_t *n_union) {
  if (!c) return NEMO_ERR_INVALID;
  if (n_success == 0)
    return fail(c, NEMO_ERR_INVALID, "no successful runs: extractProtos indexes iterProv[0] (prototype.go:80)");
  int rc = nemo_protos_partial(c, success_iters, n_success, nullptr);  // the context's own vector
  if (rc) return rc;
  return nemo_protos_finalize(c, nullptr, achieved, inter, n_inter, uni, n_union, nullptr, nullptr);
}

int nemo_fetch_run_tables(nemo_ctx *c, int which, uint32_t *out, uint64_t cap) {
  DISPATCH(node_fetch_run_tables(c, which, out, cap));
  if (!c || !out) return NEMO_ERR_INVALID;
  if (!c->protos_done) return fail(c, NEMO_ERR_STATE, "run tables before nemo_protos_partial");
  const uint64_t n = (uint64_t)c->n_runs * c->W;
  if (cap < n) return fail(c, NEMO_ERR_INVALID, "capacity %llu < %llu", (unsigned long long)cap, (unsigned long long)n);
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipEventSynchronize(c->ev_protos));
  memcpy(out, c->h_tab + (which == 0 ? 0 : n), n * 4);
  return NEMO_OK;
}

int nemo_missing_from(nemo_ctx *c, uint32_t failed_iter, const uint32_t *proto, uint32_t n_proto, uint32_t *out,
                      uint32_t *n_out) {
  DISPATCH(node_missing_from(c, failed_iter, proto, n_proto, out, n_out));
  if (!c || (!proto && n_proto)) return NEMO_ERR_INVALID;
  if (!c->protos_done) return fail(c, NEMO_ERR_STATE, "nemo_missing_from before prototypes");
  uint32_t r;
  int rc = run_index(c, failed_iter, &r);
  if (rc) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  std::vector<uint32_t> bits(c->W);
  HIPCHK(c, hipMemcpyAsync(bits.data(), c->dc.graph_tables + (size_t)r * c->W, c->W * 4, hipMemcpyDeviceToHost,
                           c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  uint32_t n = 0;
  for (uint32_t i = 0; i < n_proto; i++) {
    const uint32_t t = proto[i];
    const bool have = t < c->T && ((bits[t >> 5] >> (t & 31)) & 1u);
    if (!have) {
      if (out) out[n] = t;
      n++;
    }
  }
  if (n_out) *n_out = n;
  return NEMO_OK;
}

// d_labels != NULL: label mode, every entry's failGoals is the device label
// set [n, label...] (n <= labels_cap), e.g. broadcast from the shard that owns
// failedRuns[0]; mode is then ignored.
static int diffprov_impl(nemo_ctx *c, const uint32_t *failed_iters, size_t n_failed, int mode,
                         const uint32_t *d_labels, uint64_t labels_cap) {
  if (!c || (!failed_iters && n_failed)) return NEMO_ERR_INVALID;
  if (mode != NEMO_DIFF_REFERENCE && mode != NEMO_DIFF_PER_RUN) return fail(c, NEMO_ERR_INVALID, "unknown diff mode %d", mode);
  if (!c->loaded) return fail(c, NEMO_ERR_STATE, "nemo_diffprov without a loaded corpus (the last load failed?)");
  if (!c->marked) return fail(c, NEMO_ERR_STATE, "nemo_diffprov before nemo_mark_holds");
  // (the diff kernels read no holds flags: a deferred mark stays fused with the simplification)
  HIPCHK(c, hipSetDevice(c->device));
  c->n_entries = 0;
  if (n_failed == 0 || c->run0 < 0) return NEMO_OK;  // MATCH on run 0 finds nothing
  if (!c->ev_up_dsrc) HIPCHK(c, hipEventCreateWithFlags(&c->ev_up_dsrc, hipEventDisableTiming));
  else HIPCHK(c, hipEventSynchronize(c->ev_up_dsrc));  // the previous upload has landed
  if (int rg = hgrow(c, &c->h_dsrc, &c->h_dsrc_cap, 3 * n_failed)) return rg;
  // D_f depends on run 0 and on the label source alone (differential-provenance.go:22-43):
  // entries with the same source share one computation.  In the reference mode every
  // entry's source is failedRuns[0] (the in-place ###RUN### substitution of :43), so
  // the whole call is one computation; in the per-run mode each distinct failed run is.
  uint32_t *src = c->h_dsrc, *emap = c->h_dsrc + n_failed, *urep = c->h_dsrc + 2 * n_failed;
  c->dmap.assign(n_failed, 0);
  std::unordered_map<uint32_t, uint32_t> uniq;
  uint32_t nu = 0;
  double src_bytes = 0;  // the label sources' HBM reads (word + label per node, or the label set)
  for (size_t e = 0; e < n_failed; e++) {
    uint32_t r;
    const uint32_t it = mode == NEMO_DIFF_PER_RUN && !d_labels ? failed_iters[e] : failed_iters[0];
    int rc = run_index(c, d_labels ? failed_iters[e] : it, &r);
    if (rc) return rc;
    const uint32_t key = d_labels ? 0u : 2 * r + 1;  // label mode: one set for every entry
    auto ins = uniq.emplace(key, nu);
    if (ins.second) {
      urep[nu] = (uint32_t)e;  // the first entry of each source stands for it (nemo_pull_edges(2))
      src[nu++] = 2 * r + 1;
      src_bytes += d_labels ? 0.0 : 8.0 * (double)(c->node_off[2 * r + 2] - c->node_off[2 * r + 1]);
    }
    c->dmap[e] = emap[e] = ins.first->second;
  }
  if (d_labels) src_bytes = 4.0 * (double)labels_cap;  // read once, then L2-resident
  const bool expand = nu < n_failed;
  const uint32_t g0 = 2 * c->run0 + 1;
  const uint64_t V0 = c->node_off[g0 + 1] - c->node_off[g0];
  const uint64_t E0 = c->edge_off[g0 + 1] - c->edge_off[g0];
  const bool dx = c->dx_ok && !c->diff_legacy && (c->diff_window != 2 || c->g0_maxdeg <= nemo::dx_max_row_tiny());
  int rc;
  // capacities in whole 64-entry chunks: the per-entry buffers of corpora (batches) with a few more
  // or fewer failed runs are the same size, so the allocation cache hands the same blocks back (a
  // block no load takes is freed at the next load, and hipFree waits for the whole device)
  const uint64_t nf_cap = (n_failed + 63) & ~(uint64_t)63;
  if (n_failed > c->diff_cap) {
    for (void *q : {(void *)c->d_dsrc, (void *)c->d_dmask, (void *)c->d_miss, (void *)c->d_dbits, (void *)c->d_dumask,
                    (void *)c->d_ddepth, (void *)c->d_dtopo})
      dfree(c, q);
    c->d_dbits = c->d_dumask = nullptr;
    c->d_ddepth = nullptr;
    c->d_dtopo = nullptr;
    c->legacy_cap = 0;
    if ((rc = dalloc(c, &c->d_dsrc, 3 * nf_cap))) return rc;
    if ((rc = dalloc(c, &c->d_dmask, nf_cap * V0))) return rc;
    if ((rc = dalloc(c, &c->d_miss, 2 * nf_cap * (V0 + 1)))) return rc;
    c->diff_cap = (uint32_t)nf_cap;
  }
  if (!dx && n_failed > c->legacy_cap) {  // the one-workgroup-per-entry kernels' scratch
    for (void *q : {(void *)c->d_dbits, (void *)c->d_dumask, (void *)c->d_ddepth, (void *)c->d_dtopo}) dfree(c, q);
    c->d_dbits = c->d_dumask = nullptr;
    c->d_ddepth = nullptr;
    c->d_dtopo = nullptr;
    if ((rc = dalloc(c, &c->d_dbits, nf_cap * V0))) return rc;
    if ((rc = dalloc(c, &c->d_dumask, nf_cap * V0))) return rc;
    if ((rc = dalloc(c, &c->d_ddepth, nf_cap * V0))) return rc;
    if ((rc = dalloc(c, &c->d_dtopo, 4 * V0 + 2 * E0 + 2 + c->n_r0lab))) return rc;
    c->legacy_cap = (uint32_t)nf_cap;
  }
  const uint32_t nch = (nu + 63) / 64, w32 = (uint32_t)((V0 + 31) / 32), nu_cap = 64 * nch;
  if (dx && (nu > c->dx_nu_cap || nch > c->dx_nch_cap)) {
    for (void *q : {(void *)c->d_dxpb, (void *)c->d_dxsval, (void *)c->d_dxlpl, (void *)c->d_dxw, (void *)c->d_dxfb})
      dfree(c, q);
    c->d_dxpb = c->d_dxsval = c->d_dxlpl = c->d_dxfb = nullptr;
    c->d_dxw = nullptr;
    c->dx_nu_cap = c->dx_nch_cap = 0;
    if ((rc = dalloc(c, &c->d_dxpb, (size_t)nu_cap * w32))) return rc;
    if ((rc = dalloc(c, &c->d_dxsval, (size_t)nu_cap * V0))) return rc;
    if ((rc = dalloc(c, &c->d_dxlpl, (size_t)nu_cap + nch))) return rc;  // maxima, then the chunks' walk flags
    if ((rc = dalloc(c, &c->d_dxw, 4 * (size_t)nch * V0))) return rc;
    if ((rc = dalloc(c, &c->d_dxfb, 8 * (size_t)nch * V0))) return rc;  // 32 bytes per position and chunk
    c->dx_nu_cap = nu_cap;
    c->dx_nch_cap = nch;
  }
  if (!c->d_nmiss && (rc = dalloc(c, &c->d_nmiss, 1))) return rc;
  c->d_dmap = c->d_dsrc + n_failed;
  c->n_uniq = nu;
  // the diff kernels go on `aux` once `stream` has reached this point (the load /
  // rebuild of the graphs they read is queued there)
  hipStream_t s = c->stream;
  if (c->diff_on_aux) {
    if (!c->aux) HIPCHK(c, hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
    if ((rc = ensure_event(c, &c->ev_fork))) return rc;
    HIPCHK(c, hipEventRecord(c->ev_fork, c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->aux, c->ev_fork, 0));
    s = c->aux;
  }
  nemo::launch_to_host(c->d_dsrc, src, 3 * n_failed * 4, s);  // pinned -> device by a copy kernel (no blit queue)
  HIPCHK(c, hipEventRecord(c->ev_up_dsrc, s));
  nemo::launch_zero(c->d_nmiss, 4, s);
  // HBM lower bound: run 0's post graph once (rows both ways, node word, Kahn
  // order: 8E0 + 16V0 -- every entry re-reads it from L2), each distinct label
  // source and each entry's D mask (V0); the three reachability sweeps per
  // computed entry are counted as traversed edges, not as HBM bytes
  const double bytes = 8.0 * E0 + 16.0 * V0 + src_bytes + (double)n_failed * V0;
  c->dx_last = dx;
  if (dx) {
    nemo::DxArgs a{};
    a.p = c->dxp;
    a.nu = nu;
    a.nch = nch;
    a.src = c->d_dsrc;
    a.ref_labels = d_labels;
    a.r0lab = c->d_r0lab;
    a.r0hkey = c->d_r0hkey;
    a.r0hval = c->d_r0hval;
    a.r0hmask = c->r0hmask;
    a.r0dense = c->dxp.r0dense;
    a.nlab = c->nlab;
    a.pb = c->d_dxpb;
    a.w32 = w32;
    uint64_t maxsrc = d_labels ? labels_cap : 0;
    for (uint32_t u = 0; u < nu && !d_labels; u++)
      maxsrc = std::max<uint64_t>(maxsrc, c->node_off[src[u] + 1] - c->node_off[src[u]]);
    a.lab_per = 8192;  // one workgroup per source up to 8192 nodes: its bitmap stored whole, no atomics
    a.lab_split = (uint32_t)std::max<uint64_t>(1, (maxsrc + a.lab_per - 1) / a.lab_per);
    const size_t plane = (size_t)nch * V0;
    a.gw = c->d_dxw;
    a.bw = a.gw + plane;
    a.dw = a.bw + plane;
    a.lw = a.dw + plane;
    a.fb = reinterpret_cast<uint8_t *>(c->d_dxfb);
    a.sval = c->d_dxsval;
    a.maxlen = c->d_dxlpl;
    a.wflag = c->d_dxlpl + c->dx_nu_cap;
    a.mask = c->d_dmask;
    a.map = c->d_dmap;
    a.n_entries = (uint32_t)n_failed;
    a.missing = c->d_miss;
    a.n_missing = c->d_nmiss;
    a.window = c->diff_window;
    a.legacy_lp = c->diff_unfused;
    a.urep = c->d_dsrc + 2 * n_failed;
    a.own_mask = nu == n_failed ? 1u : 0u;
    if (c->dx_img_key < 0) {
      // g0 in Kahn order (read the Kahn order, both CSRs and the node words;
      // write positions, rows both ways, level bounds), once per load / rebuild
      c->dxp.err0 = c->dc.err + c->dxp.g0;
      if ((rc = timed_on(c, s, "k_dxprep", 16.0 * E0 + 44.0 * V0, 0,
                         [&] { nemo::launch_dx_prep(c->dc, c->dxp, c->dx_its.tsum, s); })))
        return rc;
    }
    if (c->dx_img_key != (int)c->diff_window) {
      // the walk images (read rows and Kahn levels, write records, steps and
      // misses), once per load / rebuild and window configuration (test knob)
      nemo::dx_img_configs(c->dxp.V0, c->dxp.E0, c->diff_window, c->dx_img);
      if ((rc = timed_on(c, s, "k_dximg", 2 * (16.0 * E0 + 32.0 * V0), 0,
                         [&] { nemo::launch_dx_img(c->dxp, c->dx_img, c->dx_its, s); })))
        return rc;
      c->dx_img_key = (int)c->diff_window;
    }
    for (int k = 0; k < 2; k++) a.img[k] = c->dx_img[k];
    rc = timed_on(c, s, "k_diff", bytes, (double)nu * 3 * E0, [&] { nemo::launch_dx(c->dc, a, s); });
  } else {
    nemo::DiffArgs a;
    a.g0 = g0;
    a.src = c->d_dsrc;
    a.ref_labels = d_labels;
    a.r0lab = c->d_r0lab;
    a.r0idx = c->d_r0idx;
    a.n_r0lab = c->n_r0lab;
    a.r0hkey = c->d_r0hkey;
    a.r0hval = c->d_r0hval;
    a.r0hmask = c->r0hmask;
    a.bits = c->d_dbits;
    a.depth = c->d_ddepth;
    a.tpos = c->d_dtopo;
    a.tinfo = a.tpos + V0;
    a.trp = a.tinfo + V0;
    a.tfp = a.trp + V0 + 1;
    a.trc = a.tfp + V0 + 1;
    a.tfc = a.trc + E0;
    a.r0pos = a.tfc + E0;
    a.mask = expand ? c->d_dumask : c->d_dmask;
    a.missing = c->d_miss;
    a.n_missing = c->d_nmiss;
    rc = timed_on(c, s, "k_diff", bytes, (double)nu * 3 * E0,
                  [&] {
                    // the Kahn-order relayout only when g0 may fall outside the LDS tier
                    const bool lds = c->dc.t_diff.bytes && V0 <= c->dc.t_diff.v && E0 <= c->dc.t_diff.e;
                    nemo::launch_diff(c->dc, a, nu, lds ? 0u : (uint32_t)V0, s);
                    if (expand) nemo::launch_diff_expand(c->d_dmask, c->d_dumask, c->d_dmap, V0, (uint32_t)n_failed, s);
                  });
  }
  if (rc) return rc;
  // D masks and the missing-event count -> pinned host
  if ((rc = ensure_event(c, &c->ev_diff))) return rc;
  if ((rc = hgrow(c, &c->h_mask, &c->h_mask_cap, n_failed * V0))) return rc;
  if ((rc = hgrow(c, &c->h_nmiss, &c->h_nmiss_cap, (uint64_t)1))) return rc;
  // the missing rows too, at the last call's count: nemo_fetch_missing then needs no round
  // trip of its own unless this call found more (d_miss holds n_failed (V0 + 1) rows)
  c->mrows_staged = std::min<uint64_t>(c->mrows_hint, (uint64_t)n_failed * (V0 + 1));
  if ((rc = hgrow(c, &c->h_mrows, &c->h_mrows_cap, 2 * c->mrows_staged + 2))) return rc;
  nemo::HostCopies hc;
  hc.add(c->h_mask, c->d_dmask, n_failed * V0);
  hc.add(c->h_nmiss, c->d_nmiss, 4);
  hc.add(c->h_mrows, c->d_miss, 8 * c->mrows_staged);
  nemo::launch_to_host_multi(hc, s);
  HIPCHK(c, hipEventRecord(c->ev_diff, s));
  c->aux_pending = true;
  c->n_entries = (uint32_t)n_failed;
  return NEMO_OK;
}

int nemo_diffprov(nemo_ctx *c, const uint32_t *failed_iters, size_t n_failed, int mode) {
  DISPATCH(node_diffprov(c, failed_iters, n_failed, mode));
  return diffprov_impl(c, failed_iters, n_failed, mode, nullptr, 0);
}

int nemo_diffprov_labels(nemo_ctx *c, const uint32_t *failed_iters, size_t n_failed, const uint32_t *d_labels,
                         uint64_t labels_cap) {
  DISPATCH(node_diffprov_labels(c, failed_iters, n_failed, d_labels, labels_cap));
  if (!d_labels) return c ? fail(c, NEMO_ERR_INVALID, "no label set") : NEMO_ERR_INVALID;
  return diffprov_impl(c, failed_iters, n_failed, NEMO_DIFF_REFERENCE, d_labels, labels_cap);
}

int nemo_diffprov_host_labels(nemo_ctx *c, const uint32_t *failed_iters, size_t n_failed, const uint32_t *labels,
                              uint64_t n_labels) {
  DISPATCH(node_diffprov_host_labels(c, failed_iters, n_failed, labels, n_labels));
  if (!c || (!labels && n_labels)) return NEMO_ERR_INVALID;
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if ((rc = join_aux(c))) return rc;  // the previous diff may still read d_hlab
  if (n_labels + 1 > c->hlab_cap) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    dfree(c, c->d_hlab);
    c->d_hlab = nullptr;
    c->hlab_cap = 0;
    if ((rc = dalloc(c, &c->d_hlab, n_labels + 1))) return rc;
    c->hlab_cap = n_labels + 1;
  }
  if (!c->ev_up_hlab) HIPCHK(c, hipEventCreateWithFlags(&c->ev_up_hlab, hipEventDisableTiming));
  else HIPCHK(c, hipEventSynchronize(c->ev_up_hlab));  // the previous upload has landed
  if ((rc = hgrow(c, &c->h_hlab, &c->h_hlab_cap, n_labels + 1))) return rc;
  c->h_hlab[0] = (uint32_t)n_labels;
  if (n_labels) memcpy(c->h_hlab + 1, labels, n_labels * 4);
  nemo::launch_to_host(c->d_hlab, c->h_hlab, (n_labels + 1) * 4, c->stream);  // pinned -> device by a copy kernel
  HIPCHK(c, hipEventRecord(c->ev_up_hlab, c->stream));
  return diffprov_impl(c, failed_iters, n_failed, NEMO_DIFF_REFERENCE, c->d_hlab, n_labels + 1);
}

int nemo_goal_labels(nemo_ctx *c, uint32_t iteration, int cond, uint32_t *d_out, uint64_t cap) {
  DISPATCH(node_goal_labels(c, iteration, cond, d_out, cap));
  if (!c || !d_out || (cond != 0 && cond != 1)) return NEMO_ERR_INVALID;
  if (!c->loaded) return fail(c, NEMO_ERR_STATE, "no corpus loaded");
  HIPCHK(c, hipSetDevice(c->device));
  if (int rl = ensure_load_checked(c)) return rl;
  uint32_t r;
  int rc = run_index(c, iteration, &r);
  if (rc) return rc;
  const uint32_t g = 2 * r + (uint32_t)cond;
  const uint64_t V = c->node_off[g + 1] - c->node_off[g];
  if (cap < V + 1) return fail(c, NEMO_ERR_INVALID, "label capacity %llu < %llu", (unsigned long long)cap,
                               (unsigned long long)(V + 1));
  HIPCHK(c, hipSetDevice(c->device));
  if ((rc = join_aux(c))) return rc;  // d_out may be the label set a previous diff still reads
  return timed(c, "k_goal_labels", 8.0 * (double)V, 0, [&] { nemo::launch_goal_labels(c->dc, g, d_out, c->stream); });
}

int nemo_fetch_diff_mask(nemo_ctx *c, uint32_t entry, uint8_t *out, uint64_t cap) {
  DISPATCH(node_fetch_diff_mask(c, entry, out, cap));
  if (!c || !out) return NEMO_ERR_INVALID;
  if (entry >= c->n_entries) return fail(c, NEMO_ERR_INVALID, "diff entry %u out of range", entry);
  const uint32_t g0 = 2 * c->run0 + 1;
  const uint64_t V0 = c->node_off[g0 + 1] - c->node_off[g0];
  if (cap < V0) return fail(c, NEMO_ERR_INVALID, "capacity too small");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipEventSynchronize(c->ev_diff));
  memcpy(out, c->h_mask + (size_t)entry * V0, V0);
  return NEMO_OK;
}

int nemo_fetch_diff_masks(nemo_ctx *c, uint8_t *out, uint64_t cap) {
  DISPATCH(node_fetch_diff_masks(c, out, cap));
  if (!c || !out) return NEMO_ERR_INVALID;
  if (!c->n_entries) return NEMO_OK;
  const uint32_t g0 = 2 * c->run0 + 1;
  const uint64_t n = (uint64_t)c->n_entries * (c->node_off[g0 + 1] - c->node_off[g0]);
  if (cap < n) return fail(c, NEMO_ERR_INVALID, "capacity too small");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipEventSynchronize(c->ev_diff));
  memcpy(out, c->h_mask, n);
  return NEMO_OK;
}

int nemo_diff_masks_view(nemo_ctx *c, const uint8_t **masks, uint64_t *n_entries, uint64_t *v0) {
  DISPATCH(node_diff_masks_view(c, masks, n_entries, v0));
  if (!c || !masks) return NEMO_ERR_INVALID;
  *masks = nullptr;
  if (n_entries) *n_entries = c->n_entries;
  const uint32_t g0 = c->run0 >= 0 ? 2 * c->run0 + 1 : 0;
  if (v0) *v0 = c->run0 >= 0 ? c->node_off[g0 + 1] - c->node_off[g0] : 0;
  if (!c->n_entries) return NEMO_OK;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipEventSynchronize(c->ev_diff));
  *masks = c->h_mask;
  return NEMO_OK;
}

int nemo_fetch_missing(nemo_ctx *c, nemo_missing *out, uint64_t cap, uint64_t *n_out) {
  DISPATCH(node_fetch_missing(c, out, cap, n_out));
  if (!c) return NEMO_ERR_INVALID;
  HIPCHK(c, hipSetDevice(c->device));
  uint32_t nu_rows = 0;
  if (c->n_entries) {
    HIPCHK(c, hipEventSynchronize(c->ev_diff));
    nu_rows = *c->h_nmiss;
    // the fused walks' bounded hand-off wait (k_dx.hip dx_publish) gave up: the rows are void
    if (c->dx_last && (nu_rows & DX_ERR_HANDOFF))
      return fail(c, NEMO_ERR_INVALID, "diff walks: a longest-path workgroup timed out waiting for its Bwd* hand-off");
    nu_rows &= DX_ROWS;
  }
  // rows of the distinct computations (unique index, rule), then one copy per entry
  int rc;
  if ((rc = ensure_event(c, &c->ev_misc))) return rc;
  if (nu_rows > c->mrows_staged) {  // more rows than diffprov copied with the masks
    if ((rc = hgrow(c, &c->h_mrows, &c->h_mrows_cap, 2 * (uint64_t)nu_rows + 2))) return rc;
    if ((rc = join_aux(c))) return rc;
    nemo::launch_to_host(c->h_mrows, c->d_miss, 8ull * nu_rows, c->stream);
    HIPCHK(c, hipEventRecord(c->ev_misc, c->stream));
    HIPCHK(c, hipEventSynchronize(c->ev_misc));
    c->mrows_staged = nu_rows;
  }
  c->mrows_hint = std::max<uint64_t>(256, nu_rows);
  const uint32_t *rows = c->h_mrows;
  std::vector<std::vector<uint32_t>> per(c->n_uniq);
  for (uint32_t i = 0; i < nu_rows; i++) per[rows[2 * i]].push_back(rows[2 * i + 1]);
  uint64_t n = 0;
  for (auto &v : per) std::sort(v.begin(), v.end());
  for (uint32_t e = 0; e < c->n_entries; e++) n += per[c->dmap[e]].size();
  if (n_out) *n_out = n;
  if (!out) return NEMO_OK;
  if (cap < n) return fail(c, NEMO_ERR_INVALID, "capacity too small");
  uint64_t k = 0;
  for (uint32_t e = 0; e < c->n_entries; e++)
    for (uint32_t r : per[c->dmap[e]]) {
      out[k].entry = e;
      out[k].rule = r;
      k++;
    }
  return NEMO_OK;
}

int nemo_triggers(nemo_ctx *c) {
  DISPATCH(node_triggers(c));
  if (!c) return NEMO_ERR_INVALID;
  if (!c->marked) return fail(c, NEMO_ERR_STATE, "nemo_triggers before nemo_mark_holds");
  if (int rm = ensure_marked(c)) return rm;
  HIPCHK(c, hipSetDevice(c->device));
  c->tcounts[0] = c->tcounts[1] = c->tcounts[2] = 0;
  c->trig_done = true;
  c->trig_pending = false;
  if (c->run0 < 0) return NEMO_OK;
  int rc;
  if (!c->d_tcounts && (rc = dalloc(c, &c->d_tcounts, 3))) return rc;
  if (!c->h_tcounts) HIPCHK(c, hipHostMalloc((void **)&c->h_tcounts, 16));
  if (!c->ev_trig) HIPCHK(c, hipEventCreateWithFlags(&c->ev_trig, hipEventDisableTiming));
  nemo::TrigArgs a{};
  a.g_pre = 2 * c->run0;
  a.g_post = 2 * c->run0 + 1;
  a.counts = c->d_tcounts;
  a.pre = c->d_tpre;
  a.post = c->d_tpost;
  a.async_rules = c->d_tasync;
  hipStream_t s = c->stream;
  nemo::launch_zero(c->d_tcounts, 12, s);
  rc = timed(c, "k_triggers", 0, 0, [&] { nemo::launch_triggers(c->dc, a, 1, s); });
  if (rc) return rc;
  if ((rc = hgrow(c, &c->h_tpre, &c->h_tpre_cap, 3 * c->tcap[0] + 3))) return rc;
  if ((rc = hgrow(c, &c->h_tpost, &c->h_tpost_cap, 2 * c->tcap[1] + 2))) return rc;
  if ((rc = hgrow(c, &c->h_tasync, &c->h_tasync_cap, c->tcap[2] + 1))) return rc;
  nemo::HostCopies hc;
  hc.add(c->h_tcounts, c->d_tcounts, 12);
  hc.add(c->h_tpre, c->d_tpre, 12 * c->tcap[0]);
  hc.add(c->h_tpost, c->d_tpost, 8 * c->tcap[1]);
  hc.add(c->h_tasync, c->d_tasync, 4 * c->tcap[2]);
  nemo::launch_to_host_multi(hc, s);
  HIPCHK(c, hipEventRecord(c->ev_trig, s));
  c->trig_pending = true;
  return NEMO_OK;
}

static int trig_sync(nemo_ctx *c) {
  if (!c->trig_pending) return NEMO_OK;
  HIPCHK(c, hipEventSynchronize(c->ev_trig));
  for (int i = 0; i < 3; i++) {
    if (c->h_tcounts[i] > c->tcap[i]) return fail(c, NEMO_ERR_LIMIT, "trigger rows exceed their bound");
    c->tcounts[i] = c->h_tcounts[i];
  }
  c->trig_pending = false;
  return NEMO_OK;
}

int nemo_fetch_triggers(nemo_ctx *c, uint32_t *pre, uint64_t pre_cap, uint64_t *n_pre, uint32_t *post,
                        uint64_t post_cap, uint64_t *n_post, uint32_t *async_rules, uint64_t async_cap,
                        uint64_t *n_async) {
  DISPATCH(node_fetch_triggers(c, pre, pre_cap, n_pre, post, post_cap, n_post, async_rules, async_cap, n_async));
  if (!c) return NEMO_ERR_INVALID;
  if (!c->trig_done) return fail(c, NEMO_ERR_STATE, "nemo_fetch_triggers before nemo_triggers");
  HIPCHK(c, hipSetDevice(c->device));
  if (int rt = trig_sync(c)) return rt;
  if (n_pre) *n_pre = c->tcounts[0];
  if (n_post) *n_post = c->tcounts[1];
  if (n_async) *n_async = c->tcounts[2];
  if (pre && c->tcounts[0]) {
    if (pre_cap < c->tcounts[0]) return fail(c, NEMO_ERR_INVALID, "capacity too small");
    memcpy(pre, c->h_tpre, 12 * (size_t)c->tcounts[0]);
  }
  if (post && c->tcounts[1]) {
    if (post_cap < c->tcounts[1]) return fail(c, NEMO_ERR_INVALID, "capacity too small");
    memcpy(post, c->h_tpost, 8 * (size_t)c->tcounts[1]);
  }
  if (async_rules && c->tcounts[2]) {
    if (async_cap < c->tcounts[2]) return fail(c, NEMO_ERR_INVALID, "capacity too small");
    memcpy(async_rules, c->h_tasync, 4 * (size_t)c->tcounts[2]);
  }
  if (pre) sort_rows<3>(pre, c->tcounts[0]);
  if (post) sort_rows<2>(post, c->tcounts[1]);
  if (async_rules) std::sort(async_rules, async_rules + c->tcounts[2]);
  return NEMO_OK;
}

int nemo_fetch_node_flags(nemo_ctx *c, uint32_t g_lo, uint32_t g_hi, uint8_t *out, uint64_t cap) {
  DISPATCH(node_fetch_node_flags(c, g_lo, g_hi, out, cap));
  if (!c || !out || g_lo > g_hi || g_hi > c->G) return NEMO_ERR_INVALID;
  if (!c->marked) return fail(c, NEMO_ERR_STATE, "no flags before nemo_mark_holds");
  const uint64_t a = c->node_off[g_lo], b = c->node_off[g_hi];
  if (cap < b - a) return fail(c, NEMO_ERR_INVALID, "capacity too small");
  HIPCHK(c, hipSetDevice(c->device));
  if (int rm = ensure_marked(c)) return rm;
  if (b > a) {
    HIPCHK(c, hipMemcpyAsync(out, c->dc.flags + a, b - a, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  return NEMO_OK;
}

int nemo_fetch_chains(nemo_ctx *c, nemo_chain *out, uint64_t cap, uint64_t *n_out) {
  DISPATCH(node_fetch_chains(c, out, cap, n_out));
  if (!c) return NEMO_ERR_INVALID;
  if (!c->simplified) return fail(c, NEMO_ERR_STATE, "no chains before nemo_simplify");
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  hipStream_t s = c->stream;
  if (!c->d_choff && (rc = dalloc(c, &c->d_choff, (size_t)c->G + 1))) return rc;
  rc = timed(c, "k_chain_gather", 0, 0, [&] { nemo::launch_chain_gather(c->dc, c->d_choff, nullptr, s); });
  if (rc) return rc;
  uint64_t n = 0;
  HIPCHK(c, hipMemcpyAsync(&n, c->d_choff + c->G, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  if (n_out) *n_out = n;
  if (!out) return NEMO_OK;
  if (cap < n) return fail(c, NEMO_ERR_INVALID, "capacity too small");
  if (n > c->chout_cap) {
    dfree(c, c->d_chout);
    c->d_chout = nullptr;
    if ((rc = dalloc(c, &c->d_chout, 5 * n))) return rc;
    c->chout_cap = n;
  }
  rc = timed(c, "k_chain_gather", 0, 0, [&] { nemo::launch_chain_gather(c->dc, c->d_choff, c->d_chout, s); });
  if (rc) return rc;
  static_assert(sizeof(nemo_chain) == 20, "nemo_chain layout");
  if (n) HIPCHK(c, hipMemcpyAsync(out, c->d_chout, n * 20, hipMemcpyDeviceToHost, s));
  HIPCHK(c, hipStreamSynchronize(s));
  return NEMO_OK;
}

// bulk D2H on the copy stream: the runtime's copies (SDMA if asked, else its blit kernel on the
// copy stream's CUs) or a k_to_host grid of stage_blocks workgroups
static hipError_t stage_copy(nemo_ctx *c, void *dst, const void *src, size_t n) {
  if (!n) return hipSuccess;
  if (c->stage_blocks) {
    nemo::launch_to_host(dst, src, n, c->copy, c->stage_blocks);
    return hipGetLastError();
  }
  if (c->stage_sdma) {
    if (hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDeviceNoCU, c->copy) == hipSuccess) return hipSuccess;
    (void)hipGetLastError();
    c->stage_sdma = false;
  }
  return hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, c->copy);
}

// The 2-bit node state on stream s and its copy; s has reached the point where the flags are final.
static int stage_state(nemo_ctx *c, hipStream_t s) {
  int rc;
  const uint64_t sbytes = 4 * ((c->V + 15) / 16);  // 2-bit node state
  if (!c->d_state && (rc = dalloc(c, &c->d_state, sbytes / 4 + 1))) return rc;
  rc = timed_on(c, s, "k_pack_state", (double)c->V + (double)sbytes, 0,
                [&] { nemo::launch_pack_state(c->dc.flags, c->d_state, c->V, s); });
  if (rc) return rc;
  if ((rc = hgrow(c, &c->h_flags, &c->h_flags_cap, sbytes + 16))) return rc;
  if ((rc = ensure_event(c, &c->ev_state))) return rc;
  HIPCHK(c, hipEventRecord(c->ev_state, s));
  HIPCHK(c, hipStreamWaitEvent(c->copy, c->ev_state, 0));
  HIPCHK(c, stage_copy(c, c->h_flags, c->d_state, sbytes));
  return NEMO_OK;
}

// Enqueue the chain pairs at a capacity of `cap` pairs and their bulk copy on the copy stream
// (behind the node state's, which stage_state queued first).
static int stage_enqueue(nemo_ctx *c, uint64_t cap) {
  int rc;
  hipStream_t s = c->stage_stream ? c->stage_stream : c->stream;
  const uint64_t pw = c->pairs_wide ? 2 : 1;  // u32 words per pair
  if (pw * cap > c->d_chht_cap) {
    HIPCHK(c, hipStreamSynchronize(s));
    dfree(c, c->d_chht);
    c->d_chht = nullptr;
    c->d_chht_cap = 0;
    if ((rc = dalloc(c, &c->d_chht, pw * cap + 2))) return rc;
    c->d_chht_cap = pw * cap + 2;
  }
  rc = timed_on(c, s, "k_chain_pairs", 4.0 * pw * (double)cap + 20.0 * c->G, 0,
                [&] { nemo::launch_chain_pairs(c->dc, c->d_choff, c->d_chht, cap, c->pairs_wide ? 1 : 0, s); });
  if (rc) return rc;
  if ((rc = hgrow(c, &c->h_chht, &c->h_chht_cap, pw * cap + 2))) return rc;
  nemo::launch_to_host(c->h_choff, c->d_choff, ((size_t)c->G + 1) * 8, s);
  HIPCHK(c, hipEventRecord(c->ev_ready, s));
  HIPCHK(c, hipStreamWaitEvent(c->copy, c->ev_ready, 0));
  HIPCHK(c, stage_copy(c, c->h_chht, c->d_chht, pw * cap * 4));
  HIPCHK(c, hipEventRecord(c->ev_copied, c->copy));
  c->staged_cap = cap;
  return NEMO_OK;
}

int nemo_stage_simplified(nemo_ctx *c) {
  DISPATCH(node_stage_simplified(c));
  if (!c) return NEMO_ERR_INVALID;
  if (!c->simplified) return fail(c, NEMO_ERR_STATE, "nemo_stage_simplified before nemo_simplify");
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  hipStream_t s = c->stream;
  if (!c->copy) {
    // the bulk D2H copies run as the runtime's blit kernel, PCIe-bound for ~0.5 ms
    // per step: confined to a few CUs, they no longer hold workgroup slots of
    // the LDS-tier kernel running beside them (stage_cus, default 8; 0 = any CU)
    if (c->stage_cus) {
      uint32_t mask[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (uint32_t k = 0; k < std::min(c->stage_cus, 256u); k++) mask[k >> 5] |= 1u << (k & 31);
      if (hipExtStreamCreateWithCUMask(&c->copy, 8, mask) != hipSuccess) {
        (void)hipGetLastError();
        c->copy = nullptr;
      }
    }
    if (!c->copy) HIPCHK(c, hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking));
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_ready, hipEventDisableTiming));
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_copied, hipEventDisableTiming));
  }
  if (c->staged) HIPCHK(c, hipEventSynchronize(c->ev_copied));  // host buffers are reused
  c->staged = false;
  if (!c->d_choff && (rc = dalloc(c, &c->d_choff, (size_t)c->G + 1))) return rc;
  if ((rc = hgrow(c, &c->h_choff, &c->h_choff_cap, (uint64_t)c->G + 1))) return rc;
  if (c->stage_on_aux) {  // read-only on the analysis: `stream` goes on to the triggers and pulls
    if (!c->aux) HIPCHK(c, hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
    // the node state from where nemo_simplify's flags were final (beside the chain cover), then
    // the chain pairs from here (the chain cover and whatever the caller queued since)
    if (!c->flags_final) {  // flags rewritten since nemo_simplify: pack them where `stream` is now
      if ((rc = ensure_event(c, &c->ev_flags))) return rc;
      HIPCHK(c, hipEventRecord(c->ev_flags, c->stream));
    }
    HIPCHK(c, hipStreamWaitEvent(c->aux, c->ev_flags, 0));
    if ((rc = stage_state(c, c->aux))) return rc;
    if ((rc = ensure_event(c, &c->ev_stage))) return rc;
    HIPCHK(c, hipEventRecord(c->ev_stage, c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->aux, c->ev_stage, 0));
    s = c->aux;
  } else if ((rc = stage_state(c, s))) {
    return rc;
  }
  c->stage_stream = s;
  rc = timed_on(c, s, "k_chain_gather", 0, 0, [&] { nemo::launch_chain_gather(c->dc, c->d_choff, nullptr, s); });
  if (rc) return rc;
  // the pair count is only known on the device: stage at the last count seen
  // (no host round trip); nemo_simplified_view re-stages if it was too small
  uint64_t cap = c->chht_hint;
  if (!cap) {
    if ((rc = ensure_event(c, &c->ev_misc))) return rc;
    nemo::launch_to_host(c->h_choff, c->d_choff, ((size_t)c->G + 1) * 8, s);
    HIPCHK(c, hipEventRecord(c->ev_misc, s));
    HIPCHK(c, hipEventSynchronize(c->ev_misc));
    cap = c->h_choff[c->G];
  }
  if ((rc = stage_enqueue(c, cap))) return rc;
  c->staged = true;
  return NEMO_OK;
}

int nemo_simplified_view(nemo_ctx *c, const uint8_t **state, const uint64_t **chain_off, const uint32_t **chain_ht,
                         uint64_t *n_chains, int *wide_pairs) {
  DISPATCH(node_simplified_view(c, state, chain_off, chain_ht, n_chains, wide_pairs));
  if (!c) return NEMO_ERR_INVALID;
  if (!c->staged) return fail(c, NEMO_ERR_STATE, "nothing staged: call nemo_stage_simplified");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipEventSynchronize(c->ev_copied));
  const uint64_t n = c->h_choff[c->G];
  if (n > c->staged_cap) {  // the hint was short: stage again at the real count
    // on the context's stream, behind everything queued since the first stage (work that
    // rewrites flags may follow it there; `aux` was ordered only after the first stage)
    c->stage_stream = c->stream;
    int rc = stage_enqueue(c, n);
    if (rc) return rc;
    HIPCHK(c, hipEventSynchronize(c->ev_copied));
  }
  c->chht_hint = n;
  c->staged_n = n;
  if (state) *state = c->h_flags;
  if (wide_pairs) *wide_pairs = c->pairs_wide ? 1 : 0;
  if (chain_off) *chain_off = c->h_choff;
  if (chain_ht) *chain_ht = c->h_chht;
  if (n_chains) *n_chains = c->staged_n;
  return NEMO_OK;
}

static int pull_launch(nemo_ctx *c) {
  nemo::PullArgs &a = c->pull_args;
  a.src = c->d_psrc;
  a.dst = c->d_pdst;
  a.cap = c->pull_cap;
  const uint32_t slots = c->pull_dslots;
  hipStream_t s = c->stream;
  // the simplified pull reads what nemo_simplify left (graphs, flags, chains): on `aux`, behind
  // the end of the simplification only, it overlaps the protos and hand-over kernels of `stream`
  const bool on_aux = a.which == 1 && c->pull_on_aux && c->ev_simp;
  if (on_aux) {
    if (!c->aux) HIPCHK(c, hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
    HIPCHK(c, hipStreamWaitEvent(c->aux, c->ev_simp, 0));
    s = c->aux;
  }
  double V = (double)c->V, E = (double)c->E;
  if (a.which == 2) {
    V = (double)slots * (double)a.mask_stride;
    E = (double)slots * (double)(c->edge_off[a.g0 + 1] - c->edge_off[a.g0]);
  }
  nemo::launch_zero(c->d_pcur, sizeof(unsigned long long), s);
  // algorithmic bytes: the read side (node flags, both row pointers, columns, masks)
  uint32_t rest = c->pull_rest;
  if (a.which == 2) {
    const uint64_t v0 = c->node_off[a.g0 + 1] - c->node_off[a.g0], e0 = c->edge_off[a.g0 + 1] - c->edge_off[a.g0];
    rest = !tier_fits(c->dc.t_pull, (uint32_t)std::min<uint64_t>(v0, ~0u), (uint32_t)std::min<uint64_t>(e0, ~0u), 0);
  }
  int rc = timed_on(c, s, "k_pull", 4 * E + 13 * V, E, [&] { nemo::launch_pull(c->dc, a, slots, rest, s); });
  if (rc) return rc;
  nemo::HostCopies hc;
  hc.add(c->h_poff, c->d_poff, slots * 8ull);
  hc.add(c->h_pcnt, c->d_pcnt, slots * 4ull);
  hc.add(c->h_pcur, c->d_pcur, sizeof(unsigned long long));
  nemo::launch_to_host_multi(hc, s);
  HIPCHK(c, hipEventRecord(c->ev_pull, s));
  if (on_aux) {
    if ((rc = ensure_event(c, &c->ev_auxpull))) return rc;
    HIPCHK(c, hipEventRecord(c->ev_auxpull, s));
    c->pull_aux_pending = true;
  }
  c->pull_synced = false;
  return NEMO_OK;
}

static int pull_grow(nemo_ctx *c, uint64_t total) {
  if (total <= c->pull_cap) return NEMO_OK;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  dfree(c, c->d_psrc);
  dfree(c, c->d_pdst);
  c->d_psrc = c->d_pdst = nullptr;
  c->pull_cap = 0;
  int rc;
  if ((rc = dalloc(c, &c->d_psrc, total))) return rc;
  if ((rc = dalloc(c, &c->d_pdst, total))) return rc;
  c->pull_cap = total;
  return NEMO_OK;
}

// Wait for the last pull's slot table; re-run it once if its regions overran the capacity.
static int pull_sync(nemo_ctx *c) {
  if (c->pull_synced) return NEMO_OK;
  HIPCHK(c, hipEventSynchronize(c->ev_pull));
  const uint64_t total = *c->h_pcur;
  if (total > c->pull_cap) {
    int rc = pull_grow(c, total);
    if (!rc) rc = pull_launch(c);
    if (rc) return rc;
    HIPCHK(c, hipEventSynchronize(c->ev_pull));
  }
  c->pull_hint[c->pull_which] = total;
  if (!c->pull_map.empty()) {  // shared regions: entry e takes its computed slot's (map[e] <= e)
    for (uint32_t e = c->pull_slots; e-- > 0;) {
      const uint32_t u = c->pull_map[e];
      c->h_poff[e] = c->h_poff[u];
      c->h_pcnt[e] = c->h_pcnt[u];
    }
    c->pull_map.clear();
  }
  c->pull_synced = true;
  return NEMO_OK;
}

int nemo_pull_edges(nemo_ctx *c, int which) {
  DISPATCH(node_pull_edges(c, which));
  if (!c || which < 0 || which > 2) return NEMO_ERR_INVALID;
  if (!c->loaded) return fail(c, NEMO_ERR_STATE, "no corpus loaded");
  if (which == 1 && !c->simplified) return fail(c, NEMO_ERR_STATE, "simplified pull before nemo_simplify");
  HIPCHK(c, hipSetDevice(c->device));
  int rc = ensure_load_checked(c);
  if (rc) return rc;
  const uint32_t slots = which == 2 ? c->n_entries : c->G;
  // the previous pull's slot table may still be in flight into the pinned tables: wait for it
  // only when they are about to be reallocated (a pull queued behind another on the same
  // stream overwrites the device tables in order; the host reads them in pull_sync after the
  // last pull's event)
  if (!c->pull_synced && (slots + 1 > c->pull_slot_cap || slots + 1 > c->h_pslot_cap))
    HIPCHK(c, hipEventSynchronize(c->ev_pull));
  c->pull_synced = true;
  if (which == 2 && (rc = join_aux(c))) return rc;  // the D masks
  // diff entries sharing a label source have one D mask, hence one graph: it is
  // compacted once and their slots share its region (pull_sync expands the table)
  const bool share = which == 2 && c->n_uniq < c->n_entries;
  const uint32_t dslots = share ? c->n_uniq : slots;
  if (!c->ev_pull) HIPCHK(c, hipEventCreateWithFlags(&c->ev_pull, hipEventDisableTiming));
  if (!c->h_pcur) HIPCHK(c, hipHostMalloc((void **)&c->h_pcur, sizeof(unsigned long long)));
  if (!c->d_pcur && (rc = dalloc(c, &c->d_pcur, 1))) return rc;
  if (slots + 1 > c->pull_slot_cap) {
    dfree(c, c->d_pcnt);
    dfree(c, c->d_poff);
    c->d_pcnt = nullptr;
    c->d_poff = nullptr;
    if ((rc = dalloc(c, &c->d_pcnt, (size_t)slots + 1))) return rc;
    if ((rc = dalloc(c, &c->d_poff, (size_t)slots + 1))) return rc;
    c->pull_slot_cap = slots + 1;
  }
  if (slots + 1 > c->h_pslot_cap) {
    if (c->h_pcnt) hipHostFree(c->h_pcnt);
    if (c->h_poff) hipHostFree(c->h_poff);
    c->h_pcnt = nullptr;
    c->h_poff = nullptr;
    c->h_pslot_cap = 0;
    HIPCHK(c, hipHostMalloc((void **)&c->h_pcnt, (slots + 1) * 4ull));
    HIPCHK(c, hipHostMalloc((void **)&c->h_poff, (slots + 1) * 8ull));
    c->h_pslot_cap = slots + 1;
  }
  c->pull_which = which;
  c->pull_slots = slots;
  c->pull_dslots = dslots;
  if (share) c->pull_map = c->dmap;
  else c->pull_map.clear();
  if (slots == 0) return NEMO_OK;
  nemo::PullArgs a{};
  a.which = (uint32_t)which;
  const uint32_t g0 = c->run0 >= 0 ? 2 * c->run0 + 1 : 0;
  a.g0 = g0;
  uint64_t cap;
  if (which == 2) {
    a.mask = c->d_dmask;
    a.mask_stride = c->node_off[g0 + 1] - c->node_off[g0];
    a.mask_row = share ? c->d_dsrc + 2 * c->n_entries : nullptr;  // diffprov's representative entries
    cap = (uint64_t)dslots * (c->edge_off[g0 + 1] - c->edge_off[g0]);  // D is an induced subgraph of g0
  } else if (which == 0) {
    cap = c->E;  // every edge
  } else {
    // kept edges (<= E) + collapsed edges; a pull past the estimate re-runs on fetch
    cap = std::max<uint64_t>(2 * c->E + 1024, c->pull_hint[1] + c->pull_hint[1] / 4);
  }
  a.cnt = c->d_pcnt;
  a.off = c->d_poff;
  a.cursor = c->d_pcur;
  // big graphs' chunk table (k_diff.hip MWP_CH = 4096 nodes or chains per chunk)
  a.ccnt = nullptr;
  a.maxck = 0;
  const uint64_t vg0 = c->node_off[g0 + 1] - c->node_off[g0];
  const uint32_t rows = which == 2 ? (vg0 >= NEMO_CSR_BIG ? dslots : 0u) : c->dc.n_big;
  if (rows) {
    a.maxck = (uint32_t)(2 * ((c->bigVmax + 4095) / 4096));
    const size_t need = (size_t)rows * a.maxck;
    if (need > c->pull_ck_cap) {
      HIPCHK(c, hipStreamSynchronize(c->stream));  // a previous pull may still use the chunk table
      dfree(c, c->d_pck);
      c->d_pck = nullptr;
      c->pull_ck_cap = 0;
      if ((rc = dalloc(c, &c->d_pck, need))) return rc;
      c->pull_ck_cap = need;
    }
    a.ccnt = c->d_pck;
  }
  c->pull_args = a;
  if ((rc = pull_grow(c, std::max<uint64_t>(cap, 1)))) return rc;
  return pull_launch(c);
}

uint64_t nemo_pulled_count(nemo_ctx *c, uint32_t slot) {
  DISPATCH(node_pulled_count(c, slot));
  if (!c || c->pull_which < 0 || slot >= c->pull_slots) return 0;
  if (pull_sync(c)) return 0;
  return c->h_pcnt[slot];
}

int nemo_fetch_pulled(nemo_ctx *c, uint32_t slot, uint32_t *src, uint32_t *dst, uint64_t cap, uint64_t *n_out) {
  DISPATCH(node_fetch_pulled(c, slot, src, dst, cap, n_out));
  if (!c) return NEMO_ERR_INVALID;
  if (c->pull_which < 0) return fail(c, NEMO_ERR_STATE, "nothing pulled");
  if (slot >= c->pull_slots) return fail(c, NEMO_ERR_INVALID, "slot %u out of range", slot);
  HIPCHK(c, hipSetDevice(c->device));
  int rc = pull_sync(c);
  if (rc) return rc;
  const uint64_t a = c->h_poff[slot], n = c->h_pcnt[slot];
  if (n_out) *n_out = n;
  if (!src && !dst) return NEMO_OK;
  if (cap < n) return fail(c, NEMO_ERR_INVALID, "capacity too small");
  if (n) {
    if (src) HIPCHK(c, hipMemcpyAsync(src, c->d_psrc + a, n * 4, hipMemcpyDeviceToHost, c->stream));
    if (dst) HIPCHK(c, hipMemcpyAsync(dst, c->d_pdst + a, n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  return NEMO_OK;
}

int nemo_fetch_pulled_all(nemo_ctx *c, uint64_t *off, uint32_t *cnt, uint32_t *src, uint32_t *dst, uint64_t cap,
                          uint64_t *n_used) {
  DISPATCH(node_fetch_pulled_all(c, off, cnt, src, dst, cap, n_used));
  if (!c) return NEMO_ERR_INVALID;
  if (c->pull_which < 0) return fail(c, NEMO_ERR_STATE, "nothing pulled");
  HIPCHK(c, hipSetDevice(c->device));
  int rc = pull_sync(c);
  if (rc) return rc;
  const uint64_t used = c->pull_slots ? *c->h_pcur : 0;
  if (n_used) *n_used = used;
  if (off && c->pull_slots) memcpy(off, c->h_poff, c->pull_slots * 8ull);
  if (cnt && c->pull_slots) memcpy(cnt, c->h_pcnt, c->pull_slots * 4ull);
  if (!src && !dst) return NEMO_OK;
  if (cap < used) return fail(c, NEMO_ERR_INVALID, "capacity too small");
  if (used) {
    if (src) HIPCHK(c, hipMemcpyAsync(src, c->d_psrc, used * 4, hipMemcpyDeviceToHost, c->stream));
    if (dst) HIPCHK(c, hipMemcpyAsync(dst, c->d_pdst, used * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  return NEMO_OK;
}

// Debug/inspection: copy `bytes` bytes at byte `offset` of an internal device array.
int nemo_debug_copy(nemo_ctx *c, const char *name, void *out, uint64_t offset, uint64_t bytes) {
  DISPATCH(node_debug_copy(c, name, out, offset, bytes));
  if (!c || !name || !out) return NEMO_ERR_INVALID;
  const void *base = nullptr;
  const std::string n(name);
  if (n == "topo") base = c->dc.topo;
  else if (n == "lvl") base = c->dc.lvl;
  else if (n == "nlv") base = c->dc.nlv;
  else if (n == "diff_tpos") base = c->d_dtopo;
  else if (n == "nlev") base = c->dc.nlev;
  else if (n == "fp") base = c->dc.fp;
  else if (n == "fc") base = c->dc.fc;
  else if (n == "rp") base = c->dc.rp;
  else if (n == "rc") base = c->dc.rc;
  else if (n == "flags") base = c->dc.flags;
  else if (n == "dbits") base = c->d_dbits;
  else if (n == "dmask") base = c->d_dmask;
  else if (n == "r0lab") base = c->d_r0lab;
  else if (n == "r0idx") base = c->d_r0idx;
  else if (n == "stamps") base = c->dc.stamps;
  else if (n == "sel") base = c->dc.sel;
  else if (n == "redo") base = c->dc.redo;
  else if (n == "s_a") base = c->dc.s_a;
  else if (n == "gscratch") base = c->dc.gscratch;
  else if (n == "gs_off") base = c->dc.gs_off;
  else if (n == "err") base = c->dc.err;  // worklists: [4][G+1] u32, count first (pulls, chains, load, protos)
  if (!base) return fail(c, NEMO_ERR_INVALID, "unknown array %s", name);
  HIPCHK(c, hipSetDevice(c->device));
  int rc = join_aux(c);  // the diff kernels on `aux` write dbits, dmask and the Kahn relayout
  if (rc) return rc;
  HIPCHK(c, hipMemcpyAsync(out, (const char *)base + offset, bytes, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return NEMO_OK;
}

int nemo_synchronize(nemo_ctx *c) {
  DISPATCH(node_synchronize(c));
  if (!c) return NEMO_ERR_INVALID;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->aux) HIPCHK(c, hipStreamSynchronize(c->aux));
  return NEMO_OK;
}

int nemo_timings(nemo_ctx *c, nemo_timing *out, uint32_t cap, uint32_t *n_out) {
  DISPATCH(node_timings(c, out, cap, n_out));
  if (!c) return NEMO_ERR_INVALID;
  HIPCHK(c, hipSetDevice(c->device));
  for (auto &p : c->pending) {
    HIPCHK(c, hipEventSynchronize(p.b));
    float ms = 0;
    HIPCHK(c, hipEventElapsedTime(&ms, p.a, p.b));
    Agg &g = c->agg[p.name];
    g.launches++;
    g.ms += ms;
    g.bytes += p.bytes;
    g.edges += p.edges;
    c->ev_pool.push_back(p.a);
    c->ev_pool.push_back(p.b);
  }
  c->pending.clear();
  uint32_t n = 0;
  for (auto &kv : c->agg) {
    if (out && n < cap) {
      memset(&out[n], 0, sizeof out[n]);
      strncpy(out[n].name, kv.first.c_str(), sizeof out[n].name - 1);
      out[n].launches = kv.second.launches;
      out[n].ms = kv.second.ms;
      out[n].bytes = kv.second.bytes;
      out[n].edges = kv.second.edges;
    }
    n++;
  }
  if (n_out) *n_out = n;
  return NEMO_OK;
}

int nemo_reset_timings(nemo_ctx *c) {
  DISPATCH(node_reset_timings(c));
  if (!c) return NEMO_ERR_INVALID;
  uint32_t n;
  int rc = nemo_timings(c, nullptr, 0, &n);
  c->agg.clear();
  return rc;
}

}  // extern "C"
