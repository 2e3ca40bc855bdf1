/*
 * nemohip.h — C ABI of libnemohip, the MI355X (gfx950) engine behind Nemo's
 * provenance-graph analysis.
 *
 * This is the drop-in boundary that replaces the Bolt connection + Neo4j 3.3.3
 * engine underneath the Go `graphing` package of at15/nemo.  Every entry point
 * below names the reference method (file:line, relative to the reference root)
 * whose database round trips it replaces.  The Go side (a cgo stub, see
 * INTEGRATION.md) keeps every string: it interns table names, labels, rule
 * types and node IDs into the integer arrays below and rebuilds IDs, labels,
 * `<code>` wrappers, corrections and DOT graphs from the integer results.
 *
 * Conventions
 *   - Plain C, plain pointers and sizes; no HIP, torch or C++ types.
 *   - Every function returns NEMO_OK (0) or a NEMO_ERR_* code; the message of
 *     the last failure is nemo_last_error(ctx) (reference messages reused where
 *     the reference has one, e.g. graphing/pre-post-prov.go:209).
 *   - A context is bound to one HIP device and is not re-entrant (the
 *     reference's Bolt connections are not thread-safe either:
 *     vendor/github.com/johnnadratowski/golang-neo4j-bolt-driver/driver.go:33-36).
 *   - Graph g of a corpus is run r's antecedent (pre) graph when g == 2r and its
 *     consequent (post) graph when g == 2r+1 (the two loadProv calls of
 *     graphing/pre-post-prov.go:255,269).
 *   - Node indices in every array are local to their graph (0 .. V_g-1).
 */
#ifndef NEMOHIP_H
#define NEMOHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NEMOHIP_ABI_VERSION 1

/* ---- status codes ------------------------------------------------------ */
#define NEMO_OK            0
#define NEMO_ERR_INVALID   1  /* bad argument / malformed corpus               */
#define NEMO_ERR_HIP       2  /* HIP runtime failure                           */
#define NEMO_ERR_LOAD      3  /* loadProv validation (dangling/duplicate edge)  */
#define NEMO_ERR_CYCLE     4  /* provenance graph is not acyclic               */
#define NEMO_ERR_STATE     5  /* call out of order (e.g. simplify before load)  */
#define NEMO_ERR_LIMIT     6  /* a size limit of this build was exceeded        */
#define NEMO_ERR_NOTFOUND  7  /* unknown run iteration                          */
#define NEMO_ERR_NOGPU     8  /* no usable HIP device                           */

/* ---- packed node word (input) ------------------------------------------ *
 * bit 31      : 1 = Rule node, 0 = Goal node   (Neo4j labels :Rule / :Goal,
 *               graphing/pre-post-prov.go:28,91)
 * bits 28..30 : rule type class (goals: 0)      (Rule.type, pre-post-prov.go:91)
 * bits 0..23  : interned table id               (Goal.table / Rule.table)      */
#define NEMO_NODE_RULE    0x80000000u
#define NEMO_TYPE_SHIFT   28
#define NEMO_TYPE_MASK    0x70000000u
#define NEMO_TYPE_OTHER   0u  /* any type string other than the two below      */
#define NEMO_TYPE_NEXT    1u  /* "next"  (preprocessing.go:71, corrections.go:213) */
#define NEMO_TYPE_ASYNC   2u  /* "async" (extensions.go:64, diagrams.go:53)    */
#define NEMO_TABLE_MASK   0x00FFFFFFu
#define NEMO_MAX_TABLES   16384u /* table-id universe supported by this build   */

#define NEMO_WORD(is_rule, type, table) \
  (((is_rule) ? NEMO_NODE_RULE : 0u) | ((uint32_t)(type) << NEMO_TYPE_SHIFT) | ((uint32_t)(table) & NEMO_TABLE_MASK))

/* ---- per-node result flags (output) ------------------------------------ */
#define NEMO_F_HOLDS    0x01u /* condition_holds after markConditionHolds        */
#define NEMO_F_KEPT     0x02u /* node survives cleanCopyProv (run 1000+i copy)   */
#define NEMO_F_DELETED  0x04u /* removed by collapseNextChains' DETACH DELETE     */
#define NEMO_F_HEAD     0x08u /* first rule of >= 1 accepted @next chain         */
#define NEMO_F_TAIL     0x10u /* last rule of >= 1 accepted @next chain          */

/* ---- corpus (input; replaces fi.Run/ProvData, faultinjectors/data-types.go:43-98) */
typedef struct nemo_corpus {
  uint32_t n_runs;           /* runs in this corpus (or this rank's shard)          */
  uint32_t n_tables;         /* table ids are < n_tables (<= NEMO_MAX_TABLES)       */
  uint32_t table_pre;        /* interned id of table "pre"  (UINT32_MAX if absent)  */
  uint32_t table_post;       /* interned id of table "post" (UINT32_MAX if absent)  */
  const uint32_t *iteration; /* [n_runs] Run.Iteration (data-types.go:82)          */
  const uint8_t *owned;      /* [n_runs] 1 = counted in cross-run reductions;
                                NULL = all owned (replicated run 0 on a shard: 0)   */
  const uint64_t *node_off;  /* [2*n_runs+1] first node of graph g                  */
  const uint64_t *edge_off;  /* [2*n_runs+1] first edge of graph g                  */
  const uint32_t *node_word; /* [V] NEMO_WORD(...)                                  */
  const uint32_t *label;     /* [V] interned label (exact interning, never a hash)  */
  const uint32_t *id_rank;   /* [V] rank of the node's ID string inside its graph,
                                or NULL when local index order == ID string order   */
  const uint32_t *edge_src;  /* [E] local index of the DUETO edge's source          */
  const uint32_t *edge_dst;  /* [E] local index of its target                       */
} nemo_corpus;

/* one accepted @next chain (graphing/preprocessing.go:108-138,249-305) */
typedef struct nemo_chain {
  uint32_t graph;  /* graph index g (2r or 2r+1)                                   */
  uint32_t k;      /* acceptance index: the _<k> of run_<1000+i>_<C>_<t>_collapsed_<k> */
  uint32_t head;   /* r1: local index, its table names the collapsed rule          */
  uint32_t tail;   /* rk: local index                                              */
  uint32_t len;    /* path length (relationships)                                  */
} nemo_chain;

/* one missing event of differential provenance (differential-provenance.go:82-146) */
typedef struct nemo_missing {
  uint32_t entry;  /* diff entry (index into the failed-run list)                  */
  uint32_t rule;   /* local index of the rule in run 0's post graph               */
} nemo_missing;

/* ---- run sharding --------------------------------------------
 * part_of_run[r] in [0, n_parts) for every run of the corpus: longest-first
 * (LPT) by the run's nodes + edges (pre + post graphs), each run to the least
 * loaded part, ties by index.  Host only; the node context (below) and the
 * one-process-per-GPU path use the same assignment.  The good run 0 is
 * replicated on every part by the caller (owned there by its own part only). */
int nemo_partition_runs(const nemo_corpus *corpus, uint32_t n_parts, uint32_t *part_of_run);

/* ---- context --------------------------------------------------------------
 * Replaces InitGraphDB / CloseDB (graphing/helpers.go:17-55, 58-86): no docker,
 * no 10 s sleep, no Bolt; binds one HIP device.                             */
typedef struct nemo_ctx nemo_ctx;
int nemo_ctx_create(int device, nemo_ctx **out);
/* Node context (SURVEY.md §8b Threading, §8e): one process drives `ndev`
 * devices (`devices` NULL = 0..ndev-1; ndev <= 0 = every visible device).  The
 * corpus given to nemo_load_corpus is run-sharded over them with
 * nemo_partition_runs (run 0 replicated), every entry point fans out over the
 * shards' streams and returns results in the corpus' global numbering
 * (graphs, runs, diff entries, pull slots), and the two cross-run exchanges
 * happen inside the library: the prototype vector is all-reduced with RCCL
 * (ncclSum over one communicator per device) and the reference diff mode's
 * failedRuns[0] label set is broadcast (ncclBroadcast) from its owner.  Shards
 * may share a device (a layout for testing on one GPU): they then exchange by
 * peer copies instead of RCCL.  nemo_protos_partial/_finalize take d_reduce =
 * NULL, nemo_set_stream / nemo_goal_labels / nemo_diffprov_labels are for
 * single-device contexts only.  Replaces InitGraphDB's one database for the
 * whole node (graphing/helpers.go:17-55; main.go:95 constructs one Neo4J). */
int nemo_ctx_create_node(int ndev, const int *devices, nemo_ctx **out);
/* Devices of a context (its shards' devices for a node context); returns the count. */
int nemo_node_devices(const nemo_ctx *ctx, int *devices, int cap);
void nemo_ctx_destroy(nemo_ctx *ctx);
const char *nemo_last_error(const nemo_ctx *ctx);
int nemo_abi_version(void);
/* Launch every kernel on `stream` (a hipStream_t, NULL = the context's own). */
int nemo_set_stream(nemo_ctx *ctx, void *stream);
/* Tuning / test knobs (value -1 restores the default).  None changes a result;
 * each selects which kernel tier runs, so the parity tests force every tier.
 *   "chains_lds_max"    largest chain subgraph H* (nodes) the @next-chain LDS
 *                       tiers take; larger graphs go to the component tier
 *   "chains_comp_max"   largest component the component tier runs in LDS on one
 *                       wave (larger ones take its workgroup-wide global path)
 *   "chains_glob_min_v" graphs with at least this many nodes take the deep
 *                       k_chains_glob tier (default 65536; next nemo_load_corpus)
 *   "build_lds_max"     largest graph (nodes) whose CSR + Kahn levels k_build
 *                       builds in LDS (also capped at 16384 nodes / 8192 edges
 *                       and by the corpus-sized LDS budget); from the next
 *                       nemo_load_corpus / nemo_rebuild
 *   "graph_lds_max"     largest graph (nodes) of the LDS graph tier of k_marksimp,
 *                       k_proto_lds, k_diff_lds and k_pull_lds (0 = off)
 *   "global_block"      workgroup size of the global-memory tiers: 256 or 1024
 *                       (default: 1024 when >= 1/8 of the graphs have >= 64k nodes)
 *   "stage_blocks"      nemo_stage_simplified's bulk copies: 0 = runtime copies
 *                       (default), else a copy kernel on this many workgroups
 *   "stage_sdma"        request nemo_stage_simplified's runtime copies as NoCU
 *                       (SDMA) copies (1) or plain D2H copies (0, default)
 *   "stage_cus"         CUs the copy stream's blit kernels may use (default 8,
 *                       0 = all); set before the first nemo_stage_simplified
 *   "stage_aux"         nemo_stage_simplified's hand-over kernels on the diff
 *                       stream behind the analysis queued so far (1, default)
 *                       or on the context's stream (0)
 *   "pull_aux"          the simplified pull on the diff stream behind the end of
 *                       nemo_simplify (1) or on the context's stream (0, default)
 *   "diff_fuse"         whole-graph diff walks finish LP rules, missing rows and
 *                       one-entry masks themselves (1, default) or hand them to
 *                       separate kernels (0; test knob)
 *   "build_marksimp"    k_build's graphs get their deferred mark + simplification
 *                       at the end of k_build, from the edges it holds (1), or
 *                       from k_marksimp in nemo_simplify (0, default)
 *   "load_parts"        corpora mostly of big graphs: edge uploads in this many
 *                       parts, each part's CSR build behind its own upload
 *                       (default 4; 1 = one upload, then the build)
 *   "load_async"        1: nemo_load_corpus returns once its work is queued; its
 *                       graph checks (validations, acyclicity) are reported by
 *                       the next nemo_rebuild / nemo_mark_holds / nemo_goal_labels /
 *                       nemo_pull_edges, which then leaves no corpus loaded
 *                       (0, default: nemo_load_corpus waits and reports them).
 *                       The corpus' arrays must stay valid until that call: the
 *                       uploads from page-locked memory may still be in flight
 *   "build_relax"       k_build's Kahn levels by relaxation sweeps over the edges
 *                       in registers, peeling if they give up (1), or by peeling
 *                       (0, default)
 *   "topo_ell"          deep graphs' Kahn levels by the edge-parallel k_topo_ell
 *                       (1) or one workgroup per graph, k_topo_deep (0, default) */
int nemo_set_option(nemo_ctx *ctx, const char *name, int64_t value);
/* Record a hipEvent pair around every launch (per-kernel timing, see nemo_timings). */
int nemo_set_timing(nemo_ctx *ctx, int enable);
/* Restrict the timing to these groups (comma-separated names as nemo_timings
 * reports them, e.g. "k_build"); NULL or "" = every group.  An event pair
 * costs the stream a few microseconds: a benchmark times only the kernel it
 * prices against the roofline.                                              */
int nemo_set_timing_groups(nemo_ctx *ctx, const char *groups);

/* ---- load (loadProv, graphing/pre-post-prov.go:25-213) ---------------------
 * Copies the corpus to HBM, builds forward + reverse CSR and the topological
 * levels of every graph on the device, and validates like loadProv does:
 * dangling or duplicate DUETO edges and goal->goal / rule->rule edges fail with
 * the reference's "inserted number of edges" message (pre-post-prov.go:208-210).
 * Cycles fail with NEMO_ERR_CYCLE.  Host arrays may be freed on return.     */
int nemo_load_corpus(nemo_ctx *ctx, const nemo_corpus *corpus);
/* Page-lock (hipHostRegister) / release a caller-owned host buffer, so that
 * nemo_load_corpus uploads it by DMA instead of through the runtime's staging
 * copies: for corpora loaded more than once (a batch of a pass over a corpus
 * larger than HBM).  No reference counterpart (Neo4j reads its own store).  */
int nemo_host_register(const void *ptr, uint64_t bytes);
int nemo_host_unregister(const void *ptr);
/* Re-run the device part of the load (CSR + topo) on the resident corpus.    */
int nemo_rebuild(nemo_ctx *ctx);
uint64_t nemo_num_nodes(const nemo_ctx *ctx);
uint64_t nemo_num_edges(const nemo_ctx *ctx);

/* ---- markConditionHolds for every graph (pre-post-prov.go:218-244,247-285) */
int nemo_mark_holds(nemo_ctx *ctx);

/* ---- SimplifyProv for every run (preprocessing.go:351-387):
 * cleanCopyProv (:13-63) then collapseNextChains (:66-348), pre and post.   */
int nemo_simplify(nemo_ctx *ctx);

/* ---- prototypes (prototype.go:9-256) --------------------------------------
 * Cross-run reduction vector (u32, device memory, nemo_reduce_len entries):
 *   [0, T)        cnt[t]   = #owned success runs whose proto list holds t
 *   [T, 2T)       first[t] = table bits of the first success run's list
 *   2T            achvdCond (prototype.go:70)
 *   2T+1          first list non-empty (prototype.go:80-103)
 *   2T+2          #holding "pre" goals in raw pre graphs (extensions.go:25-49)
 *   2T+3          #owned runs
 * Every entry is a sum, so a multi-GPU job all-reduces it with ncclSum.     */
size_t nemo_reduce_len(const nemo_ctx *ctx);
int nemo_protos_partial(nemo_ctx *ctx, const uint32_t *success_iters, size_t n_success,
                        uint32_t *d_reduce /* device, nemo_reduce_len() u32; NULL = the context's own */);
/* Optional: queue the (reduced) vector's copy to pinned host memory on the
 * context's stream now, behind the caller's all-reduce, so that
 * nemo_protos_finalize on the same d_reduce only waits for it (no round trip
 * of its own).  A node context reduces inside finalize: a no-op there.      */
int nemo_protos_stage(nemo_ctx *ctx, const uint32_t *d_reduce);
/* Interprets a (reduced) vector (d_reduce NULL = the context's own): inter/union
 * table ids, ascending, "post" excluded (prototype.go:106,120).  Returns counts through n_inter/n_union;
 * `inter`/`uni` may be NULL to query sizes (capacity n_tables is enough).   */
int nemo_protos_finalize(nemo_ctx *ctx, const uint32_t *d_reduce, uint32_t *achieved,
                         uint32_t *inter, uint32_t *n_inter, uint32_t *uni, uint32_t *n_union,
                         uint64_t *pre_holds_count, uint32_t *n_runs_total);
/* Host-only interpretation of a (reduced) vector held in HOST memory; needs no
 * context or device (nemo_protos_finalize = D2H + this). */
int nemo_reduce_interpret(const uint32_t *h_reduce, uint32_t n_tables, uint32_t table_post, uint32_t *achieved,
                          uint32_t *inter, uint32_t *n_inter, uint32_t *uni, uint32_t *n_union);
/* The context's own (for a node context: the all-reduced) vector to host
 * memory, nemo_reduce_len() u32: for callers that reduce across processes
 * themselves from host memory.                                              */
int nemo_fetch_reduce(nemo_ctx *ctx, uint32_t *out, uint64_t cap);
/* Single-process convenience: partial + finalize with the context's own buffer. */
int nemo_prototypes(nemo_ctx *ctx, const uint32_t *success_iters, size_t n_success,
                    uint32_t *achieved, uint32_t *inter, uint32_t *n_inter,
                    uint32_t *uni, uint32_t *n_union);
/* missingFrom (prototype.go:141-206): entries of `proto` (table ids, in the
 * caller's order) absent from the table set of the failed run's simplified
 * post graph (run 1000+f).  `out` receives them in proto order.            */
int nemo_missing_from(nemo_ctx *ctx, uint32_t failed_iter, const uint32_t *proto, uint32_t n_proto,
                      uint32_t *out, uint32_t *n_out);

/* ---- differential provenance (differential-provenance.go:18-243) ----------
 * Good = run-0 post goals whose label is absent from the post goals of the
 * label source run; D = Fwd*(Good) ∩ Bwd*(Good); missing events = deepest
 * leaf-parent rules of D.  mode NEMO_DIFF_REFERENCE reproduces the reference's
 * in-place ###RUN### substitution (:43): every entry uses failed_iters[0] as
 * label source.  NEMO_DIFF_PER_RUN uses each entry's own failed run.        */
#define NEMO_DIFF_REFERENCE 0
#define NEMO_DIFF_PER_RUN   1
int nemo_diffprov(nemo_ctx *ctx, const uint32_t *failed_iters, size_t n_failed, int mode);
/* The run-sharded form of the reference mode (differential-provenance.go:22-43:
 * every entry uses failedRuns[0]'s labels, but that run lives on one shard).
 * nemo_goal_labels writes the goal labels of run `iteration`'s pre (cond 0) or
 * post (cond 1) graph into device memory as [n, label...] (cap >= the graph's
 * nodes + 1), enqueued on the context's stream without a host round trip; the
 * owner's buffer is then broadcast (RCCL) and every shard runs
 * nemo_diffprov_labels with it: failGoals = that set for every entry. */
int nemo_goal_labels(nemo_ctx *ctx, uint32_t iteration, int cond, uint32_t *d_out, uint64_t cap);
int nemo_diffprov_labels(nemo_ctx *ctx, const uint32_t *failed_iters, size_t n_failed, const uint32_t *d_labels,
                         uint64_t labels_cap);
/* The same with the label set in host memory (the caller interned it, e.g. a
 * chunked pipeline whose failedRuns[0] was analysed with an earlier chunk). */
int nemo_diffprov_host_labels(nemo_ctx *ctx, const uint32_t *failed_iters, size_t n_failed, const uint32_t *labels,
                              uint64_t n_labels);
/* D node mask over run 0's post graph for entry e (1 byte per node).        */
int nemo_fetch_diff_mask(nemo_ctx *ctx, uint32_t entry, uint8_t *out, uint64_t cap);
/* D masks of every entry, entry-major (n_entries * V0 bytes).               */
int nemo_fetch_diff_masks(nemo_ctx *ctx, uint8_t *out, uint64_t cap);
/* Zero-copy view of every entry's D mask (n_entries x v0 bytes) in library-
 * owned pinned memory, valid until the next nemo_diffprov.                  */
int nemo_diff_masks_view(nemo_ctx *ctx, const uint8_t **masks, uint64_t *n_entries, uint64_t *v0);
/* Missing rules of every entry; goals = all D-children of each rule.        */
int nemo_fetch_missing(nemo_ctx *ctx, nemo_missing *out, uint64_t cap, uint64_t *n_out);

/* ---- corrections / extensions on run 0 (corrections.go:25-193, extensions.go:13-99)
 * pre rows (a, g, r) of findPreTriggers, post rows (g, r) of findPostTriggers,
 * async rules of GenerateExtensions (only meaningful when not all achieved).  */
int nemo_triggers(nemo_ctx *ctx);
int nemo_fetch_triggers(nemo_ctx *ctx, uint32_t *pre_rows /* 3 per row */, uint64_t pre_cap,
                        uint64_t *n_pre, uint32_t *post_rows /* 2 per row */, uint64_t post_cap,
                        uint64_t *n_post, uint32_t *async_rules, uint64_t async_cap, uint64_t *n_async);

/* ---- results ---------------------------------------------------------------- */
/* Per-node flags (NEMO_F_*) of graphs [g_lo, g_hi), concatenated.           */
int nemo_fetch_node_flags(nemo_ctx *ctx, uint32_t g_lo, uint32_t g_hi, uint8_t *out, uint64_t cap);
/* Accepted @next chains of every graph, ordered by (graph, k).              */
int nemo_fetch_chains(nemo_ctx *ctx, nemo_chain *out, uint64_t cap, uint64_t *n_out);
/* Asynchronous hand-over of the simplification (SimplifyProv,
 * preprocessing.go:351-387) to the host, in the compact form a caller needs to
 * rebuild every simplified graph: 2 bits per node (NEMO_STATE_*; node v of the
 * corpus at byte v/4, bits 2*(v%4)) and every graph's accepted chains as dense
 * (head, tail) pairs (graph-local node indices; graph g's chain k at
 * chain_off[g] + k), copied into library-owned pinned memory on a second
 * stream, overlapping whatever the caller launches next.  State + pairs
 * determine the simplified graphs exactly (collapsed rule k of graph g:
 * preds(head) -> V_g + k -> succs(tail)); full flags stay available through
 * nemo_fetch_node_flags.                                                    */
#define NEMO_STATE_ALIVE 0x1u /* node is in the simplified graph (kept, not deleted) */
#define NEMO_STATE_HOLDS 0x2u /* condition_holds                                     */
int nemo_stage_simplified(nemo_ctx *ctx);
/* Waits for the staged copies and returns views into the pinned buffers:
 * state[ceil(V/4)], chain_off[G+1] and the pairs, chain_ht[n] as u32
 * head | tail << 16 when every graph has < 65536 nodes (*wide_pairs = 0),
 * else chain_ht[2n] as (head, tail) u32 (*wide_pairs = 1).  Valid until the
 * next nemo_stage_simplified or nemo_ctx_destroy.  Out-pointers may be NULL. */
int nemo_simplified_view(nemo_ctx *ctx, const uint8_t **state, const uint64_t **chain_off,
                         const uint32_t **chain_ht, uint64_t *n_chains, int *wide_pairs);
/* Per-run table bitsets, words = ceil(n_tables/32) u32 per run:
 *   which = 0: proto list of the run (extractProtos, prototype.go:11-24)
 *   which = 1: all rule tables of the simplified post graph (missingFrom)   */
int nemo_fetch_run_tables(nemo_ctx *ctx, int which, uint32_t *out, uint64_t cap);

/* ---- edge pulls (PullPrePostProv, pre-post-prov.go:288-459; Q24) -----------
 * which = 0: raw graphs, 1: simplified graphs (run 1000+i: kept, not deleted,
 * plus collapsed rules), 2: differential graphs of every diff entry.  The
 * compacted edge lists stay in HBM; `slot` below is the graph index (which
 * 0/1) or the diff entry (which 2).  Collapsed rule k of graph g is reported
 * as node index V_g + k.                                                   */
int nemo_pull_edges(nemo_ctx *ctx, int which);
uint64_t nemo_pulled_count(nemo_ctx *ctx, uint32_t slot);
int nemo_fetch_pulled(nemo_ctx *ctx, uint32_t slot, uint32_t *src, uint32_t *dst, uint64_t cap,
                      uint64_t *n_out);
/* Every slot at once (one call where the Go side would make one per graph):
 * off[slot] / cnt[slot] (pulled-slot count entries each) locate slot s's edges
 * in src/dst, whose used extent is *n_used (regions are claimed in device
 * order, so they are not sorted by slot; they are disjoint, except that diff
 * entries sharing a label source -- one D mask, one graph -- share one
 * region).  src/dst may be NULL to query *n_used; then cap >= *n_used.     */
int nemo_fetch_pulled_all(nemo_ctx *ctx, uint64_t *off, uint32_t *cnt, uint32_t *src, uint32_t *dst, uint64_t cap,
                          uint64_t *n_used);

/* ---- native ingest of a Molly output directory (host only) ------------------
 * Replaces Molly.LoadOutput's per-run JSON decoding (faultinjectors/molly.go:
 * 15-163) and the per-element interning of loadProv (pre-post-prov.go:25-213)
 * for callers that want the corpus arrays without a Go/Python decoding pass:
 * run_<i>_{pre,post}_provenance.json of runs i = 0..n_runs-1 are parsed on
 * `threads` threads (<= 0: up to 16) and interned in the order the sequential
 * loader would intern them.  `iterations[i]` is runs.json's Run.Iteration of
 * run i (the caller parses runs.json).  Validation failures return
 * NEMO_ERR_LOAD with the reference's message in `err`.  Node IDs are returned
 * without the run_<iteration>_<cond>_ prefix molly.go adds (it is common to a
 * graph, so id_rank is unaffected).                                          */
typedef struct nemo_ingest nemo_ingest;
#define NEMO_STR_TABLE     0  /* interned table names  (index < n_tables)      */
#define NEMO_STR_LABEL     1  /* interned labels                               */
#define NEMO_STR_NODE_ID   2  /* per node: Molly ID (unprefixed)               */
#define NEMO_STR_NODE_TYPE 3  /* per node: rule type ("" for goals)            */
#define NEMO_STR_NODE_TIME 4  /* per node: goal time after the clock rewrite   */
int nemo_ingest_molly(const char *out_dir, const uint32_t *iterations, uint32_t n_runs, int threads,
                      nemo_ingest **out, char *err, size_t err_cap);
/* Pointers into the ingest's arrays (valid until nemo_ingest_free); ready for nemo_load_corpus. */
int nemo_ingest_corpus(const nemo_ingest *h, nemo_corpus *corpus);
uint64_t nemo_ingest_count(const nemo_ingest *h, int kind);
int nemo_ingest_string(const nemo_ingest *h, int kind, uint64_t index, const char **s, size_t *len);
void nemo_ingest_free(nemo_ingest *h);
/* Streaming form: the same directory parsed chunk by chunk
 * so that chunk i is loaded and analysed on the device while chunk i+1 is
 * being parsed.  Interning is shared across chunks; ids are assigned in parse
 * order (below), so they can differ from nemo_ingest_molly's when run 0 or
 * failedRuns[0] is not first in runs.json; table "pre"/"post" ids are fixed
 * by the first chunk.  nemo_ingest_next parses the next `chunk` runs into a
 * corpus and, with `with_run0`, prepends the run of iteration 0 as a
 * replicated, not-owned run to every chunk after the one holding it (the good
 * run of the diffs, differential-provenance.go:26).  Parse order: the run of
 * iteration 0, then the run at index `first_failed` (failedRuns[0], whose
 * post-goal labels every reference-mode diff uses, :22-43; -1: none), then
 * the rest in runs.json order.  So with chunk >= 2 the first chunk holds
 * both, and every chunk that holds a failed run also holds the good run.
 * Returns NEMO_ERR_NOTFOUND when no run is left; validation failures as
 * nemo_ingest_molly.  Lifetime: the ingest keeps two buffers, so the arrays
 * of chunk i stay valid until the call that returns chunk i+2; chunk i can be
 * uploaded while chunk i+1 is parsed.                                      */
typedef struct nemo_ingest_stream nemo_ingest_stream;
int nemo_ingest_open(const char *out_dir, const uint32_t *iterations, uint32_t n_runs, int64_t first_failed,
                     int threads, nemo_ingest_stream **out);
int nemo_ingest_next(nemo_ingest_stream *s, uint32_t chunk, int with_run0, nemo_corpus *corpus, char *err,
                     size_t err_cap);
uint64_t nemo_ingest_stream_count(const nemo_ingest_stream *s, int kind);
int nemo_ingest_stream_string(const nemo_ingest_stream *s, int kind, uint64_t index, const char **str, size_t *len);
void nemo_ingest_close(nemo_ingest_stream *s);

/* ---- instrumentation ------------------------------------------------------ */
typedef struct nemo_timing {
  char name[32];      /* kernel name                                        */
  uint64_t launches;  /* launches recorded since the last reset             */
  double ms;          /* summed HIP-event time                              */
  double bytes;       /* summed algorithmic bytes     */
  double edges;       /* summed edges examined                              */
} nemo_timing;
int nemo_timings(nemo_ctx *ctx, nemo_timing *out, uint32_t cap, uint32_t *n_out);
int nemo_reset_timings(nemo_ctx *ctx);
int nemo_synchronize(nemo_ctx *ctx);
/* Inspection hook for tests: copy bytes of a named internal device array
 * ("topo", "lvl", "nlev", "fp", "fc", "rp", "rc", "flags", "dbits", "dmask"). */
int nemo_debug_copy(nemo_ctx *ctx, const char *name, void *out, uint64_t offset, uint64_t bytes);

#ifdef __cplusplus
}
#endif
#endif /* NEMOHIP_H */
