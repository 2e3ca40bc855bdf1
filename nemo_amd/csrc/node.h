// node.h — internal interface between the single-device context (api.hip)
// and the node context (node.hip) that fans a corpus out over several devices.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/nemohip.h"

struct Node;

// api.hip: accessors of a context that node.hip drives through the public ABI
Node *ctx_node(const nemo_ctx *c);
nemo_ctx *ctx_new_facade(Node *n);  // a context whose every entry point dispatches to `n`
void ctx_delete_facade(nemo_ctx *c);
int ctx_fail(nemo_ctx *c, int code, const char *msg);
uint32_t *ctx_reduce_buf(nemo_ctx *c);  // the context's own reduction vector (device)
hipStream_t ctx_stream(nemo_ctx *c);
int ctx_device(const nemo_ctx *c);
int ctx_join_aux(nemo_ctx *c);  // the context's stream waits for its queued diff kernels

// node.hip: the node context's entry points (same contracts as nemohip.h)
void node_destroy(Node *n);
int node_set_stream(nemo_ctx *c, void *stream);
int node_set_option(nemo_ctx *c, const char *name, int64_t value);
int node_set_timing(nemo_ctx *c, int enable);
int node_set_timing_groups(nemo_ctx *c, const char *groups);
uint64_t node_num_nodes(const nemo_ctx *c);
uint64_t node_num_edges(const nemo_ctx *c);
int node_load_corpus(nemo_ctx *c, const nemo_corpus *in);
int node_rebuild(nemo_ctx *c);
int node_mark_holds(nemo_ctx *c);
int node_simplify(nemo_ctx *c);
size_t node_reduce_len(const nemo_ctx *c);
int node_protos_partial(nemo_ctx *c, const uint32_t *success, size_t n, uint32_t *d_red);
int node_protos_finalize(nemo_ctx *c, const uint32_t *d_red, uint32_t *achieved, uint32_t *inter, uint32_t *n_inter,
                         uint32_t *uni, uint32_t *n_union, uint64_t *pre_holds, uint32_t *n_runs_total);
int node_fetch_reduce(nemo_ctx *c, uint32_t *out, uint64_t cap);
int node_fetch_run_tables(nemo_ctx *c, int which, uint32_t *out, uint64_t cap);
int node_missing_from(nemo_ctx *c, uint32_t failed_iter, const uint32_t *proto, uint32_t n_proto, uint32_t *out,
                      uint32_t *n_out);
int node_diffprov(nemo_ctx *c, const uint32_t *failed, size_t n, int mode);
int node_diffprov_labels(nemo_ctx *c, const uint32_t *failed, size_t n, const uint32_t *d_labels, uint64_t cap);
int node_diffprov_host_labels(nemo_ctx *c, const uint32_t *failed, size_t n, const uint32_t *labels, uint64_t n_labels);
int node_goal_labels(nemo_ctx *c, uint32_t iteration, int cond, uint32_t *d_out, uint64_t cap);
int node_fetch_diff_mask(nemo_ctx *c, uint32_t entry, uint8_t *out, uint64_t cap);
int node_fetch_diff_masks(nemo_ctx *c, uint8_t *out, uint64_t cap);
int node_diff_masks_view(nemo_ctx *c, const uint8_t **masks, uint64_t *n_entries, uint64_t *v0);
int node_fetch_missing(nemo_ctx *c, nemo_missing *out, uint64_t cap, uint64_t *n_out);
int node_triggers(nemo_ctx *c);
int node_fetch_triggers(nemo_ctx *c, uint32_t *pre, uint64_t pre_cap, uint64_t *n_pre, uint32_t *post,
                        uint64_t post_cap, uint64_t *n_post, uint32_t *async_rules, uint64_t async_cap,
                        uint64_t *n_async);
int node_fetch_node_flags(nemo_ctx *c, uint32_t g_lo, uint32_t g_hi, uint8_t *out, uint64_t cap);
int node_fetch_chains(nemo_ctx *c, nemo_chain *out, uint64_t cap, uint64_t *n_out);
int node_stage_simplified(nemo_ctx *c);
int node_simplified_view(nemo_ctx *c, const uint8_t **state, const uint64_t **chain_off, const uint32_t **chain_ht,
                         uint64_t *n_chains, int *wide_pairs);
int node_pull_edges(nemo_ctx *c, int which);
uint64_t node_pulled_count(nemo_ctx *c, uint32_t slot);
int node_fetch_pulled(nemo_ctx *c, uint32_t slot, uint32_t *src, uint32_t *dst, uint64_t cap, uint64_t *n_out);
int node_fetch_pulled_all(nemo_ctx *c, uint64_t *off, uint32_t *cnt, uint32_t *src, uint32_t *dst, uint64_t cap,
                          uint64_t *n_used);
int node_debug_copy(nemo_ctx *c, const char *name, void *out, uint64_t offset, uint64_t bytes);
int node_synchronize(nemo_ctx *c);
int node_timings(nemo_ctx *c, nemo_timing *out, uint32_t cap, uint32_t *n_out);
int node_reset_timings(nemo_ctx *c);
