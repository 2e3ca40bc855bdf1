/*
 * nemo_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's provenance-graph analysis (at15/nemo,
 * graphing/ (Go) + the Cypher it sends to Neo4j 3.3.3/APOC 3.3.0.2), in the
 * O(V+E) closed forms of SURVEY.md Appendix A.  Only tests/, the smoke() of
 * __graft_entry__.py and bench.py's cpu_baseline leg may load it, and only as
 * the checker; the product (libnemohip) never links or calls it.
 *
 * Parity status: UNPINNED against the reference itself.  The reference has no
 * tests, no golden vectors and no fixtures, and neither Go, Java, Neo4j nor
 * docker exist in this container.  This restatement is checked
 * instead against oracle/cypher_literal.py, a literal path-enumerating
 * evaluator of the same Cypher statements, on random small graphs and on the
 * hand-derived quirk fixtures under tests/golden/.
 */
#ifndef NEMO_ORACLE_H
#define NEMO_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/nemohip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_opts {
  int threads;                    /* OpenMP threads over graphs (<=0: 1)        */
  const uint32_t *success_iters;  /* GetSuccessRunsIters() (molly.go:53)         */
  size_t n_success;
  const uint32_t *failed_iters;   /* GetFailedRunsIters()                       */
  size_t n_failed;
  int diff_mode;                  /* NEMO_DIFF_REFERENCE / NEMO_DIFF_PER_RUN     */
  int skip_pulls;                 /* 1: do not materialise simplified edge lists */
  const uint32_t *diff_labels;    /* non-NULL: failGoals label set of every diff entry
                                     (sharded reference mode: failedRuns[0]'s labels) */
  size_t n_diff_labels;
  int diff_only;                  /* 1: only CreateNaiveDiffProv (differential-provenance.go:18-146):
                                     load run 0's post graph and the label sources, no simplification,
                                     prototypes, pulls or triggers (implies skip_pulls)              */
} oracle_opts;

typedef struct oracle_out {
  int status;
  char err[256];
  uint64_t V, E;
  uint32_t n_graphs, words, n_tables;
  uint8_t *flags;            /* [V] NEMO_F_*                                   */
  nemo_chain *chains;        /* ordered by (graph, k)                          */
  uint64_t n_chains;
  uint32_t *proto_bits;      /* [n_runs*words] extractProtos list per run      */
  uint32_t *graph_tables;    /* [n_runs*words] rule tables of simplified post  */
  uint32_t *reduce;          /* [2T+4] see nemo_reduce_len()                    */
  uint32_t achieved;
  uint32_t *inter;  uint32_t n_inter;
  uint32_t *uni;    uint32_t n_union;
  /* differential provenance over run 0's post graph */
  int32_t run0;              /* run index of iteration 0, -1 if absent         */
  uint32_t v0;               /* nodes of run 0's post graph                    */
  uint32_t n_entries;
  uint8_t *diff_mask;        /* [n_entries * v0]                               */
  nemo_missing *missing;  uint64_t n_missing;
  /* run-0 trigger rows */
  uint32_t *pre_rows;   uint64_t n_pre;    /* (a, g, r)                       */
  uint32_t *post_rows;  uint64_t n_post;   /* (g, r)                          */
  uint32_t *async_rules; uint64_t n_async;
  /* simplified-graph edges per graph (collapsed rule k = V_g + k) */
  uint64_t *pulled_off;      /* [n_graphs+1]                                   */
  uint32_t *pulled_src, *pulled_dst;
} oracle_out;

int oracle_analyze(const nemo_corpus *c, const oracle_opts *o, oracle_out *out);
void oracle_free(oracle_out *out);

#ifdef __cplusplus
}
#endif
#endif
