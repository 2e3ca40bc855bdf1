/*
 * nemo_oracle.c — TEST INFRASTRUCTURE ONLY (see nemo_oracle.h).
 *
 * Plain-C restatement of the reference's provenance analysis.  Each function
 * cites the reference lines whose Cypher / Go it restates; the closed forms are
 * those of SURVEY.md Appendix A and are themselves checked against the literal
 * path enumerator oracle/cypher_literal.py.  Parity against the reference
 * engine is UNPINNED (no reference outputs exist; see nemo_oracle.h).
 *
 * Loaded by tests/ (checker), __graft_entry__.smoke() (checker) and bench.py's
 * cpu_baseline leg (timed as the CPU port), never by the product library.
 */
#include "nemo_oracle.h"

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define IS_RULE(w) (((w) & NEMO_NODE_RULE) != 0u)
#define TYPE(w) (((w) & NEMO_TYPE_MASK) >> NEMO_TYPE_SHIFT)
#define TABLE(w) ((w) & NEMO_TABLE_MASK)
#define NONE 0xFFFFFFFFu

typedef struct {
  uint32_t head, tail, len, rank, iter;
} chain_rec;

typedef struct {
  uint32_t V, E, cond;        /* cond = table id of "pre" / "post"            */
  const uint32_t *word, *label, *rank_in;
  const uint32_t *es, *ed;
  uint32_t *fp, *fc, *rp, *rc; /* forward / reverse CSR, rows sorted         */
  uint32_t *topo;              /* Kahn order                                  */
  uint8_t *flags;              /* slice of oracle_out.flags                   */
  chain_rec *ch;               /* accepted chains, k order                    */
  uint32_t nch;
  int err;
  char msg[200];
  /* simplified graph' edges (pulls) */
  uint32_t *ps, *pd;
  uint64_t np;
} graph_t;

static inline uint32_t rank_of(const graph_t *g, uint32_t v) { return g->rank_in ? g->rank_in[v] : v; }
static inline uint32_t indeg(const graph_t *g, uint32_t v) { return g->rp[v + 1] - g->rp[v]; }
static inline uint32_t outdeg(const graph_t *g, uint32_t v) { return g->fp[v + 1] - g->fp[v]; }

static void gerr(graph_t *g, int code, const char *fmt, ...) {
  if (g->err) return;
  g->err = code;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g->msg, sizeof g->msg, fmt, ap);
  va_end(ap);
}

static int cmp_u32(const void *a, const void *b) {
  uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
  return x < y ? -1 : x > y;
}

/* counting-sort CSR with sorted rows */
static void csr(uint32_t V, uint32_t E, const uint32_t *key, const uint32_t *val, uint32_t **pp, uint32_t **pc) {
  uint32_t *p = calloc((size_t)V + 1, sizeof *p), *c = malloc(((size_t)E + 1) * sizeof *c);
  uint32_t *cur = malloc(((size_t)V + 1) * sizeof *cur);
  for (uint32_t e = 0; e < E; e++) p[key[e] + 1]++;
  for (uint32_t v = 0; v < V; v++) p[v + 1] += p[v];
  memcpy(cur, p, ((size_t)V + 1) * sizeof *cur);
  for (uint32_t e = 0; e < E; e++) c[cur[key[e]]++] = val[e];
  for (uint32_t v = 0; v < V; v++)
    if (p[v + 1] - p[v] > 1) qsort(c + p[v], p[v + 1] - p[v], sizeof *c, cmp_u32);
  free(cur);
  *pp = p;
  *pc = c;
}

/* loadProv validation (graphing/pre-post-prov.go:150-210): MATCH goal/rule by
 * label + MERGE; a goal->goal or rule->rule edge matches nothing and a
 * duplicate edge is merged away, so relationships-created falls short of
 * len(Edges) and loadProv fails with the message at :209. */
static void load_graph(graph_t *g, uint32_t iteration) {
  for (uint32_t e = 0; e < g->E; e++)
    if (g->es[e] >= g->V || g->ed[e] >= g->V) {
      gerr(g, NEMO_ERR_INVALID, "Run %u: edge %u references node index out of range", iteration, e);
      return;
    }
  csr(g->V, g->E, g->es, g->ed, &g->fp, &g->fc);
  csr(g->V, g->E, g->ed, g->es, &g->rp, &g->rc);
  uint32_t created = 0;
  for (uint32_t u = 0; u < g->V; u++)
    for (uint32_t j = g->fp[u]; j < g->fp[u + 1]; j++) {
      uint32_t v = g->fc[j];
      int dup = j > g->fp[u] && g->fc[j - 1] == v;
      int bip = IS_RULE(g->word[u]) != IS_RULE(g->word[v]);
      if (!dup && bip) created++;
    }
  if (created != g->E)
    gerr(g, NEMO_ERR_LOAD,
         "Run %u: inserted number of edges (%u) does not equal number of antecedent provenance edges (%u)",
         iteration, created, g->E);
}

/* Kahn order; the closed forms assume a DAG (SURVEY.md Appendix A preamble) */
static void topo_sort(graph_t *g, uint32_t iteration) {
  uint32_t *d = malloc(((size_t)g->V + 1) * sizeof *d);
  g->topo = malloc(((size_t)g->V + 1) * sizeof *g->topo);
  uint32_t h = 0, t = 0;
  for (uint32_t v = 0; v < g->V; v++) {
    d[v] = indeg(g, v);
    if (!d[v]) g->topo[t++] = v;
  }
  while (h < t) {
    uint32_t u = g->topo[h++];
    for (uint32_t j = g->fp[u]; j < g->fp[u + 1]; j++)
      if (--d[g->fc[j]] == 0) g->topo[t++] = g->fc[j];
  }
  if (t != g->V) gerr(g, NEMO_ERR_CYCLE, "Run %u: provenance graph is not acyclic", iteration);
  free(d);
}

/* markConditionHolds (graphing/pre-post-prov.go:218-244, Cypher :221-227):
 *   MATCH (g:Goal)-[*1]->(r:Rule)
 *   WHERE (:Goal{table:C})-->(:Rule{table:C})-->(g)
 *     AND NOT ()-->(:Goal{table:C})-->(:Rule{table:C})-->(g)
 *   WITH g.table AS rule  MATCH (n:Goal) WHERE n.table = C OR n.table = rule
 *   SET n.condition_holds = true
 * The WITH yields no row when no g qualifies, so nothing is set then. */
static void mark_holds(graph_t *g, uint32_t n_tables) {
  uint32_t C = g->cond;
  uint8_t *tq = calloc(n_tables + 1, 1);
  int any = 0;
  for (uint32_t x = 0; x < g->V; x++) {
    uint32_t w = g->word[x];
    if (IS_RULE(w) || outdeg(g, x) == 0) continue;
    int pos = 0, neg = 0;
    for (uint32_t j = g->rp[x]; j < g->rp[x + 1]; j++) {
      uint32_t rc = g->rc[j];
      if (TABLE(g->word[rc]) != C) continue;
      for (uint32_t i = g->rp[rc]; i < g->rp[rc + 1]; i++) {
        uint32_t t = g->rc[i];
        if (TABLE(g->word[t]) != C) continue;
        pos = 1;
        if (indeg(g, t) > 0) neg = 1;
      }
    }
    if (pos && !neg) {
      tq[TABLE(w)] = 1;
      any = 1;
    }
  }
  if (any)
    for (uint32_t x = 0; x < g->V; x++) {
      uint32_t w = g->word[x];
      if (!IS_RULE(w) && (TABLE(w) == C || tq[TABLE(w)])) g->flags[x] |= NEMO_F_HOLDS;
    }
  free(tq);
}

/* cleanCopyProv (graphing/preprocessing.go:13-63): APOC export of every
 * (g1:Goal)-[*0..]->(g2:Goal) path = all goals + every rule lying between two
 * goals, i.e. with in>0 and out>0 in the bipartite graph; edges induced. */
static void clean_copy(graph_t *g) {
  for (uint32_t x = 0; x < g->V; x++)
    if (!IS_RULE(g->word[x]) || (indeg(g, x) > 0 && outdeg(g, x) > 0)) g->flags[x] |= NEMO_F_KEPT;
}

static uint32_t uf_find(uint32_t *p, uint32_t x) {
  while (p[x] != x) {
    p[x] = p[p[x]];
    x = p[x];
  }
  return x;
}

static int cmp_chain(const void *a, const void *b) {
  const chain_rec *x = a, *y = b;
  if (x->len != y->len) return x->len > y->len ? -1 : 1; /* ORDER BY len DESC */
  if (x->rank != y->rank) return x->rank < y->rank ? -1 : 1;
  return x->iter < y->iter ? -1 : x->iter > y->iter;
}

/* The greedy of collapseNextChains (preprocessing.go:108-138), literally: per
 * weakly connected component of H*, recompute du (longest H*-path from v to a
 * rule that contains an unseen node; down[] while v itself is unseen) over the
 * whole component, accept the longest such path (canonical tie-break), mark
 * it seen, repeat.  O(chains x component): kept as the cross-check of
 * greedy_incremental (tests/test_oracle_greedy.py, NEMO_ORACLE_RESCAN=1). */
#define INH(v) ((g->flags[v] & NEMO_F_DELETED) != 0)
static uint32_t greedy_rescan(graph_t *g, const uint32_t *order, const uint32_t *cnt, uint32_t ncomp,
                              const int32_t *down, int32_t *du, uint8_t *unseen, chain_rec *ch) {
  uint32_t nch = 0;
  for (uint32_t c = 0; c < ncomp; c++) {
    const uint32_t *cn = order + cnt[c];
    uint32_t m = cnt[c + 1] - cnt[c];
    for (uint32_t iter = 0;; iter++) {
      for (uint32_t i = m; i-- > 0;) {
        uint32_t v = cn[i];
        if (unseen[v]) {
          du[v] = down[v];
          continue;
        }
        int32_t d = -1;
        for (uint32_t j = g->fp[v]; j < g->fp[v + 1]; j++) {
          uint32_t w = g->fc[j];
          if (INH(w) && du[w] >= 0 && du[w] + 1 > d) d = du[w] + 1;
        }
        du[v] = d;
      }
      int32_t lmax = -1;
      uint32_t s = NONE;
      for (uint32_t i = 0; i < m; i++) {
        uint32_t v = cn[i];
        if (!IS_RULE(g->word[v])) continue;
        if (du[v] > lmax || (du[v] == lmax && s != NONE && rank_of(g, v) < rank_of(g, s))) {
          lmax = du[v];
          s = v;
        }
      }
      if (lmax < 2) break;
      uint32_t v = s;
      int u = unseen[s];
      unseen[s] = 0;
      for (int32_t rem = lmax; rem > 0; rem--) {
        uint32_t best = NONE;
        for (uint32_t j = g->fp[v]; j < g->fp[v + 1]; j++) {
          uint32_t w = g->fc[j];
          if (!INH(w)) continue;
          int32_t val = u ? down[w] : du[w];
          if (val == rem - 1 && (best == NONE || rank_of(g, w) < rank_of(g, best))) best = w;
        }
        if (best == NONE) { /* impossible by construction of du/down */
          gerr(g, NEMO_ERR_INVALID, "internal: chain walk lost its path");
          break;
        }
        v = best;
        u |= unseen[v];
        unseen[v] = 0;
      }
      ch[nch].head = s;
      ch[nch].tail = v;
      ch[nch].len = (uint32_t)lmax;
      ch[nch].rank = rank_of(g, s);
      ch[nch].iter = iter;
      nch++;
    }
  }
  return nch;
}

/* Selection entries are u64 snapshots: du at push time (high word), then the
 * complement of the ID rank, so the max is the longest and, among equals, the
 * smallest rank (cmp_chain's tie-break).  The key never changes once pushed. */
static void sel_push(uint64_t **a, size_t *n, size_t *cap, uint64_t x) {
  if (*n == *cap) {
    *cap = *cap * 2 + 64;
    *a = realloc(*a, *cap * sizeof **a);
  }
  size_t i = (*n)++;
  while (i > 0 && (*a)[(i - 1) / 2] < x) {
    (*a)[i] = (*a)[(i - 1) / 2];
    i = (i - 1) / 2;
  }
  (*a)[i] = x;
}
static uint64_t sel_pop(uint64_t *a, size_t *n) {
  uint64_t top = a[0], x = a[--*n];
  size_t i = 0;
  for (;;) {
    size_t l = 2 * i + 1, r = l + 1, m = i;
    uint64_t best = x;
    if (l < *n && a[l] > best) m = l, best = a[l];
    if (r < *n && a[r] > best) m = r;
    if (m == i) break;
    a[i] = a[m];
    i = m;
  }
  if (*n) a[i] = x;
  return top;
}
#define SEL_KEY(d, r) (((uint64_t)(uint32_t)(d) << 32) | (uint64_t)(0xFFFFFFFFu - (r)))

/* Max-heap of node indices by H* topological position (greedy_incremental's
 * propagation order: children before parents). */
typedef struct {
  uint32_t *a;
  size_t n, cap;
  const uint32_t *pos;
} pos_heap;
static void pos_push(pos_heap *h, uint32_t x) {
  if (h->n == h->cap) {
    h->cap = h->cap * 2 + 64;
    h->a = realloc(h->a, h->cap * sizeof *h->a);
  }
  size_t i = h->n++;
  while (i > 0 && h->pos[h->a[(i - 1) / 2]] < h->pos[x]) {
    h->a[i] = h->a[(i - 1) / 2];
    i = (i - 1) / 2;
  }
  h->a[i] = x;
}
static uint32_t pos_pop(pos_heap *h) {
  uint32_t top = h->a[0], x = h->a[--h->n];
  size_t i = 0;
  for (;;) {
    size_t l = 2 * i + 1, r = l + 1, m = i;
    uint32_t best = x;
    if (l < h->n && h->pos[h->a[l]] > h->pos[best]) m = l, best = h->a[l];
    if (r < h->n && h->pos[h->a[r]] > h->pos[best]) m = r;
    if (m == i) break;
    h->a[i] = h->a[m];
    i = m;
  }
  if (h->n) h->a[i] = x;
  return top;
}

/* The same greedy without the rescans.  du only decreases as nodes become
 * seen, and only a seen node's du is recursive (an unseen node's du is its
 * down[]), so accepting a chain changes du on the chain's nodes and, through
 * seen parents only, above them: those are re-evaluated children-first from a
 * heap keyed by topological position.  The next chain's head (max du, then min
 * rank, over rules) comes from a max-heap of (du, rank) snapshots whose stale
 * entries (du changed since the push) are skipped.  Components need no
 * separate loops: a chain only changes du inside its own component, so each
 * component sees the same sequence of acceptances as greedy_rescan, and
 * `iter` (a global acceptance counter here) only breaks ties between chains
 * of the same head, i.e. of the same component, in the same relative order.
 * Cost: the re-evaluations above each chain (the seen ancestors whose length
 * drops), superlinear on deep graphs (~15 min for a C5-shape 1M-node graph)
 * but far below the rescan's O(chains x component). */
static uint32_t greedy_incremental(graph_t *g, const uint32_t *hs, uint32_t nh, const int32_t *down, int32_t *du,
                                   uint8_t *unseen, chain_rec *ch) {
  const uint32_t V = g->V;
  uint32_t *pos = malloc((size_t)V * sizeof *pos);
  uint32_t *of_rank = malloc((size_t)V * sizeof *of_rank); /* ID rank -> node */
  uint8_t *queued = calloc(V, 1);
  uint32_t *path = malloc(((size_t)nh + 1) * sizeof *path);
  pos_heap prop = {NULL, 0, 0, pos};
  uint64_t *sel = NULL;
  size_t nsel = 0, capsel = 0;
  for (uint32_t v = 0; v < V; v++) of_rank[rank_of(g, v)] = v;
  for (uint32_t i = 0; i < nh; i++) {
    const uint32_t v = hs[i];
    pos[v] = i;
    du[v] = down[v];
    if (IS_RULE(g->word[v]) && du[v] >= 2) sel_push(&sel, &nsel, &capsel, SEL_KEY(du[v], rank_of(g, v)));
  }
  uint32_t nch = 0;
  while (nsel) {
    const uint64_t e = sel_pop(sel, &nsel);
    const uint32_t s = of_rank[0xFFFFFFFFu - (uint32_t)e];
    if (du[s] != (int32_t)(e >> 32)) continue; /* stale: du[s] dropped since (re-pushed then if >= 2) */
    const int32_t lmax = du[s];
    uint32_t v = s, np = 0;
    int u = unseen[s];
    unseen[s] = 0;
    path[np++] = s;
    for (int32_t rem = lmax; rem > 0; rem--) {
      uint32_t best = NONE;
      for (uint32_t j = g->fp[v]; j < g->fp[v + 1]; j++) {
        uint32_t w = g->fc[j];
        if (!INH(w)) continue;
        int32_t val = u ? down[w] : du[w];
        if (val == rem - 1 && (best == NONE || rank_of(g, w) < rank_of(g, best))) best = w;
      }
      if (best == NONE) {
        gerr(g, NEMO_ERR_INVALID, "internal: chain walk lost its path");
        break;
      }
      v = best;
      u |= unseen[v];
      unseen[v] = 0;
      path[np++] = v;
    }
    ch[nch].head = s;
    ch[nch].tail = v;
    ch[nch].len = (uint32_t)lmax;
    ch[nch].rank = rank_of(g, s);
    ch[nch].iter = nch;
    nch++;
    if (g->err) break;
    /* du of the newly seen nodes and of their seen ancestors, children first */
    for (uint32_t i = 0; i < np; i++)
      if (!queued[path[i]]) {
        queued[path[i]] = 1;
        pos_push(&prop, path[i]);
      }
    while (prop.n) {
      const uint32_t x = pos_pop(&prop);
      queued[x] = 0;
      int32_t d = -1;
      for (uint32_t j = g->fp[x]; j < g->fp[x + 1]; j++) {
        uint32_t w = g->fc[j];
        if (INH(w) && du[w] >= 0 && du[w] + 1 > d) d = du[w] + 1;
      }
      if (d == du[x]) continue;
      du[x] = d;
      if (IS_RULE(g->word[x]) && d >= 2) sel_push(&sel, &nsel, &capsel, SEL_KEY(d, rank_of(g, x)));
      for (uint32_t j = g->rp[x]; j < g->rp[x + 1]; j++) {
        uint32_t p = g->rc[j];
        if (INH(p) && !unseen[p] && !queued[p]) {
          queued[p] = 1;
          pos_push(&prop, p);
        }
      }
    }
    /* the head's own entry was consumed: it stays a candidate at an unchanged
     * length (a changed one was pushed above) */
    if (du[s] == lmax) sel_push(&sel, &nsel, &capsel, SEL_KEY(du[s], rank_of(g, s)));
  }
  free(sel);
  free(prop.a);
  free(pos);
  free(of_rank);
  free(queued);
  free(path);
  return nch;
}
#undef INH

/* collapseNextChains (graphing/preprocessing.go:66-348) on the clean copy.
 * Q13 (:70-78) lists every path r1(next)-[*1..]->(g)-[*1..]->r2(next) whose
 * nodes are goals or next rules, longest first; the Go loop (:108-138) accepts
 * a path iff it has a node not seen in an accepted path.  Neo4j's tie order is
 * unspecified, so ties are broken canonically by the lexicographic sequence of
 * node-ID ranks.  Accepted paths are maximal; the next one accepted is "the
 * first path in that order that contains an unseen node", found here per
 * weakly connected component by longest-path DP (no path enumeration).
 * DETACH DELETE (:312-340) then removes every node on a chain path. */
static void collapse(graph_t *g) {
  const uint32_t V = g->V;
  uint8_t *f = g->flags;
  uint8_t *np = calloc(V + 1, 1), *nc = calloc(V + 1, 1);
#define ISNEXT(v) (IS_RULE(g->word[v]) && TYPE(g->word[v]) == NEMO_TYPE_NEXT && (f[v] & NEMO_F_KEPT))
  for (uint32_t x = 0; x < V; x++) {
    if (IS_RULE(g->word[x])) continue;
    for (uint32_t j = g->rp[x]; j < g->rp[x + 1]; j++)
      if (ISNEXT(g->rc[j])) np[x] = 1;
    for (uint32_t j = g->fp[x]; j < g->fp[x + 1]; j++)
      if (ISNEXT(g->fc[j])) nc[x] = 1;
  }
  uint8_t *gp = calloc(V + 1, 1), *gc = calloc(V + 1, 1);
  for (uint32_t x = 0; x < V; x++) {
    if (IS_RULE(g->word[x])) {
      if (!ISNEXT(x)) continue;
      for (uint32_t j = g->rp[x]; j < g->rp[x + 1]; j++)
        if (np[g->rc[j]]) gp[x] = 1;
      for (uint32_t j = g->fp[x]; j < g->fp[x + 1]; j++)
        if (nc[g->fc[j]]) gc[x] = 1;
      if (gp[x] || gc[x]) f[x] |= NEMO_F_DELETED;
      if (!gp[x] && gc[x]) f[x] |= NEMO_F_HEAD;
      if (gp[x] && !gc[x]) f[x] |= NEMO_F_TAIL;
    } else if (np[x] && nc[x]) {
      f[x] |= NEMO_F_DELETED;
    }
  }
#undef ISNEXT
  free(np);
  free(nc);
  free(gp);
  free(gc);
#define INH(v) ((f[v] & NEMO_F_DELETED) != 0)
  /* H* in topological order, longest chain-path lengths up/down */
  uint32_t nh = 0;
  uint32_t *hs = malloc(((size_t)V + 1) * sizeof *hs);
  for (uint32_t i = 0; i < V; i++)
    if (INH(g->topo[i])) hs[nh++] = g->topo[i];
  g->ch = NULL;
  g->nch = 0;
  if (!nh) {
    free(hs);
    return;
  }
  int32_t *down = malloc((size_t)V * sizeof *down), *du = malloc((size_t)V * sizeof *du);
  uint32_t *uf = malloc((size_t)V * sizeof *uf);
  uint8_t *unseen = calloc(V, 1);
  for (uint32_t i = nh; i-- > 0;) {
    uint32_t v = hs[i];
    int32_t d = IS_RULE(g->word[v]) ? 0 : -1;
    for (uint32_t j = g->fp[v]; j < g->fp[v + 1]; j++)
      if (INH(g->fc[j]) && down[g->fc[j]] + 1 > d) d = down[g->fc[j]] + 1;
    down[v] = d;
    uf[v] = v;
    unseen[v] = 1;
  }
  for (uint32_t i = 0; i < nh; i++) {
    uint32_t v = hs[i];
    for (uint32_t j = g->fp[v]; j < g->fp[v + 1]; j++)
      if (INH(g->fc[j])) {
        uint32_t a = uf_find(uf, v), b = uf_find(uf, g->fc[j]);
        if (a != b) uf[a > b ? a : b] = a < b ? a : b;
      }
  }
  /* bucket H* by component, keeping topological order inside each */
  uint32_t *cid = malloc((size_t)V * sizeof *cid), *cnt = calloc((size_t)nh + 1, sizeof *cnt);
  uint32_t ncomp = 0;
  uint32_t *rootmap = malloc((size_t)V * sizeof *rootmap);
  for (uint32_t i = 0; i < nh; i++) rootmap[hs[i]] = NONE;
  for (uint32_t i = 0; i < nh; i++) {
    uint32_t r = uf_find(uf, hs[i]);
    if (rootmap[r] == NONE) rootmap[r] = ncomp++;
    cid[hs[i]] = rootmap[r];
    cnt[cid[hs[i]] + 1]++;
  }
  for (uint32_t c = 0; c < ncomp; c++) cnt[c + 1] += cnt[c];
  uint32_t *order = malloc((size_t)nh * sizeof *order), *cur = malloc(((size_t)ncomp + 1) * sizeof *cur);
  memcpy(cur, cnt, ((size_t)ncomp + 1) * sizeof *cur);
  for (uint32_t i = 0; i < nh; i++) order[cur[cid[hs[i]]]++] = hs[i];
  chain_rec *ch = malloc(((size_t)nh + 1) * sizeof *ch);
  uint32_t nch = 0;
  if (getenv("NEMO_ORACLE_RESCAN"))
    nch = greedy_rescan(g, order, cnt, ncomp, down, du, unseen, ch);
  else
    nch = greedy_incremental(g, hs, nh, down, du, unseen, ch);
  qsort(ch, nch, sizeof *ch, cmp_chain);
  g->ch = ch;
  g->nch = nch;
#undef INH
  free(hs);
  free(down);
  free(du);
  free(uf);
  free(unseen);
  free(cid);
  free(cnt);
  free(rootmap);
  free(order);
  free(cur);
}

/* ---- simplified graph' = clean copy − deleted + collapsed rules --------------
 * Collapsed rule k (index V+k): CREATE (repl:Rule{type:"collapsed", table =
 * r1.table}) and MERGE pred->repl->succ for pred in goal parents of r1 and succ
 * in goal children of rk, computed before the deletion
 * (graphing/preprocessing.go:145-309).  Edges to deleted nodes vanish with the
 * DETACH DELETE. */
typedef struct {
  uint32_t n;                  /* V + nch                                      */
  uint8_t *alive;              /* [n]                                          */
  uint32_t *word;              /* [n] (collapsed: rule, table of r1)           */
  uint32_t *fp, *fc, *rp, *rc; /* CSR over alive nodes                         */
} gprime_t;

static void build_gprime(const graph_t *g, gprime_t *p, uint32_t **es_out, uint32_t **ed_out, uint64_t *ne_out) {
  const uint32_t V = g->V, n = V + g->nch;
  p->n = n;
  p->alive = calloc(n + 1, 1);
  p->word = malloc(((size_t)n + 1) * sizeof *p->word);
  for (uint32_t v = 0; v < V; v++) {
    p->word[v] = g->word[v];
    p->alive[v] = (g->flags[v] & NEMO_F_KEPT) && !(g->flags[v] & NEMO_F_DELETED);
  }
  for (uint32_t k = 0; k < g->nch; k++) {
    p->word[V + k] = NEMO_NODE_RULE | TABLE(g->word[g->ch[k].head]);
    p->alive[V + k] = 1;
  }
  uint64_t cap = (uint64_t)g->E + 16;
  for (uint32_t k = 0; k < g->nch; k++)
    cap += indeg(g, g->ch[k].head) + outdeg(g, g->ch[k].tail);
  uint32_t *es = malloc(cap * sizeof *es), *ed = malloc(cap * sizeof *ed);
  uint64_t ne = 0;
  for (uint32_t u = 0; u < V; u++) {
    if (!p->alive[u]) continue;
    for (uint32_t j = g->fp[u]; j < g->fp[u + 1]; j++)
      if (p->alive[g->fc[j]]) {
        es[ne] = u;
        ed[ne++] = g->fc[j];
      }
  }
  for (uint32_t k = 0; k < g->nch; k++) {
    uint32_t h = g->ch[k].head, t = g->ch[k].tail;
    for (uint32_t j = g->rp[h]; j < g->rp[h + 1]; j++)
      if (p->alive[g->rc[j]]) {
        es[ne] = g->rc[j];
        ed[ne++] = V + k;
      }
    for (uint32_t j = g->fp[t]; j < g->fp[t + 1]; j++)
      if (p->alive[g->fc[j]]) {
        es[ne] = V + k;
        ed[ne++] = g->fc[j];
      }
  }
  csr(n, (uint32_t)ne, es, ed, &p->fp, &p->fc);
  csr(n, (uint32_t)ne, ed, es, &p->rp, &p->rc);
  *es_out = es;
  *ed_out = ed;
  *ne_out = ne;
}

static void free_gprime(gprime_t *p) {
  free(p->alive);
  free(p->word);
  free(p->fp);
  free(p->fc);
  free(p->rp);
  free(p->rc);
}

/* extractProtos' per-run query (graphing/prototype.go:11-24) on graph':
 *   MATCH path = (root:Goal)-[*1]->(r1:Rule)-[*1..]->(r2:Rule)
 *   OPTIONAL MATCH (g:Goal{run, condition:"pre", condition_holds:true})
 *   WHERE size(existsSuccess) > 0 AND not(()-->(root))
 *   ... collect(DISTINCT rule.table)
 * = tables of {r1 with a goal child that has a rule child} ∪ {rules reachable
 * from the goal children of r1}, where r1 ranges over rule children of roots;
 * empty unless the clean pre graph still has a holding goal (gate). */
static void proto_tables(const gprime_t *p, int gate, uint32_t *bits) {
  if (!gate) return;
  const uint32_t n = p->n;
  uint8_t *r1 = calloc(n + 1, 1), *seen = calloc(n + 1, 1);
  uint32_t *q = malloc(((size_t)n + 1) * sizeof *q);
  uint32_t qh = 0, qt = 0;
  for (uint32_t v = 0; v < n; v++) {
    if (!p->alive[v] || IS_RULE(p->word[v]) || p->rp[v + 1] != p->rp[v]) continue;
    for (uint32_t j = p->fp[v]; j < p->fp[v + 1]; j++) r1[p->fc[j]] = 1; /* rule children of a root */
  }
  for (uint32_t r = 0; r < n; r++) {
    if (!r1[r]) continue;
    for (uint32_t j = p->fp[r]; j < p->fp[r + 1]; j++) {
      uint32_t g2 = p->fc[j];
      if (p->fp[g2 + 1] != p->fp[g2]) bits[TABLE(p->word[r]) >> 5] |= 1u << (TABLE(p->word[r]) & 31);
      if (!seen[g2]) {
        seen[g2] = 1;
        q[qt++] = g2;
      }
    }
  }
  while (qh < qt) {
    uint32_t u = q[qh++];
    if (IS_RULE(p->word[u])) bits[TABLE(p->word[u]) >> 5] |= 1u << (TABLE(p->word[u]) & 31);
    for (uint32_t j = p->fp[u]; j < p->fp[u + 1]; j++)
      if (!seen[p->fc[j]]) {
        seen[p->fc[j]] = 1;
        q[qt++] = p->fc[j];
      }
  }
  free(r1);
  free(seen);
  free(q);
}

/* missingFrom's table set (graphing/prototype.go:143-147): every rule of the
 * simplified post graph, collapsed rules included. */
static void graph_tables(const gprime_t *p, uint32_t *bits) {
  for (uint32_t v = 0; v < p->n; v++)
    if (p->alive[v] && IS_RULE(p->word[v])) bits[TABLE(p->word[v]) >> 5] |= 1u << (TABLE(p->word[v]) & 31);
}

static int find_run(const nemo_corpus *c, uint32_t iteration) {
  for (uint32_t r = 0; r < c->n_runs; r++)
    if (c->iteration[r] == iteration) return (int)r;
  return -1;
}

static int oerr(oracle_out *out, int code, const char *fmt, ...) {
  out->status = code;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(out->err, sizeof out->err, fmt, ap);
  va_end(ap);
  return code;
}

static int cmp_u32x2(const void *a, const void *b) {
  const uint32_t *x = a, *y = b;
  for (int i = 0; i < 2; i++)
    if (x[i] != y[i]) return x[i] < y[i] ? -1 : 1;
  return 0;
}
static int cmp_u32x3(const void *a, const void *b) {
  const uint32_t *x = a, *y = b;
  for (int i = 0; i < 3; i++)
    if (x[i] != y[i]) return x[i] < y[i] ? -1 : 1;
  return 0;
}

/* differential provenance for one entry (graphing/differential-provenance.go:22-146) */
/* gf == NULL: failGoals is the given label set (the sharded reference mode's
 * broadcast of failedRuns[0]'s labels, same set by construction) */
static void diff_entry(const graph_t *g0, const graph_t *gf, const uint32_t *set, uint32_t n_set, uint8_t *D,
                       uint32_t entry, nemo_missing **miss, uint64_t *nmiss, uint64_t *capmiss) {
  const uint32_t V = g0->V;
  /* failGoals = collect(failed.label) over (failed:Goal{run: F, condition:'post'}) (:23-24) */
  uint32_t nl = 0;
  uint32_t *L = malloc(((size_t)(gf ? gf->V : n_set) + 1) * sizeof *L);
  if (gf) {
    for (uint32_t v = 0; v < gf->V; v++)
      if (!IS_RULE(gf->word[v])) L[nl++] = gf->label[v];
  } else {
    for (uint32_t i = 0; i < n_set; i++) L[nl++] = set[i];
  }
  qsort(L, nl, sizeof *L, cmp_u32);
  uint8_t *fw = calloc(V + 1, 1), *bw = calloc(V + 1, 1);
  uint32_t *q = malloc(((size_t)V + 1) * sizeof *q);
  /* pathSucc = (root:Goal{run:0,post})-[*0..]->(goal:Goal{run:0,post}), both labels
   * NOT IN failGoals (:26-27): nodes on such paths = Fwd*(Good) ∩ Bwd*(Good) */
  uint32_t qh = 0, qt = 0;
  for (uint32_t v = 0; v < V; v++) {
    if (IS_RULE(g0->word[v])) continue;
    if (!bsearch(&g0->label[v], L, nl, sizeof *L, cmp_u32)) {
      fw[v] = bw[v] = 1;
      q[qt++] = v;
    }
  }
  uint32_t ngood = qt;
  while (qh < qt) {
    uint32_t u = q[qh++];
    for (uint32_t j = g0->fp[u]; j < g0->fp[u + 1]; j++)
      if (!fw[g0->fc[j]]) {
        fw[g0->fc[j]] = 1;
        q[qt++] = g0->fc[j];
      }
  }
  qh = 0;
  qt = 0;
  for (uint32_t v = 0; v < V; v++)
    if (bw[v]) q[qt++] = v;
  (void)ngood;
  while (qh < qt) {
    uint32_t u = q[qh++];
    for (uint32_t j = g0->rp[u]; j < g0->rp[u + 1]; j++)
      if (!bw[g0->rc[j]]) {
        bw[g0->rc[j]] = 1;
        q[qt++] = g0->rc[j];
      }
  }
  for (uint32_t v = 0; v < V; v++) D[v] = fw[v] && bw[v];
  /* missing events (:82-146): deepest rules with a D-leaf child */
  int32_t *depth = malloc(((size_t)V + 1) * sizeof *depth);
  for (uint32_t i = 0; i < V; i++) {
    uint32_t v = g0->topo[i];
    if (!D[v]) continue;
    int32_t d = 0;
    for (uint32_t j = g0->rp[v]; j < g0->rp[v + 1]; j++)
      if (D[g0->rc[j]] && depth[g0->rc[j]] + 1 > d) d = depth[g0->rc[j]] + 1;
    depth[v] = d;
  }
  int32_t maxlen = -1;
  uint8_t *lp = calloc(V + 1, 1);
  for (uint32_t r = 0; r < V; r++) {
    if (!D[r] || !IS_RULE(g0->word[r])) continue;
    for (uint32_t j = g0->fp[r]; j < g0->fp[r + 1]; j++) {
      uint32_t x = g0->fc[j];
      if (!D[x]) continue;
      int leaf = 1;
      for (uint32_t i = g0->fp[x]; i < g0->fp[x + 1]; i++)
        if (D[g0->fc[i]]) leaf = 0;
      if (leaf) lp[r] = 1;
    }
    if (lp[r] && depth[r] + 1 > maxlen) maxlen = depth[r] + 1;
  }
  for (uint32_t r = 0; r < V; r++)
    if (lp[r] && depth[r] + 1 == maxlen) {
      if (*nmiss == *capmiss) {
        *capmiss = *capmiss * 2 + 16;
        *miss = realloc(*miss, *capmiss * sizeof **miss);
      }
      (*miss)[*nmiss].entry = entry;
      (*miss)[*nmiss].rule = r;
      (*nmiss)++;
    }
  free(L);
  free(fw);
  free(bw);
  free(q);
  free(depth);
  free(lp);
}

int oracle_analyze(const nemo_corpus *c, const oracle_opts *o, oracle_out *out) {
  memset(out, 0, sizeof *out);
  out->run0 = -1;
  if (!c || !o || !c->node_off || !c->edge_off) return oerr(out, NEMO_ERR_INVALID, "null corpus");
  if (c->n_tables > NEMO_MAX_TABLES) return oerr(out, NEMO_ERR_LIMIT, "too many tables");
  const uint32_t G = 2 * c->n_runs, T = c->n_tables, W = (T + 31) / 32;
  out->n_graphs = G;
  out->words = W;
  out->n_tables = T;
  out->V = c->node_off[G];
  out->E = c->edge_off[G];
  out->flags = calloc(out->V + 1, 1);
  graph_t *gs = calloc((size_t)G + 1, sizeof *gs);
  for (uint32_t gi = 0; gi < G; gi++) {
    graph_t *g = &gs[gi];
    uint64_t n0 = c->node_off[gi], e0 = c->edge_off[gi];
    g->V = (uint32_t)(c->node_off[gi + 1] - n0);
    g->E = (uint32_t)(c->edge_off[gi + 1] - e0);
    g->cond = (gi & 1) ? c->table_post : c->table_pre;
    g->word = c->node_word + n0;
    g->label = c->label + n0;
    g->rank_in = c->id_rank ? c->id_rank + n0 : NULL;
    g->es = c->edge_src + e0;
    g->ed = c->edge_dst + e0;
    g->flags = out->flags + n0;
  }
  int nth = o->threads > 0 ? o->threads : 1;
  /* diff_only: the graphs CreateNaiveDiffProv reads, run 0's post graph and each entry's label source */
  uint8_t *need = calloc((size_t)G + 1, 1);
  if (o->diff_only) {
    int r0 = find_run(c, 0);
    if (r0 >= 0) need[2 * r0 + 1] = 1;
    for (size_t e = 0; e < o->n_failed && !o->diff_labels; e++) {
      int fr = find_run(c, o->diff_mode == NEMO_DIFF_PER_RUN ? o->failed_iters[e] : o->failed_iters[0]);
      if (fr >= 0) need[2 * fr + 1] = 1;
    }
  }
  /* LoadRawProvenance (pre-post-prov.go:247-285) then SimplifyProv (preprocessing.go:351-387) */
#pragma omp parallel for schedule(dynamic, 1) num_threads(nth)
  for (uint32_t gi = 0; gi < G; gi++) {
    graph_t *g = &gs[gi];
    if (o->diff_only && !need[gi]) continue;
    load_graph(g, c->iteration[gi / 2]);
    if (!g->err) topo_sort(g, c->iteration[gi / 2]);
    if (!g->err && !o->diff_only) {
      mark_holds(g, T);
      clean_copy(g);
      collapse(g);
    }
  }
  free(need);
  for (uint32_t gi = 0; gi < G; gi++)
    if (gs[gi].err) {
      oerr(out, gs[gi].err, "%s", gs[gi].msg);
      goto done;
    }
  if (o->diff_only) goto diff;
  /* graph' per graph: proto list (post), table set (post), pulled edges */
  out->proto_bits = calloc((size_t)c->n_runs * W + 1, sizeof(uint32_t));
  out->graph_tables = calloc((size_t)c->n_runs * W + 1, sizeof(uint32_t));
#pragma omp parallel for schedule(dynamic, 1) num_threads(nth)
  for (uint32_t gi = 0; gi < G; gi++) {
    graph_t *g = &gs[gi];
    gprime_t p;
    uint32_t *es, *ed;
    uint64_t ne;
    build_gprime(g, &p, &es, &ed, &ne);
    if (gi & 1) {
      const graph_t *pre = &gs[gi - 1];
      int gate = 0; /* OPTIONAL MATCH (g:Goal{run:1000+i, condition:"pre", condition_holds:true}) */
      for (uint32_t v = 0; v < pre->V; v++)
        if (!IS_RULE(pre->word[v]) && (pre->flags[v] & NEMO_F_HOLDS) && !(pre->flags[v] & NEMO_F_DELETED)) gate = 1;
      proto_tables(&p, gate, out->proto_bits + (size_t)(gi / 2) * W);
      graph_tables(&p, out->graph_tables + (size_t)(gi / 2) * W);
    }
    free_gprime(&p);
    if (o->skip_pulls) {
      free(es);
      free(ed);
    } else {
      g->ps = es;
      g->pd = ed;
      g->np = ne;
    }
  }
  /* chains, ordered by (graph, k) */
  uint64_t nch = 0;
  for (uint32_t gi = 0; gi < G; gi++) nch += gs[gi].nch;
  out->chains = malloc((nch + 1) * sizeof *out->chains);
  out->n_chains = nch;
  nch = 0;
  for (uint32_t gi = 0; gi < G; gi++)
    for (uint32_t k = 0; k < gs[gi].nch; k++) {
      nemo_chain *x = &out->chains[nch++];
      x->graph = gi;
      x->k = k;
      x->head = gs[gi].ch[k].head;
      x->tail = gs[gi].ch[k].tail;
      x->len = gs[gi].ch[k].len;
    }
  if (!o->skip_pulls) {
    out->pulled_off = calloc((size_t)G + 1, sizeof *out->pulled_off);
    for (uint32_t gi = 0; gi < G; gi++) out->pulled_off[gi + 1] = out->pulled_off[gi] + gs[gi].np;
    out->pulled_src = malloc((out->pulled_off[G] + 1) * sizeof(uint32_t));
    out->pulled_dst = malloc((out->pulled_off[G] + 1) * sizeof(uint32_t));
    for (uint32_t gi = 0; gi < G; gi++) {
      memcpy(out->pulled_src + out->pulled_off[gi], gs[gi].ps, gs[gi].np * sizeof(uint32_t));
      memcpy(out->pulled_dst + out->pulled_off[gi], gs[gi].pd, gs[gi].np * sizeof(uint32_t));
    }
  }
  /* cross-run reduction (prototype.go:29-130, extensions.go:25-49) */
  out->reduce = calloc(2 * (size_t)T + 4, sizeof(uint32_t));
  {
    uint32_t *R = out->reduce;
    for (size_t i = 0; i < o->n_success; i++) {
      int r = find_run(c, o->success_iters[i]);
      if (r < 0 || (c->owned && !c->owned[r])) continue;
      const uint32_t *b = out->proto_bits + (size_t)r * W;
      int nonempty = 0;
      for (uint32_t t = 0; t < T; t++)
        if (b[t >> 5] >> (t & 31) & 1) nonempty = 1;
      if (nonempty) {
        R[2 * T]++;
        for (uint32_t t = 0; t < T; t++) R[t] += b[t >> 5] >> (t & 31) & 1;
      }
      if (i == 0) {
        for (uint32_t t = 0; t < T; t++) R[T + t] = b[t >> 5] >> (t & 31) & 1;
        R[2 * T + 1] = (uint32_t)nonempty;
      }
    }
    for (uint32_t r = 0; r < c->n_runs; r++) {
      if (c->owned && !c->owned[r]) continue;
      R[2 * T + 3]++;
      const graph_t *g = &gs[2 * r];
      for (uint32_t v = 0; v < g->V; v++)
        if (!IS_RULE(g->word[v]) && TABLE(g->word[v]) == c->table_pre && (g->flags[v] & NEMO_F_HOLDS))
          R[2 * T + 2]++;
    }
    if (o->n_success == 0) {
      oerr(out, NEMO_ERR_INVALID, "no successful runs: extractProtos indexes iterProv[0] (prototype.go:80)");
      goto done;
    }
    out->achieved = R[2 * T];
    out->inter = malloc(((size_t)T + 1) * sizeof(uint32_t));
    out->uni = malloc(((size_t)T + 1) * sizeof(uint32_t));
    if (R[2 * T + 1]) {
      for (uint32_t t = 0; t < T; t++) {
        if (t == c->table_post) continue;
        if (R[T + t] && R[t] == R[2 * T]) out->inter[out->n_inter++] = t;
        if (R[t] > 0) out->uni[out->n_union++] = t;
      }
    }
  }
  /* differential provenance (differential-provenance.go:18-243) */
diff:
  out->run0 = find_run(c, 0);
  if (out->run0 >= 0 && o->n_failed > 0) {
    const graph_t *g0 = &gs[2 * out->run0 + 1];
    out->v0 = g0->V;
    out->n_entries = (uint32_t)o->n_failed;
    out->diff_mask = calloc((size_t)o->n_failed * g0->V + 1, 1);
    uint64_t capm = 0;
    for (uint32_t e = 0; e < o->n_failed; e++) {
      uint32_t src = o->diff_mode == NEMO_DIFF_PER_RUN && !o->diff_labels ? o->failed_iters[e] : o->failed_iters[0];
      int fr = find_run(c, o->diff_labels ? o->failed_iters[e] : src);
      if (fr < 0) {
        oerr(out, NEMO_ERR_NOTFOUND, "unknown failed run %u", src);
        goto done;
      }
      diff_entry(g0, o->diff_labels ? NULL : &gs[2 * fr + 1], o->diff_labels, (uint32_t)o->n_diff_labels,
                 out->diff_mask + (size_t)e * g0->V, e, &out->missing, &out->n_missing, &capm);
    }
  } else if (out->run0 >= 0) {
    out->v0 = gs[2 * out->run0 + 1].V;
  }
  /* triggers on run 0 (corrections.go:30-34,121-125) and async rules (extensions.go:63-67) */
  if (out->run0 >= 0 && !o->diff_only) {
    const graph_t *gp = &gs[2 * out->run0], *gq = &gs[2 * out->run0 + 1];
    uint64_t cap = 16;
    out->pre_rows = malloc(cap * 3 * sizeof(uint32_t));
#define HOLDS(gg, v) (((gg)->flags[v] & NEMO_F_HOLDS) != 0)
    for (uint32_t x = 0; x < gp->V; x++) {
      if (IS_RULE(gp->word[x]) || HOLDS(gp, x)) continue;
      for (uint32_t j = gp->rp[x]; j < gp->rp[x + 1]; j++) {
        uint32_t a = gp->rc[j];
        int hp = 0;
        for (uint32_t i = gp->rp[a]; i < gp->rp[a + 1]; i++)
          if (HOLDS(gp, gp->rc[i])) hp = 1;
        if (!hp) continue;
        for (uint32_t i = gp->fp[x]; i < gp->fp[x + 1]; i++) {
          if (out->n_pre == cap) {
            cap *= 2;
            out->pre_rows = realloc(out->pre_rows, cap * 3 * sizeof(uint32_t));
          }
          uint32_t *row = out->pre_rows + 3 * out->n_pre++;
          row[0] = a;
          row[1] = x;
          row[2] = gp->fc[i];
        }
      }
    }
    qsort(out->pre_rows, out->n_pre, 3 * sizeof(uint32_t), cmp_u32x3);
    cap = 16;
    out->post_rows = malloc(cap * 2 * sizeof(uint32_t));
    for (uint32_t x = 0; x < gq->V; x++) {
      if (IS_RULE(gq->word[x]) || !HOLDS(gq, x) || indeg(gq, x) == 0) continue;
      for (uint32_t j = gq->fp[x]; j < gq->fp[x + 1]; j++) {
        uint32_t r = gq->fc[j];
        int ok = 0;
        for (uint32_t i = gq->fp[r]; i < gq->fp[r + 1]; i++) {
          uint32_t y = gq->fc[i];
          if (!HOLDS(gq, y) && outdeg(gq, y) > 0) ok = 1;
        }
        if (!ok) continue;
        if (out->n_post == cap) {
          cap *= 2;
          out->post_rows = realloc(out->post_rows, cap * 2 * sizeof(uint32_t));
        }
        out->post_rows[2 * out->n_post] = x;
        out->post_rows[2 * out->n_post + 1] = r;
        out->n_post++;
      }
    }
    qsort(out->post_rows, out->n_post, 2 * sizeof(uint32_t), cmp_u32x2);
    out->async_rules = malloc(((size_t)gp->V + 1) * sizeof(uint32_t));
    for (uint32_t r = 0; r < gp->V; r++) {
      if (!IS_RULE(gp->word[r]) || TYPE(gp->word[r]) != NEMO_TYPE_ASYNC) continue;
      int hp = 0, np = 0, down = 0;
      for (uint32_t j = gp->rp[r]; j < gp->rp[r + 1]; j++) {
        if (HOLDS(gp, gp->rc[j])) hp = 1;
        else np = 1;
      }
      for (uint32_t j = gp->fp[r]; j < gp->fp[r + 1]; j++) {
        uint32_t y = gp->fc[j];
        if (!HOLDS(gp, y) && outdeg(gp, y) > 0) down = 1;
      }
      if ((hp && down) || np) out->async_rules[out->n_async++] = r;
    }
#undef HOLDS
  }
done:
  for (uint32_t gi = 0; gi < G; gi++) {
    graph_t *g = &gs[gi];
    free(g->fp);
    free(g->fc);
    free(g->rp);
    free(g->rc);
    free(g->topo);
    free(g->ch);
    free(g->ps);
    free(g->pd);
  }
  free(gs);
  return out->status;
}

void oracle_free(oracle_out *o) {
  free(o->flags);
  free(o->chains);
  free(o->proto_bits);
  free(o->graph_tables);
  free(o->reduce);
  free(o->inter);
  free(o->uni);
  free(o->diff_mask);
  free(o->missing);
  free(o->pre_rows);
  free(o->post_rows);
  free(o->async_rules);
  free(o->pulled_off);
  free(o->pulled_src);
  free(o->pulled_dst);
  memset(o, 0, sizeof *o);
}
