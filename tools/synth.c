/*
 * synth.c — deterministic synthetic Molly-shaped provenance corpora (bench and
 * test input generator; SURVEY.md §8d "Synthetic inputs").
 *
 * Per condition (pre/post) one base provenance DAG is grown top-down from the
 * condition's root goals, time-layered from EOT down to 1 (Dedalus @next and
 * @async rules step one timestep back; deductive rules stay in the timestep
 * and only use tables of higher stratum, so the DAG is acyclic).  Goals are
 * keyed by (table, location, value, time) so derivations share body goals.
 * Run r then injects message omissions (drops a few @async rule instances;
 * run 0 is fault-free) and keeps what is still derivable from the roots: the
 * run's pre/post provenance.  A run whose post roots are not all derivable is
 * a failed run.  Seeds: splitmix64(seed ^ r * 0x9E3779B97F4A7C15).
 *
 * Node IDs are "goal%08u"/"rule%08u" of the base index, so inside every run
 * graph the local node order equals the ID string order (id_rank = NULL).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/nemohip.h"

#define NREG 32u /* regular tables 0..31 */
#define T_CLOCK 32u
#define T_PRE 33u
#define T_POST 34u
#define NTAB 35u
#define RULE_LABEL_BASE 0xF0000000u

typedef struct synth_params {
  uint64_t seed;
  uint32_t n_runs;       /* runs generated: iterations run_base .. run_base+n_runs-1 */
  uint32_t run_base;
  uint32_t eot, nloc, nval, target_nodes;
  double p_fault;        /* probability that a run (other than 0) has omissions */
  uint32_t max_drops;    /* async rule instances dropped in a faulty run (1..max) */
  int prepend_run0;      /* shard mode: add run 0 (not owned) when run_base > 0 */
  int threads;
  uint32_t body_extra;   /* extra body atoms per rule, uniform on 0..2*body_extra (0: Molly-like 1-3 atoms) */
} synth_params;

typedef struct synth_out {
  uint32_t n_runs, n_tables, table_pre, table_post, table_clock;
  uint32_t eot, nloc, nval;
  uint32_t *iteration;
  uint8_t *status_ok, *owned;
  uint64_t *node_off, *edge_off;
  uint32_t *node_word, *label, *edge_src, *edge_dst, *base_id;
} synth_out;

static uint64_t splitmix64(uint64_t *s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static double urand(uint64_t *s) { return (splitmix64(s) >> 11) * (1.0 / 9007199254740992.0); }
static uint32_t urange(uint64_t *s, uint32_t n) { return (uint32_t)(urand(s) * n); }

/* Zipf(s = 1.1) over the regular tables */
static double zipf_cdf[NREG];
static void zipf_init(void) {
  double acc = 0;
  for (uint32_t i = 0; i < NREG; i++) {
    acc += 1.0 / __builtin_pow(i + 1.0, 1.1);
    zipf_cdf[i] = acc;
  }
  for (uint32_t i = 0; i < NREG; i++) zipf_cdf[i] /= acc;
}
static uint32_t zipf(uint64_t *s) {
  double u = urand(s);
  for (uint32_t i = 0; i < NREG; i++)
    if (u <= zipf_cdf[i]) return i;
  return NREG - 1;
}

typedef struct {
  uint32_t n, cap;
  uint32_t *word, *label;    /* per node                                   */
  uint8_t *is_rule, *type;
  uint32_t *key_t;           /* goal time                                  */
  uint32_t ne, ecap;
  uint32_t *es, *ed;
  /* hash map goal key -> node */
  uint64_t *hkey;
  uint32_t *hval, hcap;
  uint32_t nroots;
  uint32_t *roots;
} base_t;

static uint32_t add_node(base_t *b) {
  if (b->n == b->cap) {
    b->cap = b->cap ? 2 * b->cap : 1024;
    b->word = realloc(b->word, b->cap * sizeof *b->word);
    b->label = realloc(b->label, b->cap * sizeof *b->label);
    b->is_rule = realloc(b->is_rule, b->cap);
    b->type = realloc(b->type, b->cap);
    b->key_t = realloc(b->key_t, b->cap * sizeof *b->key_t);
  }
  return b->n++;
}
static void add_edge(base_t *b, uint32_t u, uint32_t v) {
  if (b->ne == b->ecap) {
    b->ecap = b->ecap ? 2 * b->ecap : 2048;
    b->es = realloc(b->es, b->ecap * sizeof *b->es);
    b->ed = realloc(b->ed, b->ecap * sizeof *b->ed);
  }
  b->es[b->ne] = u;
  b->ed[b->ne++] = v;
}

static uint64_t gkey(uint32_t tab, uint32_t loc, uint32_t val, uint32_t t) {
  return ((((uint64_t)tab * 64 + loc) * 65536 + val) * 65536 + t) + 1;
}
static uint32_t glabel(const synth_params *p, uint32_t tab, uint32_t loc, uint32_t val, uint32_t t) {
  return (((tab * p->nloc + loc) * p->nval + val) * (p->eot + 2)) + t;
}

static uint32_t hget(base_t *b, uint64_t k, int *found) {
  uint32_t h = (uint32_t)((k * 0x9E3779B97F4A7C15ull) >> 40) & (b->hcap - 1);
  while (b->hkey[h]) {
    if (b->hkey[h] == k) {
      *found = 1;
      return h;
    }
    h = (h + 1) & (b->hcap - 1);
  }
  *found = 0;
  return h;
}

/* goal node for (tab, loc, val, t), created on first use; new goals are queued */
static uint32_t goal(base_t *b, const synth_params *p, uint32_t tab, uint32_t loc, uint32_t val, uint32_t t,
                     uint32_t **q, uint32_t *qn, uint32_t *qcap) {
  uint64_t k = gkey(tab, loc, val, t);
  int f;
  uint32_t h = hget(b, k, &f);
  if (f) return b->hval[h];
  uint32_t v = add_node(b);
  b->is_rule[v] = 0;
  b->type[v] = 0;
  b->word[v] = NEMO_WORD(0, 0, tab);
  b->label[v] = glabel(p, tab, loc, val, t);
  b->key_t[v] = t;
  b->hkey[h] = k;
  b->hval[h] = v;
  if (*qn == *qcap) {
    *qcap *= 2;
    *q = realloc(*q, *qcap * sizeof **q);
  }
  (*q)[(*qn)++] = v;
  return v;
}

static void gen_base(base_t *b, const synth_params *p, uint32_t C, uint64_t seed) {
  memset(b, 0, sizeof *b);
  b->hcap = 1;
  while (b->hcap < 4 * p->target_nodes + 64) b->hcap <<= 1;
  b->hkey = calloc(b->hcap, sizeof *b->hkey);
  b->hval = calloc(b->hcap, sizeof *b->hval);
  uint32_t qcap = 1024, qn = 0, qh = 0;
  uint32_t *q = malloc(qcap * sizeof *q);
  uint64_t s = seed;
  /* goal decoding for expansion */
  uint32_t *gt = NULL, *gl = NULL, *gv = NULL;
  uint32_t gcap = 0;
  /* roots: C(n0, 0, t) for t in [eot/2, eot]; the condition holds from then on */
  uint32_t t0 = p->eot / 2 > 1 ? p->eot / 2 : 1;
  b->roots = malloc((p->eot + 2) * sizeof *b->roots);
  b->nroots = 0;
  b->roots = realloc(b->roots, ((p->eot + 2) * (size_t)p->nloc) * sizeof *b->roots);
  for (uint32_t l = 0; l < p->nloc; l++)
    for (uint32_t t = t0; t <= p->eot; t++) b->roots[b->nroots++] = goal(b, p, C, l, 0, t, &q, &qn, &qcap);
#define KEEP(v, tab, loc, val)                                \
  do {                                                        \
    if ((v) >= gcap) {                                        \
      gcap = 2 * ((v) + 1024);                                \
      gt = realloc(gt, gcap * 4);                             \
      gl = realloc(gl, gcap * 4);                             \
      gv = realloc(gv, gcap * 4);                             \
    }                                                         \
    gt[v] = (tab);                                            \
    gl[v] = (loc);                                            \
    gv[v] = (val);                                            \
  } while (0)
  for (uint32_t i = 0; i < b->nroots; i++) KEEP(b->roots[i], C, i / (p->eot - t0 + 1), 0);
  while (qh < qn) {
    const uint32_t x = q[qh++];
    const uint32_t tab = gt[x], loc = gl[x], val = gv[x], t = b->key_t[x];
    if (tab == T_CLOCK) continue;
    if (tab != C && (b->n >= p->target_nodes || (t <= 1 && urand(&s) < 0.8) || urand(&s) < 0.04)) continue; /* EDB */
    uint32_t nder = (tab != C && urand(&s) < 0.2) ? 2 : 1;
    for (uint32_t d = 0; d < nder; d++) {
      double u = urand(&s);
      uint32_t type = u < 0.55 ? NEMO_TYPE_NEXT : (u < 0.70 ? NEMO_TYPE_ASYNC : NEMO_TYPE_OTHER);
      if (tab == C) type = NEMO_TYPE_OTHER;
      if (t <= 1) type = NEMO_TYPE_OTHER;
      if (type == NEMO_TYPE_OTHER && tab != C && tab >= NREG - 2) type = t > 1 ? NEMO_TYPE_NEXT : 99;
      if (type == 99) continue;
      uint32_t r = add_node(b);
      b->is_rule[r] = 1;
      b->type[r] = (uint8_t)type;
      b->word[r] = NEMO_WORD(1, type, tab);
      b->label[r] = RULE_LABEL_BASE + tab;
      b->key_t[r] = t;
      add_edge(b, x, r);
      double ub = urand(&s);
      uint32_t nb = ub < 0.45 ? 1 : (ub < 0.85 ? 2 : 3);
      if (p->body_extra) nb += urange(&s, 2 * p->body_extra + 1);  /* denser corpora (C5's 4 edges per node) */
      for (uint32_t k = 0; k < nb; k++) {
        uint32_t bt, bl, bv, tt;
        if (type == NEMO_TYPE_NEXT) {
          tt = t - 1;
          if (k == 0) { /* persistence: the same fact one timestep earlier */
            bt = tab;
            bl = loc;
            bv = val;
          } else {
            bt = zipf(&s);
            bl = loc;
            bv = urange(&s, p->nval);
          }
        } else if (type == NEMO_TYPE_ASYNC) {
          tt = t - 1;
          bt = zipf(&s);
          bl = urange(&s, p->nloc);
          bv = urange(&s, p->nval);
          if (k == 0) { /* the message's clock(sender, receiver, t-1, t) */
            uint32_t v = goal(b, p, T_CLOCK, bl, loc, t, &q, &qn, &qcap);
            KEEP(v, T_CLOCK, bl, loc);
            add_edge(b, r, v);
          }
        } else {
          tt = t;
          bl = loc;
          bv = urange(&s, p->nval);
          if (tab == C) {
            bt = zipf(&s);
          } else {
            uint32_t lo = tab + 1;
            bt = lo + urange(&s, NREG - lo);
          }
        }
        uint32_t v = goal(b, p, bt, bl, bv, tt, &q, &qn, &qcap);
        KEEP(v, bt, bl, bv);
        /* a rule body never lists the same goal twice (MERGE would collapse it) */
        int dup = 0;
        for (uint32_t e = b->ne; e-- > 0 && b->es[e] == r;)
          if (b->ed[e] == v) dup = 1;
        if (!dup) add_edge(b, r, v);
      }
    }
  }
#undef KEEP
  free(q);
  free(gt);
  free(gl);
  free(gv);
}

static void free_base(base_t *b) {
  free(b->word);
  free(b->label);
  free(b->is_rule);
  free(b->type);
  free(b->key_t);
  free(b->es);
  free(b->ed);
  free(b->hkey);
  free(b->hval);
  free(b->roots);
}

/* CSR of the base graph + goals-first renumbering */
typedef struct {
  uint32_t n, ne;
  uint32_t *perm;      /* base node -> final id (goals first) */
  uint32_t *inv;
  uint32_t *fp, *fc;   /* forward adjacency (final ids) */
  uint32_t *word, *label;
  uint8_t *is_rule, *type;
  uint32_t *roots, nroots;
  uint32_t *topo;      /* reverse-topological (children before parents) */
} graph_t;

static void finalize(const base_t *b, graph_t *g) {
  const uint32_t n = b->n;
  g->n = n;
  g->ne = b->ne;
  g->perm = malloc(n * 4);
  g->inv = malloc(n * 4);
  uint32_t k = 0;
  for (uint32_t v = 0; v < n; v++)
    if (!b->is_rule[v]) g->perm[v] = k++;
  for (uint32_t v = 0; v < n; v++)
    if (b->is_rule[v]) g->perm[v] = k++;
  for (uint32_t v = 0; v < n; v++) g->inv[g->perm[v]] = v;
  g->word = malloc(n * 4);
  g->label = malloc(n * 4);
  g->is_rule = malloc(n);
  g->type = malloc(n);
  for (uint32_t v = 0; v < n; v++) {
    uint32_t f = g->perm[v];
    g->word[f] = b->word[v];
    g->label[f] = b->label[v];
    g->is_rule[f] = b->is_rule[v];
    g->type[f] = b->type[v];
  }
  g->fp = calloc(n + 1, 4);
  g->fc = malloc((b->ne + 1) * 4);
  for (uint32_t e = 0; e < b->ne; e++) g->fp[g->perm[b->es[e]] + 1]++;
  for (uint32_t v = 0; v < n; v++) g->fp[v + 1] += g->fp[v];
  uint32_t *cur = malloc((n + 1) * 4);
  memcpy(cur, g->fp, (n + 1) * 4);
  for (uint32_t e = 0; e < b->ne; e++) g->fc[cur[g->perm[b->es[e]]]++] = g->perm[b->ed[e]];
  free(cur);
  g->nroots = b->nroots;
  g->roots = malloc((b->nroots + 1) * 4);
  for (uint32_t i = 0; i < b->nroots; i++) g->roots[i] = g->perm[b->roots[i]];
  /* reverse topological order by DFS post-order (graph is a DAG) */
  g->topo = malloc((n + 1) * 4);
  uint8_t *st = calloc(n, 1);
  uint32_t *stack = malloc((n + 1) * 4), *it = malloc((n + 1) * 4);
  uint32_t nt = 0;
  for (uint32_t s0 = 0; s0 < n; s0++) {
    if (st[s0]) continue;
    uint32_t sp = 0;
    stack[sp] = s0;
    it[sp++] = g->fp[s0];
    st[s0] = 1;
    while (sp) {
      uint32_t v = stack[sp - 1];
      if (it[sp - 1] < g->fp[v + 1]) {
        uint32_t w = g->fc[it[sp - 1]++];
        if (!st[w]) {
          st[w] = 1;
          stack[sp] = w;
          it[sp++] = g->fp[w];
        }
      } else {
        g->topo[nt++] = v;
        sp--;
      }
    }
  }
  free(st);
  free(stack);
  free(it);
}

static void free_graph(graph_t *g) {
  free(g->perm);
  free(g->inv);
  free(g->fp);
  free(g->fc);
  free(g->word);
  free(g->label);
  free(g->is_rule);
  free(g->type);
  free(g->roots);
  free(g->topo);
}

/* derivable part of the base graph under dropped async rules; keep[] marks the
 * run's nodes (reachable from derivable roots through live rules).  Returns
 * 1 iff every root is derivable. */
static int run_subgraph(const graph_t *g, const uint8_t *dropped, uint8_t *ok, uint8_t *keep, uint32_t *stack) {
  const uint32_t n = g->n;
  for (uint32_t i = 0; i < n; i++) {
    uint32_t v = g->topo[i];
    if (g->is_rule[v]) {
      uint8_t o = !dropped[v];
      for (uint32_t j = g->fp[v]; j < g->fp[v + 1] && o; j++) o = ok[g->fc[j]];
      ok[v] = o;
    } else {
      if (g->fp[v + 1] == g->fp[v]) {
        ok[v] = 1; /* EDB fact */
      } else {
        uint8_t o = 0;
        for (uint32_t j = g->fp[v]; j < g->fp[v + 1]; j++) o |= ok[g->fc[j]];
        ok[v] = o;
      }
    }
  }
  memset(keep, 0, n);
  uint32_t sp = 0;
  int all = 1;
  for (uint32_t i = 0; i < g->nroots; i++) {
    uint32_t r = g->roots[i];
    if (!ok[r]) {
      all = 0;
      continue;
    }
    keep[r] = 1;
    stack[sp++] = r;
  }
  while (sp) {
    uint32_t v = stack[--sp];
    for (uint32_t j = g->fp[v]; j < g->fp[v + 1]; j++) {
      uint32_t w = g->fc[j];
      if (ok[w] && !keep[w]) {
        keep[w] = 1;
        stack[sp++] = w;
      }
    }
  }
  return all;
}

typedef struct {
  uint32_t *async_rules[2];
  uint32_t nasync[2];
} async_idx;

static void pick_drops(const synth_params *p, uint32_t it, const graph_t *g, const uint32_t *ar, uint32_t na,
                       uint8_t *dropped, uint32_t cond) {
  memset(dropped, 0, g->n);
  if (it == 0 || na == 0) return;
  uint64_t s = p->seed ^ ((uint64_t)it * 0x9E3779B97F4A7C15ull) ^ (cond * 0xD1B54A32D192ED03ull);
  splitmix64(&s);
  if (urand(&s) >= p->p_fault) return;
  uint32_t k = 1 + urange(&s, p->max_drops ? p->max_drops : 1);
  for (uint32_t i = 0; i < k; i++) dropped[ar[urange(&s, na)]] = 1;
}

int synth_generate(const synth_params *p, synth_out *o) {
  memset(o, 0, sizeof *o);
  if (!p || p->nloc == 0 || p->nloc > 64 || p->nval == 0 || p->nval > 1024 || p->eot < 2 || p->eot > 4000)
    return NEMO_ERR_INVALID;
  zipf_init();
  base_t b[2];
  graph_t g[2];
  for (uint32_t c = 0; c < 2; c++) {
    uint64_t s = p->seed ^ (0xC0FFEEull + c);
    gen_base(&b[c], p, c ? T_POST : T_PRE, splitmix64(&s));
    finalize(&b[c], &g[c]);
    free_base(&b[c]);
  }
  async_idx ai;
  for (uint32_t c = 0; c < 2; c++) {
    ai.async_rules[c] = malloc((g[c].n + 1) * 4);
    ai.nasync[c] = 0;
    for (uint32_t v = 0; v < g[c].n; v++)
      if (g[c].is_rule[v] && g[c].type[v] == NEMO_TYPE_ASYNC) ai.async_rules[c][ai.nasync[c]++] = v;
  }
  const int pre0 = p->prepend_run0 && p->run_base > 0;
  const uint32_t R = p->n_runs + (pre0 ? 1 : 0);
  o->n_runs = R;
  o->n_tables = NTAB;
  o->table_pre = T_PRE;
  o->table_post = T_POST;
  o->table_clock = T_CLOCK;
  o->eot = p->eot;
  o->nloc = p->nloc;
  o->nval = p->nval;
  o->iteration = malloc(R * 4);
  o->status_ok = malloc(R);
  o->owned = malloc(R);
  for (uint32_t r = 0; r < R; r++) {
    if (pre0) {
      o->iteration[r] = r == 0 ? 0 : p->run_base + r - 1;
      o->owned[r] = r != 0;
    } else {
      o->iteration[r] = p->run_base + r;
      o->owned[r] = 1;
    }
  }
  uint64_t *nn = calloc(2 * (size_t)R + 1, 8), *ne = calloc(2 * (size_t)R + 1, 8);
  int nth = p->threads > 0 ? p->threads : 1;
  /* pass 1: sizes */
#pragma omp parallel num_threads(nth)
  {
    uint8_t *dr = malloc(g[0].n > g[1].n ? g[0].n : g[1].n);
    uint8_t *ok = malloc(g[0].n > g[1].n ? g[0].n : g[1].n);
    uint8_t *keep = malloc(g[0].n > g[1].n ? g[0].n : g[1].n);
    uint32_t *stk = malloc(4 * (size_t)(g[0].n > g[1].n ? g[0].n : g[1].n));
#pragma omp for schedule(dynamic, 16)
    for (uint32_t r = 0; r < R; r++) {
      int post_ok = 1;
      for (uint32_t c = 0; c < 2; c++) {
        pick_drops(p, o->iteration[r], &g[c], ai.async_rules[c], ai.nasync[c], dr, c);
        int all = run_subgraph(&g[c], dr, ok, keep, stk);
        if (c == 1) post_ok = all;
        uint64_t vn = 0, en = 0;
        for (uint32_t v = 0; v < g[c].n; v++)
          if (keep[v]) {
            vn++;
            for (uint32_t j = g[c].fp[v]; j < g[c].fp[v + 1]; j++) en += keep[g[c].fc[j]];
          }
        nn[2 * r + c + 1] = vn;
        ne[2 * r + c + 1] = en;
      }
      o->status_ok[r] = (uint8_t)post_ok;
    }
    free(dr);
    free(ok);
    free(keep);
    free(stk);
  }
  for (uint32_t i = 0; i < 2 * R; i++) {
    nn[i + 1] += nn[i];
    ne[i + 1] += ne[i];
  }
  o->node_off = nn;
  o->edge_off = ne;
  const uint64_t V = nn[2 * R], E = ne[2 * R];
  o->node_word = malloc((V + 1) * 4);
  o->label = malloc((V + 1) * 4);
  o->base_id = malloc((V + 1) * 4);
  o->edge_src = malloc((E + 1) * 4);
  o->edge_dst = malloc((E + 1) * 4);
  /* pass 2: fill */
#pragma omp parallel num_threads(nth)
  {
    uint32_t mx = g[0].n > g[1].n ? g[0].n : g[1].n;
    uint8_t *dr = malloc(mx), *ok = malloc(mx), *keep = malloc(mx);
    uint32_t *stk = malloc(4 * (size_t)mx), *loc = malloc(4 * (size_t)mx);
#pragma omp for schedule(dynamic, 16)
    for (uint32_t r = 0; r < R; r++) {
      for (uint32_t c = 0; c < 2; c++) {
        const graph_t *gg = &g[c];
        pick_drops(p, o->iteration[r], gg, ai.async_rules[c], ai.nasync[c], dr, c);
        run_subgraph(gg, dr, ok, keep, stk);
        uint64_t v0 = nn[2 * r + c], e0 = ne[2 * r + c];
        uint32_t k = 0;
        for (uint32_t v = 0; v < gg->n; v++)
          if (keep[v]) {
            loc[v] = k;
            o->node_word[v0 + k] = gg->word[v];
            o->label[v0 + k] = gg->label[v];
            o->base_id[v0 + k] = v;
            k++;
          }
        uint64_t e = e0;
        for (uint32_t v = 0; v < gg->n; v++) {
          if (!keep[v]) continue;
          for (uint32_t j = gg->fp[v]; j < gg->fp[v + 1]; j++) {
            uint32_t w = gg->fc[j];
            if (!keep[w]) continue;
            o->edge_src[e] = loc[v];
            o->edge_dst[e] = loc[w];
            e++;
          }
        }
      }
    }
    free(dr);
    free(ok);
    free(keep);
    free(stk);
    free(loc);
  }
  for (uint32_t c = 0; c < 2; c++) {
    free(ai.async_rules[c]);
    free_graph(&g[c]);
  }
  return NEMO_OK;
}

void synth_free(synth_out *o) {
  free(o->iteration);
  free(o->status_ok);
  free(o->owned);
  free(o->node_off);
  free(o->edge_off);
  free(o->node_word);
  free(o->label);
  free(o->edge_src);
  free(o->edge_dst);
  free(o->base_id);
  memset(o, 0, sizeof *o);
}

/* ---- Molly-format writer (the e2e bench's input; tools/synth.py to_molly in C) ----
 * runs.json + run_<i>_{pre,post}_provenance.json exactly as synth.to_molly
 * writes them (json.dump's default separators), one file per OpenMP task. */
typedef struct {
  char *p;
  size_t n, cap;
} sbuf;
static void sb_put(sbuf *b, const char *s, size_t n) {
  if (b->n + n + 1 > b->cap) {
    b->cap = (b->n + n + 1) * 2;
    b->p = realloc(b->p, b->cap);
  }
  memcpy(b->p + b->n, s, n);
  b->n += n;
}
static void sb_str(sbuf *b, const char *s) { sb_put(b, s, strlen(s)); }
static void sb_u(sbuf *b, uint64_t v) {
  char t[24];
  int k = 0;
  do t[k++] = (char)('0' + v % 10); while ((v /= 10));
  while (k) sb_put(b, &t[--k], 1);
}
static void sb_i(sbuf *b, int64_t v) {
  if (v < 0) {
    sb_put(b, "-", 1);
    v = -v;
  }
  sb_u(b, (uint64_t)v);
}
/* label text of an interned synthetic label (synth.py label_string) */
static void sb_label(sbuf *b, uint32_t lab, const char *const *names, uint32_t eot, uint32_t nloc, uint32_t nval,
                     int64_t *time_out) {
  if (lab >= RULE_LABEL_BASE) {
    sb_str(b, names[lab - RULE_LABEL_BASE]);
    return;
  }
  const uint32_t t = lab % (eot + 2);
  uint32_t rest = lab / (eot + 2);
  const uint32_t val = rest % nval;
  rest /= nval;
  const uint32_t loc = rest % nloc, tab = rest / nloc;
  const char *name = names[tab];
  sb_str(b, name);
  sb_str(b, "(n");
  sb_u(b, loc);
  if (!strcmp(name, "clock")) {
    sb_str(b, ", n");
    sb_u(b, val);
    sb_str(b, ", ");
    sb_i(b, (int64_t)t - 1);
    sb_str(b, ", ");
  } else if (!strcmp(name, "pre") || !strcmp(name, "post")) {
    sb_str(b, ", ");
  } else {
    sb_str(b, ", v");
    sb_u(b, val);
    sb_str(b, ", ");
  }
  sb_u(b, t);
  sb_str(b, ")");
  if (time_out) *time_out = t;
}
static void sb_id(sbuf *b, int rule, uint32_t base) {
  char t[16];
  snprintf(t, sizeof t, "%08u", base);
  sb_str(b, rule ? "rule" : "goal");
  sb_str(b, t);
}

int synth_write_molly(const char *dir, uint32_t n_runs, const uint32_t *iteration, const uint8_t *status_ok,
                      const uint64_t *node_off, const uint64_t *edge_off, const uint32_t *node_word,
                      const uint32_t *label, const uint32_t *edge_src, const uint32_t *edge_dst,
                      const uint32_t *base_id, uint32_t eot, uint32_t nloc, uint32_t nval, const char *const *names,
                      int threads) {
  static const char *types[3] = {"single", "next", "async"};
  int bad = 0;
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1) reduction(| : bad)
  for (int64_t g = 0; g < 2 * (int64_t)n_runs; g++) {
    const uint32_t r = (uint32_t)(g / 2);
    const char *cond = g % 2 ? "post" : "pre";
    const uint64_t n0 = node_off[g], n1 = node_off[g + 1], e0 = edge_off[g], e1 = edge_off[g + 1];
    sbuf b = {0, 0, 0};
    sb_str(&b, "{\"goals\": [");
    int first = 1;
    for (uint64_t v = n0; v < n1; v++) {
      if (node_word[v] & NEMO_NODE_RULE) continue;
      sb_str(&b, first ? "{\"id\": \"" : ", {\"id\": \"");
      first = 0;
      sb_id(&b, 0, base_id[v]);
      sb_str(&b, "\", \"label\": \"");
      int64_t t = 0;
      sb_label(&b, label[v], names, eot, nloc, nval, &t);
      sb_str(&b, "\", \"table\": \"");
      sb_str(&b, names[node_word[v] & NEMO_TABLE_MASK]);
      sb_str(&b, "\", \"time\": \"");
      sb_i(&b, t);
      sb_str(&b, "\"}");
    }
    sb_str(&b, "], \"rules\": [");
    first = 1;
    for (uint64_t v = n0; v < n1; v++) {
      if (!(node_word[v] & NEMO_NODE_RULE)) continue;
      sb_str(&b, first ? "{\"id\": \"" : ", {\"id\": \"");
      first = 0;
      sb_id(&b, 1, base_id[v]);
      sb_str(&b, "\", \"label\": \"");
      sb_label(&b, label[v], names, eot, nloc, nval, NULL);
      sb_str(&b, "\", \"table\": \"");
      sb_str(&b, names[node_word[v] & NEMO_TABLE_MASK]);
      sb_str(&b, "\", \"type\": \"");
      sb_str(&b, types[((node_word[v] >> NEMO_TYPE_SHIFT) & 7u) % 3]);
      sb_str(&b, "\"}");
    }
    sb_str(&b, "], \"edges\": [");
    for (uint64_t e = e0; e < e1; e++) {
      const uint64_t s = n0 + edge_src[e], d = n0 + edge_dst[e];
      sb_str(&b, e == e0 ? "{\"from\": \"" : ", {\"from\": \"");
      sb_id(&b, (node_word[s] & NEMO_NODE_RULE) != 0, base_id[s]);
      sb_str(&b, "\", \"to\": \"");
      sb_id(&b, (node_word[d] & NEMO_NODE_RULE) != 0, base_id[d]);
      sb_str(&b, "\"}");
    }
    sb_str(&b, "]}");
    char path[4096];
    snprintf(path, sizeof path, "%s/run_%u_%s_provenance.json", dir, r, cond);
    FILE *f = fopen(path, "wb");
    if (!f || fwrite(b.p, 1, b.n, f) != b.n) bad |= 1;
    if (f) fclose(f);
    free(b.p);
  }
  /* runs.json */
  sbuf b = {0, 0, 0};
  sb_str(&b, "[");
  for (uint32_t r = 0; r < n_runs; r++) {
    sb_str(&b, r ? ", {\"iteration\": " : "{\"iteration\": ");
    sb_u(&b, iteration[r]);
    sb_str(&b, status_ok[r] ? ", \"status\": \"success\"" : ", \"status\": \"failure\"");
    sb_str(&b, ", \"failureSpec\": {\"eot\": ");
    sb_u(&b, eot);
    sb_str(&b, ", \"eff\": ");
    sb_u(&b, eot > 3 ? eot - 2 : 1);
    sb_str(&b, ", \"maxCrashes\": 0, \"nodes\": [");
    for (uint32_t i = 0; i < nloc; i++) {
      sb_str(&b, i ? ", \"n" : "\"n");
      sb_u(&b, i);
      sb_str(&b, "\"");
    }
    sb_str(&b, "], \"crashes\": [], \"omissions\": []}, \"model\": {\"tables\": {\"pre\": [[\"n0\", \"");
    sb_u(&b, eot);
    sb_str(&b, "\"]], \"post\": [[\"n0\", \"");
    sb_u(&b, eot);
    sb_str(&b, "\"]]}}, \"messages\": []}");
  }
  sb_str(&b, "]");
  char path[4096];
  snprintf(path, sizeof path, "%s/runs.json", dir);
  FILE *f = fopen(path, "wb");
  if (!f || fwrite(b.p, 1, b.n, f) != b.n) bad |= 1;
  if (f) fclose(f);
  free(b.p);
  return bad ? -1 : 0;
}
