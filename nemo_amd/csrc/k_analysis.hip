// k_analysis.hip — markConditionHolds, cleanCopyProv, collapseNextChains and
// extractProtos as per-graph workgroup kernels (one graph per workgroup).
#include <algorithm>

#include "device.h"
#include "internal.h"
#include "marksimp.h"

namespace nemo {

// markConditionHolds (graphing/pre-post-prov.go:218-244): a goal g qualifies
// iff it has a rule child, some (C goal)->(C rule)->g exists, and no such
// pattern starts at a C goal that has a parent.  Tq = tables of qualifying
// goals (LDS bitset); if Tq is non-empty every goal whose table is C or in Tq
// holds.  Also counts holding "pre" goals for GenerateExtensions
// (extensions.go:25-49).  Resets every other flag bit of the graph.
template <int B>
__global__ __launch_bounds__(B) void k_mark(DevCorpus c, int skip_tier) {
  __shared__ uint32_t s_tq[NEMO_MAX_TABLES / 32];
  __shared__ uint32_t s_any, s_pre;
  const uint32_t g = blockIdx.x;
  if (c.err[g]) return;
  const GraphView gv = c.view(g);
  if (skip_tier && tier_fits(c.t_ms, gv.V, gv.E, gv.nlev)) return;  // k_marksimp's graph
  if (gv.V >= NEMO_CSR_BIG) return;                                      // k_mw_mark_*'s graph
  const uint32_t C = (g & 1) ? c.table_post : c.table_pre;
  for (uint32_t i = threadIdx.x; i < c.words; i += B) s_tq[i] = 0;
  if (threadIdx.x == 0) {
    s_any = 0;
    s_pre = 0;
  }
  __syncthreads();
  for (uint32_t x = threadIdx.x; x < gv.V; x += B) {
    const uint32_t w = gv.word[x];
    if (is_rule(w) || gv.outdeg(x) == 0) continue;
    bool pos = false, neg = false;
    for (uint32_t j = gv.rp[x]; j < gv.rp[x + 1]; j++) {
      const uint32_t rcn = gv.rc[j];
      if (table_of(gv.word[rcn]) != C) continue;
      for (uint32_t i = gv.rp[rcn]; i < gv.rp[rcn + 1]; i++) {
        const uint32_t t = gv.rc[i];
        if (table_of(gv.word[t]) != C) continue;
        pos = true;
        neg |= gv.indeg(t) > 0;
      }
    }
    if (pos && !neg) {
      atomicOr(&s_tq[table_of(w) >> 5], 1u << (table_of(w) & 31));
      s_any = 1;
    }
  }
  __syncthreads();
  const bool any = s_any != 0;
  uint32_t pre = 0;
  for (uint32_t x = threadIdx.x; x < gv.V; x += B) {
    const uint32_t w = gv.word[x];
    const uint32_t t = table_of(w);
    const bool h = any && !is_rule(w) && (t == C || ((s_tq[t >> 5] >> (t & 31)) & 1u));
    gv.flags[x] = h ? (uint8_t)NEMO_F_HOLDS : (uint8_t)0;
    pre += (h && t == c.table_pre) ? 1u : 0u;
  }
  if (pre) atomicAdd(&s_pre, pre);
  __syncthreads();
  if (threadIdx.x == 0) c.prehold[g] = s_pre;
}

// cleanCopyProv (preprocessing.go:13-63) + the local part of
// collapseNextChains (:66-348): KEPT = goal or rule with in>0 and out>0;
// on the clean graph a goal with a next-rule parent and a next-rule child, or
// a next rule with a next-rule grandparent or grandchild, lies on an @next
// chain and is DETACH DELETEd; heads/tails are the chain ends.
template <int B>
__global__ __launch_bounds__(B) void k_simplify_flags(DevCorpus c, int skip_tier) {
  __shared__ uint32_t s_hold;
  const uint32_t g = blockIdx.x;
  if (c.err[g]) return;
  const GraphView gv = c.view(g);
  if (skip_tier && tier_fits(c.t_ms, gv.V, gv.E, gv.nlev)) return;  // k_marksimp's graph
  if (gv.V >= NEMO_CSR_BIG) return;                                      // k_mw_simplify_*'s graph
  uint8_t *f = gv.flags;
  for (uint32_t x = threadIdx.x; x < gv.V; x += B) {
    uint8_t fl = f[x] & NEMO_F_HOLDS;
    if (!is_rule(gv.word[x]) || (gv.indeg(x) > 0 && gv.outdeg(x) > 0)) fl |= NEMO_F_KEPT;
    f[x] = fl;
  }
  __syncthreads();
#define ISNEXT(v) (is_rule(gv.word[v]) && type_of(gv.word[v]) == NEMO_TYPE_NEXT && (f[v] & NEMO_F_KEPT))
  for (uint32_t x = threadIdx.x; x < gv.V; x += B) {
    if (is_rule(gv.word[x])) continue;
    uint8_t b = 0;
    for (uint32_t j = gv.rp[x]; j < gv.rp[x + 1]; j++)
      if (ISNEXT(gv.rc[j])) b |= FT_NP;
    for (uint32_t j = gv.fp[x]; j < gv.fp[x + 1]; j++)
      if (ISNEXT(gv.fc[j])) b |= FT_NC;
    f[x] |= b;
  }
  __syncthreads();
  for (uint32_t x = threadIdx.x; x < gv.V; x += B) {
    if (!ISNEXT(x)) continue;
    bool gp = false, gc = false;
    for (uint32_t j = gv.rp[x]; j < gv.rp[x + 1]; j++) gp |= (f[gv.rc[j]] & FT_NP) != 0;
    for (uint32_t j = gv.fp[x]; j < gv.fp[x + 1]; j++) gc |= (f[gv.fc[j]] & FT_NC) != 0;
    uint8_t fl = f[x];
    if (gp || gc) fl |= NEMO_F_DELETED;
    if (!gp && gc) fl |= NEMO_F_HEAD;
    if (gp && !gc) fl |= NEMO_F_TAIL;
    f[x] = fl;
  }
#undef ISNEXT
  __syncthreads();
  bool hold = false;
  for (uint32_t x = threadIdx.x; x < gv.V; x += B) {
    if (is_rule(gv.word[x])) continue;
    uint8_t fl = f[x];
    if ((fl & FT_NP) && (fl & FT_NC)) fl |= NEMO_F_DELETED;
    f[x] = fl & (uint8_t)~(FT_NP | FT_NC);
    hold |= (fl & (NEMO_F_HOLDS | NEMO_F_DELETED)) == NEMO_F_HOLDS;
  }
  // extractProtos' gate (prototype.go:13): a holding goal of the simplified graph
  if (threadIdx.x == 0) s_hold = 0;
  __syncthreads();
  if (__any(hold) && lane_id() == 0) s_hold = 1;
  __syncthreads();
  if (threadIdx.x == 0) c.holdany[g] = s_hold;
}

// The same two kernels for the big graphs (V >= NEMO_CSR_BIG: the deep
// corpora's 1M-node graphs, few per corpus): one workgroup per graph leaves
// the chip latency-bound on dependent row reads, so each phase runs as its own
// multi-workgroup kernel over the host's list of big graphs (2D grid: x =
// chunk of the graph, y = list slot; kernel boundaries replace the barriers).
// markConditionHolds' table set Tq and its any-flag are ORed per graph into
// scratch (c.s_c at the graph's V+G slice: [0] any, [1 + w] Tq words).
#define MW_BLOCK 256
#define MW_LOOP(c, skip, ...)                                                              \
  for (uint32_t b_ = blockIdx.y; b_ < c.n_big; b_ += gridDim.y) {                          \
    const uint32_t g = c.big[b_];                                                          \
    if (c.err[g]) continue;                                                                \
    const GraphView gv = c.view(g);                                                        \
    if (skip && tier_fits(c.t_ms, gv.V, gv.E, gv.nlev)) continue;                          \
    const uint32_t t0 = blockIdx.x * MW_BLOCK + threadIdx.x, stride = gridDim.x * MW_BLOCK; \
    uint32_t *tqg = c.s_c + gv.n0 + g;                                                     \
    (void)t0, (void)stride, (void)tqg;                                                     \
    __VA_ARGS__                                                                            \
  }
__global__ __launch_bounds__(MW_BLOCK) void k_mw_mark_z(DevCorpus c, int skip) {
  MW_LOOP(c, skip, {
    if (blockIdx.x == 0) {
      for (uint32_t i = threadIdx.x; i <= c.words; i += MW_BLOCK) tqg[i] = 0;
      if (threadIdx.x == 0) c.prehold[g] = 0;
    }
  })
}
__global__ __launch_bounds__(MW_BLOCK) void k_mw_mark_a(DevCorpus c, int skip) {
  __shared__ uint32_t s_tq[NEMO_MAX_TABLES / 32];
  __shared__ uint32_t s_any;
  MW_LOOP(c, skip, {
    const uint32_t C = (g & 1) ? c.table_post : c.table_pre;
    for (uint32_t i = threadIdx.x; i < c.words; i += MW_BLOCK) s_tq[i] = 0;
    if (threadIdx.x == 0) s_any = 0;
    __syncthreads();
    for (uint32_t x = t0; x < gv.V; x += stride) {
      const uint32_t w = gv.word[x];
      if (is_rule(w) || gv.outdeg(x) == 0) continue;
      bool pos = false, neg = false;
      for (uint32_t j = gv.rp[x]; j < gv.rp[x + 1]; j++) {
        const uint32_t rcn = gv.rc[j];
        if (table_of(gv.word[rcn]) != C) continue;
        for (uint32_t i = gv.rp[rcn]; i < gv.rp[rcn + 1]; i++) {
          const uint32_t t = gv.rc[i];
          if (table_of(gv.word[t]) != C) continue;
          pos = true;
          neg |= gv.indeg(t) > 0;
        }
      }
      if (pos && !neg) {
        atomicOr(&s_tq[table_of(w) >> 5], 1u << (table_of(w) & 31));
        s_any = 1;
      }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < c.words; i += MW_BLOCK)
      if (s_tq[i]) atomicOr(&tqg[1 + i], s_tq[i]);
    if (threadIdx.x == 0 && s_any) atomicOr(&tqg[0], 1u);
    __syncthreads();
  })
}
__global__ __launch_bounds__(MW_BLOCK) void k_mw_mark_b(DevCorpus c, int skip) {
  __shared__ uint32_t s_tq[NEMO_MAX_TABLES / 32 + 1];
  MW_LOOP(c, skip, {
    const uint32_t C = (g & 1) ? c.table_post : c.table_pre;
    for (uint32_t i = threadIdx.x; i <= c.words; i += MW_BLOCK) s_tq[i] = tqg[i];
    __syncthreads();
    const bool any = s_tq[0] != 0;
    uint32_t pre = 0;
    for (uint32_t x = t0; x < gv.V; x += stride) {
      const uint32_t w = gv.word[x];
      const uint32_t t = table_of(w);
      const bool h = any && !is_rule(w) && (t == C || ((s_tq[1 + (t >> 5)] >> (t & 31)) & 1u));
      gv.flags[x] = h ? (uint8_t)NEMO_F_HOLDS : (uint8_t)0;
      pre += (h && t == c.table_pre) ? 1u : 0u;
    }
    for (int d = 32; d >= 1; d >>= 1) pre += __shfl_xor(pre, d);
    if (lane_id() == 0 && pre) atomicAdd(&c.prehold[g], pre);
    __syncthreads();
  })
}
// cleanCopyProv + collapseNextChains' local flags, one kernel per phase
__global__ __launch_bounds__(MW_BLOCK) void k_mw_simplify_1(DevCorpus c, int skip) {
  MW_LOOP(c, skip, {
    uint8_t *f = gv.flags;
    if (t0 == 0) c.holdany[g] = 0;
    for (uint32_t x = t0; x < gv.V; x += stride) {
      uint8_t fl = f[x] & NEMO_F_HOLDS;
      if (!is_rule(gv.word[x]) || (gv.indeg(x) > 0 && gv.outdeg(x) > 0)) fl |= NEMO_F_KEPT;
      f[x] = fl;
    }
  })
}
#define ISNEXT(v) (is_rule(gv.word[v]) && type_of(gv.word[v]) == NEMO_TYPE_NEXT && (f[v] & NEMO_F_KEPT))
__global__ __launch_bounds__(MW_BLOCK) void k_mw_simplify_2(DevCorpus c, int skip) {
  MW_LOOP(c, skip, {
    uint8_t *f = gv.flags;
    for (uint32_t x = t0; x < gv.V; x += stride) {
      if (is_rule(gv.word[x])) continue;
      uint8_t b = 0;
      for (uint32_t j = gv.rp[x]; j < gv.rp[x + 1]; j++)
        if (ISNEXT(gv.rc[j])) b |= FT_NP;
      for (uint32_t j = gv.fp[x]; j < gv.fp[x + 1]; j++)
        if (ISNEXT(gv.fc[j])) b |= FT_NC;
      f[x] |= b;
    }
  })
}
__global__ __launch_bounds__(MW_BLOCK) void k_mw_simplify_3(DevCorpus c, int skip) {
  MW_LOOP(c, skip, {
    uint8_t *f = gv.flags;
    for (uint32_t x = t0; x < gv.V; x += stride) {
      if (!ISNEXT(x)) continue;
      bool gp = false, gc = false;
      for (uint32_t j = gv.rp[x]; j < gv.rp[x + 1]; j++) gp |= (f[gv.rc[j]] & FT_NP) != 0;
      for (uint32_t j = gv.fp[x]; j < gv.fp[x + 1]; j++) gc |= (f[gv.fc[j]] & FT_NC) != 0;
      uint8_t fl = f[x];
      if (gp || gc) fl |= NEMO_F_DELETED;
      if (!gp && gc) fl |= NEMO_F_HEAD;
      if (gp && !gc) fl |= NEMO_F_TAIL;
      f[x] = fl;
    }
  })
}
#undef ISNEXT
__global__ __launch_bounds__(MW_BLOCK) void k_mw_simplify_4(DevCorpus c, int skip) {
  MW_LOOP(c, skip, {
    uint8_t *f = gv.flags;
    bool hold = false;
    for (uint32_t x = t0; x < gv.V; x += stride) {
      if (is_rule(gv.word[x])) continue;
      uint8_t fl = f[x];
      if ((fl & FT_NP) && (fl & FT_NC)) fl |= NEMO_F_DELETED;
      f[x] = fl & (uint8_t)~(FT_NP | FT_NC);
      hold |= (fl & (NEMO_F_HOLDS | NEMO_F_DELETED)) == NEMO_F_HOLDS;
    }
    if (__any(hold) && lane_id() == 0) c.holdany[g] = 1;  // extractProtos' gate (prototype.go:13)
  })
}
#undef MW_LOOP

// extractProtos' per-run query (prototype.go:11-24) and missingFrom's table
// set (:143-147) on the simplified post graph, without materialising it:
// collapsed rule k is reached through its head (preds(r1) = goal parents of
// the head) and leads to the goal children of its tail.
//
// Global tier (post graphs k_proto_lds does not take: the deep corpora's 1M-
// node graphs), push form as k_proto_lds below.  The phases that are single
// passes over a graph run as multi-workgroup kernels over a device list of
// those runs (2D grid: x = chunk of the graph, y = list slot, kernel
// boundaries between phases); only the Kahn-level sweep keeps one workgroup
// per graph, and it issues a node's child pushes as independent
// batched parent loads.  Per-node SB_* bits live in c.sb (HBM); a collapsed
// rule's reach goes through per-tail chain lists built here (cl_first /
// cl_next, the graph's chains only).
#define PG_BLOCK 256
#define PG_SWEEP 64  // one wave per graph: a level has a few dozen nodes
#define SB_NR 0x20u      // goal has a REG or TAIL parent (not a root)

// k_proto_lds takes the graphs within its LDS tier (and its chain cap) that
// k_build built: their edges in source Kahn order are in c.e2 / c.posoff
__device__ __forceinline__ bool proto_lds_fits(const DevCorpus &c, const GraphView &gv) {
  return lds_fits(c, gv.V, gv.E, gv.nlev) && c.nch[gv.g] <= proto_chain_cap(gv.V) && c.bld_bytes &&
         gv.V <= c.bld_v && gv.E <= c.bld_e && !c.redo[gv.g];
}
__host__ __device__ __forceinline__ uint32_t *proto_list(const DevCorpus &c) { return c.sel + 3 * ((size_t)c.G + 1); }

__global__ __launch_bounds__(NEMO_BLOCK) void k_proto_sel(DevCorpus c) {
  const uint32_t r = blockIdx.x * NEMO_BLOCK + threadIdx.x;
  bool need = false;
  if (r < c.n_runs) {
    const uint32_t g = 2 * r + 1;
    need = !c.err[g] && !c.err[g - 1] && !proto_lds_fits(c, c.view(g));
  }
  uint32_t *lst = proto_list(c);
  wave_append(need, r, lst + 1, lst);
}

// per-run table bitsets accumulated per workgroup in LDS, ORed out once
struct PgBits {
  uint32_t w[NEMO_MAX_TABLES / 32];
};
__device__ __forceinline__ void pg_bits_clear(PgBits &b, uint32_t W) {
  for (uint32_t i = threadIdx.x; i < W; i += PG_BLOCK) b.w[i] = 0;
}
__device__ __forceinline__ void pg_bits_flush(PgBits &b, uint32_t *dst, uint32_t W) {
  for (uint32_t i = threadIdx.x; i < W; i += PG_BLOCK)
    if (b.w[i]) atomicOr(&dst[i], b.w[i]);
}
#define PG_LOOP(c, ...)                                                         \
  const uint32_t *lst_ = proto_list(c);                                         \
  const uint32_t nl_ = lst_[0];                                                 \
  for (uint32_t b_ = blockIdx.y; b_ < nl_; b_ += gridDim.y) {                   \
    const uint32_t r = lst_[1 + b_], g = 2 * r + 1;                             \
    const GraphView gv = c.view(g);                                             \
    __VA_ARGS__                                                                 \
  }
#define DEL(v) ((f[v] & NEMO_F_DELETED) != 0)
#define REG(v) ((f[v] & (NEMO_F_KEPT | NEMO_F_DELETED)) == NEMO_F_KEPT)
#define RULEISH(v) (REG(v) || (f[v] & NEMO_F_HEAD))

// clear the graph's SB bytes, its bitset rows and its chains' head lists
__global__ __launch_bounds__(PG_BLOCK) void k_pg_init(DevCorpus c) {
  PG_LOOP(c, {
    uint8_t *sb = c.sb + gv.n0;
    const uint32_t stride = gridDim.x * PG_BLOCK, t0 = blockIdx.x * PG_BLOCK + threadIdx.x;
    for (uint32_t x = t0; x < gv.V; x += stride) {
      sb[x] = 0;
      if (gv.flags[x] & NEMO_F_TAIL) c.cl_first[gv.n0 + x] = NEMO_NONE;  // every tail, linked below
    }
    if (blockIdx.x == 0)
      for (uint32_t i = threadIdx.x; i < c.words; i += PG_BLOCK) {
        c.proto_bits[(size_t)r * c.words + i] = 0;
        c.graph_tables[(size_t)r * c.words + i] = 0;
      }
  })
}
__global__ __launch_bounds__(PG_BLOCK) void k_pg_link(DevCorpus c) {
  PG_LOOP(c, {
    const uint32_t *ch = c.chain + 5 * gv.n0;
    for (uint32_t k = blockIdx.x * PG_BLOCK + threadIdx.x; k < c.nch[g]; k += gridDim.x * PG_BLOCK)
      c.cl_next[gv.n0 + k] = atomicExch(&c.cl_first[gv.n0 + ch[5 * k + 1]], k);
  })
}
// missingFrom's table set; not-root marks pushed from REG / TAIL rules; HASRC goals
__global__ __launch_bounds__(PG_BLOCK) void k_pg_a(DevCorpus c) {
  __shared__ PgBits s_t;
  PG_LOOP(c, {
    const uint8_t *f = gv.flags;
    uint8_t *sbg = c.sb;  // corpus-wide: or8 on n0 + x (n0 need not be 4-aligned)
    pg_bits_clear(s_t, c.words);
    __syncthreads();
    for (uint32_t x = blockIdx.x * PG_BLOCK + threadIdx.x; x < gv.V; x += gridDim.x * PG_BLOCK) {
      const uint32_t w = gv.word[x], j0 = gv.fp[x], j1 = gv.fp[x + 1];
      if (is_rule(w)) {
        if (RULEISH(x)) atomicOr(&s_t.w[table_of(w) >> 5], 1u << (table_of(w) & 31));
        if (REG(x) || (f[x] & NEMO_F_TAIL))
          for (uint32_t j = j0; j < j1; j++) or8(sbg, gv.n0 + gv.fc[j], SB_NR);
      } else if (!DEL(x)) {
        bool hasrc = false;
        for (uint32_t j = j0; j < j1 && !hasrc; j++) hasrc = RULEISH(gv.fc[j]);
        if (hasrc) or8(sbg, gv.n0 + x, SB_HASRC);
      }
    }
    __syncthreads();
    pg_bits_flush(s_t, c.graph_tables + (size_t)r * c.words, c.words);
    __syncthreads();
  })
}
// R1: the rule children of roots (a push to a non-REG/HEAD rule is never read)
__global__ __launch_bounds__(PG_BLOCK) void k_pg_b(DevCorpus c) {
  PG_LOOP(c, {
    const uint8_t *f = gv.flags;
    const uint8_t *sb = c.sb + gv.n0;
    for (uint32_t x = blockIdx.x * PG_BLOCK + threadIdx.x; x < gv.V; x += gridDim.x * PG_BLOCK) {
      if (is_rule(gv.word[x]) || DEL(x) || (sb[x] & SB_NR)) continue;
      for (uint32_t j = gv.fp[x]; j < gv.fp[x + 1]; j++) or8(c.sb, gv.n0 + gv.fc[j], SB_R1);
    }
  })
}
// G2 below R1 rules (regular, and collapsed through their chain's tail), with
// the R1 tables whose rule has a live goal child that has a rule child
__global__ __launch_bounds__(PG_BLOCK) void k_pg_c(DevCorpus c) {
  __shared__ PgBits s_s;
  PG_LOOP(c, {
    const uint8_t *f = gv.flags;
    const uint8_t *sb = c.sb + gv.n0;
    pg_bits_clear(s_s, c.words);
    __syncthreads();
    const uint32_t stride = gridDim.x * PG_BLOCK, t0 = blockIdx.x * PG_BLOCK + threadIdx.x;
    auto below = [&](uint32_t src, uint32_t table) {
      bool add = false;
      for (uint32_t j = gv.fp[src]; j < gv.fp[src + 1]; j++) {
        const uint32_t q = gv.fc[j];
        if (DEL(q)) continue;
        or8(c.sb, gv.n0 + q, SB_G2);
        add |= (sb[q] & SB_HASRC) != 0;
      }
      if (add) atomicOr(&s_s.w[table >> 5], 1u << (table & 31));
    };
    for (uint32_t x = t0; x < gv.V; x += stride) {
      const uint32_t w = gv.word[x];
      if (is_rule(w) && REG(x) && (sb[x] & SB_R1)) below(x, table_of(w));
    }
    const uint32_t *ch = c.chain + 5 * gv.n0;
    for (uint32_t k = t0; k < c.nch[g]; k += stride) {
      const uint32_t h = ch[5 * k];
      if (sb[h] & SB_R1) below(ch[5 * k + 1], table_of(gv.word[h]));
    }
    __syncthreads();
    pg_bits_flush(s_s, c.proto_bits + (size_t)r * c.words, c.words);
    __syncthreads();
  })
}
// rules reachable from G2: one wave per graph, one wave barrier per Kahn level
// (pull form: a node's parents lie on earlier levels, whose bits are final).
// Deep graphs have ~20k levels of a few dozen nodes, so the sweep is a chain
// of latencies, and one wave per graph lets many graphs share a CU (a
// 1024-thread workgroup had 15 idle waves per level and one graph per CU).
// The wave walks 64-position chunks of the Kahn order with a three-stage
// pipeline: the Kahn order of chunk k+2 and the static data of chunk k+1
// (node word, flags, row bounds, own SB byte) are loaded while chunk k reads
// its parents' SB bytes, so a chunk's critical path is the parent ids (PG_BATCH
// at a time) and their flag / SB bytes, not the four dependent loads before.
#define PG_BATCH 8  // parents of a node staged ahead (more: read in the chunk's own pass)
// One wave per graph walks the Kahn order in 64-position chunks.  A chunk's
// reads that do not depend on the sweep are staged ahead in a five-stage
// pipeline: chunk k+4's node ids, chunk k+3's static node data (word, flags,
// parent row, own SB byte), chunk k+2's first parents, chunk k+1's parents'
// flags; chunk k itself then waits on one round trip, its parents' SB bytes
// (written by earlier chunks of this wave: the level fence orders them).
// Every stage's loads of an iteration are issued together, chunk k's first.
__global__ __launch_bounds__(PG_SWEEP) void k_pg_sweep(DevCorpus c) {
  const uint32_t *lst = proto_list(c);
  const uint32_t ngr = lst[0];
  const uint32_t lane = threadIdx.x;
  for (uint32_t b = blockIdx.x; b < ngr; b += gridDim.x) {
    const uint32_t r = lst[1 + b], g = 2 * r + 1;
    const GraphView gv = c.view(g);
    const uint32_t nlev = gv.nlev;
    if (nlev == 0) continue;
    const uint8_t *__restrict__ f = gv.flags;
    uint8_t *sb = c.sb + gv.n0;
    const uint32_t *__restrict__ topo = gv.topo;
    const uint32_t *ch = c.chain + 5 * gv.n0, nch = c.nch[g];
    const uint32_t *clf = c.cl_first + gv.n0, *cln = c.cl_next + gv.n0;
    // chunk cursors (level, start, end): levels are contiguous, so the next
    // level starts where this one ends and only its end is loaded
    struct Cur {
      uint32_t l, s, e;
    };
    auto adv = [&](Cur q) {
      if (q.s + PG_SWEEP < q.e) {
        q.s += PG_SWEEP;
      } else {
        q.l++;
        q.s = q.e;
        q.e = q.l < nlev ? gv.lvl[q.l + 1] : q.e;
      }
      return q;
    };
    struct It {
      uint32_t x, w, fx, j0, j1, sbx;
      uint32_t p[PG_BATCH], fp[PG_BATCH];
    };
    auto ld_x = [&](const Cur &q) { return q.s + lane < q.e ? topo[q.s + lane] : NEMO_NONE; };
    auto ld_static = [&](uint32_t x) {
      It t;
      t.x = x;
      t.w = t.fx = t.j0 = t.j1 = t.sbx = 0;
      if (x != NEMO_NONE) {
        t.w = gv.word[x];
        t.fx = f[x];
        t.j0 = gv.rp[x];
        t.j1 = gv.rp[x + 1];
        t.sbx = sb[x];
      }
      return t;
    };
    auto ld_par = [&](It &t) {
#pragma unroll
      for (int q = 0; q < PG_BATCH; q++) t.p[q] = t.j0 + q < t.j1 ? gv.rc[t.j0 + q] : NEMO_NONE;
    };
    auto ld_pflag = [&](It &t) {
#pragma unroll
      for (int q = 0; q < PG_BATCH; q++) t.fp[q] = t.p[q] != NEMO_NONE ? f[t.p[q]] : 0u;
    };
    Cur c0{0, gv.lvl[0], gv.lvl[1]};
    Cur c1 = adv(c0), c2 = adv(c1), c3 = adv(c2), c4 = adv(c3);
    // prologue: chunk k through stage 3, k+1 through 2, k+2 through 1, k+3's ids
    It A = ld_static(ld_x(c0)), B = ld_static(ld_x(c1)), C = ld_static(ld_x(c2));
    uint32_t xD = ld_x(c3);
    ld_par(A);
    ld_par(B);
    ld_pflag(A);
    while (c0.l < nlev) {
      // chunk k's parents' SB bytes first, then every prefetch stage
      uint32_t bp[PG_BATCH];
#pragma unroll
      for (int q = 0; q < PG_BATCH; q++) bp[q] = A.p[q] != NEMO_NONE ? sb[A.p[q]] : 0u;
      const uint32_t xE = ld_x(c4);
      It D = ld_static(xD);
      ld_par(C);
      ld_pflag(B);
      // chunk k
      const uint32_t x = A.x, fx = A.fx;
      const bool rule = is_rule(A.w);
      const bool live = x != NEMO_NONE && (rule ? ((fx & (NEMO_F_KEPT | NEMO_F_DELETED)) == NEMO_F_KEPT ||
                                                    (fx & NEMO_F_HEAD))
                                                 : (fx & NEMO_F_DELETED) == 0);
      if (live) {
        // a rule is reached from a live G2 / RCH goal parent; a goal from an RCH
        // regular rule parent, or a tail parent one of whose chains has an RCH head
        const uint32_t want = rule ? (SB_G2 | SB_RCH) : SB_RCH;
        bool rch = false;
        auto parent = [&](uint32_t pq, uint32_t fpq, uint32_t bpq) {
          if (rule) {
            rch |= !(fpq & NEMO_F_DELETED) && (bpq & want);
          } else if ((fpq & (NEMO_F_KEPT | NEMO_F_DELETED)) == NEMO_F_KEPT) {
            rch |= (bpq & SB_RCH) != 0;
          } else if (fpq & NEMO_F_TAIL) {
            uint32_t hops = 0;
            for (uint32_t k = clf[pq]; k < nch && hops++ < nch && !rch; k = cln[k]) rch = (sb[ch[5 * k]] & SB_RCH) != 0;
          }
        };
#pragma unroll
        for (int q = 0; q < PG_BATCH; q++)
          if (A.p[q] != NEMO_NONE && !rch) parent(A.p[q], A.fp[q], bp[q]);
        for (uint32_t j = A.j0 + PG_BATCH; j < A.j1 && !rch; j++) {  // rows past the staged parents
          const uint32_t pq = gv.rc[j];
          parent(pq, f[pq], sb[pq]);
        }
        if (rch) sb[x] = (uint8_t)(A.sbx | SB_RCH);  // only x sets its own RCH bit
      }
      if (c1.l != c0.l) __syncthreads();  // the next chunk starts a level: this level's bits are final
      A = B;
      B = C;
      C = D;
      xD = xE;
      c0 = c1;
      c1 = c2;
      c2 = c3;
      c3 = c4;
      c4 = adv(c4);
    }
  }
}
// tables of the reached rules; then extractProtos' gate (prototype.go:13)
__global__ __launch_bounds__(PG_BLOCK) void k_pg_d(DevCorpus c) {
  __shared__ PgBits s_s;
  PG_LOOP(c, {
    const uint8_t *f = gv.flags;
    const uint8_t *sb = c.sb + gv.n0;
    pg_bits_clear(s_s, c.words);
    __syncthreads();
    for (uint32_t x = blockIdx.x * PG_BLOCK + threadIdx.x; x < gv.V; x += gridDim.x * PG_BLOCK) {
      const uint32_t w = gv.word[x];
      if (is_rule(w) && RULEISH(x) && (sb[x] & SB_RCH)) atomicOr(&s_s.w[table_of(w) >> 5], 1u << (table_of(w) & 31));
    }
    __syncthreads();
    pg_bits_flush(s_s, c.proto_bits + (size_t)r * c.words, c.words);
    __syncthreads();
  })
}
__global__ __launch_bounds__(NEMO_BLOCK) void k_pg_gate(DevCorpus c) {
  const uint32_t *lst = proto_list(c);
  for (uint32_t b = blockIdx.x * NEMO_BLOCK + threadIdx.x; b < lst[0]; b += gridDim.x * NEMO_BLOCK) {
    const uint32_t r = lst[1 + b];
    // OPTIONAL MATCH (g:Goal{run:1000+i, condition:"pre", condition_holds:true}) on the simplified pre graph
    const bool gt = c.holdany[2 * r] != 0;
    c.gate[r] = gt ? 1 : 0;
    if (!gt)
      for (uint32_t i = 0; i < c.words; i++) c.proto_bits[(size_t)r * c.words + i] = 0;
  }
}
#undef DEL
#undef REG
#undef RULEISH
#undef PG_LOOP

// k_proto's LDS tier, edge-parallel push form.  The graph's forward edges are
// laid out in LDS in the Kahn order of their source (e2[]: src << 16 | dst,
// built from the HBM CSR + Kahn order by one degree scan), so every phase is
// one pass over a contiguous edge range with one edge per thread -- no
// per-node child loops -- and the reachability sweep touches, per Kahn level,
// exactly the edges leaving that level (elo[] offsets).  Per node one u16:
// low byte = flags (NEMO_F_* | PAB_RULE), high byte = PB_* bits ORed by LDS
// atomics.  LDS ~2 B/node + 4 B/edge (device.h lds_tier_bytes).  Same
// predicates as k_proto's global tier:
//   ROOT  goal, not deleted, no REG or TAIL parent        (push PB_NR from REG/TAIL rules)
//   R1    REG/HEAD rule with a ROOT parent                  (push from ROOT goals)
//   G2    live goal below an R1 REG rule or below the tail of a chain with an R1 head
//         (tails of chains with an R1 head carry PB_R1T and push like R1 REG rules)
//   RCH   Kahn-level sweep: live G2/RCH goals reach their REG/HEAD rule children,
//         RCH REG rules their live goal children; a chain whose head is RCH marks
//         its tail PB_RCHT (the tail lies two levels below the head or deeper)
//         and the tail pushes RCH to its live goal children at its own level.
#define PROTO_BLOCK 512
#define PCH_DONE 0x8000u  // chain tail word: the head's reach was pushed
#define PAB_RULE 0x80u    // rule bit in the flags byte (NEMO_F_* use bits 0-4)
#define PB_NR 0x01u
#define PB_HASRC 0x02u
#define PB_R1 0x04u
#define PB_G2 0x08u
#define PB_RCH 0x10u
#define PB_R1T 0x20u
#define PB_ADDT 0x40u
#define PB_RCHT 0x80u
__global__ __launch_bounds__(PROTO_BLOCK) void k_proto_lds(DevCorpus c) {
  extern __shared__ __align__(16) uint8_t dyn[];
  const uint32_t r = blockIdx.x;
  const uint32_t g = 2 * r + 1;
  if (c.err[g] || c.err[g - 1]) return;
  const GraphView gv = c.view(g);
  if (!proto_lds_fits(c, gv)) return;
  const uint32_t V = gv.V, E = gv.E, L = gv.nlev, W = c.words, tid = threadIdx.x;
  STAMP(0);
  const uint32_t nch = c.nch[g];
  ProtoLds P = proto_carve(dyn, V, E, L, W, proto_chain_cap(V));
  uint32_t *s_s = P.words, *s_t = P.words + W;
  uint16_t *ab = P.ab;
  uint32_t *ab32 = (uint32_t *)P.ab;
  for (uint32_t i = tid; i < 2 * W; i += PROTO_BLOCK) P.words[i] = 0;
  // the forward edges in source Kahn order (k_build's e2) staged; each level's
  // first edge from the Kahn position its level starts at
  {
    const StageDesc d[1] = {{c.e2 + gv.e0, P.e2, E, ST_U32}};
    stage_lds<1, PROTO_BLOCK>(d);
  }
  for (uint32_t l = tid; l <= L; l += PROTO_BLOCK) P.elo[l] = l < L ? (uint16_t)c.posoff[gv.n0 + gv.lvl[l]] : (uint16_t)E;
  // chain k = tid + q PROTO_BLOCK in registers: head | tail << 16 (bit 31: PCH_DONE << 16)
  static_assert(PROTO_BLOCK == 512, "proto_chain_cap assumes 512 threads");
  uint32_t chp[PROTO_CHQ];
#pragma unroll
  for (int q = 0; q < PROTO_CHQ; q++) {
    const uint32_t k = tid + q * PROTO_BLOCK;
    chp[q] = k < nch ? (c.chain[5 * (gv.n0 + k)] & 0xFFFFu) | (c.chain[5 * (gv.n0 + k) + 1] << 16) : 0u;
  }
  // node bytes; missingFrom's table set (prototype.go:143-147): the tables of the REG / HEAD rules
  for (uint32_t v = tid; v < V; v += PROTO_BLOCK) {
    const uint32_t w = gv.word[v], f = gv.flags[v];
    const bool rule = is_rule(w);
    ab[v] = (uint16_t)(f | (rule ? PAB_RULE : 0u));
    if (rule && (((f & (NEMO_F_KEPT | NEMO_F_DELETED)) == NEMO_F_KEPT) || (f & NEMO_F_HEAD)))
      atomicOr(&s_t[table_of(w) >> 5], 1u << (table_of(w) & 31));
  }
  // OPTIONAL MATCH (g:Goal{run:1000+i, condition:"pre", condition_holds:true}) on the simplified pre graph
  const bool gt = c.holdany[g - 1] != 0;
  __syncthreads();
  STAMP(1);
#define XRULE(x) (((x) & PAB_RULE) != 0)
#define XDEL(x) (((x) & NEMO_F_DELETED) != 0)
#define XREG(x) (((x) & (NEMO_F_KEPT | NEMO_F_DELETED)) == NEMO_F_KEPT)
#define XRULEISH(x) (XREG(x) || ((x) & NEMO_F_HEAD))
#define XSB(x) ((x) >> 8)
#define SET(v, bits) atomicOr(&ab32[(v) >> 1], (uint32_t)(bits) << (8u + 16u * ((v) & 1u)))
#define EDGES(lo, hi, BODY)                                    \
  for (uint32_t e = (lo) + tid; e < (hi); e += PROTO_BLOCK) {  \
    const uint32_t sd_ = P.e2[e], s = sd_ >> 16, d = sd_ & 0xFFFFu; \
    const uint32_t as = ab[s], ad = ab[d];                     \
    BODY                                                       \
  }
  // not-root marks from REG / TAIL rules; goals with a REG / HEAD rule child
  EDGES(0, E, {
    if (XRULE(as)) {
      if (XREG(as) || (as & NEMO_F_TAIL)) SET(d, PB_NR);
    } else if (!XDEL(as) && XRULEISH(ad)) {
      SET(s, PB_HASRC);
    }
  })
  __syncthreads();
  STAMP(2);
  // R1: REG / HEAD rule children of roots
  EDGES(0, E, {
    if (!XRULE(as) && !XDEL(as) && !(XSB(as) & PB_NR) && XRULEISH(ad)) SET(d, PB_R1);
  })
  __syncthreads();
#pragma unroll
  for (int q = 0; q < PROTO_CHQ; q++)
    if (tid + q * PROTO_BLOCK < nch && (XSB(ab[chp[q] & 0xFFFFu]) & PB_R1)) SET(chp[q] >> 16, PB_R1T);
  __syncthreads();
  STAMP(3);
  // G2 below R1 REG rules and below the tails of chains with an R1 head; the
  // pushing rule is marked PB_ADDT when such a goal has a rule child
  EDGES(0, E, {
    if (XRULE(as) && ((XREG(as) && (XSB(as) & PB_R1)) || (XSB(as) & PB_R1T)) && !XDEL(ad)) {
      SET(d, PB_G2);
      if (XSB(ad) & PB_HASRC) SET(s, PB_ADDT);
    }
  })
  __syncthreads();
  STAMP(4);
  for (uint32_t v = tid; v < V; v += PROTO_BLOCK) {
    const uint32_t x = ab[v];
    if (XRULE(x) && XREG(x) && (XSB(x) & PB_ADDT)) {
      const uint32_t t = table_of(gv.word[v]);
      atomicOr(&s_s[t >> 5], 1u << (t & 31));
    }
  }
#pragma unroll
  for (int q = 0; q < PROTO_CHQ; q++) {
    if (tid + q * PROTO_BLOCK >= nch) continue;
    const uint32_t h = chp[q] & 0xFFFFu;
    if ((XSB(ab[h]) & PB_R1) && (XSB(ab[chp[q] >> 16]) & PB_ADDT)) {
      const uint32_t t = table_of(gv.word[h]);
      atomicOr(&s_s[t >> 5], 1u << (t & 31));
    }
  }
  STAMP(5);
  // rules reachable from G2: per Kahn level, the edges leaving it (a node's
  // bits are final when its level starts: every parent lies on an earlier level)
  for (uint32_t l = 0; l < L; l++) {
    EDGES(P.elo[l], P.elo[l + 1], {
      const uint32_t sb = XSB(as);
      const bool act = XRULE(as) ? ((XREG(as) && (sb & PB_RCH)) || (sb & PB_RCHT)) : (!XDEL(as) && (sb & (PB_G2 | PB_RCH)));
      if (act && (XRULE(as) ? !XDEL(ad) : XRULEISH(ad))) SET(d, PB_RCH);
    })
#pragma unroll
    for (int q = 0; q < PROTO_CHQ; q++) {
      const uint32_t t = chp[q] >> 16;
      if (tid + q * PROTO_BLOCK >= nch || (t & PCH_DONE) || !(XSB(ab[chp[q] & 0xFFFFu]) & PB_RCH)) continue;
      chp[q] |= PCH_DONE << 16;
      SET(t, PB_RCHT);
    }
    __syncthreads();
  }
  STAMP(6);
  // tables of the reached rules (RCH is only ever set on REG / HEAD rules and live goals)
  for (uint32_t v = tid; v < V; v += PROTO_BLOCK) {
    const uint32_t x = ab[v];
    if (XRULE(x) && (XSB(x) & PB_RCH)) {
      const uint32_t t = table_of(gv.word[v]);
      atomicOr(&s_s[t >> 5], 1u << (t & 31));
    }
  }
#undef XRULE
#undef XDEL
#undef XREG
#undef XRULEISH
#undef XSB
#undef SET
#undef EDGES
  __syncthreads();
  for (uint32_t i = tid; i < W; i += PROTO_BLOCK) {
    c.proto_bits[(size_t)r * W + i] = gt ? s_s[i] : 0u;
    c.graph_tables[(size_t)r * W + i] = s_t[i];
  }
  if (tid == 0) c.gate[r] = gt ? 1 : 0;
  STAMP(7);
}


// markConditionHolds + cleanCopyProv + the local part of collapseNextChains
// fused for the LDS-tier graphs, straight from the input edge list
// (marksimp.h).  LDS holds ~4 B per node (u16 node word, flags, one aux byte),
// so the CU is filled by waves, not capped by LDS.  Same outputs as the
// CSR-walking kernels (pre-post-prov.go:218-244, preprocessing.go:13-348).
// skip_built: the graphs k_build's fused tail already did (ms_built_by_build).
__global__ __launch_bounds__(MS_BLOCK) void k_marksimp(DevCorpus c, int skip_built) {
  extern __shared__ __align__(16) uint8_t dyn[];
  __shared__ uint32_t s_misc[3];
  const uint32_t g = blockIdx.x;
  if (c.err[g]) return;
  const GraphView gv = c.view(g);
  if (!tier_fits(c.t_ms, gv.V, gv.E, gv.nlev)) return;
  if (skip_built && ms_built_by_build(c, g, gv.V, gv.E)) return;
  const uint32_t E = gv.E, tid = threadIdx.x;
  const uint32_t *es = c.esrc + gv.e0, *ed = c.edst + gv.e0;
  // every input load issued back to back: the edges (src << 16 | dst) of the
  // first MS_EPT x block, then the node words (inside marksimp_graph)
  uint32_t sd[MS_EPT];
  auto load = [&](uint32_t base) {
#pragma unroll
    for (int q = 0; q < MS_EPT; q++) {
      const uint32_t e = base + tid + q * MS_BLOCK;
      sd[q] = e < E ? (es[e] << 16) | ed[e] : 0xFFFFFFFFu;
    }
  };
  load(0);
  marksimp_graph<MS_BLOCK, MS_EPT, false>(c, g, gv.V, E, gv.word, gv.flags, sd, E <= MS_EPT * MS_BLOCK, load, dyn, s_misc);
}

// Cross-run reduction vector (nemo_reduce_len): per-table counts over owned
// success runs with a non-empty list, the first success run's list, achvdCond
// (prototype.go:29-130) and the holding-"pre"-goal count (extensions.go:25-49).
// Counts are summed per workgroup in LDS, then one global atomic per table.
#define RED_LDS_TABLES 4096
__global__ __launch_bounds__(NEMO_BLOCK) void k_reduce(DevCorpus c, const uint8_t *is_success, const uint8_t *owned,
                                                        uint32_t first_run, uint32_t *red) {
  __shared__ uint32_t s_cnt[RED_LDS_TABLES];
  __shared__ uint32_t s_misc[3];
  const uint32_t T = c.n_tables, W = c.words;
  const bool lds = T <= RED_LDS_TABLES;
  for (uint32_t t = threadIdx.x; t < T && lds; t += NEMO_BLOCK) s_cnt[t] = 0;
  if (threadIdx.x < 3) s_misc[threadIdx.x] = 0;
  __syncthreads();
  for (uint32_t r = blockIdx.x * NEMO_BLOCK + threadIdx.x; r < c.n_runs; r += gridDim.x * NEMO_BLOCK) {
    const bool own = owned == nullptr || owned[r];
    if (!own) continue;
    atomicAdd(&s_misc[0], 1u);
    if (c.prehold[2 * r]) atomicAdd(&s_misc[1], c.prehold[2 * r]);
    const uint32_t *b = c.proto_bits + (size_t)r * W;
    bool nonempty = false;
    for (uint32_t i = 0; i < W; i++) nonempty |= b[i] != 0u;
    if (r == first_run) {
      red[2 * T + 1] = nonempty ? 1u : 0u;
      for (uint32_t i = 0; i < W; i++)
        for (uint32_t m = b[i]; m; m &= m - 1) red[T + 32 * i + __builtin_ctz(m)] = 1u;
    }
    if (!is_success[r] || !nonempty) continue;
    atomicAdd(&s_misc[2], 1u);
    for (uint32_t i = 0; i < W; i++)
      for (uint32_t m = b[i]; m; m &= m - 1) {
        const uint32_t t = 32 * i + __builtin_ctz(m);
        if (lds) atomicAdd(&s_cnt[t], 1u);
        else atomicAdd(&red[t], 1u);
      }
  }
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < T && lds; t += NEMO_BLOCK)
    if (s_cnt[t]) atomicAdd(&red[t], s_cnt[t]);
  if (threadIdx.x == 0) {
    if (s_misc[0]) atomicAdd(&red[2 * T + 3], s_misc[0]);
    if (s_misc[1]) atomicAdd(&red[2 * T + 2], s_misc[1]);
    if (s_misc[2]) atomicAdd(&red[2 * T], s_misc[2]);
  }
}

static dim3 mw_grid(const DevCorpus &c) { return dim3(std::max(1u, c.pg_chunks), std::min(c.n_big, 65535u)); }
void launch_mark(const DevCorpus &c, bool skip_tier, hipStream_t s, bool per_graph) {
  const int sk = skip_tier ? 1 : 0;
  if (!per_graph) {
  } else if (c.gblock == 1024)
    hipLaunchKernelGGL(k_mark<1024>, dim3(c.G), dim3(1024), 0, s, c, sk);
  else
    hipLaunchKernelGGL(k_mark<NEMO_BLOCK>, dim3(c.G), dim3(NEMO_BLOCK), 0, s, c, sk);
  if (!c.n_big) return;
  hipLaunchKernelGGL(k_mw_mark_z, mw_grid(c), dim3(MW_BLOCK), 0, s, c, sk);
  hipLaunchKernelGGL(k_mw_mark_a, mw_grid(c), dim3(MW_BLOCK), 0, s, c, sk);
  hipLaunchKernelGGL(k_mw_mark_b, mw_grid(c), dim3(MW_BLOCK), 0, s, c, sk);
}
void launch_simplify(const DevCorpus &c, bool skip_tier, hipStream_t s, bool per_graph) {
  const int sk = skip_tier ? 1 : 0;
  if (!per_graph) {
  } else if (c.gblock == 1024)
    hipLaunchKernelGGL(k_simplify_flags<1024>, dim3(c.G), dim3(1024), 0, s, c, sk);
  else
    hipLaunchKernelGGL(k_simplify_flags<NEMO_BLOCK>, dim3(c.G), dim3(NEMO_BLOCK), 0, s, c, sk);
  if (!c.n_big) return;
  hipLaunchKernelGGL(k_mw_simplify_1, mw_grid(c), dim3(MW_BLOCK), 0, s, c, sk);
  hipLaunchKernelGGL(k_mw_simplify_2, mw_grid(c), dim3(MW_BLOCK), 0, s, c, sk);
  hipLaunchKernelGGL(k_mw_simplify_3, mw_grid(c), dim3(MW_BLOCK), 0, s, c, sk);
  hipLaunchKernelGGL(k_mw_simplify_4, mw_grid(c), dim3(MW_BLOCK), 0, s, c, sk);
}
void launch_marksimp(const DevCorpus &c, hipStream_t s, bool skip_built) {
  if (!c.t_ms.bytes) return;
  const uint32_t b = c.t_ms.bytes;
  hipFuncSetAttribute((const void *)k_marksimp, hipFuncAttributeMaxDynamicSharedMemorySize, (int)b);
  hipLaunchKernelGGL(k_marksimp, dim3(c.G), dim3(MS_BLOCK), b, s, c, skip_built ? 1 : 0);
}
void launch_proto(const DevCorpus &c, hipStream_t s, bool tiers) {
  if (c.lds_bytes) {
    hipFuncSetAttribute((const void *)k_proto_lds, hipFuncAttributeMaxDynamicSharedMemorySize, (int)c.lds_bytes);
    hipLaunchKernelGGL(k_proto_lds, dim3(c.n_runs), dim3(PROTO_BLOCK), c.lds_bytes, s, c);
  }
  if (!c.n_runs || !tiers) return;  // !tiers: the host knows the global tier's list is empty
  launch_zero(proto_list(c), sizeof(uint32_t), s);
  hipLaunchKernelGGL(k_proto_sel, dim3((c.n_runs + NEMO_BLOCK - 1) / NEMO_BLOCK), dim3(NEMO_BLOCK), 0, s, c);
  const dim3 grid(c.pg_chunks, std::min(c.n_runs, 256u));
  hipLaunchKernelGGL(k_pg_init, grid, dim3(PG_BLOCK), 0, s, c);
  hipLaunchKernelGGL(k_pg_link, grid, dim3(PG_BLOCK), 0, s, c);
  hipLaunchKernelGGL(k_pg_a, grid, dim3(PG_BLOCK), 0, s, c);
  hipLaunchKernelGGL(k_pg_b, grid, dim3(PG_BLOCK), 0, s, c);
  hipLaunchKernelGGL(k_pg_c, grid, dim3(PG_BLOCK), 0, s, c);
  hipLaunchKernelGGL(k_pg_sweep, dim3(std::min(c.n_runs, 2048u)), dim3(PG_SWEEP), 0, s, c);
  hipLaunchKernelGGL(k_pg_d, grid, dim3(PG_BLOCK), 0, s, c);
  hipLaunchKernelGGL(k_pg_gate, dim3(std::min((c.n_runs + NEMO_BLOCK - 1) / NEMO_BLOCK, 64u)), dim3(NEMO_BLOCK), 0, s, c);
}
void launch_reduce(const DevCorpus &c, const uint8_t *is_success, const uint8_t *owned, uint32_t first_run,
                   uint32_t *red, hipStream_t s) {
  uint32_t blocks = (c.n_runs + NEMO_BLOCK - 1) / NEMO_BLOCK;
  if (blocks == 0) blocks = 1;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(k_reduce, dim3(blocks), dim3(NEMO_BLOCK), 0, s, c, is_success, owned, first_run, red);
}

}  // namespace nemo
