// k_chains.hip — the greedy @next chain cover of collapseNextChains
// (graphing/preprocessing.go:70-138) on the clean copy, one graph per
// workgroup.
//
// Q13 lists every path r1(next)-[*1..]->(g)-[*1..]->r2(next) over goals and
// next rules, ORDER BY len DESC; the Go loop accepts a path iff it holds a node
// no accepted path holds.  Neo4j's tie order is unspecified; ties are broken by
// the lexicographic sequence of node-ID ranks.  Acceptance only interacts
// inside a weakly connected component of the chain subgraph H* (the nodes
// k_simplify_flags marks DELETED), and inside a component the next accepted
// path is "the first path in that order containing an unseen node":
//   du(v) = longest H* path from v to a next rule that contains an unseen
//           node (down(v) if v is unseen),
//   start = the min-rank next rule with the component's maximal du,
//   walk  = at every step the min-rank child that can still complete the length.
// k_chains (first tier) does not iterate at all: a path is accepted iff it is
// first(v), the first path in sorted order through some node v (when first(v)
// comes up, v is unseen; an accepted path's fresh node has no earlier path).
// first(v) = best_prefix(v) ++ best_suffix(v): the lexicographically least
// longest path from a head to v (ranked per prefix length) and the least
// longest path from v to a tail (min-rank child with down = down-1).  The
// witnesses of a path are contiguous on it, so its representative is the
// witness whose best parent does not continue into it: up(v)==0 or
// nxt(bp(v)) != v.  The whole chain subgraph H* of a graph is staged in LDS.
// Graphs whose H* exceeds the LDS tile go to k_chains_big: per weakly
// connected component, the greedy iterated literally ("next accepted = first
// path holding an unseen node"), one wave per component in LDS, or a
// workgroup-wide sweep over global memory for the largest components.  Both
// tiers produce the same acceptance index k = rank of (len desc, lex asc).
#include <algorithm>

#include "device.h"
#include "internal.h"

namespace nemo {

#define CM 256  // nodes of a component staged in LDS
#define CE 768  // intra-component edges staged in LDS

struct CompLDS {
  uint32_t node[CM];  // graph-local node ids, topological (level, id) order
  uint32_t rank[CM];
  uint32_t key[CM];   // level
  uint16_t coff[CM + 1];
  uint16_t child[CE];
  uint16_t seg[CM + 1];
  int16_t down[CM];
  int16_t du[CM];
  uint8_t flag[CM];   // 1 = rule, 2 = unseen
};


#define CF_RULE 1u
#define CF_UNSEEN 2u

__device__ __forceinline__ uint32_t uf_find(uint32_t *p, uint32_t x) {
  uint32_t y = ld_relaxed(&p[x]);
  while (y != x) {
    x = y;
    y = ld_relaxed(&p[x]);
  }
  return x;
}

// One wave: the whole greedy of one component held in LDS.  Returns false if
// the component does not fit (caller leaves it to the fallback).
__device__ bool wave_component(const GraphView &gv, CompLDS &L, const uint32_t *nodes, uint32_t m,
                               const uint32_t *lev, uint32_t *cidx, uint32_t *tmp, uint32_t *nch) {
  const uint32_t lane = lane_id();
  const uint8_t *f = gv.flags;
  // topological order inside the component: sort by (level, node id)
  for (uint32_t i = lane; i < m; i += 64) {
    const uint32_t v = nodes[i];
    L.key[i] = lev[v];
    L.rank[i] = v;
  }
  wsync();
  for (uint32_t i = lane; i < m; i += 64) {
    const uint32_t ki = L.key[i], vi = L.rank[i];
    uint32_t pos = 0;
    for (uint32_t j = 0; j < m; j++) {
      const uint32_t kj = L.key[j], vj = L.rank[j];
      pos += (kj < ki) || (kj == ki && vj < vi);
    }
    L.node[pos] = vi;
  }
  wsync();
  for (uint32_t i = lane; i < m; i += 64) {
    const uint32_t v = L.node[i];
    cidx[v] = i;
    L.key[i] = lev[v];
    L.rank[i] = gv.rank_of(v);
    L.flag[i] = (uint8_t)((is_rule(gv.word[v]) ? CF_RULE : 0u) | CF_UNSEEN);
  }
  __threadfence_block();
  wsync();
  // level segments
  uint32_t nseg = 0;
  for (uint32_t base = 0; base < m; base += 64) {
    const uint32_t i = base + lane;
    const bool st = i < m && (i == 0 || L.key[i] != L.key[i - 1]);
    const uint64_t b = __ballot(st);
    if (st) L.seg[nseg + mbcnt(b)] = (uint16_t)i;
    nseg += (uint32_t)__popcll(b);
  }
  if (lane == 0) L.seg[nseg] = (uint16_t)m;
  // intra-component adjacency (children in H*)
  uint32_t ne = 0;
  for (uint32_t base = 0; base < m; base += 64) {
    const uint32_t i = base + lane;
    uint32_t n = 0, v = 0;
    if (i < m) {
      v = L.node[i];
      for (uint32_t j = gv.fp[v]; j < gv.fp[v + 1]; j++) n += (f[gv.fc[j]] & NEMO_F_DELETED) != 0;
    }
    uint32_t tot;
    const uint32_t off = ne + wave_exscan(n, &tot);
    if (i < m) L.coff[i] = (uint16_t)off;
    if (ne + tot <= CE && i < m) {
      uint32_t k = off;
      for (uint32_t j = gv.fp[v]; j < gv.fp[v + 1]; j++) {
        const uint32_t w = gv.fc[j];
        if (f[w] & NEMO_F_DELETED) L.child[k++] = (uint16_t)cidx[w];
      }
    }
    ne += tot;
  }
  if (ne > CE) return false;
  if (lane == 0) L.coff[m] = (uint16_t)ne;
  wsync();
  // down(i): longest H* path from i to a next rule
  for (uint32_t s = nseg; s-- > 0;) {
    for (uint32_t i = L.seg[s] + lane; i < L.seg[s + 1]; i += 64) {
      int32_t d = (L.flag[i] & CF_RULE) ? 0 : -1;
      for (uint32_t j = L.coff[i]; j < L.coff[i + 1]; j++) d = max(d, (int32_t)L.down[L.child[j]] + 1);
      L.down[i] = (int16_t)d;
    }
    wsync();
  }
  for (uint32_t iter = 0;; iter++) {
    for (uint32_t s = nseg; s-- > 0;) {
      for (uint32_t i = L.seg[s] + lane; i < L.seg[s + 1]; i += 64) {
        int32_t d;
        if (L.flag[i] & CF_UNSEEN) {
          d = L.down[i];
        } else {
          d = -1;
          for (uint32_t j = L.coff[i]; j < L.coff[i + 1]; j++) {
            const int32_t x = L.du[L.child[j]];
            if (x >= 0) d = max(d, x + 1);
          }
        }
        L.du[i] = (int16_t)d;
      }
      wsync();
    }
    unsigned long long mine = 0;
    uint32_t mi = 0;
    for (uint32_t i = lane; i < m; i += 64) {
      if (!(L.flag[i] & CF_RULE) || L.du[i] < 2) continue;
      const unsigned long long k = ((unsigned long long)(uint32_t)L.du[i] << 32) | (0xFFFFFFFFu - L.rank[i]);
      if (k > mine) {
        mine = k;
        mi = i;
      }
    }
    const unsigned long long best = wave_max_u64(mine);
    if (best == 0) break;
    if (mine == best) {  // exactly one lane: ranks are unique
      uint32_t v = mi;
      int32_t rem = L.du[mi];
      bool u = (L.flag[mi] & CF_UNSEEN) != 0;
      L.flag[mi] &= (uint8_t)~CF_UNSEEN;
      while (rem > 0) {
        uint32_t bc = 0xFFFFu, br = NEMO_NONE;
        for (uint32_t j = L.coff[v]; j < L.coff[v + 1]; j++) {
          const uint32_t w = L.child[j];
          const int32_t val = u ? L.down[w] : L.du[w];
          if (val == rem - 1 && L.rank[w] < br) {
            bc = w;
            br = L.rank[w];
          }
        }
        if (bc == 0xFFFFu) break;  // unreachable by construction
        v = bc;
        u |= (L.flag[v] & CF_UNSEEN) != 0;
        L.flag[v] &= (uint8_t)~CF_UNSEEN;
        rem--;
      }
      const uint32_t k = atomicAdd(nch, 1u);
      uint32_t *t = tmp + 5 * k;
      t[0] = L.node[mi];
      t[1] = L.node[v];
      t[2] = (uint32_t)L.du[mi];
      t[3] = L.rank[mi];
      t[4] = iter;
    }
    wsync();
  }
  // covered: the fallback (if any) must treat these nodes as seen
  for (uint32_t i = lane; i < m; i += 64) gv.flags[L.node[i]] |= FT_SEEN;
  return true;
}


// ---- first tier: first(v) over an LDS-resident chain subgraph ------------------
// Two instantiations (launch_chains): <1664, 120> keeps the LDS image at
// 40 KB, so four workgroups share a CU, and takes the graphs it can; the
// <2048, 512> tier then runs only the graphs the first one handed back.
//   HCAP: H* nodes (and H* edges per direction) staged in LDS
//   UCAP: Kahn levels of the graph / distinct prefix lengths (longest chain path + 2)
#define NIL16 0xFFFFu
#define CF_ROWS 20  // nodes per thread per compaction round (fast front)
#ifndef CF_Q
#define CF_Q 4      // ... taken CF_Q consecutive nodes per load
#endif
#define CF_EPT 32   // input edges per thread per adjacency round (fast front)
#ifndef PR_GROUP_MIN
#define PR_GROUP_MIN 96  // prefix ranks: levels above this many nodes rank by groups, smaller ones by counting all keys
#endif
#ifndef CH_K
#define CH_K 3      // up/down sweeps: parents (children) of a node read together
#endif

template <int HCAP, int UCAP>
struct ChainsLDS {
  static constexpr int ECAP = HCAP;
  static_assert(HCAP % 32 == 0 && HCAP <= 2048 && UCAP >= HCAP / 32 + 64, "isrule words; rank bitmap + 64 prefix words in cur[]");
  uint16_t crank[HCAP];  // rank of the node's ID among H* nodes
  int16_t up[HCAP], down[HCAP];
  uint16_t nxt[HCAP], bp[HCAP], po[HCAP];
  uint16_t ub[HCAP];
  uint32_t cur[UCAP];
  uint16_t uoff[UCAP];
  uint16_t seg[HCAP + 1];
  uint32_t isrule[HCAP / 32];  // bitmap
  union __align__(16) {
    struct {
      uint16_t pcoff[HCAP + 2], par[ECAP];  // live until the prefix ranks are done
      uint16_t ccoff[HCAP + 2], child[ECAP];  // (+2: ccoff 4-byte aligned for packed u16 atomics)
    } adj;
    struct {
      uint16_t pad[HCAP + 2 + ECAP + 6];   // keeps bk 16-byte aligned, past par[]
      uint32_t bk[HCAP + 4];               // level keys, or group counters + members; over ccoff/child
    } rk;
    unsigned long long kk[HCAP];           // bitonic sort of ranks; later the chain sort keys
  } u;
};

template <int HCAP, int UCAP>
__device__ __forceinline__ void chains_graph(const DevCorpus c, const uint32_t g) {
  constexpr uint32_t ECAP = HCAP;
  __shared__ ChainsLDS<HCAP, UCAP> L;
  __shared__ uint32_t s_lds[NEMO_WAVES];
  __shared__ uint32_t s_nch, s_maxup, s_fail;
  if (c.err[g] || c.gs_off[g] != ~0ull) return;  // deep graphs: k_chains_glob
  const GraphView gv = c.view(g);
  const uint8_t *f = gv.flags;
  uint32_t *hs = c.s_a + gv.n0 + g;    // compact index -> graph-local node
  uint32_t *hidx = c.s_f + gv.n0 + g;  // graph-local node -> compact index
  uint32_t *tmp = c.chain_tmp + c.tmp_off[g];
  const uint32_t tid = threadIdx.x;
  const uint32_t cap = min((uint32_t)HCAP, c.hcap_limit);
  STAMP(0);
  for (uint32_t w = tid; w < HCAP / 32; w += NEMO_BLOCK) L.isrule[w] = 0;
#define INH(v) ((f[v] & NEMO_F_DELETED) != 0)
#define RULE(i) ((L.isrule[(i) >> 5] >> ((i) & 31)) & 1u)
  const uint32_t ns = gv.nlev;
  uint32_t n = 0;
  if (gv.V <= 6u * HCAP && ns + 1 < UCAP) {
    // Fast front (graphs whose node map fits LDS).  Every HBM access of the
    // compaction is issued in two rounds per CF_ROWS x 256 topo positions (the
    // Kahn order, then the flag/word/rank gathers); positions are compacted
    // in (row, wave, lane) order = topo order with ballots and per-row wave
    // counts; each H* node's level goes into a histogram whose scan is the
    // level segmentation; ranks via the rank bitmap; the H* adjacency comes
    // from the coalesced input edge list with packed-u16 LDS counters.
    uint32_t *bm = (uint32_t *)L.u.kk;  // [1024] rank bitmap
    uint32_t *pre = bm + 1024;          // [1025] prefix popcounts
    uint32_t *hist = L.cur;             // H* nodes per level -> segment starts
    uint16_t *hmap = (uint16_t *)L.up;  // graph-local node -> compact index (spans up..ub)
    const uint32_t nw = (gv.V + 31) >> 5;
    for (uint32_t w = tid; w < nw; w += NEMO_BLOCK) bm[w] = 0;
    for (uint32_t l = tid; l <= ns; l += NEMO_BLOCK) hist[l] = 0;
    for (uint32_t v = tid; v < gv.V; v += NEMO_BLOCK) hmap[v] = 0xFFFFu;
    if (tid == 0) {
      s_nch = 0;
      s_maxup = 0;
      s_fail = 0;
    }
    __syncthreads();
    STAMP(10);
    // H* in level order (any order inside a level: every later tie-break is by
    // ID rank).  Node-order reads are coalesced: flags, level, word, rank.
    const uint32_t *nlv = c.nlv + gv.n0;
    uint32_t lev[CF_ROWS], rk[CF_ROWS], hm = 0, rl = 0;
    // node of slot q: CF_Q consecutive nodes per thread and load, so the
    // flags come four to a u32 and the levels, words (and ranks) four to a
    // 16-byte load
    auto xq = [&](uint32_t sbase, int q) { return sbase + CF_Q * ((q / CF_Q) * NEMO_BLOCK + tid) + (q % CF_Q); };
    auto rows = [&](uint32_t sbase) {
      uint8_t fl[CF_ROWS];
      uint32_t wd[CF_ROWS];
#pragma unroll
      for (int g4 = 0; g4 < CF_ROWS / CF_Q; g4++) {
        const uint32_t x0 = xq(sbase, g4 * CF_Q);
        if (CF_Q == 4 && x0 + 3 < gv.V) {  // a whole quad inside the graph
          uint32_t f4;
          __builtin_memcpy(&f4, f + x0, 4);
          uint4 l4, w4;
          __builtin_memcpy(&l4, nlv + x0, 16);
          __builtin_memcpy(&w4, gv.word + x0, 16);
          const uint32_t l[4] = {l4.x, l4.y, l4.z, l4.w}, w[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
          for (int b = 0; b < CF_Q; b++) {
            fl[g4 * CF_Q + b] = (uint8_t)(f4 >> (8 * b));
            lev[g4 * CF_Q + b] = l[b];
            wd[g4 * CF_Q + b] = w[b];
            rk[g4 * CF_Q + b] = gv.rank_of(x0 + b);
          }
        } else {
#pragma unroll
          for (int b = 0; b < CF_Q; b++) {
            const int q = g4 * CF_Q + b;
            const uint32_t x = x0 + b;
            const bool in = x < gv.V;
            fl[q] = in ? f[x] : (uint8_t)0;
            lev[q] = in ? nlv[x] : 0u;
            wd[q] = in ? gv.word[x] : 0u;
            rk[q] = in ? gv.rank_of(x) : 0u;
          }
        }
      }
      hm = rl = 0;
#pragma unroll
      for (int q = 0; q < CF_ROWS; q++) {
        hm |= ((fl[q] & NEMO_F_DELETED) ? 1u : 0u) << q;
        rl |= (is_rule(wd[q]) ? 1u : 0u) << q;
      }
    };
    const bool one = gv.V <= CF_ROWS * NEMO_BLOCK;  // one round: the rows stay in registers
    for (uint32_t sbase = 0; sbase < gv.V; sbase += CF_ROWS * NEMO_BLOCK) {
      rows(sbase);
#pragma unroll
      for (int q = 0; q < CF_ROWS; q++)
        if ((hm >> q) & 1u) atomicAdd(&hist[lev[q]], 1u);
    }
    __syncthreads();
    STAMP(11);
    n = block_scan_inplace(hist, ns + 1, s_lds);  // level starts; hist[ns] = n
    if (n == 0) {
      if (tid == 0) c.nch[g] = 0;
      return;
    }
    if (n > cap) {  // too large for the LDS tier: k_chains_big takes the graph
      if (tid == 0) c.nch[g] = NEMO_NONE;
      return;
    }
    for (uint32_t l = tid; l <= ns; l += NEMO_BLOCK) L.seg[l] = (uint16_t)hist[l];
    __syncthreads();
    for (uint32_t sbase = 0; sbase < gv.V; sbase += CF_ROWS * NEMO_BLOCK) {
      if (!one) rows(sbase);
#pragma unroll
      for (int q = 0; q < CF_ROWS; q++) {
        if (!((hm >> q) & 1u)) continue;
        const uint32_t x = xq(sbase, q);
        const uint32_t i = atomicAdd(&hist[lev[q]], 1u);
        hs[i] = x;
        hmap[x] = (uint16_t)i;
        if ((rl >> q) & 1u) atomicOr(&L.isrule[i >> 5], 1u << (i & 31));
        atomicOr(&bm[rk[q] >> 5], 1u << (rk[q] & 31));
        L.crank[i] = (uint16_t)rk[q];  // the ID rank until the prefix popcounts exist
      }
    }
    __syncthreads();
    __threadfence_block();
    STAMP(1);
    for (uint32_t w = tid; w < nw; w += NEMO_BLOCK) pre[w] = __popc(bm[w]);
    __syncthreads();
    block_scan_inplace(pre, nw, s_lds);
    for (uint32_t i = tid; i < n; i += NEMO_BLOCK) {
      const uint32_t rr = L.crank[i];
      L.crank[i] = (uint16_t)(pre[rr >> 5] + __popc(bm[rr >> 5] & ((1u << (rr & 31)) - 1u)));
    }
    __syncthreads();
    STAMP(2);
    // H* adjacency from the edge list: count, scan, scatter (row order is
    // irrelevant below: every consumer takes a max/min over the row)
    uint32_t *cc32 = (uint32_t *)L.u.adj.ccoff, *pc32 = (uint32_t *)L.u.adj.pcoff;
    for (uint32_t w = tid; w < (HCAP + 2) / 2; w += NEMO_BLOCK) {
      cc32[w] = 0;
      pc32[w] = 0;
    }
    __syncthreads();
    const uint32_t *es = c.esrc + gv.e0, *ed = c.edst + gv.e0;
    // one round (E <= CF_EPT x block, the common case): the H*-mapped edges of
    // pass 0 stay in registers for pass 1, so the edge list is read once
    const bool one_e = gv.E <= CF_EPT * NEMO_BLOCK;
    uint32_t ab[CF_EPT];
    for (int pass = 0; pass < 2; pass++) {
      for (uint32_t ebase = 0; ebase < gv.E; ebase += CF_EPT * NEMO_BLOCK) {
        if (!(one_e && pass == 1)) {
          uint32_t sd[CF_EPT];  // (four consecutive edges per thread and 16-byte load)
#pragma unroll
          for (int g4 = 0; g4 < CF_EPT / 4; g4++) {
            const uint32_t e0 = ebase + 4 * (g4 * NEMO_BLOCK + tid);
            uint32_t xs[4], ys[4];
            if (e0 + 3 < gv.E) {
              uint4 a4, b4;
              __builtin_memcpy(&a4, es + e0, 16);
              __builtin_memcpy(&b4, ed + e0, 16);
              xs[0] = a4.x, xs[1] = a4.y, xs[2] = a4.z, xs[3] = a4.w;
              ys[0] = b4.x, ys[1] = b4.y, ys[2] = b4.z, ys[3] = b4.w;
            } else {
#pragma unroll
              for (int b = 0; b < 4; b++) {
                xs[b] = e0 + b < gv.E ? es[e0 + b] : 0u;
                ys[b] = e0 + b < gv.E ? ed[e0 + b] : 0u;
              }
            }
#pragma unroll
            for (int b = 0; b < 4; b++) sd[4 * g4 + b] = e0 + b < gv.E ? (xs[b] << 16) | ys[b] : 0xFFFFFFFFu;
          }
#pragma unroll
          for (int q = 0; q < CF_EPT; q++) {
            ab[q] = 0xFFFFFFFFu;
            if (sd[q] == 0xFFFFFFFFu) continue;
            const uint32_t a = hmap[sd[q] >> 16], b = hmap[sd[q] & 0xFFFFu];
            if (a != 0xFFFFu && b != 0xFFFFu) ab[q] = (a << 16) | b;
          }
        }
#pragma unroll
        for (int q = 0; q < CF_EPT; q++) {
          if (ab[q] == 0xFFFFFFFFu) continue;
          const uint32_t a = ab[q] >> 16, b = ab[q] & 0xFFFFu;
          const uint32_t sa = 16u * (a & 1u), sb = 16u * (b & 1u);
          if (pass == 0) {
            atomicAdd(&cc32[a >> 1], 1u << sa);
            atomicAdd(&pc32[b >> 1], 1u << sb);
          } else {
            L.u.adj.child[(atomicAdd(&cc32[a >> 1], 1u << sa) >> sa) & 0xFFFFu] = (uint16_t)b;
            L.u.adj.par[(atomicAdd(&pc32[b >> 1], 1u << sb) >> sb) & 0xFFFFu] = (uint16_t)a;
          }
        }
      }
      __syncthreads();
      if (pass == 0) {
        const uint32_t tc = block_scan_inplace(L.u.adj.ccoff, n + 1, s_lds);
        const uint32_t tp = block_scan_inplace(L.u.adj.pcoff, n + 1, s_lds);
        if (tc > ECAP || tp > ECAP) {
          if (tid == 0) c.nch[g] = NEMO_NONE;
          return;
        }
      }
    }
    // the cursors now hold row ends: shift them into row starts
    {
      uint32_t ce[(HCAP + NEMO_BLOCK - 1) / NEMO_BLOCK], pe[(HCAP + NEMO_BLOCK - 1) / NEMO_BLOCK];
#pragma unroll
      for (int q = 0; q < (HCAP + NEMO_BLOCK - 1) / NEMO_BLOCK; q++) {
        const uint32_t i = q * NEMO_BLOCK + tid;
        ce[q] = i < n ? L.u.adj.ccoff[i] : 0u;
        pe[q] = i < n ? L.u.adj.pcoff[i] : 0u;
      }
      __syncthreads();
#pragma unroll
      for (int q = 0; q < (HCAP + NEMO_BLOCK - 1) / NEMO_BLOCK; q++) {
        const uint32_t i = q * NEMO_BLOCK + tid;
        if (i < n) {
          L.u.adj.ccoff[i + 1] = (uint16_t)ce[q];
          L.u.adj.pcoff[i + 1] = (uint16_t)pe[q];
        }
      }
      if (tid == 0) {
        L.u.adj.ccoff[0] = 0;
        L.u.adj.pcoff[0] = 0;
      }
      __syncthreads();
    }
    STAMP(3);
  } else {
  // ordered compaction of H* in Kahn order (chunks of 4 positions per thread);
  // pc[p] = #H* nodes before topo position p gives every level's segment
  uint32_t *pc = c.s_b + gv.n0 + g;
  for (uint32_t base = 0; base < gv.V; base += 4 * NEMO_BLOCK) {
    const uint32_t i0 = base + 4 * tid;
    uint32_t v[4], cnt = 0;
    bool p[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      v[q] = i0 + q < gv.V ? gv.topo[i0 + q] : 0u;
      p[q] = i0 + q < gv.V && INH(v[q]);
      cnt += p[q];
    }
    uint32_t tot;
    uint32_t off = n + block_exscan(cnt, &tot, s_lds);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      if (i0 + q < gv.V) pc[i0 + q] = off;
      if (p[q]) {
        if (off < cap) hs[off] = v[q];
        off++;
      }
    }
    n += tot;
  }
  if (n == 0) {
    if (tid == 0) c.nch[g] = 0;
    return;
  }
  if (n > cap) {  // too large for the LDS tier: k_chains_big takes the graph
    if (tid == 0) c.nch[g] = NEMO_NONE;
    return;
  }
  __threadfence_block();
  __syncthreads();
  if (ns > HCAP) {
    if (tid == 0) c.nch[g] = NEMO_NONE;
    return;
  }
  for (uint32_t l = tid; l <= ns; l += NEMO_BLOCK) L.seg[l] = (uint16_t)(l == ns ? n : pc[gv.lvl[l]]);
  if (tid == 0) {
    s_nch = 0;
    s_maxup = 0;
    s_fail = 0;
  }
  STAMP(1);
  // compact ID ranks: crank(v) = #H* nodes of smaller ID rank.  Small graphs
  // set one bit per H* node in a rank bitmap and take prefix popcounts; larger
  // ones sort (rank, index) pairs with an LDS bitonic network.
  // graph-local node -> compact index (NONE outside H*): in LDS over the
  // not-yet-used up..ub arrays when the graph is small enough, else global
  uint16_t *hmap = (uint16_t *)L.up;  // spans up, down, nxt, bp, po, ub
  const bool lmap = gv.V <= 6u * HCAP;
  if (lmap) {
    for (uint32_t v = tid; v < gv.V; v += NEMO_BLOCK) hmap[v] = 0xFFFFu;
    __syncthreads();
  }
  for (uint32_t i = tid; i < n; i += NEMO_BLOCK) {
    const uint32_t v = hs[i];
    if (lmap)
      hmap[v] = (uint16_t)i;
    else
      hidx[v] = i;
    if (is_rule(gv.word[v])) atomicOr(&L.isrule[i >> 5], 1u << (i & 31));
  }
  if (gv.V <= 32768) {
    uint32_t *bm = (uint32_t *)L.u.kk;            // [1024] rank bitmap
    uint32_t *pre = bm + 1024;                    // [1025] prefix popcounts
    const uint32_t nw = (gv.V + 31) >> 5;
    for (uint32_t w = tid; w < nw; w += NEMO_BLOCK) bm[w] = 0;
    __syncthreads();
    for (uint32_t i = tid; i < n; i += NEMO_BLOCK) {
      const uint32_t r = gv.rank_of(hs[i]);
      atomicOr(&bm[r >> 5], 1u << (r & 31));
    }
    __syncthreads();
    for (uint32_t w = tid; w < nw; w += NEMO_BLOCK) pre[w] = __popc(bm[w]);
    __syncthreads();
    block_scan_inplace(pre, nw, s_lds);
    for (uint32_t i = tid; i < n; i += NEMO_BLOCK) {
      const uint32_t r = gv.rank_of(hs[i]);
      L.crank[i] = (uint16_t)(pre[r >> 5] + __popc(bm[r >> 5] & ((1u << (r & 31)) - 1u)));
    }
    __syncthreads();
  } else {
    uint32_t N2 = 1;
    while (N2 < n) N2 <<= 1;
    if (N2 > HCAP) {  // the network needs a power of two: the next tier
      if (tid == 0) c.nch[g] = NEMO_NONE;
      return;
    }
    for (uint32_t i = tid; i < N2; i += NEMO_BLOCK)
      L.u.kk[i] = i < n ? (((unsigned long long)gv.rank_of(hs[i]) << 16) | i) : ~0ull;
    __syncthreads();
    for (uint32_t k = 2; k <= N2; k <<= 1) {
      for (uint32_t j = k >> 1; j > 0; j >>= 1) {
        for (uint32_t i = tid; i < N2; i += NEMO_BLOCK) {
          const uint32_t ixj = i ^ j;
          if (ixj > i) {
            const unsigned long long x = L.u.kk[i], y = L.u.kk[ixj];
            const bool up = (i & k) == 0;
            if ((x > y) == up) {
              L.u.kk[i] = y;
              L.u.kk[ixj] = x;
            }
          }
        }
        __syncthreads();
      }
    }
    for (uint32_t q = tid; q < n; q += NEMO_BLOCK) L.crank[L.u.kk[q] & 0xFFFFu] = (uint16_t)q;
  }
  __threadfence_block();
  __syncthreads();
  STAMP(2);
  // compact child / parent lists
  auto hx = [&](uint32_t w) -> uint32_t {
    if (lmap) {
      const uint32_t h = hmap[w];
      return h == 0xFFFFu ? NEMO_NONE : h;
    }
    return INH(w) ? hidx[w] : NEMO_NONE;
  };
  uint32_t ce = 0, pe = 0;
  for (uint32_t base = 0; base < n; base += NEMO_BLOCK) {
    const uint32_t i = base + tid;
    uint32_t nc = 0, np = 0, fb = 0, fe = 0, rb = 0, re = 0;
    if (i < n) {
      const uint32_t v = hs[i];
      fb = gv.fp[v];
      fe = gv.fp[v + 1];
      rb = gv.rp[v];
      re = gv.rp[v + 1];
      for (uint32_t j = fb; j < fe; j++) nc += hx(gv.fc[j]) != NEMO_NONE;
      for (uint32_t j = rb; j < re; j++) np += hx(gv.rc[j]) != NEMO_NONE;
    }
    uint32_t tc, tp;
    const uint32_t oc = ce + block_exscan(nc, &tc, s_lds);
    const uint32_t op = pe + block_exscan(np, &tp, s_lds);
    if (i < n) {
      L.u.adj.ccoff[i] = (uint16_t)min(oc, (uint32_t)ECAP);
      L.u.adj.pcoff[i] = (uint16_t)min(op, (uint32_t)ECAP);
      if (oc + nc <= ECAP) {
        uint32_t k = oc;
        for (uint32_t j = fb; j < fe; j++) {
          const uint32_t h = hx(gv.fc[j]);
          if (h != NEMO_NONE) L.u.adj.child[k++] = (uint16_t)h;
        }
      }
      if (op + np <= ECAP) {
        uint32_t k = op;
        for (uint32_t j = rb; j < re; j++) {
          const uint32_t h = hx(gv.rc[j]);
          if (h != NEMO_NONE) L.u.adj.par[k++] = (uint16_t)h;
        }
      }
    }
    ce += tc;
    pe += tp;
  }
  if (ce > ECAP || pe > ECAP) {
    if (tid == 0) c.nch[g] = NEMO_NONE;
    return;
  }
  if (tid == 0) {
    L.u.adj.ccoff[n] = (uint16_t)ce;
    L.u.adj.pcoff[n] = (uint16_t)pe;
  }
  __syncthreads();
  STAMP(3);
  }
  // up: longest H* path from a next rule ending here; down/nxt/tail: the
  // lexicographically least longest continuation to a next rule
  // both sweeps at once, each by ONE wave and without a barrier: wave 0 walks
  // the levels forward (up), wave 1 backward (down).  A wave's LDS operations
  // complete in order, so a level reads the values its own wave wrote for the
  // levels before; the two waves touch disjoint arrays.  A node's first
  // CH_K parents (children) are read together, clamped (their values are
  // discarded past the row's end), so a level costs a few LDS round trips.
  if (tid < 128) {
    const bool fwd = tid < 64;
    const uint32_t lane = tid & 63u;
    for (uint32_t s = 0; s < ns; s++) {
      const uint32_t sl = fwd ? s : ns - 1 - s;
      const uint32_t e = L.seg[sl + 1];
      for (uint32_t i = L.seg[sl] + lane; i < e; i += 64) {
        const bool ru = RULE(i);
        if (fwd) {
          int32_t d = ru ? 0 : -1;
          const uint32_t j0 = L.u.adj.pcoff[i], j1 = L.u.adj.pcoff[i + 1];
          uint32_t p[CH_K];
          int32_t v[CH_K];
#pragma unroll
          for (int q = 0; q < CH_K; q++) p[q] = min((uint32_t)L.u.adj.par[min(j0 + q, ECAP - 1u)], (uint32_t)HCAP - 1u);
#pragma unroll
          for (int q = 0; q < CH_K; q++) v[q] = L.up[p[q]];
#pragma unroll
          for (int q = 0; q < CH_K; q++) d = j0 + q < j1 ? max(d, v[q] + 1) : d;
          for (uint32_t j = j0 + CH_K; j < j1; j++) d = max(d, (int32_t)L.up[L.u.adj.par[j]] + 1);
          L.up[i] = (int16_t)d;
        } else {
          // one pass: the deepest child, ties to the smallest ID rank
          int32_t best = -1;
          uint32_t bc = NIL16, br = NEMO_NONE;
          auto take = [&](uint32_t w, int32_t dw, uint32_t rw) {
            if (dw > best || (dw == best && rw < br)) {
              best = dw;
              bc = w;
              br = rw;
            }
          };
          const uint32_t j0 = L.u.adj.ccoff[i], j1 = L.u.adj.ccoff[i + 1];
          uint32_t w[CH_K], rw[CH_K];
          int32_t dw[CH_K];
#pragma unroll
          for (int q = 0; q < CH_K; q++) w[q] = min((uint32_t)L.u.adj.child[min(j0 + q, ECAP - 1u)], (uint32_t)HCAP - 1u);
#pragma unroll
          for (int q = 0; q < CH_K; q++) {
            dw[q] = L.down[w[q]];
            rw[q] = L.crank[w[q]];
          }
#pragma unroll
          for (int q = 0; q < CH_K; q++)
            if (j0 + q < j1) take(w[q], dw[q], rw[q]);
          for (uint32_t j = j0 + CH_K; j < j1; j++) {
            const uint32_t x = L.u.adj.child[j];
            take(x, L.down[x], L.crank[x]);
          }
          int32_t d = best >= 0 ? best + 1 : (ru ? 0 : -1);
          if (ru && d < 0) d = 0;
          if (d > 0 && best < 0) bc = NIL16;
          L.down[i] = (int16_t)d;
          L.nxt[i] = (uint16_t)(d > 0 ? bc : NIL16);
          if (d < 0) s_fail = 1;  // a goal without a chain continuation: impossible on H*
        }
      }
      wsync();  // the level's writes before the next level's reads (compiler order; the wave's DS ops are in order)
    }
  }
  __syncthreads();
  {
    uint32_t m = 0;
    for (uint32_t i = tid; i < n; i += NEMO_BLOCK) m = max(m, (uint32_t)max((int32_t)L.up[i], 0));
    for (int d = 32; d >= 1; d >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, d));
    if (lane_id() == 0) atomicMax(&s_maxup, m);
    __syncthreads();
  }
  STAMP(4);
  // bucket by up value (counting sort in LDS)
  const uint32_t maxup = s_maxup;
  if (maxup + 2 > UCAP) {
    if (tid == 0) c.nch[g] = NEMO_NONE;
    return;
  }
  for (uint32_t k = tid; k <= maxup + 1; k += NEMO_BLOCK) L.cur[k] = 0;
  __syncthreads();
  for (uint32_t i = tid; i < n; i += NEMO_BLOCK) atomicAdd(&L.cur[L.up[i]], 1u);
  __syncthreads();
  block_scan_inplace(L.cur, maxup + 2, s_lds);
  for (uint32_t k = tid; k <= maxup + 1; k += NEMO_BLOCK) L.uoff[k] = (uint16_t)L.cur[k];
  __syncthreads();
  for (uint32_t i = tid; i < n; i += NEMO_BLOCK) L.ub[atomicAdd(&L.cur[L.up[i]], 1u)] = (uint16_t)i;
  __syncthreads();
  // prefix ranks: po(v) = rank of best_prefix(v) among the prefixes of its
  // length; key = (po(bp(v)), crank(v)) is unique inside a level.  The best
  // parent is fixed up front where only one parent has up == up(v) - 1 (the
  // usual case), so a level only waits on its parents' po.  fpos(v) = the po
  // of v's first sibling (keys below (po(bp(v)), 0)) feeds the preorder.
  constexpr uint32_t MULTI16 = 0xFFFEu;
  uint16_t *fpos = L.seg;  // seg[] is dead after the sweeps
  for (uint32_t i = tid; i < n; i += NEMO_BLOCK) {
    const int32_t k = L.up[i];
    uint32_t cand = NIL16, cnt = 0;
    if (k > 0) {
      const uint32_t q1 = L.u.adj.pcoff[i + 1];
      for (uint32_t q = L.u.adj.pcoff[i]; q < q1; q++) {
        const uint32_t p = L.u.adj.par[q];
        if (L.up[p] == k - 1) {
          cnt++;
          cand = p;
        }
      }
    }
    L.bp[i] = (uint16_t)(cnt > 1 ? MULTI16 : cand);
  }
  __syncthreads();
  // Per level: roots rank by ID (bitmap + prefix popcounts); small levels
  // count keys directly (broadcast reads); large levels group nodes by
  // po(bp) (histogram + scan = group bases, cursors scatter the members) and
  // rank inside the few-member groups.
  for (uint32_t k = 0; k <= maxup; k++) {
    const uint32_t a = L.uoff[k], b = L.uoff[k + 1];
    const uint32_t m = b - a, m4 = (m + 3) & ~3u;
    if (k == 0) {
      uint32_t *bmr = L.cur, *pcr = L.cur + HCAP / 32;  // cur[] is dead after the bucketing
      for (uint32_t w = tid; w < HCAP / 32; w += NEMO_BLOCK) bmr[w] = 0;
      __syncthreads();
      for (uint32_t j = a + tid; j < b; j += NEMO_BLOCK) {
        const uint32_t cr = L.crank[L.ub[j]];
        atomicOr(&bmr[cr >> 5], 1u << (cr & 31));
      }
      __syncthreads();
      if (tid < 64) {
        uint32_t tot;
        pcr[tid] = wave_exscan(tid < HCAP / 32 ? __popc(bmr[tid]) : 0u, &tot);
      }
      __syncthreads();
      for (uint32_t j = a + tid; j < b; j += NEMO_BLOCK) {
        const uint32_t i = L.ub[j], cr = L.crank[i];
        L.po[i] = (uint16_t)(pcr[cr >> 5] + __popc(bmr[cr >> 5] & ((1u << (cr & 31)) - 1u)));
        fpos[i] = 0;
      }
      __syncthreads();
      continue;
    }
    const bool grouped = m > PR_GROUP_MIN;
    const uint32_t mp = a - L.uoff[k - 1];  // size of level k-1: po(bp) < mp
    uint32_t *cnt = L.u.rk.bk, *grp = L.u.rk.bk + mp + 1;
    if (grouped) {
      for (uint32_t w = tid; w <= mp; w += NEMO_BLOCK) cnt[w] = 0;
      __syncthreads();
    }
    for (uint32_t j = a + tid; j < b; j += NEMO_BLOCK) {
      const uint32_t i = L.ub[j];
      uint32_t bpo;
      const uint32_t cand = L.bp[i];
      if (cand != MULTI16) {
        bpo = L.po[cand];
      } else {
        uint32_t bpi = NIL16;
        bpo = NEMO_NONE;
        const uint32_t q1 = L.u.adj.pcoff[i + 1];
        for (uint32_t q = L.u.adj.pcoff[i]; q < q1; q++) {
          const uint32_t p = L.u.adj.par[q];
          if ((uint32_t)L.up[p] == k - 1 && L.po[p] < bpo) {
            bpi = p;
            bpo = L.po[p];
          }
        }
        L.bp[i] = (uint16_t)bpi;
      }
      if (grouped) atomicAdd(&cnt[bpo], 1u);
      else L.u.rk.bk[j - a] = (bpo << 16) | L.crank[i];
    }
    if (!grouped)
      for (uint32_t j = m + tid; j < m4; j += NEMO_BLOCK) L.u.rk.bk[j] = 0xFFFFFFFFu;
    __syncthreads();
    if (!grouped) {
      const uint4 *bk4 = (const uint4 *)L.u.rk.bk;
      for (uint32_t j = a + tid; j < b; j += NEMO_BLOCK) {
        const uint32_t me = L.u.rk.bk[j - a], lo = me & 0xFFFF0000u;
        uint32_t pos = 0, fp = 0;
#pragma unroll 8
        for (uint32_t q = 0; q < m4 / 4; q++) {
          const uint4 x = bk4[q];
          pos += (x.x < me) + (x.y < me) + (x.z < me) + (x.w < me);
          fp += (x.x < lo) + (x.y < lo) + (x.z < lo) + (x.w < lo);
        }
        const uint32_t i = L.ub[j];
        L.po[i] = (uint16_t)pos;
        fpos[i] = (uint16_t)fp;
      }
    } else {
      block_scan_inplace(cnt, mp + 1, s_lds);  // group bases
      for (uint32_t j = a + tid; j < b; j += NEMO_BLOCK) {
        const uint32_t i = L.ub[j];
        const uint32_t slot = atomicAdd(&cnt[L.po[L.bp[i]]], 1u);
        grp[slot] = ((uint32_t)L.crank[i] << 16) | i;
      }
      __syncthreads();  // cnt[g] = end of group g = base of group g + 1
      for (uint32_t j = a + tid; j < b; j += NEMO_BLOCK) {
        const uint32_t i = L.ub[j], bpo = L.po[L.bp[i]], cr = L.crank[i];
        const uint32_t base = bpo ? cnt[bpo - 1] : 0u, end = cnt[bpo];
        uint32_t r = 0;
        for (uint32_t q = base; q < end; q++) r += (grp[q] >> 16) < cr;
        L.po[i] = (uint16_t)(base + r);
        fpos[i] = (uint16_t)base;
      }
    }
    __syncthreads();
  }
  STAMP(5);
  // one representative per accepted path
  for (uint32_t i = tid; i < n; i += NEMO_BLOCK) {
    const bool rep = L.up[i] == 0 || L.nxt[L.bp[i]] != i;
    if (!rep) continue;
    uint32_t h = i, t = i;  // head: root of the bp chain; tail: end of the nxt chain
    while (L.up[h] > 0) h = L.bp[h];
    while (L.nxt[t] != NIL16) t = L.nxt[t];
    const uint32_t k = atomicAdd(&s_nch, 1u);
    // packed record: compact head | tail << 16, length | representative << 16
    tmp[2 * k] = h | (t << 16);
    tmp[2 * k + 1] = (uint32_t)(L.up[i] + L.down[i]) | (i << 16);
  }
  __threadfence_block();
  __syncthreads();
  const uint32_t nch = s_nch;
  STAMP(6);
  // Acceptance order.  For equal lengths, the lexicographic order of accepted
  // paths is the preorder of their representatives in the best-prefix forest
  // (bp pointers; roots = heads; children in ID-rank order, which is po order
  // inside a level): an ancestor's path comes first, otherwise the first
  // divergence decides.  S = subtree sizes (bottom-up), pre = preorder
  // (top-down, exclusive scans of sizes in po order).
  {
    // pre(v) = up(v) + sum over v and its bp ancestors a of off(a), where
    // off(a) = total size of a's earlier siblings = A[first sibling .. a) over
    // the sizes laid out in (level, po) order; the ancestor sums come from
    // pointer jumping (log2(maxup) rounds instead of one pass per level).
    uint32_t *S = (uint32_t *)L.u.kk;  // subtree sizes
    uint32_t *A = S + HCAP;            // sizes in (level, po) order -> exclusive scan
    for (uint32_t i = tid; i < n; i += NEMO_BLOCK) S[i] = 1;
    __syncthreads();
    for (uint32_t k = maxup; k >= 1; k--) {
      for (uint32_t j = L.uoff[k] + tid; j < L.uoff[k + 1]; j += NEMO_BLOCK) {
        const uint32_t i = L.ub[j];
        atomicAdd(&S[L.bp[i]], S[i]);
      }
      __syncthreads();
    }
    for (uint32_t i = tid; i < n; i += NEMO_BLOCK) A[L.uoff[L.up[i]] + L.po[i]] = S[i];
    __syncthreads();
    block_scan_inplace(A, n, s_lds);
    uint16_t *va = L.nxt, *vb = L.crank;                            // dead once the records are written
    uint16_t *pa = (uint16_t *)L.u.kk, *pb = pa + HCAP;              // over S (dead once A is built)
    for (uint32_t i = tid; i < n; i += NEMO_BLOCK) {
      const uint32_t k = L.up[i], base = L.uoff[k];
      va[i] = (uint16_t)(A[base + L.po[i]] - A[base + fpos[i]]);
      pa[i] = (uint16_t)(k ? L.bp[i] : NIL16);
    }
    __syncthreads();
    for (uint32_t r = 1; r <= maxup; r <<= 1) {
      for (uint32_t i = tid; i < n; i += NEMO_BLOCK) {
        const uint32_t p = pa[i];
        if (p != NIL16) {
          vb[i] = (uint16_t)(va[i] + va[p]);
          pb[i] = pa[p];
        } else {
          vb[i] = va[i];
          pb[i] = (uint16_t)NIL16;
        }
      }
      __syncthreads();
      uint16_t *t = va;
      va = vb;
      vb = t;
      t = pa;
      pa = pb;
      pb = t;
    }
    uint16_t *pre = va;
    for (uint32_t i = tid; i < n; i += NEMO_BLOCK) pre[i] = (uint16_t)(pre[i] + L.up[i]);
    __syncthreads();
    // tie-free keys (len desc, preorder asc): every key is unique, so a
    // chain's position is the number of smaller keys (broadcast LDS reads,
    // four keys per read)
    uint32_t *key = (uint32_t *)L.u.kk;
    uint32_t *ord = key + ((nch + 3) & ~3u);
    for (uint32_t q = tid; q < ((nch + 3) & ~3u); q += NEMO_BLOCK) {
      uint32_t k = 0xFFFFFFFFu;
      if (q < nch) {
        const uint32_t len = tmp[2 * q + 1] & 0xFFFFu, rep = tmp[2 * q + 1] >> 16;
        k = ((0xFFFFu - len) << 16) | pre[rep];
      }
      key[q] = k;
    }
    __syncthreads();
    const uint4 *k4 = (const uint4 *)key;
    for (uint32_t q = tid; q < nch; q += NEMO_BLOCK) {
      const uint32_t me = key[q];
      uint32_t pos = 0;
      for (uint32_t j = 0; j < (nch + 3) / 4; j++) {
        const uint4 x = k4[j];
        pos += (x.x < me) + (x.y < me) + (x.z < me) + (x.w < me);
      }
      ord[pos] = q;
    }
    __syncthreads();
  }
  uint32_t *out = c.chain + 5 * gv.n0;
  const uint32_t *ord = (const uint32_t *)L.u.kk + ((nch + 3) & ~3u);
  for (uint32_t pos = tid; pos < nch; pos += NEMO_BLOCK) {
    const uint32_t q = ord[pos];
    uint32_t *w = out + 5 * pos;
    w[0] = hs[tmp[2 * q] & 0xFFFFu];
    w[1] = hs[tmp[2 * q] >> 16];
    w[2] = tmp[2 * q + 1] & 0xFFFFu;
    w[3] = gv.rank_of(w[0]);
    w[4] = 0;
  }
#ifdef NEMO_STAMPS
  __syncthreads();
#endif
  STAMP(8);
  STAMP(9);
  if (tid == 0) {
    c.nch[g] = nch;
    if (s_fail) c.err[g] = NEMO_ERR_INVALID;
  }
#undef INH
#undef RULE
}

__global__ __launch_bounds__(NEMO_BLOCK) void k_chains_big(DevCorpus c) {
  __shared__ CompLDS s_comp[NEMO_WAVES];
  __shared__ uint32_t s_lds[NEMO_WAVES];
  __shared__ uint32_t s_n, s_flag, s_nch, s_ncomp, s_big;
  const uint32_t g = blockIdx.x;
  if (c.err[g] || c.nch[g] != NEMO_NONE || c.gs_off[g] != ~0ull) return;  // k_chains / k_chains_glob
  const GraphView gv = c.view(g);
  uint8_t *f = gv.flags;
  uint32_t *hs = c.s_a + gv.n0 + g;                   // H* in topological order
  uint32_t *hl = c.s_b + gv.n0 + g;                   // H* level offsets
  uint32_t *par = c.s_c + gv.n0 + g;                  // union-find parent
  uint32_t *lev = (uint32_t *)(c.s_d + gv.n0);        // Kahn level of H* nodes
  uint32_t *ccomp = c.s_f + gv.n0 + g;                // component id
  uint32_t *cnodes = c.s_g + gv.n0 + g;               // nodes bucketed by component
  uint32_t *coff = (uint32_t *)(c.s_e + gv.n0);       // [ncomp+1] bucket offsets, then cursors
  uint32_t *roots = c.chain + 5 * gv.n0;              // temp until the final sort
  uint32_t *cidx = c.cl_next + gv.n0;                // graph-local -> component-local
  uint32_t *tmp = c.chain_tmp + c.tmp_off[g];
  const uint32_t wave = threadIdx.x >> 6;
  if (threadIdx.x == 0) {
    s_n = 0;
    s_nch = 0;
    s_ncomp = 0;
    s_big = 0;
    hl[0] = 0;
  }
  __syncthreads();
#define INH(v) ((f[v] & NEMO_F_DELETED) != 0)
  for (uint32_t l = 0; l < gv.nlev; l++) {
    const uint32_t a = gv.lvl[l], b = gv.lvl[l + 1];
    for (uint32_t base = a; base < b; base += NEMO_BLOCK) {
      const uint32_t i = base + threadIdx.x;
      uint32_t v = 0;
      bool p = false;
      if (i < b) {
        v = gv.topo[i];
        p = INH(v);
        if (p) {
          lev[v] = l;
          par[v] = v;
        }
      }
      wave_append(p, v, hs, &s_n);
    }
    __syncthreads();
    if (threadIdx.x == 0) hl[l + 1] = s_n;
    __syncthreads();
  }
  const uint32_t nh = s_n;
  if (nh == 0) {
    if (threadIdx.x == 0) c.nch[g] = 0;
    return;
  }
  // weakly connected components of H* (hook to the smaller root + compress)
  for (;;) {
    if (threadIdx.x == 0) s_flag = 0;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nh; i += NEMO_BLOCK) {
      const uint32_t v = hs[i];
      for (uint32_t j = gv.fp[v]; j < gv.fp[v + 1]; j++) {
        const uint32_t w = gv.fc[j];
        if (!INH(w)) continue;
        const uint32_t a = uf_find(par, v), b = uf_find(par, w);
        if (a != b) {
          atomicMin(&par[max(a, b)], min(a, b));
          s_flag = 1;
        }
      }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nh; i += NEMO_BLOCK) atomicMin(&par[hs[i]], uf_find(par, hs[i]));
    __syncthreads();
    if (!s_flag) break;
    __syncthreads();
  }
  // bucket H* by component
  for (uint32_t base = 0; base < nh; base += NEMO_BLOCK) {
    const uint32_t i = base + threadIdx.x;
    const uint32_t v = i < nh ? hs[i] : 0;
    wave_append(i < nh && par[v] == v, v, roots, &s_ncomp);
  }
  __syncthreads();
  const uint32_t ncomp = s_ncomp;
  for (uint32_t k = threadIdx.x; k < ncomp; k += NEMO_BLOCK) {
    ccomp[roots[k]] = k;
    coff[k] = 0;
  }
  if (threadIdx.x == 0) coff[ncomp] = 0;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nh; i += NEMO_BLOCK) {
    const uint32_t v = hs[i];
    const uint32_t k = ccomp[par[v]];
    if (par[v] != v) ccomp[v] = k;
    atomicAdd(&coff[k], 1u);
  }
  __syncthreads();
  block_scan_inplace(coff, ncomp + 1, s_lds);
  uint32_t *cur = coff + ncomp + 1;
  for (uint32_t k = threadIdx.x; k < ncomp; k += NEMO_BLOCK) cur[k] = coff[k];
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nh; i += NEMO_BLOCK) {
    const uint32_t v = hs[i];
    cnodes[atomicAdd(&cur[ccomp[v]], 1u)] = v;
  }
  __syncthreads();
  // one wave per component, LDS-resident
  for (uint32_t k = wave; k < ncomp; k += NEMO_WAVES) {
    const uint32_t a = coff[k], m = coff[k + 1] - a;
    bool ok = false;
    if (m <= CM && m <= c.comp_limit) ok = wave_component(gv, s_comp[wave], cnodes + a, m, lev, cidx, tmp, &s_nch);
    if (!ok && lane_id() == 0) s_big = 1;
  }
  __syncthreads();
  if (s_big) {
    // fallback for components beyond the LDS tile: workgroup-wide sweeps over
    // global memory; LDS-handled components are all FT_SEEN already.
    int32_t *down = c.s_d + gv.n0;
    int32_t *du = (int32_t *)(c.cl_first + gv.n0);
    unsigned long long *best = c.s_e + gv.n0;
    for (uint32_t l = gv.nlev; l-- > 0;) {
      for (uint32_t i = hl[l] + threadIdx.x; i < hl[l + 1]; i += NEMO_BLOCK) {
        const uint32_t v = hs[i];
        int32_t d = is_rule(gv.word[v]) ? 0 : -1;
        for (uint32_t j = gv.fp[v]; j < gv.fp[v + 1]; j++) {
          const uint32_t w = gv.fc[j];
          if (INH(w)) d = max(d, down[w] + 1);
        }
        down[v] = d;
        best[v] = 0ull;
      }
      __syncthreads();
    }
    for (uint32_t iter = 0;; iter++) {
      for (uint32_t l = gv.nlev; l-- > 0;) {
        for (uint32_t i = hl[l] + threadIdx.x; i < hl[l + 1]; i += NEMO_BLOCK) {
          const uint32_t v = hs[i];
          int32_t d;
          if (!(f[v] & FT_SEEN)) {
            d = down[v];
          } else {
            d = -1;
            for (uint32_t j = gv.fp[v]; j < gv.fp[v + 1]; j++) {
              const uint32_t w = gv.fc[j];
              if (INH(w) && du[w] >= 0) d = max(d, du[w] + 1);
            }
          }
          du[v] = d;
        }
        __syncthreads();
      }
      for (uint32_t i = threadIdx.x; i < nh; i += NEMO_BLOCK) {
        const uint32_t v = hs[i];
        if (is_rule(gv.word[v]) && du[v] >= 2) {
          const unsigned long long key = ((unsigned long long)(uint32_t)du[v] << 32) | (0xFFFFFFFFu - gv.rank_of(v));
          atomicMax(&best[par[v]], key);
        }
      }
      if (threadIdx.x == 0) s_flag = 0;
      __syncthreads();
      for (uint32_t i = threadIdx.x; i < nh; i += NEMO_BLOCK) {
        const uint32_t s = hs[i];
        if (!is_rule(gv.word[s]) || du[s] < 2) continue;
        const unsigned long long key = ((unsigned long long)(uint32_t)du[s] << 32) | (0xFFFFFFFFu - gv.rank_of(s));
        if (best[par[s]] != key) continue;
        int32_t rem = du[s];
        bool u = !(f[s] & FT_SEEN);
        f[s] |= FT_SEEN;
        uint32_t v = s;
        while (rem > 0) {
          uint32_t bc = NEMO_NONE, br = NEMO_NONE;
          for (uint32_t j = gv.fp[v]; j < gv.fp[v + 1]; j++) {
            const uint32_t w = gv.fc[j];
            if (!INH(w)) continue;
            const int32_t val = u ? down[w] : du[w];
            const uint32_t rw = gv.rank_of(w);
            if (val == rem - 1 && (bc == NEMO_NONE || rw < br)) {
              bc = w;
              br = rw;
            }
          }
          if (bc == NEMO_NONE) break;
          v = bc;
          u |= !(f[v] & FT_SEEN);
          f[v] |= FT_SEEN;
          rem--;
        }
        const uint32_t k = atomicAdd(&s_nch, 1u);
        uint32_t *t = tmp + 5 * k;
        t[0] = s;
        t[1] = v;
        t[2] = (uint32_t)du[s];
        t[3] = gv.rank_of(s);
        t[4] = iter;
        s_flag = 1;
      }
      __syncthreads();
      for (uint32_t i = threadIdx.x; i < nh; i += NEMO_BLOCK) best[hs[i]] = 0ull;
      const bool more = s_flag != 0;
      __syncthreads();
      if (!more) break;
    }
  }
  // acceptance order k = rank of (len desc, head rank asc, iteration asc)
  const uint32_t n = s_nch;
  uint32_t *out = c.chain + 5 * gv.n0;
  for (uint32_t i = threadIdx.x; i < n; i += NEMO_BLOCK) {
    const uint32_t li = tmp[5 * i + 2], ri = tmp[5 * i + 3], ii = tmp[5 * i + 4];
    uint32_t k = 0;
    for (uint32_t j = 0; j < n; j++) {
      const uint32_t lj = tmp[5 * j + 2], rj = tmp[5 * j + 3], ij = tmp[5 * j + 4];
      k += (lj > li) || (lj == li && (rj < ri || (rj == ri && ij < ii)));
    }
#pragma unroll
    for (int q = 0; q < 5; q++) out[5 * k + q] = tmp[5 * i + q];
  }
  for (uint32_t i = threadIdx.x; i < nh; i += NEMO_BLOCK) f[hs[i]] &= (uint8_t)~FT_SEEN;
#undef INH
  if (threadIdx.x == 0) c.nch[g] = n;
}

// The second tier lists the graphs the first handed back (k_chains_sel) and
// runs a small grid over that list: one early-exit workgroup per graph of the
// 52.5 KB tier cost ~29 us per step at C3, where the list is empty.
__global__ __launch_bounds__(NEMO_BLOCK) void k_chains_sel(DevCorpus c) {
  const uint32_t g = blockIdx.x * NEMO_BLOCK + threadIdx.x;
  const bool need = g < c.G && !c.err[g] && c.gs_off[g] == ~0ull && c.nch[g] == NEMO_NONE;
  uint32_t *sel = c.sel + c.G + 1;
  wave_append(need, g, sel + 1, sel);
}

// The first tier's H* cap: at 1280 its LDS image is 31.7 KB, so five workgroups share a CU
// (with the register budget cut to five waves per SIMD: 96 VGPRs, 52 B of spills); the chain
// cover's level loops are latency-bound, and at C3 this took k_chains 2.01 -> 1.72 ms against
// 1664 (41 KB, four per CU).  Larger H* go to k_chains_list (2048) as before.
#ifndef CH_HCAP
#define CH_HCAP 1280
#endif
#ifndef CH_WPE
#define CH_WPE 5
#endif
#define CH_WPE_ATTR __attribute__((amdgpu_waves_per_eu(CH_WPE)))
template <int HCAP, int UCAP>
__global__ __launch_bounds__(NEMO_BLOCK) CH_WPE_ATTR void k_chains(DevCorpus c) {
  chains_graph<HCAP, UCAP>(c, blockIdx.x);
}

// The list gets a kernel of its own, so the first tier's stays at 119 VGPRs
// (four waves per SIMD); this one is held to three, as its LDS allows.
template <int HCAP, int UCAP>
__global__ __launch_bounds__(NEMO_BLOCK) __attribute__((amdgpu_waves_per_eu(3))) void k_chains_list(DevCorpus c) {
  const uint32_t *sel = c.sel + c.G + 1;
  const uint32_t n = sel[0];
  for (uint32_t k = blockIdx.x; k < n; k += gridDim.x) {
    chains_graph<HCAP, UCAP>(c, sel[1 + k]);
    __syncthreads();  // the LDS image of this graph is done before the next one
  }
}

#define CHAINS_GRID 1024u
void launch_chains(const DevCorpus &c, hipStream_t s, bool tiers) {
  if (!c.G) return;
  hipLaunchKernelGGL((k_chains<CH_HCAP, 120>), dim3(c.G), dim3(NEMO_BLOCK), 0, s, c);
  if (!tiers) {  // the host knows the first tier hands nothing back (api.hip tiers_known)
    launch_chains_glob(c, s);
    return;
  }
  launch_zero(c.sel + c.G + 1, sizeof(uint32_t), s);
  hipLaunchKernelGGL(k_chains_sel, dim3((c.G + NEMO_BLOCK - 1) / NEMO_BLOCK), dim3(NEMO_BLOCK), 0, s, c);
  hipLaunchKernelGGL((k_chains_list<2048, 512>), dim3(std::min(c.G, CHAINS_GRID)), dim3(NEMO_BLOCK), 0, s, c);
  hipLaunchKernelGGL(k_chains_big, dim3(c.G), dim3(NEMO_BLOCK), 0, s, c);
  launch_chains_glob(c, s);
}

}  // namespace nemo
