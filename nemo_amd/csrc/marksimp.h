// marksimp.h — markConditionHolds + cleanCopyProv + the local part of
// collapseNextChains for one graph held by one workgroup, straight from its
// edge list in registers (pre-post-prov.go:218-244, preprocessing.go:13-348).
// Shared by k_marksimp (k_analysis.hip: its own launch, the edges loaded from
// HBM) and k_build's fused tail (k_load.hip: the edges still in the registers
// the CSR build loaded them into).  Every rule is a predicate over a node's in-
// or out-edges, so each phase is one pass over the edges that ORs bits into
// per-node LDS bytes.
#pragma once
#include "device.h"

namespace nemo {

#define MS_BLOCK 256
#define MS_EPT 32
#define A_IN 0x01u   // in-degree > 0
#define A_OUT 0x02u  // out-degree > 0
#define A_PC 0x04u   // node of table C with a parent of table C (pos source)
#define A_NC 0x08u   // ... one of which has a parent itself (neg source)
#define A_POS 0x10u  // child of an A_PC node
#define A_NEG 0x20u  // child of an A_NC node
#define A_GP 0x40u   // kept next rule: a parent goal has a kept next-rule parent
#define A_GC 0x80u   // kept next rule: a child goal has a kept next-rule child

// byte v of a 4-aligned byte array (LDS, or a corpus-wide array with v the global index)
__device__ __forceinline__ void or8(uint8_t *b, uint64_t v, uint32_t bits) {
  atomicOr((uint32_t *)b + (v >> 2), bits << (8u * (uint32_t)(v & 3u)));
}

// Graph g was done by k_build's fused tail (DevCorpus::ms_fuse at its launch):
// a graph within k_build's caps that it did not leave to the global tier.  The
// caller also checks err[g] == 0 and the t_ms tier, as the tail does.
__device__ __forceinline__ bool ms_built_by_build(const DevCorpus &c, uint32_t g, uint32_t V, uint32_t E) {
  return c.bld_bytes != 0u && V <= c.bld_v && E <= c.bld_e && !c.redo[g];
}

// Graph g (V nodes, E edges, node words `word`) -> final flags `out`, prehold[g],
// holdany[g].  sd holds edges (src << 16 | dst; ~0u = none) of the first
// EPT x B slice; when `one` is false, load(base) refills sd with the slice at
// `base` (a graph of more than EPT x B edges).  ONE: the caller knows E <= EPT x B
// (k_build): one pass per phase, no loop (a loop around the invariant slice
// had its address math hoisted, and spilled inside k_build's register budget).  dyn: marksimp_bytes(V, c.words)
// of LDS (device.h: table bitset, u16 node words, flags and aux bytes).  The
// caller's workgroup is B threads and every thread calls this.
template <int B, int EPT, bool ONE, class Load>
__device__ __forceinline__ void marksimp_graph(const DevCorpus &c, uint32_t g, uint32_t V, uint32_t E,
                                               const uint32_t *word, uint8_t *out, uint32_t (&sd)[EPT], bool one,
                                               Load &&load, uint8_t *dyn, uint32_t *s_misc) {
  const uint32_t W = c.words, tid = threadIdx.x;
  uint8_t *p = dyn;
  uint32_t *tq = (uint32_t *)p;
  p += lds_align(8u * W);
  uint16_t *nw = (uint16_t *)p;
  p += lds_align(2u * V);
  uint8_t *fl = p;
  p += lds_align(V);
  uint8_t *ax = p;
  uint32_t &s_any = s_misc[0], &s_pre = s_misc[1], &s_hold = s_misc[2];
  for (uint32_t base = 0; base < V; base += 8 * B) {
    uint32_t w[8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint32_t v = base + q * B + tid;
      w[q] = v < V ? word[v] : 0u;
    }
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint32_t v = base + q * B + tid;
      if (v < V) nw[v] = nw_of(w[q]);
    }
  }
  for (uint32_t i = tid; i < W; i += B) tq[i] = 0;
  for (uint32_t i = tid; i < (V + 3) / 4; i += B) ((uint32_t *)ax)[i] = 0;
  if (tid == 0) {
    s_any = 0;
    s_pre = 0;
    s_hold = 0;
  }
  __syncthreads();
  // one pass over the edges: fn(src, dst) for every edge of the graph
  auto edges = [&](auto fn) {
    auto slice = [&] {
#pragma unroll
      for (int q = 0; q < EPT; q++)
        if (sd[q] != 0xFFFFFFFFu) fn(sd[q] >> 16, sd[q] & 0xFFFFu);
    };
    if constexpr (ONE) {
      slice();
    } else {
      for (uint32_t base = 0; base < E; base += EPT * B) {
        if (!one) load(base);
        slice();
      }
    }
  };
  const uint32_t C = (g & 1) ? c.table_post : c.table_pre;
#define NTAB(v) (nw[v] & NW_TABLE)
#define NRULE(v) ((nw[v] & NW_RULE) != 0)
  // degrees, and the (T:C)->(Rc:C) edges of markConditionHolds' pattern
  edges([&](uint32_t s, uint32_t d) {
    or8(ax, s, A_OUT);
    or8(ax, d, A_IN);
    if (NTAB(s) == C && NTAB(d) == C) or8(ax, d, A_PC);
  });
  __syncthreads();
  // negative pattern: X->(T':C)->(R':C); then pos/neg onto the goals below Rc
  edges([&](uint32_t s, uint32_t d) {
    if ((ax[s] & A_IN) && NTAB(s) == C && NTAB(d) == C) or8(ax, d, A_NC);
  });
  __syncthreads();
  edges([&](uint32_t s, uint32_t d) {
    const uint32_t a = ax[s];
    if (a & (A_PC | A_NC)) or8(ax, d, ((a & A_PC) ? A_POS : 0u) | ((a & A_NC) ? A_NEG : 0u));
  });
  __syncthreads();
  // qualifying tables Tq: goals with a rule child, the positive and not the negative pattern
  bool any = false;
  for (uint32_t x = tid; x < V; x += B) {
    const uint32_t a = ax[x];
    if (NRULE(x) || !(a & A_OUT) || (a & (A_POS | A_NEG)) != A_POS) continue;
    atomicOr(&tq[NTAB(x) >> 5], 1u << (NTAB(x) & 31));
    any = true;
  }
  if (__any(any) && lane_id() == 0) s_any = 1;
  __syncthreads();
  // holds + cleanCopyProv's KEPT (preprocessing.go:13-63)
  const bool anyq = s_any != 0;
  uint32_t pre = 0;
  for (uint32_t x4 = tid; x4 < (V + 3) / 4; x4 += B) {
    uint32_t packed = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const uint32_t x = 4 * x4 + b;
      if (x >= V) break;
      const uint32_t t = NTAB(x), a = ax[x];
      const bool rule = NRULE(x);
      const bool h = anyq && !rule && (t == C || ((tq[t >> 5] >> (t & 31)) & 1u));
      uint32_t f = h ? NEMO_F_HOLDS : 0u;
      if (!rule || (a & (A_IN | A_OUT)) == (A_IN | A_OUT)) f |= NEMO_F_KEPT;
      packed |= f << (8 * b);
      pre += (h && t == c.table_pre) ? 1u : 0u;
    }
    ((uint32_t *)fl)[x4] = packed;
  }
  for (int d = 32; d >= 1; d >>= 1) pre += __shfl_xor(pre, d);
  if (lane_id() == 0 && pre) atomicAdd(&s_pre, pre);
  __syncthreads();
  // collapseNextChains' local rules (preprocessing.go:66-348): goals with a
  // kept next-rule parent / child ...
#define ISNEXT(v) ((nw[v] & NW_NEXT) && (fl[v] & NEMO_F_KEPT))
  edges([&](uint32_t s, uint32_t d) {
    if (ISNEXT(s) && !NRULE(d)) or8(fl, d, FT_NP);
    if (ISNEXT(d) && !NRULE(s)) or8(fl, s, FT_NC);
  });
  __syncthreads();
  // ... and next rules with a next grandparent / grandchild
  edges([&](uint32_t s, uint32_t d) {
    if (ISNEXT(d) && (fl[s] & FT_NP)) or8(ax, d, A_GP);
    if (ISNEXT(s) && (fl[d] & FT_NC)) or8(ax, s, A_GC);
  });
  __syncthreads();
  bool hold = false;
  for (uint32_t x = tid; x < V; x += B) {
    uint32_t f = fl[x];
    if (ISNEXT(x)) {
      const bool gp = (ax[x] & A_GP) != 0, gc = (ax[x] & A_GC) != 0;
      if (gp || gc) f |= NEMO_F_DELETED;
      if (!gp && gc) f |= NEMO_F_HEAD;
      if (gp && !gc) f |= NEMO_F_TAIL;
    } else if (!NRULE(x)) {
      if ((f & FT_NP) && (f & FT_NC)) f |= NEMO_F_DELETED;
      f &= ~(FT_NP | FT_NC);
      hold |= (f & (NEMO_F_HOLDS | NEMO_F_DELETED)) == NEMO_F_HOLDS;
    }
    out[x] = (uint8_t)f;
  }
#undef ISNEXT
#undef NTAB
#undef NRULE
  if (__any(hold) && lane_id() == 0) s_hold = 1;
  __syncthreads();
  if (tid == 0) {
    c.prehold[g] = s_pre;
    c.holdany[g] = s_hold;
  }
}

}  // namespace nemo
