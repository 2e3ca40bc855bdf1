// device.h — gfx950 device helpers shared by the libnemohip kernels.
//
// Execution model: one 256-thread workgroup (4 wave64s)
// owns one provenance graph; per-node state lives in graph-local slices of
// global arrays (L2-resident while the workgroup works on its graph), and
// level-synchronous sweeps walk the graph's Kahn levels with one workgroup
// barrier per level.  Frontier queues are filled with wave-aggregated appends
// (ballot + mbcnt, one LDS atomic per wave).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nemohip.h"

#define NEMO_BLOCK 256
#define NEMO_CSR_BIG 8192u  // graphs of at least this many nodes: multi-workgroup CSR build (k_csrb_*)
#define CB_MAXB 8192u       // the bucketed CSR build's buckets per graph (of 2048 nodes): V <= 16M
#ifndef CB_NB
#define CB_NB 2048u         // nodes per bucket of the bucketed CSR build
#endif
#ifndef CB_CHUNK
#define CB_CHUNK 16384u     // edges per histogram / partition chunk of the bucketed CSR build
#endif
#define NEMO_WAVES (NEMO_BLOCK / 64)
#define NEMO_NONE 0xFFFFFFFFu

// scratch flag bits (second byte array `sb`)
#define SB_ROOT 0x01u
#define SB_HASRC 0x02u
#define SB_R1 0x04u
#define SB_G2 0x08u
#define SB_RCH 0x10u
// transient bits in the flags byte (cleared before a phase returns)
#define FT_NP 0x20u   // goal: has a kept next-rule parent
#define FT_NC 0x40u   // goal: has a kept next-rule child
#define FT_SEEN 0x80u // chain greedy: node covered by an accepted chain

__device__ __forceinline__ bool is_rule(uint32_t w) { return (w & NEMO_NODE_RULE) != 0u; }
__device__ __forceinline__ uint32_t type_of(uint32_t w) { return (w & NEMO_TYPE_MASK) >> NEMO_TYPE_SHIFT; }
__device__ __forceinline__ uint32_t table_of(uint32_t w) { return w & NEMO_TABLE_MASK; }

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Wave-aggregated append of `val` (where pred) to q[*tail++]; one LDS atomic per wave.
__device__ __forceinline__ void wave_append(bool pred, uint32_t val, uint32_t *q, uint32_t *tail) {
  const uint64_t m = __ballot(pred);
  if (m == 0) return;
  const int leader = __ffsll((long long)m) - 1;
  uint32_t base = 0;
  if ((int)lane_id() == leader) base = atomicAdd(tail, (uint32_t)__popcll(m));
  base = __builtin_amdgcn_readlane(base, leader);  // leader is wave-uniform: no LDS round trip
  if (pred) q[base + mbcnt(m)] = val;
}

// Inclusive wave scan by DPP (six VALU adds, no LDS permutes): Hillis-Steele
// within each 16-lane row (row_shr 1, 2, 4, 8; lanes shifted past the row's
// start read 0), then row 0's total into row 1 and row 2's into row 3
// (row_bcast:15), then rows 0-1's total into rows 2-3 (row_bcast:31).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  uint32_t v = x;
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return v;
}

// The same by LDS permutes (__shfl_up).  DPP is the faster form where measured
// (k_build, k_pull_lds); k_chains measured 1.76 -> 2.0 ms with it, so the
// default stays the permute form.
__device__ __forceinline__ uint32_t wave_incl_scan_shfl(uint32_t x) {
  const uint32_t lane = lane_id();
  uint32_t v = x;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t y = __shfl_up(v, d);
    if (lane >= (uint32_t)d) v += y;
  }
  return v;
}

// Block-wide exclusive scan of one u32 per thread; `lds` holds B/64 u32.
template <int B = NEMO_BLOCK, bool DPP = false>
__device__ __forceinline__ uint32_t block_exscan(uint32_t x, uint32_t *total, uint32_t *lds) {
  constexpr int NW = B / 64;
  const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
  const uint32_t v = DPP ? wave_incl_scan(x) : wave_incl_scan_shfl(x);
  if (lane == 63) lds[w] = v;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NW; i++) {
    uint32_t s = lds[i];
    off += (i < (int)w) ? s : 0u;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return off + v - x;
}

// In-place exclusive scan of a[0..n) by one workgroup of B threads; returns the total.
// Each round takes PER consecutive elements per thread: 4 for LDS arrays (few
// bank conflicts), 16 for HBM arrays (16 independent loads in flight per
// thread, so a long scan costs few latency-bound rounds).
template <int B = NEMO_BLOCK, int PER = 4, bool DPP = false, typename T>
__device__ __forceinline__ uint32_t block_scan_inplace(T *a, uint32_t n, uint32_t *lds) {
  uint32_t carry = 0;
  for (uint32_t base = 0; base < n; base += B * PER) {
    const uint32_t i0 = base + threadIdx.x * PER;
    uint32_t x[PER], s = 0;
#pragma unroll
    for (int k = 0; k < PER; k++) {
      x[k] = (i0 + k < n) ? a[i0 + k] : 0u;
      s += x[k];
    }
    uint32_t tot;
    uint32_t ex = block_exscan<B, DPP>(s, &tot, lds) + carry;
#pragma unroll
    for (int k = 0; k < PER; k++) {
      if (i0 + k < n) a[i0 + k] = (T)ex;
      ex += x[k];
    }
    carry += tot;
  }
  __syncthreads();  // the writes above land after block_exscan's last barrier
  return carry;
}

__device__ __forceinline__ uint32_t ld_relaxed(const uint32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Intra-wave LDS hand-off: lanes of one wave run in lockstep and DS ops of a
// wave complete in order, so ordering the compiler is all that is needed.
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <bool DPP = false>
__device__ __forceinline__ uint32_t wave_exscan(uint32_t x, uint32_t *total) {
  if (DPP) {
    const uint32_t v = wave_incl_scan(x);
    *total = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
    return v - x;
  }
  const uint32_t v = wave_incl_scan_shfl(x);
  *total = __shfl(v, 63);
  return v - x;
}

__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const unsigned long long y = __shfl_xor(v, d);
    v = y > v ? y : v;
  }
  return v;
}

// Graph-local view.  Arrays indexed per node use base n0 (+g for the V+1-sized
// ones), arrays indexed per edge use base e0.
struct GraphView {
  uint32_t g, V, E;
  uint64_t n0, e0;
  const uint32_t *word, *label, *rank;
  const uint32_t *fp, *fc, *rp, *rc;  // local CSR (rows sorted)
  const uint32_t *topo, *lvl;          // Kahn order, level offsets into topo
  uint32_t nlev;
  uint8_t *flags;

  __device__ __forceinline__ uint32_t rank_of(uint32_t v) const { return rank ? rank[v] : v; }
  __device__ __forceinline__ uint32_t indeg(uint32_t v) const { return rp[v + 1] - rp[v]; }
  __device__ __forceinline__ uint32_t outdeg(uint32_t v) const { return fp[v + 1] - fp[v]; }
};

// One kernel's LDS graph tier: graphs with V <= v, E <= e and nlev <= l are
// staged by that kernel's LDS variant (bytes = its dynamic LDS; 0 = tier off).
// Each kernel's image differs, so each has its own caps (api.hip set_lds_tier).
struct Tier {
  uint32_t v, e, l, bytes;
};

// Device-side arrays of a loaded corpus (all graphs concatenated).
struct DevCorpus {
  uint32_t G, n_runs, n_tables, words, table_pre, table_post;
  uint32_t hcap_limit;                   // largest chain subgraph H* k_chains stages in LDS (test knob)
  uint32_t comp_limit;                   // largest H* component k_chains_big stages in LDS (test knob)
  uint32_t bld_v, bld_e, bld_bytes;      // k_build's LDS caps and image size (0 = tier off)
  uint32_t lds_v, lds_e, lds_l;          // k_proto_lds's LDS tier caps (V, E, Kahn levels); 0 = tier off
  uint32_t lds_bytes;                    // dynamic LDS of k_proto_lds
  Tier t_ms, t_diff, t_pull;             // the LDS tiers of k_marksimp, k_diff_lds, k_pull_lds
  uint32_t gblock;                       // workgroup size of the global-tier kernels (256, or 1024 for deep corpora)
  uint32_t glob_block;                   // k_chains_glob's workgroup size (256 or 512)
  uint32_t glob_stop;                    // diagnostic (stamps build): k_chains_glob returns after phase k (0: none)
  uint32_t glob_prep;                    // 1: k_glob_prep builds the deep graphs' H* order and adjacency (identity ranks)
  uint32_t topo_ell;                     // 1: deep graphs' Kahn levels by k_topo_ell (child records in gscratch)
  uint32_t ms_fuse;                      // 1: k_build's tail runs marksimp_graph on its graphs (marksimp.h)
  uint32_t bld_relax;                    // 1: k_build's Kahn levels by relaxation sweeps (peeling if they give up)
  uint32_t n_glob;                       // deep graphs (gs_off != ~0)
  const uint32_t *glob_list;             // [n_glob] their graph ids
  uint32_t *team;                        // k_glob_prep's team scratch (barrier counters, phase sums)
  uint32_t n_cu;                         // compute units of the device
  uint32_t pg_chunks;                    // k_pg_* workgroups per listed graph (by the largest post graph)
  const uint64_t *node_off, *edge_off;
  const uint32_t *word, *label, *rank;  // rank may be null
  const uint32_t *esrc, *edst;
  uint32_t *fp, *fc, *rp, *rc;           // fp/rp: V+G entries (graph g at n0+g)
  uint32_t *topo, *lvl, *nlev;           // lvl: V+G entries
  uint32_t *nlv;                         // [V] Kahn level of every node
  uint32_t *e2, *posoff;                 // post graphs built by k_build: forward edges in source Kahn order
                                         // (src << 16 | dst, [E]) and each Kahn position's first edge ([V])
  uint8_t *flags, *sb;                   // V
  uint32_t *s_a, *s_b, *s_c;             // V+G scratch
  int32_t *s_d;                          // V scratch
  unsigned long long *s_e;               // V scratch
  uint32_t *s_f, *s_g;                   // V+G scratch
  uint32_t *err;                         // [G] NEMO_ERR_* of the graph (0 = fine)
  uint32_t *created;                     // [G] loadProv relationships-created
  uint32_t *prehold;                     // [G] #holding "pre" goals (pre graphs)
  uint32_t *holdany;                     // [G] 1 iff a holding goal survives simplification
  uint8_t *redo;                         // [G] k_build left the graph to the global tier
  uint32_t *gscratch;                    // k_chains_glob scratch (deep graphs), null if none
  const uint64_t *gs_off;                // [G] u32 offset of the graph's region, ~0 = not deep
  uint32_t *chain;                       // [5*V] sorted chains (head, tail, len, rank, iter) at n0
  uint32_t *chain_tmp;                   // [5*V of the graphs k_chains_glob does not take]
  const uint64_t *tmp_off;               // [G] u32 offset of the graph's chain_tmp region
  uint32_t *nch;                         // [G]
  uint32_t *sel;                         // [4 (G + 1)] fallback-tier worklists (count first): k_pull's, k_chains', k_csr/k_topo's, k_pg_*'s (runs)
  const uint32_t *big;                   // graphs of >= 8192 nodes (host list): the multi-workgroup CSR build
  uint32_t n_big;
  // its bucketed form (null cb_hist: the atomic form): (bucket, chunk) counts per big graph at
  // cb_hoff[b], (key, value) edge scratch, the largest bucket and chunk counts (the grid)
  uint32_t *cb_hist, *cb_key, *cb_val;
  const uint64_t *cb_hoff;
  uint32_t cb_maxbk, cb_maxck;
  uint32_t *cl_first;                    // [V] first chain of a tail (k_proto's global tier; scratch elsewhere)
  uint32_t *cl_next;                     // [V] next chain with the same tail
  uint32_t *proto_bits, *graph_tables;   // [n_runs*words]
  uint8_t *gate;                         // [n_runs]
  unsigned long long *stamps;            // diagnostic builds only: [16*G] phase stamps

  __device__ __forceinline__ GraphView view(uint32_t g) const {
    GraphView v;
    v.g = g;
    v.n0 = node_off[g];
    v.e0 = edge_off[g];
    v.V = (uint32_t)(node_off[g + 1] - v.n0);
    v.E = (uint32_t)(edge_off[g + 1] - v.e0);
    v.word = word + v.n0;
    v.label = label + v.n0;
    v.rank = rank ? rank + v.n0 : nullptr;
    v.fp = fp + v.n0 + g;
    v.rp = rp + v.n0 + g;
    v.fc = fc + v.e0;
    v.rc = rc + v.e0;
    v.topo = topo + v.n0;
    v.lvl = lvl + v.n0 + g;
    v.nlev = nlev[g];
    v.flags = flags + v.n0;
    return v;
  }
};

// ---- LDS graph tier ------------------------------------------------------------
// A graph with V <= lds_v, E <= lds_e and nlev <= lds_l is staged into LDS as
// u16 CSR rows (both directions), u16 Kahn order and level offsets, a u16 node
// word (bit 15 rule, bit 14 @next rule, low 14 bits table) and two bytes of
// node state; the kernel then walks it without touching HBM.  The host sizes
// the caps from the corpus so that two workgroups fit a CU.  Graphs outside
// the caps run the global-memory kernels.
#define NW_RULE 0x8000u
#define NW_NEXT 0x4000u
#define NW_TABLE 0x3FFFu
__host__ __device__ __forceinline__ uint32_t lds_align(uint32_t b) { return (b + 15u) & ~15u; }
// slot hash of an interned label (the diff's failGoals table, api.hip / k_diff.hip)
__host__ __device__ __forceinline__ uint32_t hash_label(uint32_t x) {
  x *= 0x9E3779B1u;
  return x ^ (x >> 15);
}
// k_proto_lds's chains (head, tail) held in registers, PROTO_CHQ per thread of its
// PROTO_BLOCK: graphs with more run the global tier
#define PROTO_CHQ 4
__host__ __device__ __forceinline__ uint32_t proto_chain_cap(uint32_t) { return PROTO_CHQ * 512u; }
// k_proto_lds's image: table bitsets, u16 node bytes, per-level edge offsets, the
// forward edges in source Kahn order (u32 pairs): 39 KB at C3, four workgroups per CU
__host__ __device__ __forceinline__ uint32_t lds_tier_bytes(uint32_t v, uint32_t e, uint32_t l, uint32_t words) {
  return lds_align(8u * words) + lds_align(2u * (v + 1u)) + lds_align(2u * (l + 1u)) + lds_align(4u * e);
}

__device__ __forceinline__ bool lds_fits(const DevCorpus &c, uint32_t V, uint32_t E, uint32_t nlev) {
  return c.lds_bytes != 0u && V <= c.lds_v && E <= c.lds_e && nlev <= c.lds_l;
}
__host__ __device__ __forceinline__ bool tier_fits(const Tier &t, uint32_t V, uint32_t E, uint32_t nlev) {
  return t.bytes != 0u && V <= t.v && E <= t.e && nlev <= t.l;
}
// LDS images of the other tiered kernels (k_analysis.hip / k_diff.hip carve them)
__host__ __device__ __forceinline__ uint32_t marksimp_bytes(uint32_t v, uint32_t words) {
  return lds_align(8u * words) + lds_align(2u * v) + 2u * lds_align(v);
}
__host__ __device__ __forceinline__ uint32_t diff_lds_bytes(uint32_t v, uint32_t e, uint32_t l) {
  return 2u * lds_align(2u * (v + 1u)) + 2u * lds_align(2u * e) + lds_align(4u * ((v + 31u) / 32u)) + lds_align(v);
}
__host__ __device__ __forceinline__ uint32_t pull_lds_bytes(uint32_t v, uint32_t e) {
  return lds_align(2u * (v + 1u)) + lds_align(2u * e) + lds_align(8u * ((v + 63u) / 64u));
}

struct ProtoLds {
  uint32_t *words;      // 2 * c.words u32 of table bitsets
  uint16_t *ab;         // per node: flags byte | PB_* byte << 8 (u32-packed pairs for atomics)
  uint16_t *elo;        // per Kahn level: first edge of e2[] whose source is on it
  uint32_t *e2;         // forward edges in source Kahn order: src << 16 | dst
};

// Carve k_proto_lds's dynamic LDS for a graph of V nodes / E edges / L levels.
__device__ __forceinline__ ProtoLds proto_carve(void *base, uint32_t V, uint32_t E, uint32_t L, uint32_t words,
                                                uint32_t chain_cap) {
  (void)chain_cap;
  uint8_t *p = (uint8_t *)base;
  ProtoLds g;
  g.words = (uint32_t *)p;
  p += lds_align(8u * words);
  g.ab = (uint16_t *)p;
  p += lds_align(2u * (V + 1u));
  g.elo = (uint16_t *)p;
  p += lds_align(2u * (L + 1u));
  g.e2 = (uint32_t *)p;
  return g;
}

// Batched HBM -> LDS staging.  Every source is read in 16-B aligned chunks
// (a chunk may start before the slice or end after it: slices live inside
// page-granular allocations and the extra lanes are dropped), and each thread
// keeps STAGE_DEPTH chunks in flight, so a whole ~5k-node graph arrives in a
// handful of HBM round trips instead of one per loop iteration.
enum StageKind : uint32_t { ST_U16 = 0, ST_U8 = 1, ST_WORD = 2, ST_U32 = 3 };
struct StageDesc {
  const void *src;
  void *dst;
  uint32_t n;     // elements
  uint32_t kind;  // ST_U16: u32 -> u16; ST_U8: u8 -> u8; ST_WORD: node word -> NW_* u16
};
#define STAGE_DEPTH 8

__device__ __forceinline__ uint16_t nw_of(uint32_t w) {
  return (uint16_t)((is_rule(w) ? NW_RULE : 0u) | ((is_rule(w) && type_of(w) == NEMO_TYPE_NEXT) ? NW_NEXT : 0u) |
                    (table_of(w) & NW_TABLE));
}

// Every descriptor index below is a compile-time constant after unrolling, so
// the descriptors stay in registers (a dynamically indexed local array would
// live in scratch memory).
template <int ND, int BLOCK = NEMO_BLOCK>
__device__ __forceinline__ void stage_lds(const StageDesc (&d)[ND]) {
  uint32_t first[ND + 1], skip[ND];
  first[0] = 0;
#pragma unroll
  for (int i = 0; i < ND; i++) {
    const uint32_t es = d[i].kind == ST_U8 ? 1u : 4u;
    const uint32_t a = (uint32_t)((uintptr_t)d[i].src & 15u) / es;  // elements before the slice in its chunk
    const uint32_t per = 16u / es;
    skip[i] = a;
    first[i + 1] = first[i] + (d[i].n ? (d[i].n + a + per - 1) / per : 0u);
  }
  const uint32_t total = first[ND];
  for (uint32_t base = 0; base < total; base += STAGE_DEPTH * BLOCK) {
    uint4 v[STAGE_DEPTH];
#pragma unroll
    for (int q = 0; q < STAGE_DEPTH; q++) {
      const uint32_t k = base + q * BLOCK + threadIdx.x;
      const uint8_t *p = nullptr;
#pragma unroll
      for (int i = 0; i < ND; i++)
        if (k >= first[i] && k < first[i + 1])
          p = (const uint8_t *)((uintptr_t)d[i].src & ~(uintptr_t)15) + 16u * (k - first[i]);
      v[q] = p ? *(const uint4 *)p : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < STAGE_DEPTH; q++) {
      const uint32_t k = base + q * BLOCK + threadIdx.x;
      const uint32_t w[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
      for (int i = 0; i < ND; i++) {
        if (!(k >= first[i] && k < first[i + 1])) continue;
        const int32_t n = (int32_t)d[i].n;
        if (d[i].kind == ST_U8) {
          const int32_t e0 = 16 * (int32_t)(k - first[i]) - (int32_t)skip[i];
          uint8_t *o = (uint8_t *)d[i].dst;
#pragma unroll
          for (int b = 0; b < 16; b++)
            if (e0 + b >= 0 && e0 + b < n) o[e0 + b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
        } else if (d[i].kind == ST_U32) {
          const int32_t e0 = 4 * (int32_t)(k - first[i]) - (int32_t)skip[i];
          uint32_t *o = (uint32_t *)d[i].dst;
#pragma unroll
          for (int b = 0; b < 4; b++)
            if (e0 + b >= 0 && e0 + b < n) o[e0 + b] = w[b];
        } else {
          const int32_t e0 = 4 * (int32_t)(k - first[i]) - (int32_t)skip[i];
          uint16_t *o = (uint16_t *)d[i].dst;
          const bool word = d[i].kind == ST_WORD;
#pragma unroll
          for (int b = 0; b < 4; b++)
            if (e0 + b >= 0 && e0 + b < n) o[e0 + b] = word ? nw_of(w[b]) : (uint16_t)w[b];
        }
      }
    }
  }
}

#ifdef NEMO_STAMPS
// diagnostic build only: per-phase s_memtime stamps of thread 0 (never in the product build)
#define STAMP(k)                                                                          \
  do {                                                                                    \
    if (threadIdx.x == 0 && c.stamps) {                                                   \
      unsigned long long t_;                                                              \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");          \
      c.stamps[16 * (size_t)blockIdx.x + (k)] = t_;                                       \
    }                                                                                     \
  } while (0)
// the same for a 2-D grid (block index x + y * gridDim.x)
#define STAMP2(k)                                                                               \
  do {                                                                                          \
    if (threadIdx.x == 0 && c.stamps) {                                                         \
      unsigned long long t_;                                                                    \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                \
      c.stamps[16 * ((size_t)blockIdx.y * gridDim.x + blockIdx.x) + (k)] = t_;                  \
    }                                                                                           \
  } while (0)
// phase accumulators: TICK waits for the wave's outstanding memory operations,
// so a phase is charged with the latency of the loads it issued
// diagnostic early exit after phase k of a stamped kernel (per-phase HBM counters)
#define GSTOP(k)                                   \
  do {                                             \
    if (c.glob_stop == (k)) {                      \
      if (threadIdx.x == 0) c.nch[blockIdx.x] = 0; \
      return;                                      \
    }                                              \
  } while (0)
#define TICK(t) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory")
#else
#define STAMP(k) \
  do {           \
  } while (0)
#define STAMP2(k) \
  do {            \
  } while (0)
#define GSTOP(k) \
  do {           \
  } while (0)
#endif
