// k_diff.hip — differential provenance (differential-provenance.go:18-146),
// edge pulls (pre-post-prov.go:288-459, Q24) and the run-0 trigger patterns of
// corrections.go:30-34,121-125 / extensions.go:63-67.
#include "device.h"
#include "internal.h"

namespace nemo {

#define DB_F 0x01u
#define DB_B 0x02u
#define DB_PRESENT 0x04u
#define DB_LEAF 0x08u
#define DB_D 0x10u
#define DB_LP 0x20u

// LDS image of run 0's post graph for k_diff_lds: u16 rows both ways, a rule
// bitmap and the entry's node bits (~5V + 4E bytes, three workgroups per CU
// at the tier caps, so a few hundred diff entries run in one round); the Kahn
// order (coalesced, one load per level) and the depths stay in HBM.
struct DiffLds {
  uint16_t *rp, *fp, *rc, *fc;
  uint32_t *rule;
  uint8_t *bits;
};
__device__ __forceinline__ DiffLds diff_carve(void *base, uint32_t V, uint32_t E, uint32_t L) {
  uint8_t *p = (uint8_t *)base;
  DiffLds d;
  d.rp = (uint16_t *)p;
  p += lds_align(2u * (V + 1u));
  d.fp = (uint16_t *)p;
  p += lds_align(2u * (V + 1u));
  d.rc = (uint16_t *)p;
  p += lds_align(2u * E);
  d.fc = (uint16_t *)p;
  p += lds_align(2u * E);
  d.rule = (uint32_t *)p;
  p += lds_align(4u * ((V + 31u) / 32u));
  d.bits = p;
  return d;
}
__device__ __forceinline__ bool diff_lds_fits(const DevCorpus &c, const GraphView &gv) {
  return tier_fits(c.t_diff, gv.V, gv.E, gv.nlev);
}

// failGoals = collect(failed.label) (:23-24): every run-0 post goal whose label
// is a post-goal label of the source graph gets DB_PRESENT.  Each thread takes
// DL_BATCH source nodes and walks their hash probes together, so a pass costs
// a few rounds of independent loads rather than a binary search per node.
// The label source is the post graph of the entry's source run, or (label
// mode) a label set handed over in device memory as [n, label...]: the set of
// failedRuns[0]'s post-goal labels broadcast from the shard that owns it.
#define DL_BATCH 8
struct LabelSrc {
  const uint32_t *label, *word;  // word == nullptr: every entry is a goal label
  uint32_t n;
};
__device__ __forceinline__ LabelSrc diff_label_src(const DevCorpus &c, const DiffArgs &a, uint32_t e) {
  if (a.ref_labels) return {a.ref_labels + 1, nullptr, a.ref_labels[0]};
  const GraphView s = c.view(a.src[e]);
  return {s.label, s.word, s.V};
}
template <int B = NEMO_BLOCK>
__device__ __forceinline__ void diff_fail_goals(const DiffArgs &a, const LabelSrc &src, uint8_t *bits,
                                                const uint32_t *idx) {
  for (uint32_t base = 0; base < src.n; base += DL_BATCH * B) {
    uint32_t lab[DL_BATCH], h[DL_BATCH], pos[DL_BATCH], live = 0;
#pragma unroll
    for (int q = 0; q < DL_BATCH; q++) {
      const uint32_t x = base + q * B + threadIdx.x;
      const bool in = x < src.n && (!src.word || !is_rule(src.word[x]));
      lab[q] = in ? src.label[x] : 0u;
      h[q] = hash_label(lab[q]) & a.r0hmask;
      pos[q] = NEMO_NONE;
      live |= (in ? 1u : 0u) << q;
    }
    while (live) {
      uint32_t k[DL_BATCH];
#pragma unroll
      for (int q = 0; q < DL_BATCH; q++) k[q] = ((live >> q) & 1u) ? a.r0hkey[h[q]] : 0u;
#pragma unroll
      for (int q = 0; q < DL_BATCH; q++) {
        if (!((live >> q) & 1u)) continue;
        if (k[q] == lab[q] + 1u) {
          pos[q] = h[q];
          live &= ~(1u << q);
        } else if (k[q] == 0u) {
          live &= ~(1u << q);
        } else {
          h[q] = (h[q] + 1u) & a.r0hmask;
        }
      }
    }
#pragma unroll
    for (int q = 0; q < DL_BATCH; q++)
      if (pos[q] != NEMO_NONE) pos[q] = a.r0hval[pos[q]];
#pragma unroll
    for (int q = 0; q < DL_BATCH; q++)
      if (pos[q] != NEMO_NONE)
        for (uint32_t i = pos[q]; i < a.n_r0lab && a.r0lab[i] == lab[q]; i++) bits[idx[i]] = DB_PRESENT;
  }
}

// ---- global tier: run 0's post graph relaid in Kahn order, windowed sweeps ----
// A level-synchronous sweep over a deep graph (C5: ~4900 Kahn levels of ~200
// nodes) done node by node costs several dependent gathers per level, and a
// diff entry is one workgroup, so those gathers all queue on one CU.  All
// entries share g0, so g0 is first relaid once per diffprov call by
// whole-GPU kernels (k_dprep_*): nodes in Kahn order, rows of parents and
// children as Kahn positions, the level and rule bit packed per position.
// Every entry then works in Kahn-position space: its bits and depths are
// contiguous, a window of DW_N consecutive positions (~20 levels) is staged
// with coalesced loads (links inside the window become LDS links, links
// before/after it read final values), and the window's levels are swept in
// LDS with one barrier each.
#define DW_N 4096u    // Kahn positions per window
#define DW_E 8192u    // in-window links past each node's first two, staged in LDS
#define DW_SPILL 0xFFFFu
struct DiffWin {
  uint32_t off[DW_N];     // first extra link of node k
  int32_t dep[DW_N];      // depth (mode 2)
  uint16_t ln[DW_N];      // extra link count, DW_SPILL = re-read the row from HBM
  uint16_t adj[DW_E];     // window-local index of each extra in-window link
  uint16_t u0[DW_N], u1[DW_N];  // first two in-window links (DW_SPILL = none)
  uint8_t val[DW_N];      // F / B bit (modes 0, 1), D bit (mode 2)
  uint32_t lv[DW_N];      // Kahn level
};

// g0 in Kahn order, pass 1 (one thread per position): inverse order, row
// lengths, level << 1 | rule
__global__ __launch_bounds__(NEMO_BLOCK) void k_dprep_a(DevCorpus c, DiffArgs a) {
  const GraphView gv = c.view(a.g0);
  if (diff_lds_fits(c, gv)) return;
  const uint32_t i = blockIdx.x * NEMO_BLOCK + threadIdx.x;
  if (i == 0) {
    a.trp[gv.V] = 0;
    a.tfp[gv.V] = 0;
  }
  if (i >= gv.V) return;
  const uint32_t v = gv.topo[i];
  a.tpos[v] = i;
  a.trp[i] = gv.rp[v + 1] - gv.rp[v];
  a.tfp[i] = gv.fp[v + 1] - gv.fp[v];
  a.tinfo[i] = (c.nlv[gv.n0 + v] << 1) | (is_rule(gv.word[v]) ? 1u : 0u);
}
// pass 2 (one workgroup): row starts
__global__ __launch_bounds__(1024) void k_dprep_scan(DevCorpus c, DiffArgs a) {
  __shared__ uint32_t s_red[16];
  const GraphView gv = c.view(a.g0);
  if (diff_lds_fits(c, gv)) return;
  block_scan_inplace<1024, 16>(a.trp, gv.V + 1, s_red);
  block_scan_inplace<1024, 16>(a.tfp, gv.V + 1, s_red);
}
// pass 3 (one thread per position): rows as Kahn positions; label nodes as positions
__global__ __launch_bounds__(NEMO_BLOCK) void k_dprep_b(DevCorpus c, DiffArgs a) {
  const GraphView gv = c.view(a.g0);
  if (diff_lds_fits(c, gv)) return;
  const uint32_t i = blockIdx.x * NEMO_BLOCK + threadIdx.x;
  if (i < a.n_r0lab) a.r0pos[i] = a.tpos[a.r0idx[i]];
  if (i >= gv.V) return;
  const uint32_t v = gv.topo[i];
  uint32_t o = a.trp[i];
  for (uint32_t j = gv.rp[v]; j < gv.rp[v + 1]; j++) a.trc[o++] = a.tpos[gv.rc[j]];
  o = a.tfp[i];
  for (uint32_t j = gv.fp[v]; j < gv.fp[v + 1]; j++) a.tfc[o++] = a.tpos[gv.fc[j]];
}

// mode 0: F = Good | any F parent        (Fwd*(Good), forward over parents)
// mode 1: B = Good | any B child; D = F&B (Bwd*(Good), backward over children)
// mode 2: depth = max(0, depth(p) + 1 over D parents p), D nodes only
// bits/depth are indexed by Kahn position.  Thread t owns window positions
// t, t + B, ...: its nodes' level and accumulator stay in registers.
template <int B, int MODE>
__device__ __noinline__ void diff_window_sweep(uint32_t V, const DiffArgs &a, uint8_t *bits, int32_t *depth,
                                               DiffWin &W, uint32_t *s_red, unsigned long long *st) {
#ifdef NEMO_STAMPS
  unsigned long long acc_s = 0, acc_l = 0, acc_w = 0, t_a, t_b;
#define DW_T(t) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory")
#endif
  constexpr int PT = (int)(DW_N / B);
  constexpr bool FWD = MODE != 1;
  constexpr uint32_t NIL = 0xFFFFFFFFu;
  const uint32_t tid = threadIdx.x;
  const uint32_t *ptr = FWD ? a.trp : a.tfp, *col = FWD ? a.trc : a.tfc;
  const uint32_t nwin = (V + DW_N - 1) / DW_N;
  for (uint32_t wi = 0; wi < nwin; wi++) {
    // forward: windows in Kahn order; backward: from the end
    const uint32_t w0 = FWD ? wi * DW_N : (V > (wi + 1) * DW_N ? V - (wi + 1) * DW_N : 0u);
    const uint32_t w1 = FWD ? min(V, w0 + DW_N) : V - wi * DW_N;
    const uint32_t n = w1 - w0;
#ifdef NEMO_STAMPS
    DW_T(t_a);
#endif
    uint32_t r0[PT], r1[PT], lev[PT], p0[PT], p1[PT], cx[PT];
    int32_t x[PT];
    uint8_t ob[PT];
#pragma unroll
    for (int q = 0; q < PT; q++) {
      const uint32_t k = tid + q * B, i = w0 + k;
      const bool in = k < n;
      const uint32_t info = in ? a.tinfo[i] : 0u;
      r0[q] = in ? ptr[i] : 0u;
      r1[q] = in ? ptr[i + 1] : 0u;
      lev[q] = in ? info >> 1 : NIL;
      ob[q] = in ? bits[i] : 0u;
      const bool good = in && !(info & 1u) && !(ob[q] & DB_PRESENT);
      x[q] = MODE == 2 ? 0 : (good ? 1 : 0);
      if (MODE == 2 && !(ob[q] & DB_D)) r1[q] = r0[q];  // only D nodes get a depth
      if (MODE != 2 && good) r1[q] = r0[q];             // Good: set regardless of neighbours
    }
#pragma unroll
    for (int q = 0; q < PT; q++) {
      p0[q] = r1[q] > r0[q] ? col[r0[q]] : NIL;
      p1[q] = r1[q] > r0[q] + 1 ? col[r0[q] + 1] : NIL;
    }
    // links leaving the window read final values; links inside it go to LDS
#pragma unroll
    for (int q = 0; q < PT; q++) {
      uint32_t u0 = NIL, u1 = NIL;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const uint32_t p = h ? p1[q] : p0[q];
        if (p == NIL) continue;
        const bool inw = FWD ? p >= w0 : p < w1;
        uint32_t u = NIL;
        if (MODE == 2) {
          const uint8_t bp = bits[p];
          if (bp & DB_D) {
            if (inw) u = p - w0;
            else x[q] = max(x[q], depth[p] + 1);
          }
        } else if (inw) {
          u = p - w0;
        } else if (bits[p] & (MODE == 0 ? DB_F : DB_B)) {
          x[q] = 1;
        }
        if (h) u1 = u;
        else u0 = u;
      }
      const uint32_t k = tid + q * B;
      if (k < n) {
        W.u0[k] = u0 == NIL ? (uint16_t)DW_SPILL : (uint16_t)u0;
        W.u1[k] = u1 == NIL ? (uint16_t)DW_SPILL : (uint16_t)u1;
      }
    }
    // the rest of long rows (rare)
#pragma unroll
    for (int q = 0; q < PT; q++) {
      cx[q] = 0;
      for (uint32_t j = r0[q] + 2; j < r1[q]; j++) {
        const uint32_t p = col[j];
        const bool inw = FWD ? p >= w0 : p < w1;
        if (MODE == 2) {
          if (!(bits[p] & DB_D)) continue;
          if (inw) cx[q]++;
          else x[q] = max(x[q], depth[p] + 1);
        } else if (inw) {
          cx[q]++;
        } else if (bits[p] & (MODE == 0 ? DB_F : DB_B)) {
          x[q] = 1;
        }
      }
    }
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < PT; q++) sum += cx[q];
    uint32_t tot;
    uint32_t base = block_exscan<B>(sum, &tot, s_red);
#pragma unroll
    for (int q = 0; q < PT; q++) {
      const uint32_t k = tid + q * B;
      if (k >= n) continue;
      if (MODE == 2) {
        W.dep[k] = x[q];
        W.val[k] = (ob[q] & DB_D) ? 1 : 0;
      } else {
        W.val[k] = (uint8_t)x[q];
      }
      W.lv[k] = lev[q];
      W.ln[k] = 0;
      if (!cx[q]) continue;
      const bool spill = base + cx[q] > DW_E;
      W.off[k] = base;
      W.ln[k] = spill ? (uint16_t)DW_SPILL : (uint16_t)cx[q];
      if (!spill) {
        uint32_t o = base;
        for (uint32_t j = r0[q] + 2; j < r1[q]; j++) {
          const uint32_t p = col[j];
          const bool inw = FWD ? p >= w0 : p < w1;
          if (inw && (MODE != 2 || (bits[p] & DB_D))) W.adj[o++] = (uint16_t)(p - w0);
        }
      }
      base += cx[q];
    }
    __syncthreads();
#ifdef NEMO_STAMPS
    DW_T(t_b);
    acc_s += t_b - t_a;
    t_a = t_b;
#endif
    // the window's levels, walked by ONE wave: a level is a few LDS round trips
    // and no workgroup barrier (a wave's LDS operations complete in order);
    // positions are level-sorted, so a level is a contiguous run
    if (tid < 64) {
      const uint32_t lane = lane_id();
      uint32_t k = 0;
      while (k < n) {
        const uint32_t q = k + lane, kk = FWD ? q : n - 1u - q;
        const bool in = q < n;
        const uint32_t lv = in ? W.lv[kk] : NIL;
        const uint32_t l = __builtin_amdgcn_readfirstlane(lv);
        const bool mine = in && lv == l;
        const uint64_t m = __ballot(mine);
        if (mine) {
          const uint32_t v0 = W.u0[kk], v1 = W.u1[kk], ln = W.ln[kk];
          if (MODE != 2) {
            if (!W.val[kk]) {
              const uint32_t a0 = W.val[v0 != DW_SPILL ? v0 : kk], a1 = W.val[v1 != DW_SPILL ? v1 : kk];
              uint32_t hv = (v0 != DW_SPILL ? a0 : 0u) | (v1 != DW_SPILL ? a1 : 0u);
              if (!hv && ln) {
                if (ln != DW_SPILL) {
                  const uint32_t o = W.off[kk];
                  for (uint32_t t = 0; t < ln; t++) hv |= W.val[W.adj[o + t]];
                } else {
                  const uint32_t i = w0 + kk;
                  for (uint32_t j = ptr[i] + 2; j < ptr[i + 1]; j++) {
                    const uint32_t p = col[j];
                    if (FWD ? p >= w0 : p < w1) hv |= W.val[p - w0];
                  }
                }
              }
              if (hv) W.val[kk] = 1;
            }
          } else if (W.val[kk]) {  // D nodes get a depth
            const int32_t a0 = W.dep[v0 != DW_SPILL ? v0 : kk], a1 = W.dep[v1 != DW_SPILL ? v1 : kk];
            int32_t d = W.dep[kk];
            if (v0 != DW_SPILL) d = max(d, a0 + 1);
            if (v1 != DW_SPILL) d = max(d, a1 + 1);
            if (ln) {
              if (ln != DW_SPILL) {
                const uint32_t o = W.off[kk];
                for (uint32_t t = 0; t < ln; t++) d = max(d, W.dep[W.adj[o + t]] + 1);
              } else {
                const uint32_t i = w0 + kk;
                for (uint32_t j = ptr[i] + 2; j < ptr[i + 1]; j++) {
                  const uint32_t p = col[j];
                  if (p >= w0 && (bits[p] & DB_D)) d = max(d, W.dep[p - w0] + 1);
                }
              }
            }
            W.dep[kk] = d;
          }
        }
        k += (uint32_t)__popcll(m);
        wsync();
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PT; q++) {
      const uint32_t k = tid + q * B;
      if (k < n) x[q] = MODE == 2 ? W.dep[k] : (int32_t)W.val[k];
    }
#ifdef NEMO_STAMPS
    DW_T(t_b);
    acc_l += t_b - t_a;
    t_a = t_b;
#endif
#pragma unroll
    for (int q = 0; q < PT; q++) {
      const uint32_t k = tid + q * B, i = w0 + k;
      if (k >= n) continue;
      if (MODE == 0) {
        if (x[q]) bits[i] = ob[q] | DB_F;
      } else if (MODE == 1) {
        if (x[q]) bits[i] = ob[q] | DB_B | ((ob[q] & DB_F) ? DB_D : 0u);
      } else if (ob[q] & DB_D) {
        depth[i] = x[q];
      }
    }
    // the window's HBM writes must be performed before the next window (or
    // sweep) stages: a workgroup barrier alone does not wait for them
    __threadfence();
    __syncthreads();
#ifdef NEMO_STAMPS
    DW_T(t_b);
    acc_w += t_b - t_a;
#endif
  }
#ifdef NEMO_STAMPS
  if (tid == 0 && st) {
    st[3 * MODE] = acc_s;
    st[3 * MODE + 1] = acc_l;
    st[3 * MODE + 2] = acc_w;
  }
#undef DW_T
#endif
}

// One workgroup per diff entry, all over run 0's post graph g0 (in Kahn order):
//   Good = goals of g0 whose label is absent from the source run's post goals
//   D    = Fwd*(Good) ∩ Bwd*(Good)                       (:22-32, APOC export)
//   missing = D rules with a D-leaf child at maximal depth (:82-98)
template <int B>
__global__ __launch_bounds__(B) void k_diff(DevCorpus c, DiffArgs a) {
  __shared__ DiffWin W;
  __shared__ uint32_t s_red[B / 64];
  __shared__ int32_t s_max;
  const uint32_t e = blockIdx.x;
  const GraphView gv = c.view(a.g0);
  if (diff_lds_fits(c, gv)) return;  // k_diff_lds's graph
  const LabelSrc src = diff_label_src(c, a, e);
  const uint32_t V = gv.V;
  uint8_t *bits = a.bits + (size_t)e * V;     // by Kahn position
  int32_t *depth = a.depth + (size_t)e * V;   // by Kahn position
  uint8_t *mask = a.mask + (size_t)e * V;     // by node
#ifdef NEMO_STAMPS
  unsigned long long *st = c.stamps ? c.stamps + 16 * (size_t)e : nullptr, tk;
#define DK_T(slot)                      \
  do {                                  \
    TICK(tk);                           \
    if (threadIdx.x == 0 && st) st[slot] = tk; \
  } while (0)
#else
  unsigned long long *st = nullptr;
#define DK_T(slot) \
  do {             \
  } while (0)
#endif
  DK_T(9);
  if (threadIdx.x == 0) s_max = -1;
  for (uint32_t i = threadIdx.x; i < V; i += B) bits[i] = 0;
  __threadfence();
  __syncthreads();
  diff_fail_goals<B>(a, src, bits, a.r0pos);
  __threadfence();
  __syncthreads();
  DK_T(10);
  diff_window_sweep<B, 0>(V, a, bits, depth, W, s_red, st);
  diff_window_sweep<B, 1>(V, a, bits, depth, W, s_red, st);
  diff_window_sweep<B, 2>(V, a, bits, depth, W, s_red, st);
  DK_T(11);
  // D mask (by node); goal leaves of D (no D child)
  for (uint32_t i = threadIdx.x; i < V; i += B) {
    const uint8_t b = bits[i];
    mask[gv.topo[i]] = (b & DB_D) ? 1 : 0;
    if (!(b & DB_D) || (a.tinfo[i] & 1u)) continue;
    bool leaf = true;
    for (uint32_t j = a.tfp[i]; j < a.tfp[i + 1]; j++)
      if (bits[a.tfc[j]] & DB_D) leaf = false;
    if (leaf) bits[i] = b | DB_LEAF;
  }
  __threadfence();
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < V; i += B) {
    if (!(bits[i] & DB_D) || !(a.tinfo[i] & 1u)) continue;
    bool lp = false;
    for (uint32_t j = a.tfp[i]; j < a.tfp[i + 1]; j++)
      if ((bits[a.tfc[j]] & (DB_D | DB_LEAF)) == (DB_D | DB_LEAF)) lp = true;
    if (lp) {
      bits[i] |= DB_LP;
      atomicMax(&s_max, depth[i] + 1);
    }
  }
  __threadfence();
  __syncthreads();
  const int32_t mx = s_max;
  for (uint32_t i = threadIdx.x; i < V; i += B) {
    if ((bits[i] & DB_LP) && depth[i] + 1 == mx) {
      const uint32_t k = atomicAdd(a.n_missing, 1u);
      a.missing[2 * k] = e;
      a.missing[2 * k + 1] = gv.topo[i];
    }
  }
  DK_T(12);
#undef DK_T
}

// k_diff over the LDS graph tier: the same three level sweeps (Fwd*, Bwd*,
// depth) with run 0's post graph rows and the entry's node bits in LDS, so
// the dependent parent/child probes of a level are LDS round trips.
__global__ __launch_bounds__(NEMO_BLOCK) void k_diff_lds(DevCorpus c, DiffArgs a) {
  extern __shared__ __align__(16) uint8_t dyn[];
  __shared__ int32_t s_max;
  const uint32_t e = blockIdx.x, tid = threadIdx.x;
  const GraphView gv = c.view(a.g0);
  if (!diff_lds_fits(c, gv)) return;  // k_diff's graph
  const LabelSrc src = diff_label_src(c, a, e);
  const uint32_t V = gv.V, nl = gv.nlev;
  DiffLds L = diff_carve(dyn, V, gv.E, nl);
  uint8_t *mask = a.mask + (size_t)e * V;
  int32_t *depth = a.depth + (size_t)e * V;  // HBM: only D nodes touch it
  {
    const StageDesc d[4] = {{gv.rp, L.rp, V + 1, ST_U16}, {gv.fp, L.fp, V + 1, ST_U16},
                            {gv.rc, L.rc, gv.E, ST_U16},  {gv.fc, L.fc, gv.E, ST_U16}};
    stage_lds<4, NEMO_BLOCK>(d);
  }
  for (uint32_t w = tid; w < (V + 31) / 32; w += NEMO_BLOCK) L.rule[w] = 0;
  for (uint32_t v = tid; v < V; v += NEMO_BLOCK) L.bits[v] = 0;
  if (tid == 0) s_max = -1;
  __syncthreads();
  for (uint32_t base = 0; base < V; base += NEMO_BLOCK) {
    const uint32_t v = base + tid;
    const uint64_t m = __ballot(v < V && is_rule(gv.word[v]));
    if ((lane_id() & 31) == 0 && v < V) {
      const uint32_t b = (uint32_t)(m >> (lane_id() & 32));
      if (b) atomicOr(&L.rule[v >> 5], b);
    }
  }
  uint8_t *bits = L.bits;
  diff_fail_goals(a, src, bits, a.r0idx);
  __syncthreads();
#define LRULE(v) ((L.rule[(v) >> 5] >> ((v) & 31)) & 1u)
#define GOOD(v) (!LRULE(v) && !(bits[v] & DB_PRESENT))
  for (uint32_t l = 0; l < nl; l++) {
    for (uint32_t i = gv.lvl[l] + tid; i < gv.lvl[l + 1]; i += NEMO_BLOCK) {
      const uint32_t v = gv.topo[i];
      bool fw = GOOD(v);
      for (uint32_t j = L.rp[v]; j < L.rp[v + 1] && !fw; j++) fw = (bits[L.rc[j]] & DB_F) != 0;
      if (fw) bits[v] |= DB_F;
    }
    __syncthreads();
  }
  for (uint32_t l = nl; l-- > 0;) {
    for (uint32_t i = gv.lvl[l] + tid; i < gv.lvl[l + 1]; i += NEMO_BLOCK) {
      const uint32_t v = gv.topo[i];
      bool bw = GOOD(v);
      for (uint32_t j = L.fp[v]; j < L.fp[v + 1] && !bw; j++) bw = (bits[L.fc[j]] & DB_B) != 0;
      uint8_t b = bits[v];
      if (bw) b |= DB_B;
      if ((b & DB_F) && bw) b |= DB_D;
      bits[v] = b;
    }
    __syncthreads();
  }
#undef GOOD
  // longest path from a D root (Kahn-level DP restricted to D)
  for (uint32_t l = 0; l < nl; l++) {
    for (uint32_t i = gv.lvl[l] + tid; i < gv.lvl[l + 1]; i += NEMO_BLOCK) {
      const uint32_t v = gv.topo[i];
      const uint8_t b = bits[v];
      if (!(b & DB_D)) continue;
      uint32_t d = 0;
      for (uint32_t j = L.rp[v]; j < L.rp[v + 1]; j++) {
        const uint32_t p = L.rc[j];
        if (bits[p] & DB_D) d = max(d, (uint32_t)depth[p] + 1u);
      }
      depth[v] = (int32_t)d;
      if (!LRULE(v)) {
        bool leaf = true;
        for (uint32_t j = L.fp[v]; j < L.fp[v + 1]; j++)
          if (bits[L.fc[j]] & DB_D) leaf = false;
        if (leaf) bits[v] = b | DB_LEAF;
      }
    }
    __syncthreads();
  }
  for (uint32_t v = tid; v < V; v += NEMO_BLOCK) mask[v] = (bits[v] & DB_D) ? 1 : 0;
  for (uint32_t r = tid; r < V; r += NEMO_BLOCK) {
    if (!(bits[r] & DB_D) || !LRULE(r)) continue;
    bool lp = false;
    for (uint32_t j = L.fp[r]; j < L.fp[r + 1]; j++) {
      const uint32_t x = L.fc[j];
      if ((bits[x] & (DB_D | DB_LEAF)) == (DB_D | DB_LEAF)) lp = true;
    }
    if (lp) {
      bits[r] |= DB_LP;
      atomicMax(&s_max, depth[r] + 1);
    }
  }
  __syncthreads();
  const int32_t mx = s_max;
  for (uint32_t r = tid; r < V; r += NEMO_BLOCK) {
    if ((bits[r] & DB_LP) && depth[r] + 1 == mx) {
      const uint32_t k = atomicAdd(a.n_missing, 1u);
      a.missing[2 * k] = e;
      a.missing[2 * k + 1] = r;
    }
  }
#undef LRULE
}

// ---- edge pulls: which 0 = raw, 1 = simplified (graph'), 2 = diff entry ---------
__device__ __forceinline__ bool pull_alive(uint32_t which, const uint8_t *f, const uint8_t *m, uint32_t v) {
  if (which == 0) return true;
  if (which == 1) return (f[v] & (NEMO_F_KEPT | NEMO_F_DELETED)) == NEMO_F_KEPT;
  return m[v] != 0;
}

// exclusive scan of cnt[0..n) into off[0..n], one workgroup: every thread
// sums a contiguous slice (independent loads), one block scan of the slice
// sums, then each slice is written from its base
#define SCAN_BLOCK 1024
__global__ __launch_bounds__(SCAN_BLOCK) void k_scan64(const uint32_t *cnt, uint64_t *off, uint32_t n) {
  __shared__ unsigned long long s_w[SCAN_BLOCK / 64];
  const uint32_t t = threadIdx.x, lane = lane_id(), wv = t >> 6;
  const uint32_t per = (n + SCAN_BLOCK - 1) / SCAN_BLOCK;
  const uint32_t lo = min(n, t * per), hi = min(n, lo + per);
  unsigned long long sum = 0;
  for (uint32_t i = lo; i < hi; i++) sum += cnt[i];
  unsigned long long inc = sum;  // inclusive scan inside the wave
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const unsigned long long y = __shfl_up(inc, d);
    if (lane >= d) inc += y;
  }
  if (lane == 63) s_w[wv] = inc;
  __syncthreads();
  if (t == 0) {
    unsigned long long run = 0;
    for (uint32_t w = 0; w < SCAN_BLOCK / 64; w++) {
      const unsigned long long x = s_w[w];
      s_w[w] = run;
      run += x;
    }
  }
  __syncthreads();
  unsigned long long o = s_w[wv] + inc - sum;
  for (uint32_t i = lo; i < hi; i++) {
    off[i] = o;
    o += cnt[i];
  }
  if (t == SCAN_BLOCK - 1) off[n] = s_w[wv] + inc;
}

// One pass per slot (graph, or diff entry over run 0's post graph): count the
// slot's edges, claim a contiguous region with one global atomic (slots land
// in any order; each slot's edges stay in reference order), then write rows
// in node order, each row in CSR order, then collapsed edges by k
// (pred->V+k for the head's goal parents, V+k->succ for the tail's goal
// children).  A region past a.cap is not written: the host re-runs the pull
// with the capacity the cursor reports.
template <int B>
__device__ __forceinline__ void pull_slot(const DevCorpus c, const PullArgs a, const uint32_t slot) {
  __shared__ uint32_t s_lds[(B / 64)];
  __shared__ uint32_t s_cnt;
  __shared__ unsigned long long s_base;
  const uint32_t g = a.which == 2 ? a.g0 : slot;
  if (c.err[g]) {
    if (threadIdx.x == 0) {
      a.cnt[slot] = 0;
      a.off[slot] = 0;
    }
    return;
  }
  const GraphView gv = c.view(g);
  if (tier_fits(c.t_pull, gv.V, gv.E, gv.nlev)) return;  // k_pull_lds's graph or diff entry
  if (a.ccnt && gv.V >= NEMO_CSR_BIG) return;             // k_mwp_*'s graph
  const uint8_t *m = a.mask ? a.mask + (size_t)(a.mask_row ? a.mask_row[slot] : slot) * a.mask_stride : nullptr;
  const uint32_t *ch = c.chain + 5 * gv.n0;
  const uint32_t nch = a.which == 1 ? c.nch[g] : 0u;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  uint32_t n = 0;
  for (uint32_t u = threadIdx.x; u < gv.V; u += B) {
    if (!pull_alive(a.which, gv.flags, m, u)) continue;
    for (uint32_t j = gv.fp[u]; j < gv.fp[u + 1]; j++) n += pull_alive(a.which, gv.flags, m, gv.fc[j]);
  }
  for (uint32_t k = threadIdx.x; k < nch; k += B) {
    const uint32_t h = ch[5 * k], t = ch[5 * k + 1];
    for (uint32_t j = gv.rp[h]; j < gv.rp[h + 1]; j++) n += pull_alive(1, gv.flags, m, gv.rc[j]);
    for (uint32_t j = gv.fp[t]; j < gv.fp[t + 1]; j++) n += pull_alive(1, gv.flags, m, gv.fc[j]);
  }
  for (int d = 32; d >= 1; d >>= 1) n += __shfl_xor(n, d);
  if (lane_id() == 0 && n) atomicAdd(&s_cnt, n);
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long base = atomicAdd(a.cursor, (unsigned long long)s_cnt);
    s_base = base;
    a.off[slot] = base;
    a.cnt[slot] = s_cnt;
  }
  __syncthreads();
  uint64_t pos = s_base;
  if (pos + s_cnt > a.cap) return;
  for (uint32_t base = 0; base < gv.V; base += B) {
    const uint32_t u = base + threadIdx.x;
    uint32_t n = 0;
    const bool au = u < gv.V && pull_alive(a.which, gv.flags, m, u);
    if (au)
      for (uint32_t j = gv.fp[u]; j < gv.fp[u + 1]; j++) n += pull_alive(a.which, gv.flags, m, gv.fc[j]);
    uint32_t tot;
    uint64_t o = pos + block_exscan<B>(n, &tot, s_lds);
    if (au)
      for (uint32_t j = gv.fp[u]; j < gv.fp[u + 1]; j++) {
        const uint32_t v = gv.fc[j];
        if (!pull_alive(a.which, gv.flags, m, v)) continue;
        a.src[o] = u;
        a.dst[o] = v;
        o++;
      }
    pos += tot;
  }
  for (uint32_t base = 0; base < nch; base += B) {
    const uint32_t k = base + threadIdx.x;
    uint32_t n = 0, h = 0, t = 0;
    if (k < nch) {
      h = ch[5 * k];
      t = ch[5 * k + 1];
      for (uint32_t j = gv.rp[h]; j < gv.rp[h + 1]; j++) n += pull_alive(1, gv.flags, m, gv.rc[j]);
      for (uint32_t j = gv.fp[t]; j < gv.fp[t + 1]; j++) n += pull_alive(1, gv.flags, m, gv.fc[j]);
    }
    uint32_t tot;
    uint64_t o = pos + block_exscan<B>(n, &tot, s_lds);
    if (k < nch) {
      for (uint32_t j = gv.rp[h]; j < gv.rp[h + 1]; j++) {
        const uint32_t p = gv.rc[j];
        if (!pull_alive(1, gv.flags, m, p)) continue;
        a.src[o] = p;
        a.dst[o] = gv.V + k;
        o++;
      }
      for (uint32_t j = gv.fp[t]; j < gv.fp[t + 1]; j++) {
        const uint32_t q = gv.fc[j];
        if (!pull_alive(1, gv.flags, m, q)) continue;
        a.src[o] = gv.V + k;
        a.dst[o] = q;
        o++;
      }
    }
    pos += tot;
  }
}

// The same pull for big graphs (V >= NEMO_CSR_BIG), spread over MWP_CH-node
// chunks: one workgroup per graph walked ~1M rows as a latency-bound loop.
// Three kernels: each chunk counts its edges (node chunks, then chain
// chunks); one workgroup per slot scans its chunk counts into offsets and
// claims the slot's region; each chunk writes its edges from its offset in
// the same order as pull_slot (rows in node order, each row in CSR order,
// then collapsed edges by k).  Slot rows: the big-graph list (raw /
// simplified) or the diff entries.
#define MWP_CH 4096u
#define MWP_BLOCK 256
struct MwpSlot {
  uint32_t slot, g, nnc, nt;
  const uint8_t *m;
};
__device__ __forceinline__ bool mwp_slot(const DevCorpus &c, const PullArgs &a, uint32_t y, MwpSlot &s,
                                         GraphView &gv) {
  if (a.which == 2) {
    s.slot = y;
    s.g = a.g0;
  } else {
    if (y >= c.n_big) return false;
    s.g = s.slot = c.big[y];
  }
  if (c.err[s.g]) return false;
  gv = c.view(s.g);
  if (tier_fits(c.t_pull, gv.V, gv.E, gv.nlev) || gv.V < NEMO_CSR_BIG) return false;
  const uint32_t nch = a.which == 1 ? c.nch[s.g] : 0u;
  s.nnc = (gv.V + MWP_CH - 1) / MWP_CH;
  s.nt = s.nnc + (nch + MWP_CH - 1) / MWP_CH;
  s.m = a.mask ? a.mask + (size_t)(a.mask_row ? a.mask_row[s.slot] : s.slot) * a.mask_stride : nullptr;
  return true;
}
// edges of node u (raw / simplified / diff row) or of chain k (collapsed edges)
__device__ __forceinline__ uint32_t mwp_row_count(const PullArgs &a, const GraphView &gv, const uint8_t *m,
                                                  uint32_t u) {
  uint32_t n = 0;
  if (pull_alive(a.which, gv.flags, m, u))
    for (uint32_t j = gv.fp[u]; j < gv.fp[u + 1]; j++) n += pull_alive(a.which, gv.flags, m, gv.fc[j]);
  return n;
}
__device__ __forceinline__ uint32_t mwp_chain_count(const GraphView &gv, const uint8_t *m, uint32_t h, uint32_t t) {
  uint32_t n = 0;
  for (uint32_t j = gv.rp[h]; j < gv.rp[h + 1]; j++) n += pull_alive(1, gv.flags, m, gv.rc[j]);
  for (uint32_t j = gv.fp[t]; j < gv.fp[t + 1]; j++) n += pull_alive(1, gv.flags, m, gv.fc[j]);
  return n;
}
__global__ __launch_bounds__(MWP_BLOCK) void k_mwp_count(DevCorpus c, PullArgs a) {
  __shared__ uint32_t s_n;
  MwpSlot s;
  GraphView gv;
  if (!mwp_slot(c, a, blockIdx.y, s, gv) || blockIdx.x >= s.nt) return;
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  uint32_t n = 0;
  if (blockIdx.x < s.nnc) {
    const uint32_t u0 = blockIdx.x * MWP_CH, u1 = min(gv.V, u0 + MWP_CH);
    for (uint32_t u = u0 + threadIdx.x; u < u1; u += MWP_BLOCK) n += mwp_row_count(a, gv, s.m, u);
  } else {
    const uint32_t *ch = c.chain + 5 * gv.n0, nch = c.nch[s.g];
    const uint32_t k0 = (blockIdx.x - s.nnc) * MWP_CH, k1 = min(nch, k0 + MWP_CH);
    for (uint32_t k = k0 + threadIdx.x; k < k1; k += MWP_BLOCK) n += mwp_chain_count(gv, s.m, ch[5 * k], ch[5 * k + 1]);
  }
  for (int d = 32; d >= 1; d >>= 1) n += __shfl_xor(n, d);
  if (lane_id() == 0 && n) atomicAdd(&s_n, n);
  __syncthreads();
  if (threadIdx.x == 0) a.ccnt[(size_t)blockIdx.y * a.maxck + blockIdx.x] = s_n;
}
__global__ __launch_bounds__(MWP_BLOCK) void k_mwp_scan(DevCorpus c, PullArgs a) {
  __shared__ uint32_t s_lds[MWP_BLOCK / 64];
  MwpSlot s;
  GraphView gv;
  if (!mwp_slot(c, a, blockIdx.x, s, gv)) return;
  const uint32_t tot = block_scan_inplace<MWP_BLOCK>(a.ccnt + (size_t)blockIdx.x * a.maxck, s.nt, s_lds);
  if (threadIdx.x == 0) {
    a.off[s.slot] = atomicAdd(a.cursor, (unsigned long long)tot);
    a.cnt[s.slot] = tot;
  }
}
__global__ __launch_bounds__(MWP_BLOCK) void k_mwp_write(DevCorpus c, PullArgs a) {
  __shared__ uint32_t s_lds[MWP_BLOCK / 64];
  MwpSlot s;
  GraphView gv;
  if (!mwp_slot(c, a, blockIdx.y, s, gv) || blockIdx.x >= s.nt) return;
  if (a.off[s.slot] + a.cnt[s.slot] > a.cap) return;  // the host re-runs the pull with room
  uint64_t pos = a.off[s.slot] + a.ccnt[(size_t)blockIdx.y * a.maxck + blockIdx.x];
  if (blockIdx.x < s.nnc) {
    const uint32_t u0 = blockIdx.x * MWP_CH, u1 = min(gv.V, u0 + MWP_CH);
    for (uint32_t base = u0; base < u1; base += MWP_BLOCK) {
      const uint32_t u = base + threadIdx.x;
      const uint32_t n = u < u1 ? mwp_row_count(a, gv, s.m, u) : 0u;
      uint32_t tot;
      uint64_t o = pos + block_exscan<MWP_BLOCK>(n, &tot, s_lds);
      if (n)
        for (uint32_t j = gv.fp[u]; j < gv.fp[u + 1]; j++) {
          const uint32_t v = gv.fc[j];
          if (!pull_alive(a.which, gv.flags, s.m, v)) continue;
          a.src[o] = u;
          a.dst[o] = v;
          o++;
        }
      pos += tot;
    }
  } else {
    const uint32_t *ch = c.chain + 5 * gv.n0, nch = c.nch[s.g];
    const uint32_t k0 = (blockIdx.x - s.nnc) * MWP_CH, k1 = min(nch, k0 + MWP_CH);
    for (uint32_t base = k0; base < k1; base += MWP_BLOCK) {
      const uint32_t k = base + threadIdx.x;
      uint32_t h = 0, t = 0, n = 0;
      if (k < k1) {
        h = ch[5 * k];
        t = ch[5 * k + 1];
        n = mwp_chain_count(gv, s.m, h, t);
      }
      uint32_t tot;
      uint64_t o = pos + block_exscan<MWP_BLOCK>(n, &tot, s_lds);
      if (n) {
        for (uint32_t j = gv.rp[h]; j < gv.rp[h + 1]; j++) {
          const uint32_t p = gv.rc[j];
          if (!pull_alive(1, gv.flags, s.m, p)) continue;
          a.src[o] = p;
          a.dst[o] = gv.V + k;
          o++;
        }
        for (uint32_t j = gv.fp[t]; j < gv.fp[t + 1]; j++) {
          const uint32_t q = gv.fc[j];
          if (!pull_alive(1, gv.flags, s.m, q)) continue;
          a.src[o] = gv.V + k;
          a.dst[o] = q;
          o++;
        }
      }
      pos += tot;
    }
  }
}

// Raw / simplified pulls: the graphs k_pull_lds leaves (errors, past the LDS
// caps) are listed first, so k_pull runs a small grid over that list instead
// of one mostly-empty workgroup per graph (~20k early exits cost ~38 us at C3).
__global__ __launch_bounds__(NEMO_BLOCK) void k_pull_sel(DevCorpus c, uint32_t slots) {
  const uint32_t g = blockIdx.x * NEMO_BLOCK + threadIdx.x;
  bool need = false;
  if (g < slots) {
    if (c.err[g]) {
      need = true;
    } else {
      const GraphView gv = c.view(g);
      need = !tier_fits(c.t_pull, gv.V, gv.E, gv.nlev);
    }
  }
  wave_append(need, g, c.sel + 1, c.sel);
}

#define PULL_GRID 2048u
template <int B>
__global__ __launch_bounds__(B) void k_pull(DevCorpus c, PullArgs a) {
  // diff pulls: one workgroup per entry (gridDim.x == slots)
  const bool list = a.which != 2;
  const uint32_t n = list ? c.sel[0] : gridDim.x;
  for (uint32_t k = blockIdx.x; k < n; k += gridDim.x) {
    pull_slot<B>(c, a, list ? c.sel[1 + k] : k);
    __syncthreads();  // LDS of this graph is done before the next one starts
  }
}


// k_pull over the LDS graph tier (raw / simplified graphs, and the diff
// entries over run 0's graph, D mask in place of the flags): the forward rows
// and a liveness bitmap staged in LDS (the reverse rows are read from HBM for
// the chain heads only).  Thread t owns nodes k * PULL_BLOCK + t: their edge
// counts, then their in-wave output offsets, stay in registers (u16 pairs),
// and one wave scans the per-(k, wave) totals, so the output order is k_pull's.
// The image is ~2V + 2E bytes (26 KB at C3): six workgroups share a CU.
#define PULL_BLOCK 256
#define PULL_K 24  // nodes per thread: the tier's node cap is PULL_K * PULL_BLOCK
struct PullLds {
  uint16_t *fp, *fc;
  uint32_t *bits;  // node v alive = bit v (which 1: KEPT and not DELETED; which 2: D mask)
};
__device__ __forceinline__ PullLds pull_carve(void *base, uint32_t V, uint32_t E) {
  uint8_t *p = (uint8_t *)base;
  PullLds L;
  L.fp = (uint16_t *)p;
  p += lds_align(2u * (V + 1u));
  L.fc = (uint16_t *)p;
  p += lds_align(2u * E);
  L.bits = (uint32_t *)p;
  return L;
}

__global__ __launch_bounds__(PULL_BLOCK) void k_pull_lds(DevCorpus c, PullArgs a) {
  constexpr uint32_t NW = PULL_BLOCK / 64;
  static_assert(PULL_K * NW <= 128 && PULL_K % 2 == 0, "one wave scans the (k, wave) totals, two per lane");
  extern __shared__ __align__(16) uint8_t dyn[];
  __shared__ uint32_t s_lds[NW];
  __shared__ uint32_t s_pre[PULL_K * NW];
  __shared__ uint32_t s_cnt, s_nn;
  __shared__ unsigned long long s_base;
  const uint32_t which = a.which, slot = blockIdx.x, tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  const uint32_t g = which == 2 ? a.g0 : slot;
  if (c.err[g]) {  // the empty slot (k_pull, which also writes it, runs only when the host sees graphs past the tier)
    if (tid == 0) {
      a.cnt[slot] = 0;
      a.off[slot] = 0;
    }
    return;
  }
  const GraphView gv = c.view(g);
  if (!tier_fits(c.t_pull, gv.V, gv.E, gv.nlev)) return;
  const uint32_t V = gv.V;
  PullLds L = pull_carve(dyn, V, gv.E);
  if (which != 0 && V) {
    // diff pulls read the entry's D mask where the others read the flags
    const uint8_t *fsrc = which == 2 ? a.mask + (size_t)(a.mask_row ? a.mask_row[slot] : slot) * a.mask_stride : gv.flags;
    uint32_t f[PULL_K];
#pragma unroll
    for (int k = 0; k < PULL_K; k++) f[k] = fsrc[min(k * PULL_BLOCK + tid, V - 1u)];  // unconditional: one wait
#pragma unroll
    for (int k = 0; k < PULL_K; k++) {
      if (k * PULL_BLOCK >= V) break;
      const bool al = which == 1 ? (f[k] & (NEMO_F_KEPT | NEMO_F_DELETED)) == NEMO_F_KEPT : f[k] != 0u;
      const uint64_t m = __ballot(al && k * PULL_BLOCK + tid < V);
      const uint32_t n0 = k * PULL_BLOCK + 64u * w;
      if (lane == 0 && n0 < V) *reinterpret_cast<uint64_t *>(L.bits + (n0 >> 5)) = m;
    }
  }
  {
    const StageDesc d[2] = {{gv.fp, L.fp, V + 1, ST_U16}, {gv.fc, L.fc, gv.E, ST_U16}};
    stage_lds<2, PULL_BLOCK>(d);
  }
  if (tid == 0) s_cnt = 0;
  __syncthreads();
  const uint32_t *bits = L.bits;
#define ALIVE(v) (which == 0 || ((bits[(v) >> 5] >> ((v) & 31u)) & 1u))
  uint32_t cp[PULL_K / 2];  // per node k: in-wave output offset (u16 halves)
#pragma unroll
  for (int k = 0; k < PULL_K; k++) {
    if (k * PULL_BLOCK >= V) break;
    const uint32_t u = k * PULL_BLOCK + tid;
    uint32_t n = 0;
    if (u < V && ALIVE(u))
      for (uint32_t j = L.fp[u]; j < L.fp[u + 1]; j++) n += ALIVE(L.fc[j]);
    uint32_t tot;
    const uint32_t ex = wave_exscan<true>(n, &tot);
    if (lane == 0) s_pre[k * NW + w] = tot;
    if (k & 1) cp[k >> 1] |= ex << 16;
    else cp[k >> 1] = ex;
  }
  const uint32_t *ch = c.chain + 5 * gv.n0;
  const uint32_t nch = which == 1 ? c.nch[g] : 0u;
  uint32_t nc = 0;
  for (uint32_t k = tid; k < nch; k += PULL_BLOCK) {
    const uint32_t h = ch[5 * k], t = ch[5 * k + 1];
    for (uint32_t j = gv.rp[h]; j < gv.rp[h + 1]; j++) nc += ALIVE(gv.rc[j]);
    for (uint32_t j = L.fp[t]; j < L.fp[t + 1]; j++) nc += ALIVE(L.fc[j]);
  }
  for (int d = 32; d >= 1; d >>= 1) nc += __shfl_xor(nc, d);
  if (lane == 0 && nc) atomicAdd(&s_cnt, nc);
  __syncthreads();
  if (w == 0) {
    // (k, wave) totals in node order -> exclusive offsets; then the graph's region
    const uint32_t nk = ((V + PULL_BLOCK - 1) / PULL_BLOCK) * NW, i0 = 2u * lane;
    const uint32_t x0 = i0 < nk ? s_pre[i0] : 0u, x1 = i0 + 1u < nk ? s_pre[i0 + 1u] : 0u;
    uint32_t nn;
    const uint32_t ex = wave_exscan<true>(x0 + x1, &nn);
    if (i0 < nk) s_pre[i0] = ex;
    if (i0 + 1u < nk) s_pre[i0 + 1u] = ex + x0;
    if (lane == 0) {
      const uint32_t tot = nn + s_cnt;
      const unsigned long long base = atomicAdd(a.cursor, (unsigned long long)tot);
      s_base = base;
      s_nn = nn;
      a.off[slot] = base;
      a.cnt[slot] = tot;
    }
  }
  __syncthreads();
  const uint64_t base = s_base;
  const uint32_t nn = s_nn;
  if (base + nn + s_cnt > a.cap) return;
#pragma unroll
  for (int k = 0; k < PULL_K; k++) {
    if (k * PULL_BLOCK >= V) break;
    const uint32_t u = k * PULL_BLOCK + tid;
    if (u >= V || !ALIVE(u)) continue;
    uint64_t o = base + s_pre[k * NW + w] + ((cp[k >> 1] >> (16 * (k & 1))) & 0xFFFFu);
    for (uint32_t j = L.fp[u]; j < L.fp[u + 1]; j++) {
      const uint32_t v = L.fc[j];
      if (!ALIVE(v)) continue;
      a.src[o] = u;
      a.dst[o] = v;
      o++;
    }
  }
  uint64_t pos = base + nn;
  for (uint32_t kb = 0; kb < nch; kb += PULL_BLOCK) {
    const uint32_t k = kb + tid;
    uint32_t n = 0, h = 0, t = 0;
    if (k < nch) {
      h = ch[5 * k];
      t = ch[5 * k + 1];
      for (uint32_t j = gv.rp[h]; j < gv.rp[h + 1]; j++) n += ALIVE(gv.rc[j]);
      for (uint32_t j = L.fp[t]; j < L.fp[t + 1]; j++) n += ALIVE(L.fc[j]);
    }
    uint32_t tot;
    uint64_t o = pos + block_exscan<PULL_BLOCK, true>(n, &tot, s_lds);
    if (k < nch) {
      for (uint32_t j = gv.rp[h]; j < gv.rp[h + 1]; j++) {
        const uint32_t p = gv.rc[j];
        if (!ALIVE(p)) continue;
        a.src[o] = p;
        a.dst[o] = V + k;
        o++;
      }
      for (uint32_t j = L.fp[t]; j < L.fp[t + 1]; j++) {
        const uint32_t q = L.fc[j];
        if (!ALIVE(q)) continue;
        a.src[o] = V + k;
        a.dst[o] = q;
        o++;
      }
    }
    pos += tot;
  }
#undef ALIVE
}

// Raw pulls (which 0) over the LDS graph tier: every edge survives, so a graph's
// region is its forward CSR verbatim (CSR edge j -> base + j): no staging, no
// counts, no LDS, so the CU holds as many workgroups as registers allow.
#define PULLR_BATCH 8
__global__ __launch_bounds__(PULL_BLOCK) void k_pull_raw(DevCorpus c, PullArgs a) {
  __shared__ unsigned long long s_base;
  const uint32_t g = blockIdx.x, tid = threadIdx.x;
  if (c.err[g]) {
    if (tid == 0) {
      a.cnt[g] = 0;
      a.off[g] = 0;
    }
    return;
  }
  const GraphView gv = c.view(g);
  if (!tier_fits(c.t_pull, gv.V, gv.E, gv.nlev)) return;
  const uint32_t V = gv.V, E = gv.E;
  if (tid == 0) {
    const unsigned long long base = atomicAdd(a.cursor, (unsigned long long)E);
    s_base = base;
    a.off[g] = base;
    a.cnt[g] = E;
  }
  __syncthreads();
  const uint64_t base = s_base;
  if (base + E > a.cap) return;
  uint32_t *src = a.src + base, *dst = a.dst + base;
  for (uint32_t j0 = 0; j0 < E; j0 += PULLR_BATCH * PULL_BLOCK) {
    uint32_t y[PULLR_BATCH];
#pragma unroll
    for (int q = 0; q < PULLR_BATCH; q++) y[q] = gv.fc[min(j0 + q * PULL_BLOCK + tid, E - 1u)];
#pragma unroll
    for (int q = 0; q < PULLR_BATCH; q++)
      if (j0 + q * PULL_BLOCK + tid < E) dst[j0 + q * PULL_BLOCK + tid] = y[q];
  }
  for (uint32_t u0 = 0; u0 < V; u0 += PULLR_BATCH * PULL_BLOCK) {
    uint32_t lo[PULLR_BATCH], hi[PULLR_BATCH];
#pragma unroll
    for (int q = 0; q < PULLR_BATCH; q++) {
      const uint32_t u = min(u0 + q * PULL_BLOCK + tid, V - 1u);
      lo[q] = gv.fp[u];
      hi[q] = gv.fp[u + 1];
    }
#pragma unroll
    for (int q = 0; q < PULLR_BATCH; q++) {
      const uint32_t u = u0 + q * PULL_BLOCK + tid;
      if (u < V)
        for (uint32_t j = lo[q]; j < hi[q]; j++) src[j] = u;
    }
  }
}

// ---- small-result hand-over -------------------------------------------------------
// Copies device results straight into pinned host memory with a kernel: the
// stores cross PCIe from the CUs, so these small copies never queue behind
// the bulk staging transfers.
__global__ __launch_bounds__(NEMO_BLOCK) void k_to_host(uint8_t *__restrict__ dst, const uint8_t *__restrict__ src,
                                                         uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * NEMO_BLOCK;
  const uint64_t t = (uint64_t)blockIdx.x * NEMO_BLOCK + threadIdx.x;
  if ((((uintptr_t)dst | (uintptr_t)src) & 15u) == 0) {
    const uint64_t n16 = n >> 4;
    for (uint64_t i = t; i < n16; i += stride) ((uint4 *)dst)[i] = ((const uint4 *)src)[i];
    for (uint64_t i = (n16 << 4) + t; i < n; i += stride) dst[i] = src[i];
  } else {
    for (uint64_t i = t; i < n; i += stride) dst[i] = src[i];
  }
}

// Several small copies in one launch (blockIdx.y = segment): each launch on the
// analysis stream costs a dispatch and a wait of its own.
__global__ __launch_bounds__(NEMO_BLOCK) void k_to_host_multi(HostCopies h) {
  const HostCopy &g = h.seg[blockIdx.y];
  uint8_t *__restrict__ dst = g.dst;
  const uint8_t *__restrict__ src = g.src;
  const uint64_t n = g.n, stride = (uint64_t)gridDim.x * NEMO_BLOCK;
  const uint64_t t = (uint64_t)blockIdx.x * NEMO_BLOCK + threadIdx.x;
  if ((((uintptr_t)dst | (uintptr_t)src) & 15u) == 0) {
    const uint64_t n16 = n >> 4;
    for (uint64_t i = t; i < n16; i += stride) ((uint4 *)dst)[i] = ((const uint4 *)src)[i];
    for (uint64_t i = (n16 << 4) + t; i < n; i += stride) dst[i] = src[i];
  } else {
    for (uint64_t i = t; i < n; i += stride) dst[i] = src[i];
  }
}

// PCIe-bound copies: a few dozen workgroups keep the link busy (each lane's 16-byte store to
// host memory is microseconds in flight); a 1024-block grid of them held every CU's wave slots
// for the ~100 us of the reference-mode D-mask copy, and the analysis stream's next kernel
// (k_chains) could not start beside it
#define TO_HOST_BLOCKS 64u
void launch_to_host_multi(const HostCopies &h, hipStream_t s) {
  uint64_t blocks = 1;
  for (uint32_t k = 0; k < h.n; k++)
    blocks = std::max<uint64_t>(blocks, (h.seg[k].n + 16ull * NEMO_BLOCK - 1) / (16ull * NEMO_BLOCK));
  if (!h.n) return;
  if (blocks > TO_HOST_BLOCKS) blocks = TO_HOST_BLOCKS;
  hipLaunchKernelGGL(k_to_host_multi, dim3((uint32_t)blocks, h.n), dim3(NEMO_BLOCK), 0, s, h);
}

void launch_to_host(void *dst, const void *src, uint64_t bytes, hipStream_t s, uint32_t max_blocks) {
  if (!bytes) return;
  uint64_t blocks = (bytes + 16ull * NEMO_BLOCK - 1) / (16ull * NEMO_BLOCK);
  if (blocks > max_blocks) blocks = max_blocks;
  hipLaunchKernelGGL(k_to_host, dim3((uint32_t)blocks), dim3(NEMO_BLOCK), 0, s, (uint8_t *)dst, (const uint8_t *)src,
                     bytes);
}

// Device memset as a kernel: rocclr's fill blits queue behind a bulk copy
// blit running on the copy stream, so the per-step clears on the analysis
// stream are plain vector stores instead.
__global__ __launch_bounds__(NEMO_BLOCK) void k_zero(uint32_t *__restrict__ dst, uint64_t words) {
  const uint64_t stride = (uint64_t)gridDim.x * NEMO_BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * NEMO_BLOCK + threadIdx.x; i < words; i += stride) dst[i] = 0u;
}

void launch_zero(void *dst, uint64_t bytes, hipStream_t s) {
  const uint64_t words = bytes / 4;  // callers clear whole u32 / u64 arrays
  if (!words) return;
  uint64_t blocks = (words + NEMO_BLOCK - 1) / NEMO_BLOCK;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(k_zero, dim3((uint32_t)blocks), dim3(NEMO_BLOCK), 0, s, (uint32_t *)dst, words);
}

// ---- run-0 trigger patterns ------------------------------------------------------
// phase 0 counts, phase 1 writes (capacities sized from the counts).
#define TRIG_SPLIT 16
__global__ __launch_bounds__(NEMO_BLOCK) void k_triggers(DevCorpus c, TrigArgs a, int phase) {
  const GraphView gp = c.view(a.g_pre), gq = c.view(a.g_post);
  // TRIG_SPLIT workgroups per pattern, nodes strided over them (row order is free)
  const uint32_t pat = blockIdx.x % 3, x0 = (blockIdx.x / 3) * NEMO_BLOCK + threadIdx.x;
  const uint32_t step = (gridDim.x / 3) * NEMO_BLOCK;
#define HOLDS(gg, v) (((gg).flags[v] & NEMO_F_HOLDS) != 0)
  if (pat == 0) {
    // findPreTriggers (corrections.go:30-34): (a:Rule)->(g:Goal{holds:false})->(r:Rule), (h{holds})->(a)
    for (uint32_t x = x0; x < gp.V; x += step) {
      if (is_rule(gp.word[x]) || HOLDS(gp, x)) continue;
      for (uint32_t j = gp.rp[x]; j < gp.rp[x + 1]; j++) {
        const uint32_t ar = gp.rc[j];
        bool hp = false;
        for (uint32_t i = gp.rp[ar]; i < gp.rp[ar + 1]; i++) hp |= HOLDS(gp, gp.rc[i]);
        if (!hp) continue;
        const uint32_t n = gp.outdeg(x);
        if (!n) continue;
        const uint32_t k = atomicAdd(&a.counts[0], n);
        if (phase == 1)
          for (uint32_t i = 0; i < n; i++) {
            a.pre[3 * (k + i)] = ar;
            a.pre[3 * (k + i) + 1] = x;
            a.pre[3 * (k + i) + 2] = gp.fc[gp.fp[x] + i];
          }
      }
    }
  } else if (pat == 1) {
    // findPostTriggers (corrections.go:121-125)
    for (uint32_t x = x0; x < gq.V; x += step) {
      if (is_rule(gq.word[x]) || !HOLDS(gq, x) || gq.indeg(x) == 0) continue;
      for (uint32_t j = gq.fp[x]; j < gq.fp[x + 1]; j++) {
        const uint32_t r = gq.fc[j];
        bool ok = false;
        for (uint32_t i = gq.fp[r]; i < gq.fp[r + 1]; i++) {
          const uint32_t y = gq.fc[i];
          ok |= !HOLDS(gq, y) && gq.outdeg(y) > 0;
        }
        if (!ok) continue;
        const uint32_t k = atomicAdd(&a.counts[1], 1u);
        if (phase == 1) {
          a.post[2 * k] = x;
          a.post[2 * k + 1] = r;
        }
      }
    }
  } else {
    // GenerateExtensions' async rules (extensions.go:63-67)
    for (uint32_t r = x0; r < gp.V; r += step) {
      const uint32_t w = gp.word[r];
      if (!is_rule(w) || type_of(w) != NEMO_TYPE_ASYNC) continue;
      bool hp = false, np = false, down = false;
      for (uint32_t j = gp.rp[r]; j < gp.rp[r + 1]; j++) {
        if (HOLDS(gp, gp.rc[j])) hp = true;
        else np = true;
      }
      for (uint32_t j = gp.fp[r]; j < gp.fp[r + 1]; j++) {
        const uint32_t y = gp.fc[j];
        down |= !HOLDS(gp, y) && gp.outdeg(y) > 0;
      }
      if ((hp && down) || np) {
        const uint32_t k = atomicAdd(&a.counts[2], 1u);
        if (phase == 1) a.async_rules[k] = r;
      }
    }
  }
#undef HOLDS
}

// gather every graph's sorted chains into one array (graph, k, head, tail, len)
__global__ __launch_bounds__(NEMO_BLOCK) void k_chain_gather(DevCorpus c, const uint64_t *off, uint32_t *out) {
  const uint32_t g = blockIdx.x;
  const uint32_t n = c.nch[g];
  const uint32_t *ch = c.chain + 5 * c.node_off[g];
  uint32_t *o = out + 5 * off[g];
  for (uint32_t k = threadIdx.x; k < n; k += NEMO_BLOCK) {
    o[5 * k] = g;
    o[5 * k + 1] = k;
    o[5 * k + 2] = ch[5 * k];
    o[5 * k + 3] = ch[5 * k + 1];
    o[5 * k + 4] = ch[5 * k + 2];
  }
}

// Dense (head, tail) pairs of every graph's accepted chains, graph g's chain k
// at off[g] + k: with the node flags this is the whole simplified graph
// (preprocessing.go:249-340 materialises exactly head.preds -> c -> tail.succs).
// Pairs are (head, tail) u32 when `wide`, else packed head | tail << 16 (every
// graph under 65536 nodes), halving the hand-over.
__global__ __launch_bounds__(NEMO_BLOCK) void k_chain_pairs(DevCorpus c, const uint64_t *off, uint32_t *out,
                                                             uint64_t cap, int wide) {
  const uint32_t g = blockIdx.x;
  const uint32_t n = c.nch[g];
  if (off[g] + n > cap) return;  // the host re-stages with the capacity off[G] asks for
  const uint32_t *ch = c.chain + 5 * c.node_off[g];
  if (wide) {
    uint2 *o = reinterpret_cast<uint2 *>(out) + off[g];
    for (uint32_t k = threadIdx.x; k < n; k += NEMO_BLOCK) o[k] = make_uint2(ch[5 * k], ch[5 * k + 1]);
  } else {
    uint32_t *o = out + off[g];
    for (uint32_t k = threadIdx.x; k < n; k += NEMO_BLOCK) o[k] = ch[5 * k] | (ch[5 * k + 1] << 16);
  }
}

void launch_chain_pairs(const DevCorpus &c, const uint64_t *off, uint32_t *out, uint64_t cap, int wide,
                        hipStream_t s) {
  hipLaunchKernelGGL(k_chain_pairs, dim3(c.G), dim3(NEMO_BLOCK), 0, s, c, off, out, cap, wide);
}

// Node state for the host, 2 bits per node (4 per byte, node v at byte v/4):
// bit 0 = the node survives into the simplified graph (KEPT, not DELETED),
// bit 1 = condition_holds.  One thread packs 16 nodes into a u32.
__global__ __launch_bounds__(NEMO_BLOCK) void k_pack_state(const uint8_t *__restrict__ flags, uint32_t *out,
                                                            uint64_t V) {
  const uint64_t w = (uint64_t)blockIdx.x * NEMO_BLOCK + threadIdx.x;
  if (16 * w >= V) return;
  uint8_t f[16];
  if (16 * w + 16 <= V) {
    *reinterpret_cast<uint4 *>(f) = reinterpret_cast<const uint4 *>(flags)[w];
  } else {
    for (int b = 0; b < 16; b++) f[b] = 16 * w + b < V ? flags[16 * w + b] : (uint8_t)0;
  }
  uint32_t x = 0;
#pragma unroll
  for (int b = 0; b < 16; b++) {
    const uint32_t alive = (f[b] & (NEMO_F_KEPT | NEMO_F_DELETED)) == NEMO_F_KEPT;
    const uint32_t holds = (f[b] & NEMO_F_HOLDS) != 0;
    x |= (alive | (holds << 1)) << (2 * b);
  }
  out[w] = x;
}

void launch_pack_state(const uint8_t *flags, uint32_t *out, uint64_t V, hipStream_t s) {
  const uint64_t words = (V + 15) / 16;
  if (!words) return;
  hipLaunchKernelGGL(k_pack_state, dim3((uint32_t)((words + NEMO_BLOCK - 1) / NEMO_BLOCK)), dim3(NEMO_BLOCK), 0, s,
                     flags, out, V);
}

void launch_chain_gather(const DevCorpus &c, uint64_t *off, uint32_t *out, hipStream_t s) {
  hipLaunchKernelGGL(k_scan64, dim3(1), dim3(SCAN_BLOCK), 0, s, c.nch, off, c.G);
  if (out) hipLaunchKernelGGL(k_chain_gather, dim3(c.G), dim3(NEMO_BLOCK), 0, s, c, off, out);
}

void launch_diff(const DevCorpus &c, const DiffArgs &a, uint32_t n_entries, uint32_t V0, hipStream_t s) {
  if (V0) {  // g0 in Kahn order for the global tier (each kernel returns at once for an LDS-tier g0)
    const uint32_t nb = (std::max(V0, a.n_r0lab) + NEMO_BLOCK - 1) / NEMO_BLOCK;
    hipLaunchKernelGGL(k_dprep_a, dim3(nb), dim3(NEMO_BLOCK), 0, s, c, a);
    hipLaunchKernelGGL(k_dprep_scan, dim3(1), dim3(1024), 0, s, c, a);
    hipLaunchKernelGGL(k_dprep_b, dim3(nb), dim3(NEMO_BLOCK), 0, s, c, a);
  }
  if (c.t_diff.bytes) {
    const uint32_t bytes = c.t_diff.bytes;
    hipFuncSetAttribute((const void *)k_diff_lds, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    hipLaunchKernelGGL(k_diff_lds, dim3(n_entries), dim3(NEMO_BLOCK), bytes, s, c, a);
  }
  if (c.gblock == 1024)
    hipLaunchKernelGGL(k_diff<1024>, dim3(n_entries), dim3(1024), 0, s, c, a);
  else
    hipLaunchKernelGGL(k_diff<NEMO_BLOCK>, dim3(n_entries), dim3(NEMO_BLOCK), 0, s, c, a);
}
// entries sharing a label source: copy the shared mask to each entry's row, 16 B per lane
__global__ __launch_bounds__(NEMO_BLOCK) void k_diff_expand(uint8_t *__restrict__ mask, const uint8_t *__restrict__ umask,
                                                         const uint32_t *__restrict__ map, uint64_t V0) {
  const uint32_t e = blockIdx.y;
  const uint8_t *src = umask + (uint64_t)map[e] * V0;
  uint8_t *dst = mask + (uint64_t)e * V0;
  for (uint64_t i = blockIdx.x * (uint64_t)NEMO_BLOCK + threadIdx.x; i < V0; i += (uint64_t)gridDim.x * NEMO_BLOCK)
    dst[i] = src[i];
}
void launch_diff_expand(uint8_t *mask, const uint8_t *umask, const uint32_t *map, uint64_t V0, uint32_t n_entries,
                        hipStream_t s) {
  if (!V0 || !n_entries) return;
  const uint32_t gx = (uint32_t)std::min<uint64_t>(64, (V0 + NEMO_BLOCK - 1) / NEMO_BLOCK);
  hipLaunchKernelGGL(k_diff_expand, dim3(gx, n_entries), dim3(NEMO_BLOCK), 0, s, mask, umask, map, V0);
}
void launch_pull(const DevCorpus &c, const PullArgs &a, uint32_t slots, uint32_t rest, hipStream_t s) {
  if (c.t_pull.bytes && slots && a.which == 0) {
    hipLaunchKernelGGL(k_pull_raw, dim3(slots), dim3(PULL_BLOCK), 0, s, c, a);
  } else if (c.t_pull.bytes && slots) {
    const uint32_t bytes = c.t_pull.bytes;
    hipFuncSetAttribute((const void *)k_pull_lds, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    hipLaunchKernelGGL(k_pull_lds, dim3(slots), dim3(PULL_BLOCK), bytes, s, c, a);
  }
  // k_pull's selection and grid only when the host counted graphs past the LDS
  // tier (`rest`; errors write their empty slots in the LDS kernels too)
  const bool global = !c.t_pull.bytes || rest;
  uint32_t grid = slots;
  if (!slots) return;
  if (!global) {
  } else if (a.which != 2) {
    launch_zero(c.sel, sizeof(uint32_t), s);
    hipLaunchKernelGGL(k_pull_sel, dim3((slots + NEMO_BLOCK - 1) / NEMO_BLOCK), dim3(NEMO_BLOCK), 0, s, c, slots);
    grid = std::min(slots, PULL_GRID);
  }
  if (global) {
    if (c.gblock == 1024)
      hipLaunchKernelGGL(k_pull<1024>, dim3(grid), dim3(1024), 0, s, c, a);
    else
      hipLaunchKernelGGL(k_pull<NEMO_BLOCK>, dim3(grid), dim3(NEMO_BLOCK), 0, s, c, a);
  }
  if (!a.ccnt) return;
  const uint32_t rows = a.which == 2 ? slots : c.n_big;
  if (!rows) return;
  hipLaunchKernelGGL(k_mwp_count, dim3(a.maxck, rows), dim3(MWP_BLOCK), 0, s, c, a);
  hipLaunchKernelGGL(k_mwp_scan, dim3(rows), dim3(MWP_BLOCK), 0, s, c, a);
  hipLaunchKernelGGL(k_mwp_write, dim3(a.maxck, rows), dim3(MWP_BLOCK), 0, s, c, a);
}
// failGoals' label set of one graph (differential-provenance.go:23-24) into
// device memory as [n, label...]: the hand-over a sharded reference-mode
// diff broadcasts from the shard owning failedRuns[0].  Order is irrelevant
// (the set only gates run 0's goals), duplicates are harmless.
__global__ __launch_bounds__(NEMO_BLOCK) void k_goal_labels(DevCorpus c, uint32_t g, uint32_t *out) {
  const GraphView gv = c.view(g);
  for (uint32_t base = blockIdx.x * NEMO_BLOCK; base < gv.V; base += gridDim.x * NEMO_BLOCK) {
    const uint32_t v = base + threadIdx.x;
    const bool goal = v < gv.V && !is_rule(gv.word[v]);
    wave_append(goal, goal ? gv.label[v] : 0u, out + 1, out);
  }
}
void launch_goal_labels(const DevCorpus &c, uint32_t g, uint32_t *out, hipStream_t s) {
  launch_zero(out, sizeof(uint32_t), s);
  hipLaunchKernelGGL(k_goal_labels, dim3(256), dim3(NEMO_BLOCK), 0, s, c, g, out);
}

void launch_triggers(const DevCorpus &c, const TrigArgs &a, int phase, hipStream_t s) {
  hipLaunchKernelGGL(k_triggers, dim3(3 * TRIG_SPLIT), dim3(NEMO_BLOCK), 0, s, c, a, phase);
}

}  // namespace nemo
