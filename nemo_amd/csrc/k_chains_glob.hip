// k_chains_glob.hip — collapseNextChains' greedy chain cover
// (graphing/preprocessing.go:70-138) for deep graphs: the closed form of
// k_chains (accepted paths = {first(v) : v in H*}, acceptance order = length
// desc then the preorder of the representatives in the best-prefix forest)
// with every per-node array in a global scratch region, so it scales to
// chain subgraphs of hundreds of thousands of nodes and thousands of levels
// (1M-node graphs, EOT ~ 2000).  One 256- or 512-thread
// workgroup per graph; the chain tails come out of the down sweep, the chain
// heads and ancestor sums out of one top-down pass over the up-levels, the
// final order a stable counting sort of the preorder-ordered chains by
// length.  The graphs are the
// ones the host gave a scratch region (DevCorpus::gs_off, V >= glob_min_v);
// k_chains and k_chains_big skip them.
#include <algorithm>

#include "device.h"
#include "internal.h"

namespace nemo {

// One workgroup per deep graph of GB threads (256 or 512, the kernel's
// template argument) and ~37 KB of LDS, so that two to four share a CU: each
// graph's level walks are latency chains run by one wave, so a CU makes
// progress on several graphs at once (a 1024-thread, 146 KB workgroup held a
// whole CU for one graph).
#define GA_B 4   // row entries loaded together while building the H* adjacency (a long row's tail)
#define GA_N 4   // H* nodes per thread per round of the adjacency
#define GA_F 6   // ... and the first entries of each of their rows
#ifndef GA_BM
#define GA_BM 1  // membership tested in the rank bitmap first (identity ranks; C5 k_chains 230.6 -> 226.7 ms)
#endif
#define GU 8     // elements per thread per round of the HBM passes (pointer jumping, bucketing)
#define CP 16    // Kahn positions per thread per round of the H* compaction
#define GNIL 0xFFFFFFFFu

// Scratch layout (u32 units) for a graph of V nodes and E edges.  The
// preorder's buffers (va, vb, pa, pb) reuse the pointer-jumping buffers
// (ha, hb, ta, tb): the heads and tails are read for the last time when the
// representatives are recorded, before the preorder starts.  The
// representatives themselves (5 words each, at most V) go where the H*
// adjacency was (child, par: dead once the prefix ranks are done), padded to
// 5V words when 2E is less.
struct GlobScratch {
  uint32_t *bm, *bmpre, *crank, *rule;
  uint32_t *ccoff, *pcoff, *child, *par;
  uint32_t *cend, *pend;        // row ends (rows are laid out by full degree; ha / hb until the pointer jumping)
  int32_t *up, *down;
  uint32_t *nxt, *bp, *po, *fpos, *ub, *uoff, *cnt, *grp;
  uint32_t *ha, *hb, *ta, *tb;  // pointer-jumping buffers (heads, tails)
  uint32_t *S, *A, *va, *vb, *pa, *pb;
  uint32_t *tmp;                // [5 * V] representatives (over child / par)
  uint32_t *meta;               // [16]: [0] H* node count written by k_glob_prep
  unsigned long long *key;      // up to 2V keys (power-of-two padded chain count)
};

uint64_t glob_words(uint64_t V, uint64_t E) {
  const uint64_t w = (V + 31) / 32 + 2;
  const uint64_t adj = std::max<uint64_t>(2 * E, 5 * V);  // child + par, or the representatives
  return 2 * w + 2 * (V + 1) + adj + 2 * (V + 2) + 16 * V + 4 * V + 16 + 64;
}

__device__ inline GlobScratch glob_carve(uint32_t *p, uint32_t V, uint32_t E) {
  GlobScratch s;
  const uint32_t w = (V + 31) / 32 + 2;
  auto take = [&](uint64_t n) {
    uint32_t *q = p;
    p += n;
    return q;
  };
  s.bm = take(w);
  s.bmpre = take(w);
  s.crank = take(V);
  s.rule = take(V);
  s.ccoff = take(V + 1);
  s.pcoff = take(V + 1);
  s.child = take(E);
  s.par = take(E);
  s.tmp = s.child;
  if (5ull * V > 2ull * E) take(5ull * V - 2ull * E);
  s.up = (int32_t *)take(V);
  s.down = (int32_t *)take(V);
  s.nxt = take(V);
  s.bp = take(V);
  s.po = take(V);
  s.fpos = take(V);
  s.ub = take(V);
  s.uoff = take(V + 2);
  s.cnt = take(V + 2);
  s.grp = take(V);
  s.ha = take(V);
  s.hb = take(V);
  s.ta = take(V);
  s.tb = take(V);
  s.S = take(V);
  s.A = take(V);
  s.cend = s.ha;
  s.pend = s.hb;
  s.va = s.ha;
  s.vb = s.hb;
  s.pa = s.ta;
  s.pb = s.tb;
  s.meta = take(16);
  p = (uint32_t *)(((uintptr_t)p + 7) & ~(uintptr_t)7);
  s.key = (unsigned long long *)p;
  return s;
}

#define GS_RING 2048u  // values kept in LDS (power of two)
#define GS_WN 512u     // nodes per window
#define GS_E 1024u     // extra in-ring links per window (past the packed ones)
struct GSweepLds {
  int32_t rv[GS_RING];   // up / down by ring slot (index & (GS_RING - 1))
  uint32_t rc[GS_RING];  // down: crank by ring slot
  int32_t init[GS_WN];   // up: value over the parents outside the ring; down: best such child's down
  uint32_t ibc[GS_WN], ibr[GS_WN];  // down: that child and its crank; ibc then nxt
  uint32_t rt[GS_RING];  // down: tail (end of the nxt chain) by ring slot
  uint32_t ibt[GS_WN];   // down: the staged far best child's tail
  uint32_t lev[GS_WN];   // Kahn level
  uint64_t lk[GS_WN][2]; // first GS_KEEP in-ring links (u16 offsets from the ring base)
  uint16_t aoff[GS_WN], acnt[GS_WN];  // GS_MORE: link t in [GS_KEEP, acnt) at adj[aoff + t - GS_KEEP]
  uint16_t adj[GS_E];    // extra in-ring links
  uint8_t flg[GS_WN];    // bit 0 rule, GS_MORE, GS_SPILL
};

// four consecutive entries [i, i + 4) of an HBM array (one 16-byte load when
// all four exist, `fill` past n)
template <typename T>
__device__ __forceinline__ void ld4(const T *p, uint32_t i, uint32_t n, T *o, T fill) {
  if (i + 3 < n) {
    __builtin_memcpy(o, p + i, 16);
  } else {
#pragma unroll
    for (int b = 0; b < 4; b++) o[b] = i + b < n ? p[i + b] : fill;
  }
}

template <int GB>
__device__ __forceinline__ uint32_t gmax_u32(uint32_t v, uint32_t *lds) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, d));
  if (lane_id() == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t m = 0;
  for (int i = 0; i < GB / 64; i++) m = max(m, lds[i]);
  __syncthreads();
  return m;
}


// up / down of the chain subgraph H* as windowed sweeps.  The compact index
// orders H* by Kahn level, so a node's H* parents have smaller indices and its
// children larger ones.  Deep graphs have ~20k levels of a few dozen H* nodes:
// a level-synchronous sweep over HBM scratch pays a chain of dependent HBM
// round trips and a 16-wave barrier per level.  Here the index range is cut
// into GS_WN-node windows; the whole workgroup stages a window (coalesced):
// links that leave the ring of the last GS_RING values are resolved from HBM
// (their values are final), the others become an LDS adjacency list of ring
// offsets.  Then ONE wave walks the window's levels with every value in LDS:
// a level costs a few LDS round trips and no barrier (a wave's LDS operations
// complete in order).  A window whose in-ring links overflow GS_E leaves its
// last nodes' rows in HBM (re-read in the sweep).
//   up   (forward):  up(i)   = max(rule ? 0 : -1, up(p) + 1 over H* parents p)
//   down (backward): the child w of greatest (down(w), -crank(w)); down(i) =
//                    down(w) + 1, or rule ? 0 : -1 without children; nxt(i) = w
#define GS_MORE 0x2u   // more than GS_KEEP in-ring links: the rest in the window's list
#define GS_SPILL 0x4u  // ... or, past the list's capacity, in HBM
#define GS_KEEP 8      // in-ring links packed per node (u16 each, GS_NOLINK = none)
#ifndef GS_SB
#define GS_SB 4        // row entries per row and step while staging a window
#endif
#define GS_NOLINK 0xFFFFu
#define GS_RW 8        // row entries per load round when a node's extra in-ring links are listed
#ifndef GS_PF
#define GS_PF 1        // next window's per-node staging data loaded during this window's sweep
#endif
template <bool UP, int GB>
__device__ __forceinline__ void glob_sweep(GlobScratch &S, const uint32_t n, const uint32_t *hs, const uint32_t *nlv,
                                           uint32_t *s_fail, GSweepLds &L, uint32_t *s_red, unsigned long long *st) {
#ifdef NEMO_STAMPS
  unsigned long long acc_s = 0, acc_w = 0, t_a = 0, t_b = 0, iters = 0, spills = 0;
#endif
  constexpr uint32_t M = GS_RING - 1u;
  constexpr uint32_t PT = GS_WN / GB;  // window nodes per thread
  const uint32_t tid = threadIdx.x, lane = lane_id();
  const uint32_t *off = UP ? S.pcoff : S.ccoff, *oend = UP ? S.pend : S.cend, *col = UP ? S.par : S.child;
  const uint32_t nwin = (n + GS_WN - 1) / GS_WN;
  auto win = [&](uint32_t wi, uint32_t &w0, uint32_t &w1) {
    w0 = UP ? wi * GS_WN : (n > (wi + 1) * GS_WN ? n - (wi + 1) * GS_WN : 0u);
    w1 = UP ? min(n, w0 + GS_WN) : n - wi * GS_WN;
  };
  // a window's per-node data (row bounds, rule flag, node, crank) does not
  // depend on the sweep, so the next window's is loaded before this window's
  // sweep starts (GS_PF): wave 0 sweeps while those loads are in flight
  uint32_t pr0[PT], pr1[PT], prl[PT], phs[PT], pcr[PT];
  auto prefetch = [&](uint32_t wi) {
    uint32_t a, b;
    win(wi, a, b);
#pragma unroll
    for (int q = 0; q < PT; q++) {
      const uint32_t k = tid + q * GB, i = a + k;
      const bool in = wi < nwin && k < b - a;
      pr0[q] = in ? off[i] : 0u;
      pr1[q] = in ? oend[i] : 0u;
      prl[q] = in ? S.rule[i] : 0u;
      phs[q] = in ? hs[i] : 0u;
      pcr[q] = in && !UP ? S.crank[i] : 0u;
    }
  };
  if (GS_PF) prefetch(0);
  for (uint32_t wi = 0; wi < nwin; wi++) {
    uint32_t w0, w1;
    win(wi, w0, w1);
    const uint32_t nw = w1 - w0;
    // ring = [base, base + GS_RING) around the window; link offsets relative to base
    const uint32_t base = UP ? (w1 > GS_RING ? w1 - GS_RING : 0u) : w0;
#ifdef NEMO_STAMPS
    TICK(t_a);
#endif
    // ---- stage (whole workgroup): node k = tid + q * GB ----
    uint32_t r0[PT], r1[PT], cnt[PT], keep[PT][GS_KEEP];
#pragma unroll
    for (int q = 0; q < PT; q++) {
      const uint32_t k = tid + q * GB, i = w0 + k;
      const bool in = k < nw;
      r0[q] = GS_PF ? pr0[q] : (in ? off[i] : 0u);
      r1[q] = GS_PF ? pr1[q] : (in ? oend[i] : 0u);
      cnt[q] = 0;
    }
    // the PT rows walked together, GS_SB entries of each per step: every load of
    // a step (columns, then the far values) in flight at once
    uint32_t rl[PT], lv[PT], cr[PT];
    int32_t dd[PT];
    uint32_t bc[PT], br[PT], bt[PT];
#pragma unroll
    for (int q = 0; q < PT; q++) {
      const uint32_t k = tid + q * GB, i = w0 + k;
      const bool in = k < nw;
      rl[q] = GS_PF ? prl[q] : (in ? S.rule[i] : 0u);
      lv[q] = in ? nlv[GS_PF ? phs[q] : hs[i]] : 0u;
      cr[q] = GS_PF ? pcr[q] : (in && !UP ? S.crank[i] : 0u);
      dd[q] = UP ? (rl[q] ? 0 : -1) : -1;
      bc[q] = br[q] = bt[q] = GNIL;
    }
    bool more = false;
#pragma unroll
    for (int q = 0; q < PT; q++) more |= r0[q] < r1[q];
    for (uint32_t t = 0; more; t += GS_SB) {
      uint32_t p[PT][GS_SB];
      bool far[PT][GS_SB];
#pragma unroll
      for (int q = 0; q < PT; q++)
#pragma unroll
        for (int h = 0; h < GS_SB; h++) p[q][h] = r0[q] + t + h < r1[q] ? col[r0[q] + t + h] : GNIL;
      int32_t fv[PT][GS_SB];
      uint32_t fr[PT][GS_SB], ft[PT][GS_SB];
#pragma unroll
      for (int q = 0; q < PT; q++)
#pragma unroll
        for (int h = 0; h < GS_SB; h++) {
          far[q][h] = p[q][h] != GNIL && (UP ? p[q][h] < base : p[q][h] >= base + GS_RING);
          fv[q][h] = far[q][h] ? (UP ? S.up[p[q][h]] : S.down[p[q][h]]) : 0;
          fr[q][h] = far[q][h] && !UP ? S.crank[p[q][h]] : 0u;
          ft[q][h] = far[q][h] && !UP ? S.ta[p[q][h]] : 0u;
        }
      more = false;
#pragma unroll
      for (int q = 0; q < PT; q++) {
#pragma unroll
        for (int h = 0; h < GS_SB; h++) {  // in row order: the kept links' order is the row's
          if (p[q][h] == GNIL) continue;
          if (!far[q][h]) {
            if (cnt[q] < GS_KEEP) keep[q][min(cnt[q], (uint32_t)GS_KEEP - 1u)] = p[q][h] - base;
            cnt[q]++;
          } else if (UP) {
            dd[q] = max(dd[q], fv[q][h] + 1);
          } else if (fv[q][h] > dd[q] || (fv[q][h] == dd[q] && fr[q][h] < br[q])) {
            dd[q] = fv[q][h];
            bc[q] = p[q][h];
            br[q] = fr[q][h];
            bt[q] = ft[q][h];
          }
        }
        more |= r0[q] + t + GS_SB < r1[q];
      }
    }
#pragma unroll
    for (int q = 0; q < PT; q++) {
      const uint32_t k = tid + q * GB, i = w0 + k;
      if (k >= nw) continue;
      L.lev[k] = lv[q];
      L.flg[k] = (uint8_t)rl[q];
      L.init[k] = dd[q];
      if (!UP) {
        L.ibc[k] = bc[q];
        L.ibr[k] = br[q];
        L.ibt[k] = bt[q];
        L.rc[i & M] = cr[q];
      }
    }
    // first GS_KEEP links packed per node; the rest in the window's list
    // (offsets by a block scan of the extra counts), past its capacity in HBM
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < PT; q++) sum += cnt[q] > GS_KEEP ? cnt[q] - GS_KEEP : 0u;
    uint32_t tot;
    uint32_t o = block_exscan<GB>(sum, &tot, s_red);
#pragma unroll
    for (int q = 0; q < PT; q++) {
      const uint32_t k = tid + q * GB;
      if (k >= nw) continue;
      uint64_t lk[2] = {0, 0};
#pragma unroll
      for (int t = 0; t < GS_KEEP; t++)
        lk[t >> 2] |= (uint64_t)((uint32_t)t < cnt[q] ? keep[q][t] : GS_NOLINK) << (16 * (t & 3));
      L.lk[k][0] = lk[0];
      L.lk[k][1] = lk[1];
      if (cnt[q] <= GS_KEEP) continue;
      const uint32_t extra = cnt[q] - GS_KEEP;
      const bool fits = o + extra <= GS_E;
      L.flg[k] |= fits ? GS_MORE : (GS_MORE | GS_SPILL);
      L.aoff[k] = (uint16_t)(fits ? o : 0u);  // adj index of link t = aoff + t - GS_KEEP
      L.acnt[k] = (uint16_t)(fits ? cnt[q] : GS_KEEP);
      if (fits) {  // the row again, GS_RW entries per load round (one at a time was a chain of round trips)
        uint32_t x = 0;
        for (uint32_t j = r0[q]; j < r1[q]; j += GS_RW) {
          uint32_t pv[GS_RW];
#pragma unroll
          for (int h = 0; h < GS_RW; h++) pv[h] = j + h < r1[q] ? col[j + h] : GNIL;
#pragma unroll
          for (int h = 0; h < GS_RW; h++) {
            const uint32_t p = pv[h];
            if (p != GNIL && (UP ? p >= base : p < base + GS_RING)) {
              if (x >= GS_KEEP) L.adj[o + x - GS_KEEP] = (uint16_t)(p - base);
              x++;
            }
          }
        }
      }
      o += extra;
    }
    __syncthreads();
#ifdef NEMO_STAMPS
    TICK(t_b);
    acc_s += t_b - t_a;
    t_a = t_b;
#endif
    if (GS_PF) prefetch(wi + 1);
    // ---- sweep (wave 0): the window's nodes level by level ----
    // Everything but the ring values is static, so the next batch's node data
    // (level, first links, staged far value) is read while the current batch
    // waits on its ring reads: a level's critical path is one LDS round trip
    // for the links' values and the write of its own.
    if (tid < 64) {
      uint32_t k = 0;
      auto fetch = [&](uint32_t k0, uint32_t &lv, uint64_t (&lk)[2], int32_t &ini, uint32_t &bc, uint32_t &br,
                       uint32_t &bt, uint32_t &fl) {
        const uint32_t q = k0 + lane, kk = UP ? q : nw - 1u - q;
        const bool in = q < nw;
        const uint32_t kc = in ? kk : 0u;
        lv = in ? L.lev[kc] : GNIL;
        lk[0] = L.lk[kc][0];
        lk[1] = L.lk[kc][1];
        ini = L.init[kc];
        fl = L.flg[kc];
        if (!UP) {
          bc = L.ibc[kc];
          br = L.ibr[kc];
          bt = L.ibt[kc];
        }
      };
      uint32_t lv, bc = 0, br = 0, bt = 0, fl;
      uint64_t lk[2];
      int32_t ini;
      fetch(0, lv, lk, ini, bc, br, bt, fl);
      while (k < nw) {
        const uint32_t q = k + lane, kk = UP ? q : nw - 1u - q;
        const uint32_t l = __builtin_amdgcn_readfirstlane(lv);
        const bool mine = q < nw && lv == l;
        const uint64_t m = __ballot(mine);  // contiguous from lane 0: nodes are sorted by level
        const uint32_t kn = k + (uint32_t)__popcll(m);
        uint32_t lv2, bc2 = 0, br2 = 0, bt2 = 0, fl2;
        uint64_t lk2[2];
        int32_t ini2;
        fetch(kn, lv2, lk2, ini2, bc2, br2, bt2, fl2);
        if (mine) {
          const uint32_t i = w0 + kk;
          uint32_t u[GS_KEEP];
#pragma unroll
          for (int h = 0; h < GS_KEEP; h++) u[h] = (uint32_t)(lk[h >> 2] >> (16 * (h & 3))) & 0xFFFFu;
          if (UP) {
            int32_t d = ini, v[GS_KEEP];
#pragma unroll
            for (int h = 0; h < GS_KEEP; h++) v[h] = L.rv[(base + u[h]) & M];
            // keep the reads issued together: sunk into the conditional uses
            // below, each would be its own LDS round trip
            asm volatile("" ::: "memory");
#pragma unroll
            for (int h = 0; h < GS_KEEP; h++) d = max(d, u[h] != GS_NOLINK ? v[h] + 1 : d);
            if (fl & GS_MORE) {  // links past the first four: the window's list, or HBM
              const uint32_t ao = L.aoff[kk], ac = L.acnt[kk];
              for (uint32_t t = GS_KEEP; t < ac; t += 4) {  // four links' reads in flight per round
                uint32_t a4[4];
                int32_t v4[4];
#pragma unroll
                for (int h = 0; h < 4; h++) a4[h] = L.adj[ao + min(t + h, ac - 1u) - GS_KEEP];
#pragma unroll
                for (int h = 0; h < 4; h++) v4[h] = L.rv[(base + a4[h]) & M];
#pragma unroll
                for (int h = 0; h < 4; h++) d = max(d, v4[h] + 1);  // clamped duplicates are harmless in a max
              }
              if (fl & GS_SPILL)
                for (uint32_t j = off[i]; j < oend[i]; j++) {
                  const uint32_t p = col[j];
                  d = max(d, (p >= base ? L.rv[p & M] : S.up[p]) + 1);
                }
            }
            L.rv[i & M] = d;
          } else {
            int32_t best = ini;
            auto take = [&](uint32_t w, int32_t dw, uint32_t rw, uint32_t tw) {
              if (dw > best || (dw == best && rw < br)) {
                best = dw;
                bc = w;
                br = rw;
                bt = tw;
              }
            };
            int32_t dv[GS_KEEP];
            uint32_t rr[GS_KEEP], tt[GS_KEEP];
#pragma unroll
            for (int h = 0; h < GS_KEEP; h++) {
              dv[h] = L.rv[(base + u[h]) & M];
              rr[h] = L.rc[(base + u[h]) & M];
              tt[h] = L.rt[(base + u[h]) & M];
            }
            asm volatile("" ::: "memory");
#pragma unroll
            for (int h = 0; h < GS_KEEP; h++)
              if (u[h] != GS_NOLINK) take(base + u[h], dv[h], rr[h], tt[h]);
            if (fl & GS_MORE) {
              const uint32_t ao = L.aoff[kk], ac = L.acnt[kk];
              for (uint32_t t = GS_KEEP; t < ac; t += 4) {  // four links' reads in flight per round
                uint32_t w4[4], r4[4], t4[4];
                int32_t d4[4];
#pragma unroll
                for (int h = 0; h < 4; h++) w4[h] = base + L.adj[ao + min(t + h, ac - 1u) - GS_KEEP];
#pragma unroll
                for (int h = 0; h < 4; h++) {
                  d4[h] = L.rv[w4[h] & M];
                  r4[h] = L.rc[w4[h] & M];
                  t4[h] = L.rt[w4[h] & M];
                }
#pragma unroll
                for (int h = 0; h < 4; h++) take(w4[h], d4[h], r4[h], t4[h]);  // a clamped repeat cannot win twice
              }
              if (fl & GS_SPILL)
                for (uint32_t j = off[i]; j < oend[i]; j++) {
                  const uint32_t w = col[j];
                  if (w < base + GS_RING) take(w, L.rv[w & M], L.rc[w & M], L.rt[w & M]);
                  else take(w, S.down[w], S.crank[w], S.ta[w]);
                }
            }
            int32_t d = best >= 0 ? best + 1 : ((fl & 1u) ? 0 : -1);
            L.rv[i & M] = d;
            L.rt[i & M] = d > 0 ? bt : i;   // tail: the end of the nxt chain
            L.ibc[kk] = d > 0 ? bc : GNIL;  // nxt (the staged far best is consumed)
            if (d < 0) *s_fail = 1;  // a goal without a chain continuation: impossible on H*
          }
        }
#ifdef NEMO_STAMPS
        iters++;
        spills += __ballot(mine && (fl & GS_MORE)) != 0 ? 1u : 0u;
#endif
        k = kn;
        lv = lv2;
        lk[0] = lk2[0];
        lk[1] = lk2[1];
        ini = ini2;
        bc = bc2;
        br = br2;
        bt = bt2;
        fl = fl2;
        wsync();
      }
    }
    __syncthreads();
    // ---- the window's values to HBM (no global store inside the sweep: a later
    // load there would wait for it), performed before the next window stages ----
    for (uint32_t k = tid; k < nw; k += GB) {
      const uint32_t i = w0 + k;
      if (UP) {
        S.up[i] = L.rv[i & M];
      } else {
        S.down[i] = L.rv[i & M];
        S.nxt[i] = L.ibc[k];
        S.ta[i] = L.rt[i & M];
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#ifdef NEMO_STAMPS
    TICK(t_b);
    acc_w += t_b - t_a;
#endif
  }
#ifdef NEMO_STAMPS
  if (threadIdx.x == 0 && st) {
    st[UP ? 10 : 12] = acc_s;
    st[UP ? 11 : 13] = acc_w;
    if (UP) {
      st[14] = iters | (spills << 32);
      st[15] = n;
    }
  }
#endif
}

// ---- k_glob_prep: H* compaction and adjacency by XCD teams ---------------------------
// The first two phases of the deep-graph chain cover translate between two
// orders: node order (the CSR, the flags) and H* in Kahn order (the sweeps'
// compact index).  One workgroup per graph did that with scattered stores
// into a V-word node -> index map and gathers from it, beside ~600 other
// graphs doing the same, so every such access went to HBM (C5, r05a:
// 198 GB of the kernel's 406 GB per launch, 64 of its 218 ms).  Here a team of
// PT_M workgroups (the blocks of one `blockIdx % 8` class: one XCD under the
// observed round-robin placement) takes one graph at a time, so the graph's
// membership bitmap and its compact-node -> H* index map (~2 MB) stay in the
// team's L2 while it is scattered and gathered.  Correctness does not depend on
// the placement: team members hand phases over with agent-scope release /
// acquire barriers.  Identity ID ranks only (corpora with a rank array keep the
// per-graph phases of k_chains_glob).
#define PT_TEAMS 8   // teams (blockIdx % 8)
#define PT_M 32      // workgroups per team
#ifndef PT_B
#define PT_B 512     // threads per workgroup (1024 spilled registers)
#endif
#define PT_CP 4      // Kahn positions per thread and round of the compaction
#define PT_WORDS 256 // team scratch words: barrier counter + 2 x 3 x PT_M phase sums
#define PT_GN 2      // H* nodes per thread and round of the adjacency
#ifndef PT_F
#define PT_F 4       // ... and row entries per node and load round
#endif
#define PT_RB 512    // LDS entries per wave and node slot for assembling adjacency ranges

// team barrier: every wave's stores drained, one lane releases and arrives,
// polls the team's counter (relaxed, L1-bypassing loads) and acquires
__device__ __forceinline__ void team_sync(uint32_t *ctr, uint32_t target) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// compact node index (rank among H* nodes in node order) of member y
__device__ __forceinline__ uint32_t pt_no(const uint2 *hb, uint32_t y) {
  const uint2 w = hb[y >> 5];
  return w.y + __popc(w.x & ((1u << (y & 31)) - 1u));
}

__global__ __launch_bounds__(PT_B) void k_glob_prep(DevCorpus c) {
  __shared__ uint32_t s_lds[PT_B / 64];
  __shared__ uint32_t s_base[3];
  __shared__ uint32_t s_rbuf[PT_B / 64][PT_GN * PT_RB];
  const uint32_t team = blockIdx.x % PT_TEAMS, r = blockIdx.x / PT_TEAMS, tid = threadIdx.x;
  const uint32_t M = gridDim.x / PT_TEAMS;  // members per team (<= PT_M)
  uint32_t *ts = c.team + (size_t)team * PT_WORDS, *ctr = ts;
  uint32_t epoch = 0;
  for (uint32_t k = team, it = 0; k < c.n_glob; k += PT_TEAMS, it++) {
    const uint32_t g = c.glob_list[k];
    if (c.err[g]) continue;  // every member reads the same flag: the whole team skips
    const GraphView gv = c.view(g);
    const uint32_t V = gv.V, E = gv.E;
    GlobScratch S = glob_carve(c.gscratch + c.gs_off[g], V, E);
    uint2 *hb = reinterpret_cast<uint2 *>(S.bm);  // per 32 nodes: H* bits, H* nodes before the word
    uint32_t *nolo = S.S;                         // compact node index -> H* (Kahn order) index
    uint32_t *rb = S.ta;                          // rule bits in node order
    // P2 -> P3: each H* node's CSR row bounds, in H* order (the sweeps' buffers, free until then)
    uint32_t *cst = reinterpret_cast<uint32_t *>(S.up), *pst = reinterpret_cast<uint32_t *>(S.down);
    uint32_t *hs = c.s_a + gv.n0 + g;
    uint32_t *cnt = ts + 1 + (it & 1) * 3 * PT_M;  // this graph's phase sums (graph parity: the next
                                                 // graph's writes never meet this graph's late reads)
    const uint32_t nw = (V + 31) / 32;
    // ---- P0: membership bitmap in node order (32 nodes per thread: two 16-byte flag loads) ----
    {
      const uint32_t a = (uint32_t)((uint64_t)nw * r / M), b = (uint32_t)((uint64_t)nw * (r + 1) / M);
      uint32_t sum = 0;
      for (uint32_t w = a + tid; w < b; w += PT_B) {
        const uint32_t v0 = 32 * w;
        uint32_t bits = 0;
        if (v0 + 31 < V) {
          uint4 fa, fb;
          __builtin_memcpy(&fa, gv.flags + v0, 16);
          __builtin_memcpy(&fb, gv.flags + v0 + 16, 16);
          const uint32_t fw[8] = {fa.x, fa.y, fa.z, fa.w, fb.x, fb.y, fb.z, fb.w};
#pragma unroll
          for (int q = 0; q < 32; q++) bits |= ((fw[q >> 2] >> (8 * (q & 3))) & NEMO_F_DELETED ? 1u : 0u) << q;
        } else {
          for (uint32_t v = v0; v < V; v++) bits |= (gv.flags[v] & NEMO_F_DELETED ? 1u : 0u) << (v - v0);
        }
        hb[w].x = bits;
        sum += __popc(bits);
        // rule bits of the same 32 nodes (node words streamed here, not gathered in Kahn order in P2)
        uint32_t rbits = 0;
        if (v0 + 31 < V) {
#pragma unroll
          for (int q4 = 0; q4 < 8; q4++) {
            uint4 w4;
            __builtin_memcpy(&w4, gv.word + v0 + 4 * q4, 16);
            rbits |= (is_rule(w4.x) ? 1u : 0u) << (4 * q4);
            rbits |= (is_rule(w4.y) ? 1u : 0u) << (4 * q4 + 1);
            rbits |= (is_rule(w4.z) ? 1u : 0u) << (4 * q4 + 2);
            rbits |= (is_rule(w4.w) ? 1u : 0u) << (4 * q4 + 3);
          }
        } else {
          for (uint32_t v = v0; v < V; v++) rbits |= (is_rule(gv.word[v]) ? 1u : 0u) << (v - v0);
        }
        rb[w] = rbits;
      }
      uint32_t tot;
      block_exscan<PT_B>(sum, &tot, s_lds);
      if (tid == 0) cnt[r] = tot;
    }
    team_sync(ctr, ++epoch * M);
    // ---- P1: word prefixes; H* nodes per Kahn slice ----
    {
      if (tid < 64) {
        uint32_t x = tid < r ? cnt[tid] : 0u;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) x += (uint32_t)__shfl_xor((int)x, d);
        if (tid == 0) s_base[0] = x;
      }
      __syncthreads();
      const uint32_t a = (uint32_t)((uint64_t)nw * r / M), b = (uint32_t)((uint64_t)nw * (r + 1) / M);
      uint32_t o = s_base[0];
      for (uint32_t w0 = a; w0 < b; w0 += PT_B) {
        const uint32_t w = w0 + tid;
        const uint32_t bits = w < b ? hb[w].x : 0u;
        uint32_t tot;
        const uint32_t ex = block_exscan<PT_B>(__popc(bits), &tot, s_lds);
        if (w < b) hb[w].y = o + ex;
        o += tot;
      }
      const uint32_t pa = (uint32_t)((uint64_t)V * r / M), pb = (uint32_t)((uint64_t)V * (r + 1) / M);
      uint32_t hc = 0;
      for (uint32_t p0 = pa + tid * PT_CP; p0 < pb; p0 += PT_B * PT_CP) {
        uint32_t x[PT_CP];
#pragma unroll
        for (int q = 0; q < PT_CP; q++) x[q] = p0 + q < pb ? gv.topo[p0 + q] : 0u;
#pragma unroll
        for (int q = 0; q < PT_CP; q++) hc += p0 + q < pb ? (hb[x[q] >> 5].x >> (x[q] & 31)) & 1u : 0u;
      }
      uint32_t tot;
      block_exscan<PT_B>(hc, &tot, s_lds);
      if (tid == 0) cnt[PT_M + r] = tot;
    }
    team_sync(ctr, ++epoch * M);
    // ---- P2: compaction of the Kahn slice (H* index, node, rule flag, compact rank, the
    // node -> index map, full degrees prefixed within the slice) ----
    {
      if (tid < 64) {
        uint32_t x = tid < r ? cnt[PT_M + tid] : 0u, t = tid < M ? cnt[PT_M + tid] : 0u;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
          x += (uint32_t)__shfl_xor((int)x, d);
          t += (uint32_t)__shfl_xor((int)t, d);
        }
        if (tid == 0) {
          s_base[0] = x;
          if (r == 0) S.meta[0] = t;
        }
      }
      __syncthreads();
      const uint32_t pa = (uint32_t)((uint64_t)V * r / M), pb = (uint32_t)((uint64_t)V * (r + 1) / M);
      const uint32_t wv = tid >> 6, lane = lane_id();
      uint32_t i = s_base[0], oc = 0, op = 0;
      // wave wv takes 64 * PT_CP consecutive positions, lane-interleaved (position
      // c0 + 64 q + lane), so each store instruction below writes consecutive H*
      // indices: whole lines, not one dword per line and lane
      for (uint32_t b0 = pa; b0 < pb; b0 += PT_B * PT_CP) {
        const uint32_t c0 = b0 + wv * 64u * PT_CP;
        uint32_t x[PT_CP], hx[PT_CP];
#pragma unroll
        for (int q = 0; q < PT_CP; q++) {
          const uint32_t p = c0 + 64u * q + lane;
          x[q] = p < pb ? gv.topo[p] : 0u;
        }
#pragma unroll
        for (int q = 0; q < PT_CP; q++) {
          const uint2 w = hb[x[q] >> 5];
          const bool h = c0 + 64u * q + lane < pb && ((w.x >> (x[q] & 31)) & 1u);
          hx[q] = h ? w.y + __popc(w.x & ((1u << (x[q] & 31)) - 1u)) : GNIL;
        }
        uint32_t rl[PT_CP], fa[PT_CP], fb[PT_CP], ra[PT_CP], rb2[PT_CP];
#pragma unroll
        for (int q = 0; q < PT_CP; q++) {
          const bool h = hx[q] != GNIL;
          rl[q] = h ? (rb[x[q] >> 5] >> (x[q] & 31)) & 1u : 0u;
          fa[q] = h ? gv.fp[x[q]] : 0u;
          fb[q] = h ? gv.fp[x[q] + 1] : 0u;
          ra[q] = h ? gv.rp[x[q]] : 0u;
          rb2[q] = h ? gv.rp[x[q] + 1] : 0u;
        }
        // offsets within the wave in (q, lane) order, then the waves' bases
        uint32_t jq[PT_CP], cq[PT_CP], pq[PT_CP], wn = 0, wc = 0, wp = 0;
#pragma unroll
        for (int q = 0; q < PT_CP; q++) {
          uint32_t t;
          jq[q] = wn + wave_exscan(hx[q] != GNIL ? 1u : 0u, &t);
          wn += t;
          cq[q] = wc + wave_exscan(fb[q] - fa[q], &t);
          wc += t;
          pq[q] = wp + wave_exscan(rb2[q] - ra[q], &t);
          wp += t;
        }
        uint32_t tn, tc, tp;
        const uint32_t bn = __builtin_amdgcn_readfirstlane(block_exscan<PT_B>(lane == 0 ? wn : 0u, &tn, s_lds));
        const uint32_t bc = __builtin_amdgcn_readfirstlane(block_exscan<PT_B>(lane == 0 ? wc : 0u, &tc, s_lds));
        const uint32_t bp = __builtin_amdgcn_readfirstlane(block_exscan<PT_B>(lane == 0 ? wp : 0u, &tp, s_lds));
#pragma unroll
        for (int q = 0; q < PT_CP; q++) {
          if (hx[q] == GNIL) continue;
          const uint32_t j = i + bn + jq[q];
          hs[j] = x[q];
          S.rule[j] = rl[q];
          S.crank[j] = hx[q];
          nolo[hx[q]] = j;
          S.ccoff[j] = oc + bc + cq[q];  // within the slice; P3 adds the slices before it
          S.pcoff[j] = op + bp + pq[q];
          cst[j] = fa[q];
          S.cend[j] = fb[q];
          pst[j] = ra[q];
          S.pend[j] = rb2[q];
        }
        i += tn;
        oc += tc;
        op += tp;
      }
      if (tid == 0) {
        cnt[2 * PT_M + r] = oc;
        cnt[r] = op;  // P0's slot: its last readers passed the barrier before P2
      }
    }
    team_sync(ctr, ++epoch * M);
    // ---- P3: the H* adjacency in H* indices, rows laid out by full degree; the slice's
    // rows at its offsets (the row pointers made global) ----
    {
      if (tid < 64) {
        uint32_t l = tid < r ? cnt[PT_M + tid] : 0u, oc = tid < r ? cnt[2 * PT_M + tid] : 0u,
                 op = tid < r ? cnt[tid] : 0u;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
          l += (uint32_t)__shfl_xor((int)l, d);
          oc += (uint32_t)__shfl_xor((int)oc, d);
          op += (uint32_t)__shfl_xor((int)op, d);
        }
        if (tid == 0) {
          s_base[0] = l;
          s_base[1] = oc;
          s_base[2] = op;
        }
      }
      __syncthreads();
      const uint32_t lo = s_base[0], hi = lo + cnt[PT_M + r], cb = s_base[1], pb = s_base[2];
      if (r == M - 1 && tid == 0) {
        S.ccoff[hi] = cb + cnt[2 * PT_M + r];
        S.pcoff[hi] = pb + cnt[r];
      }
      // rows of 64 consecutive H* nodes (a wave, one node per lane) fill one range
      // of the adjacency (full-degree layout): assembled in LDS and stored whole
      // (one dword per lane into a different line per row was a partial-line
      // write each); a range past PT_RB entries is stored directly
      uint32_t *rbuf = s_rbuf[tid >> 6];
      const uint32_t lane = lane_id();
      auto rows = [&](const uint32_t *st, const uint32_t *col, uint32_t *off, uint32_t *endp, uint32_t *out,
                      uint32_t ob) {
        for (uint32_t i0 = lo + tid; __any(i0 < hi); i0 += PT_B * PT_GN) {
          uint32_t a[PT_GN], e[PT_GN], o[PT_GN], k[PT_GN], rs[PT_GN], rl[PT_GN];
#pragma unroll
          for (int q = 0; q < PT_GN; q++) {
            const uint32_t i = i0 + q * PT_B;
            a[q] = i < hi ? st[i] : 0u;
            e[q] = i < hi ? endp[i] : 0u;  // the row's CSR end (P2), replaced by its H* end below
            o[q] = i < hi ? off[i] + ob : 0u;
            k[q] = 0;
          }
#pragma unroll
          for (int q = 0; q < PT_GN; q++) {  // the wave's range: [first active lane's row, last one's end)
            uint32_t ee = i0 + q * PT_B < hi ? o[q] + (e[q] - a[q]) : 0u;
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) ee = max(ee, (uint32_t)__shfl_xor((int)ee, d));
            rs[q] = __builtin_amdgcn_readfirstlane(o[q]);
            rl[q] = ee > rs[q] ? ee - rs[q] : 0u;
            if (rl[q] <= PT_RB)
              for (uint32_t t = lane; t < rl[q]; t += 64) rbuf[q * PT_RB + t] = GNIL;
          }
          wsync();
          for (uint32_t t = 0;; t += PT_F) {
            bool more = false;
            uint32_t y[PT_GN][PT_F];
#pragma unroll
            for (int q = 0; q < PT_GN; q++)
#pragma unroll
              for (int h = 0; h < PT_F; h++) y[q][h] = a[q] + t + h < e[q] ? col[a[q] + t + h] : GNIL;
            uint2 w[PT_GN][PT_F];
#pragma unroll
            for (int q = 0; q < PT_GN; q++)
#pragma unroll
              for (int h = 0; h < PT_F; h++) w[q][h] = y[q][h] != GNIL ? hb[y[q][h] >> 5] : make_uint2(0, 0);
            uint32_t m[PT_GN][PT_F];
#pragma unroll
            for (int q = 0; q < PT_GN; q++)
#pragma unroll
              for (int h = 0; h < PT_F; h++) {
                const uint32_t yy = y[q][h] & 31u;
                m[q][h] = (w[q][h].x >> yy) & 1u ? nolo[w[q][h].y + __popc(w[q][h].x & ((1u << yy) - 1u))] : GNIL;
              }
#pragma unroll
            for (int q = 0; q < PT_GN; q++) {
#pragma unroll
              for (int h = 0; h < PT_F; h++)
                if (m[q][h] != GNIL) {
                  if (rl[q] <= PT_RB) rbuf[q * PT_RB + o[q] + k[q] - rs[q]] = m[q][h];
                  else out[o[q] + k[q]] = m[q][h];
                  k[q]++;
                }
              more |= a[q] + t + PT_F < e[q];
            }
            if (!__any(more)) break;
          }
          wsync();
#pragma unroll
          for (int q = 0; q < PT_GN; q++) {
            if (rl[q] <= PT_RB)
              for (uint32_t t = lane; t < rl[q]; t += 64) out[rs[q] + t] = rbuf[q * PT_RB + t];
            const uint32_t i = i0 + q * PT_B;
            if (i >= hi) continue;
            off[i] = o[q];
            endp[i] = o[q] + k[q];
          }
          wsync();
        }
      };
      rows(cst, gv.fc, S.ccoff, S.cend, S.child, cb);
      rows(pst, gv.rc, S.pcoff, S.pend, S.par, pb);
    }
  }
}

template <int GB>
__global__ __launch_bounds__(GB, 1024 / GB) void k_chains_glob(DevCorpus c) {
  static_assert(GS_WN % GB == 0, "whole window nodes per thread");
  __shared__ uint32_t s_lds[GB / 64];
  __shared__ uint32_t s_nch, s_fail;
  __shared__ __align__(16) GSweepLds s_gs;
  const uint32_t g = blockIdx.x, tid = threadIdx.x;
  if (c.err[g] || c.gs_off[g] == ~0ull) return;
  const GraphView gv = c.view(g);
  const uint32_t V = gv.V, E = gv.E;
  GlobScratch S = glob_carve(c.gscratch + c.gs_off[g], V, E);
  uint32_t *hs = c.s_a + gv.n0 + g;    // compact index -> graph-local node
  uint32_t *hidx = c.s_f + gv.n0 + g;  // graph-local node -> compact index
  uint32_t *tmp = S.tmp;
  const uint8_t *f = gv.flags;
  const uint32_t *nlv = c.nlv + gv.n0;
  const uint32_t nw = (V + 31) / 32;
  if (tid == 0) {
    s_nch = 0;
    s_fail = 0;
  }
  STAMP(0);
  // With k_glob_prep (identity ranks) the H* compaction, the compact ranks and the
  // adjacency are done: only the H* node count is read here.
  const bool idrank = gv.rank == nullptr;
  uint32_t n = 0;
  if (c.glob_prep) {
    n = S.meta[0];
  } else {
    // ---- H* in level order, compact ID ranks ------------------------------------
    // a stream compaction of the Kahn order (level-sorted already) by the H*
    // flag: block scans over CP positions per thread, no counter atomics
    for (uint32_t w = tid; w < nw; w += GB) S.bm[w] = 0;
    // every node's compact index, GNIL outside H* (a coalesced pass): the
    // adjacency then tests a neighbour's membership and maps it with one gather
    // With identity ID ranks (no rank array) the rank bitmap is the H* flag in
    // node order, stored a word per half-wave (no scattered atomics)
    // (each thread 32 consecutive nodes: their flags in two 16-byte loads, the
    // map in eight 16-byte stores, the bitmap word built in a register)
    for (uint32_t v0 = 32 * tid; v0 < V; v0 += 32 * GB) {
      uint32_t bits = 0;
      if (v0 + 31 < V) {
        uint4 fa, fb;
        __builtin_memcpy(&fa, f + v0, 16);
        __builtin_memcpy(&fb, f + v0 + 16, 16);
        const uint32_t fw[8] = {fa.x, fa.y, fa.z, fa.w, fb.x, fb.y, fb.z, fb.w};
  #pragma unroll
        for (int k = 0; k < 32; k++) bits |= ((fw[k >> 2] >> (8 * (k & 3))) & NEMO_F_DELETED ? 1u : 0u) << k;
        const uint4 nil = make_uint4(GNIL, GNIL, GNIL, GNIL);
  #pragma unroll
        for (int k = 0; k < 8; k++) __builtin_memcpy(hidx + v0 + 4 * k, &nil, 16);
      } else {
        for (uint32_t v = v0; v < V; v++) {
          bits |= (f[v] & NEMO_F_DELETED ? 1u : 0u) << (v - v0);
          hidx[v] = GNIL;
        }
      }
      if (idrank) S.bm[v0 >> 5] = bits;
    }
    __syncthreads();
    for (uint32_t base = 0; base < V; base += GB * CP) {
      const uint32_t p0 = base + tid * CP;
      uint32_t x[CP], cl = 0;
      bool h[CP];
  #pragma unroll
      for (int q = 0; q < CP; q++) x[q] = p0 + q < V ? gv.topo[p0 + q] : 0u;
  #pragma unroll
      for (int q = 0; q < CP; q++) {
        h[q] = p0 + q < V && (f[x[q]] & NEMO_F_DELETED);
        cl += h[q] ? 1u : 0u;
      }
      uint32_t tot;
      uint32_t i = block_exscan<GB>(cl, &tot, s_lds) + n;
  #pragma unroll
      for (int q = 0; q < CP; q++) {
        if (p0 + q >= V || !h[q]) continue;
        hs[i] = x[q];
        hidx[x[q]] = i;
        S.rule[i] = is_rule(gv.word[x[q]]) ? 1u : 0u;
        const uint32_t r = gv.rank_of(x[q]);
        S.crank[i] = r;
        if (!idrank) atomicOr(&S.bm[r >> 5], 1u << (r & 31));
        i++;
      }
      n += tot;
    }
  }
  __syncthreads();
  if (n == 0) {
    if (tid == 0) c.nch[g] = 0;
    return;
  }
  if (!c.glob_prep) {
    // (GU entries per thread and round below: each round's loads, then its
    // gathers, in flight together)
    for (uint32_t w0 = tid; w0 < nw; w0 += GB * GU) {
      uint32_t x[GU];
  #pragma unroll
      for (int q = 0; q < GU; q++) x[q] = w0 + q * GB < nw ? S.bm[w0 + q * GB] : 0u;
  #pragma unroll
      for (int q = 0; q < GU; q++)
        if (w0 + q * GB < nw) S.bmpre[w0 + q * GB] = __popc(x[q]);
    }
    __syncthreads();
    block_scan_inplace<GB, 16>(S.bmpre, nw, s_lds);
    for (uint32_t i0 = tid; i0 < n; i0 += GB * GU) {
      uint32_t r[GU], bp_[GU], bw[GU];
  #pragma unroll
      for (int q = 0; q < GU; q++) r[q] = i0 + q * GB < n ? S.crank[i0 + q * GB] : 0u;
  #pragma unroll
      for (int q = 0; q < GU; q++) {
        bp_[q] = S.bmpre[r[q] >> 5];
        bw[q] = S.bm[r[q] >> 5];
      }
  #pragma unroll
      for (int q = 0; q < GU; q++)
        if (i0 + q * GB < n) S.crank[i0 + q * GB] = bp_[q] + __popc(bw[q] & ((1u << (r[q] & 31)) - 1u));
    }
    STAMP(1);
    GSTOP(1);
    // ---- H* adjacency (rows in any order: every consumer takes a max/min) ---------
    // From the graph's own CSR rows, one H* node per thread: a row's children
    // (or parents) in batches of GA_B with their loads in flight together, no
    // atomics.  Each H* row is laid out by the node's full degree (one scan of
    // the degrees, no counting pass over the neighbours' flags); the H*
    // entries fill its front and cend / pend mark where they stop.  (Counting
    // and scattering the whole edge list with cursor atomics cost a
    // latency-bound pass over all E edges per direction; walking four nodes'
    // rows in lockstep, one entry per row and step, was slower: the step count
    // is the longest of the rows.)
    auto hrow = [&](const uint32_t *ptr, const uint32_t *col, uint32_t x, uint32_t j00, uint32_t *out) -> uint32_t {
      uint32_t k = 0;
      const uint32_t j1 = ptr[x + 1];
      for (uint32_t j = j00; j < j1; j += GA_B) {
        uint32_t y[GA_B];
  #pragma unroll
        for (int q = 0; q < GA_B; q++) y[q] = j + q < j1 ? col[j + q] : 0u;
        uint32_t hy[GA_B];
  #pragma unroll
        for (int q = 0; q < GA_B; q++) hy[q] = j + q < j1 ? hidx[y[q]] : GNIL;
  #pragma unroll
        for (int q = 0; q < GA_B; q++)
          if (hy[q] != GNIL) out[k++] = hy[q];
      }
      return k;
    };
    for (uint32_t i0 = tid; i0 < n; i0 += GB * GU) {
      uint32_t x[GU];
  #pragma unroll
      for (int q = 0; q < GU; q++) x[q] = i0 + q * GB < n ? hs[i0 + q * GB] : 0u;
  #pragma unroll
      for (int q = 0; q < GU; q++) {
        const uint32_t i = i0 + q * GB;
        const uint32_t fa = gv.fp[x[q]], fb = gv.fp[x[q] + 1], ra = gv.rp[x[q]], rb = gv.rp[x[q] + 1];
        if (i < n) {
          S.ccoff[i] = fb - fa;
          S.pcoff[i] = rb - ra;
        }
      }
    }
    if (tid == 0) {
      S.ccoff[n] = 0;
      S.pcoff[n] = 0;
    }
    __syncthreads();
    block_scan_inplace<GB, 16>(S.ccoff, n + 1, s_lds);
    block_scan_inplace<GB, 16>(S.pcoff, n + 1, s_lds);
    // the rows written GA_N nodes per thread at a time: their bounds, first
    // GA_F entries and those entries' compact indices each a round of loads in
    // flight together (one node at a time was a chain of three dependent
    // round trips per node and direction); longer rows finish by themselves
    auto hrows = [&](const uint32_t *ptr, const uint32_t *col, const uint32_t *off, uint32_t *endp, uint32_t *out) {
      for (uint32_t i0 = tid; i0 < n; i0 += GB * GA_N) {
        uint32_t x[GA_N], a[GA_N], b[GA_N], o[GA_N], k[GA_N];
  #pragma unroll
        for (int q = 0; q < GA_N; q++) {
          const uint32_t i = i0 + q * GB;
          x[q] = i < n ? hs[i] : 0u;
          o[q] = i < n ? off[i] : 0u;
          k[q] = 0;
        }
  #pragma unroll
        for (int q = 0; q < GA_N; q++) {
          a[q] = ptr[x[q]];
          b[q] = i0 + q * GB < n ? ptr[x[q] + 1] : a[q];
        }
        uint32_t y[GA_N][GA_F], hy[GA_N][GA_F];
  #pragma unroll
        for (int q = 0; q < GA_N; q++)
  #pragma unroll
          for (int h = 0; h < GA_F; h++) y[q][h] = a[q] + h < b[q] ? col[a[q] + h] : 0u;
  #if GA_BM
        // identity ranks: S.bm is the H* flag in node order (119 KB per 1M-node
        // graph, cache-resident), so only members' compact indices are gathered
        if (idrank) {
          uint32_t w[GA_N][GA_F];
  #pragma unroll
          for (int q = 0; q < GA_N; q++)
  #pragma unroll
            for (int h = 0; h < GA_F; h++) w[q][h] = a[q] + h < b[q] ? S.bm[y[q][h] >> 5] : 0u;
  #pragma unroll
          for (int q = 0; q < GA_N; q++)
  #pragma unroll
            for (int h = 0; h < GA_F; h++) hy[q][h] = (w[q][h] >> (y[q][h] & 31)) & 1u ? hidx[y[q][h]] : GNIL;
        } else
  #endif
  #pragma unroll
        for (int q = 0; q < GA_N; q++)
  #pragma unroll
          for (int h = 0; h < GA_F; h++) hy[q][h] = a[q] + h < b[q] ? hidx[y[q][h]] : GNIL;
  #pragma unroll
        for (int q = 0; q < GA_N; q++) {
  #pragma unroll
          for (int h = 0; h < GA_F; h++)
            if (hy[q][h] != GNIL) out[o[q] + k[q]++] = hy[q][h];
          if (b[q] > a[q] + GA_F) k[q] += hrow(ptr, col, x[q], a[q] + GA_F, out + o[q] + k[q]);
          if (i0 + q * GB < n) endp[i0 + q * GB] = o[q] + k[q];
        }
      }
    };
    hrows(gv.fp, gv.fc, S.ccoff, S.cend, S.child);
    hrows(gv.rp, gv.rc, S.pcoff, S.pend, S.par);
    __syncthreads();
  }
  STAMP(2);
  GSTOP(2);
  // ---- up (forward) and down/nxt (backward): windowed single-wave sweeps -----------
#ifdef NEMO_STAMPS
  unsigned long long *gst = c.stamps ? c.stamps + 16 * (size_t)blockIdx.x : nullptr;
#else
  unsigned long long *gst = nullptr;
#endif
  glob_sweep<true, GB>(S, n, hs, nlv, &s_fail, s_gs, s_lds, gst);
  glob_sweep<false, GB>(S, n, hs, nlv, &s_fail, s_gs, s_lds, gst);
  STAMP(3);
  GSTOP(3);
  uint32_t mu = 0, ml = 0;
  for (uint32_t b0 = 0; b0 < n; b0 += 16 * GB) {  // four quads of consecutive nodes per thread and round
    int32_t u[16], d[16];
#pragma unroll
    for (int g4 = 0; g4 < 4; g4++) {
      const uint32_t i = b0 + 4 * (g4 * GB + tid);
      ld4(S.up, i, n, u + 4 * g4, 0);
      ld4(S.down, i, n, d + 4 * g4, 0);
    }
#pragma unroll
    for (int q = 0; q < 16; q++) {
      mu = max(mu, (uint32_t)max(u[q], 0));
      ml = max(ml, (uint32_t)max(u[q] + d[q], 0));
    }
  }
  const uint32_t maxup = gmax_u32<GB>(mu, s_lds);
  const uint32_t maxlen = gmax_u32<GB>(ml, s_lds);
  // ---- bucket by up -----------------------------------------------------------------
  // (counters in LDS -- the sweeps' memory, free now -- when the up range fits)
  constexpr uint32_t LW = sizeof(GSweepLds) / 4;
  uint32_t *const lw = reinterpret_cast<uint32_t *>(&s_gs);
  if (maxup + 2 <= LW) {
    uint32_t *lc = lw;
    for (uint32_t k = tid; k <= maxup + 1; k += GB) lc[k] = 0;
    __syncthreads();
    for (uint32_t i0 = tid; i0 < n; i0 += GB * GU) {
      int32_t u[GU];
#pragma unroll
      for (int q = 0; q < GU; q++) u[q] = i0 + q * GB < n ? S.up[i0 + q * GB] : -1;
#pragma unroll
      for (int q = 0; q < GU; q++)
        if (u[q] >= 0) atomicAdd(&lc[u[q]], 1u);
    }
    __syncthreads();
    block_scan_inplace<GB>(lc, maxup + 2, s_lds);
    for (uint32_t k = tid; k <= maxup + 1; k += GB) S.uoff[k] = lc[k];
    __syncthreads();
    for (uint32_t i0 = tid; i0 < n; i0 += GB * GU) {
      int32_t u[GU];
#pragma unroll
      for (int q = 0; q < GU; q++) u[q] = i0 + q * GB < n ? S.up[i0 + q * GB] : -1;
#pragma unroll
      for (int q = 0; q < GU; q++)
        if (u[q] >= 0) S.ub[atomicAdd(&lc[u[q]], 1u)] = i0 + q * GB;
    }
  } else {
    for (uint32_t k = tid; k <= maxup + 1; k += GB) S.uoff[k] = 0;
    __syncthreads();
    for (uint32_t i = tid; i < n; i += GB) atomicAdd(&S.uoff[S.up[i]], 1u);
    __syncthreads();
    block_scan_inplace<GB, 16>(S.uoff, maxup + 2, s_lds);
    for (uint32_t k = tid; k <= maxup + 1; k += GB) S.cnt[k] = S.uoff[k];
    __syncthreads();
    for (uint32_t i = tid; i < n; i += GB) S.ub[atomicAdd(&S.cnt[S.up[i]], 1u)] = i;
  }
  // best parent fixed up front where only one parent has up == up(v) - 1
  // (GU nodes per thread and round, the first BP_K parents of each read together,
  // then their up values: two rounds of loads in flight instead of a chain per parent)
  constexpr uint32_t MULTI = 0xFFFFFFFEu;
  constexpr int BP_K = 3;
  for (uint32_t i0 = tid; i0 < n; i0 += GB * GU) {
    int32_t k[GU];
    uint32_t r0[GU], r1[GU], cand[GU], cn[GU], pp[GU][BP_K];
#pragma unroll
    for (int q = 0; q < GU; q++) {
      const uint32_t i = i0 + q * GB;
      const bool in = i < n;
      k[q] = in ? S.up[i] : 0;
      r0[q] = in ? S.pcoff[i] : 0u;
      r1[q] = in ? S.pend[i] : 0u;
    }
#pragma unroll
    for (int q = 0; q < GU; q++)
#pragma unroll
      for (int h = 0; h < BP_K; h++) pp[q][h] = k[q] > 0 && r0[q] + h < r1[q] ? S.par[r0[q] + h] : GNIL;
    int32_t uu[GU][BP_K];
#pragma unroll
    for (int q = 0; q < GU; q++)
#pragma unroll
      for (int h = 0; h < BP_K; h++) uu[q][h] = pp[q][h] != GNIL ? S.up[pp[q][h]] : -2;
#pragma unroll
    for (int q = 0; q < GU; q++) {
      cn[q] = 0;
      cand[q] = GNIL;
#pragma unroll
      for (int h = 0; h < BP_K; h++)
        if (pp[q][h] != GNIL && uu[q][h] == k[q] - 1) {
          cn[q]++;
          cand[q] = pp[q][h];
        }
    }
#pragma unroll
    for (int q = 0; q < GU; q++) {
      const uint32_t i = i0 + q * GB;
      if (i >= n) continue;
      if (k[q] > 0)
        for (uint32_t j = r0[q] + BP_K; j < r1[q]; j++) {  // the rest of the row (rare)
          const uint32_t pj = S.par[j];
          if (S.up[pj] == k[q] - 1) {
            cn[q]++;
            cand[q] = pj;
          }
        }
      S.bp[i] = cn[q] > 1 ? MULTI : cand[q];
    }
  }
  __syncthreads();
  STAMP(4);
  GSTOP(4);
  // ---- prefix ranks per up-level: roots by ID rank, then groups by po(bp) -----------
  for (uint32_t k = 0; k <= maxup; k++) {
    const uint32_t a = S.uoff[k], b = S.uoff[k + 1];
    if (k == 0) {
      const uint32_t rw = (n + 31) / 32;
      for (uint32_t w = tid; w < rw; w += GB) S.bm[w] = 0;
      __syncthreads();
      for (uint32_t j = a + tid; j < b; j += GB) {
        const uint32_t cr = S.crank[S.ub[j]];
        atomicOr(&S.bm[cr >> 5], 1u << (cr & 31));
      }
      __syncthreads();
      for (uint32_t w = tid; w < rw; w += GB) S.bmpre[w] = __popc(S.bm[w]);
      __syncthreads();
      block_scan_inplace<GB, 16>(S.bmpre, rw, s_lds);
      for (uint32_t j = a + tid; j < b; j += GB) {
        const uint32_t i = S.ub[j], cr = S.crank[i];
        S.po[i] = S.bmpre[cr >> 5] + __popc(S.bm[cr >> 5] & ((1u << (cr & 31)) - 1u));
        S.fpos[i] = 0;
      }
      __syncthreads();
      continue;
    }
    const uint32_t mp = a - S.uoff[k - 1];  // size of level k-1: po(bp) < mp
    if (b - a <= GB && mp + 1 + GB <= LW) {
      // one node per thread, its (node, crank, po(bp)) kept in registers; the
      // group counters and the groups' cranks in LDS (the sweeps' memory)
      uint32_t *lcnt = lw, *lgrp = lw + LW - GB;
      const uint32_t j = a + tid;
      const bool act = j < b;
      for (uint32_t w = tid; w <= mp; w += GB) lcnt[w] = 0;
      const uint32_t i = act ? S.ub[j] : 0u;
      uint32_t bpi = act ? S.bp[i] : 0u;
      const uint32_t cr = act ? S.crank[i] : 0u;
      if (act && bpi == MULTI) {
        uint32_t bpo = GNIL;
        for (uint32_t q = S.pcoff[i]; q < S.pend[i]; q++) {
          const uint32_t p = S.par[q];
          if ((uint32_t)S.up[p] == k - 1 && S.po[p] < bpo) {
            bpi = p;
            bpo = S.po[p];
          }
        }
        S.bp[i] = bpi;
      }
      const uint32_t bpo = act ? S.po[bpi] : 0u;
      __syncthreads();
      if (act) atomicAdd(&lcnt[bpo], 1u);
      __syncthreads();
      block_scan_inplace<GB>(lcnt, mp + 1, s_lds);  // group bases
      if (act) lgrp[atomicAdd(&lcnt[bpo], 1u)] = cr;
      __syncthreads();  // lcnt[q] = end of group q = base of group q + 1
      if (act) {
        const uint32_t base = bpo ? lcnt[bpo - 1] : 0u, end = lcnt[bpo];
        uint32_t r = 0;
        for (uint32_t q = base; q < end; q++) r += lgrp[q] < cr;
        S.po[i] = base + r;
        S.fpos[i] = base;
      }
      __syncthreads();
      continue;
    }
    if (mp + 1 + 2 * (b - a) <= LW) {
      // the level's group counters, its members' cranks and their po(bp) in LDS
      // (the sweeps' memory): device-scope atomics run at the memory side, and a
      // level's histogram and cursors were ~2 per node of them
      uint32_t *lcnt = lw, *lgrp = lw + mp + 1, *lbpo = lgrp + (b - a);
      for (uint32_t w = tid; w <= mp; w += GB) lcnt[w] = 0;
      __syncthreads();
      for (uint32_t j0 = a + tid; j0 < b; j0 += GB * GU) {
        uint32_t i[GU], bpi[GU], bpo[GU];
#pragma unroll
        for (int q = 0; q < GU; q++) i[q] = j0 + q * GB < b ? S.ub[j0 + q * GB] : 0u;
#pragma unroll
        for (int q = 0; q < GU; q++) bpi[q] = j0 + q * GB < b ? S.bp[i[q]] : 0u;
#pragma unroll
        for (int q = 0; q < GU; q++) {
          if (j0 + q * GB >= b || bpi[q] != MULTI) continue;
          uint32_t best = GNIL, bo = GNIL;
          for (uint32_t qq = S.pcoff[i[q]]; qq < S.pend[i[q]]; qq++) {
            const uint32_t p = S.par[qq];
            if ((uint32_t)S.up[p] == k - 1 && S.po[p] < bo) {
              best = p;
              bo = S.po[p];
            }
          }
          bpi[q] = best;
          S.bp[i[q]] = best;
        }
#pragma unroll
        for (int q = 0; q < GU; q++) bpo[q] = j0 + q * GB < b ? S.po[bpi[q]] : 0u;
#pragma unroll
        for (int q = 0; q < GU; q++) {
          if (j0 + q * GB >= b) continue;
          lbpo[j0 + q * GB - a] = bpo[q];
          atomicAdd(&lcnt[bpo[q]], 1u);
        }
      }
      __syncthreads();
      block_scan_inplace<GB>(lcnt, mp + 1, s_lds);  // group bases
      for (uint32_t j0 = a + tid; j0 < b; j0 += GB * GU) {
        uint32_t i[GU], cr[GU];
#pragma unroll
        for (int q = 0; q < GU; q++) i[q] = j0 + q * GB < b ? S.ub[j0 + q * GB] : 0u;
#pragma unroll
        for (int q = 0; q < GU; q++) cr[q] = j0 + q * GB < b ? S.crank[i[q]] : 0u;
#pragma unroll
        for (int q = 0; q < GU; q++)
          if (j0 + q * GB < b) lgrp[atomicAdd(&lcnt[lbpo[j0 + q * GB - a]], 1u)] = cr[q];
      }
      __syncthreads();  // lcnt[q] = end of group q = base of group q + 1
      for (uint32_t j0 = a + tid; j0 < b; j0 += GB * GU) {
        uint32_t i[GU], cr[GU];
#pragma unroll
        for (int q = 0; q < GU; q++) i[q] = j0 + q * GB < b ? S.ub[j0 + q * GB] : 0u;
#pragma unroll
        for (int q = 0; q < GU; q++) cr[q] = j0 + q * GB < b ? S.crank[i[q]] : 0u;
#pragma unroll
        for (int q = 0; q < GU; q++) {
          if (j0 + q * GB >= b) continue;
          const uint32_t bo = lbpo[j0 + q * GB - a];
          const uint32_t base = bo ? lcnt[bo - 1] : 0u, end = lcnt[bo];
          uint32_t r = 0;
          for (uint32_t qq = base; qq < end; qq++) r += lgrp[qq] < cr[q];
          S.po[i[q]] = base + r;
          S.fpos[i[q]] = base;
        }
      }
      __syncthreads();
      continue;
    }
    for (uint32_t w = tid; w <= mp; w += GB) S.cnt[w] = 0;
    __syncthreads();
    for (uint32_t j = a + tid; j < b; j += GB) {
      const uint32_t i = S.ub[j];
      uint32_t bpi = S.bp[i];
      if (bpi == MULTI) {
        uint32_t bpo = GNIL;
        for (uint32_t q = S.pcoff[i]; q < S.pend[i]; q++) {
          const uint32_t p = S.par[q];
          if ((uint32_t)S.up[p] == k - 1 && S.po[p] < bpo) {
            bpi = p;
            bpo = S.po[p];
          }
        }
        S.bp[i] = bpi;
      }
      atomicAdd(&S.cnt[S.po[bpi]], 1u);
    }
    __syncthreads();
    block_scan_inplace<GB, 16>(S.cnt, mp + 1, s_lds);  // group bases
    for (uint32_t j = a + tid; j < b; j += GB) {
      const uint32_t i = S.ub[j];
      S.grp[atomicAdd(&S.cnt[S.po[S.bp[i]]], 1u)] = i;
    }
    __syncthreads();  // cnt[q] = end of group q = base of group q + 1
    for (uint32_t j = a + tid; j < b; j += GB) {
      const uint32_t i = S.ub[j], bpo = S.po[S.bp[i]], cr = S.crank[i];
      const uint32_t base = bpo ? S.cnt[bpo - 1] : 0u, end = S.cnt[bpo];
      uint32_t r = 0;
      for (uint32_t q = base; q < end; q++) r += S.crank[S.grp[q]] < cr;
      S.po[i] = base + r;
      S.fpos[i] = base;
    }
    __syncthreads();
  }
  STAMP(5);
  GSTOP(5);
  // ---- preorder of the representatives: pre(v) = up(v) + sum of off over v and its bp
  // ancestors, off = sizes of the earlier siblings (sizes laid out in (level, po) order).
  // Subtree sizes bottom-up, then ONE top-down pass over the up-levels adds each
  // node's best parent's sum to its own and copies the parent's head (the root
  // of its bp path); the tails (ends of the nxt chains) came out of the down
  // sweep.  (Pointer jumping made ~12 rounds of random gathers over the whole
  // H* for each of heads, tails and the preorder sums.)
  uint32_t *va = S.va, *hd = S.hb, *tl = S.ta;
  for (uint32_t i = tid; i < n; i += GB) S.S[i] = 1;
  __syncthreads();
  // subtree sizes bottom-up: a level's sizes summed into its parents' slots in
  // LDS (indexed by the parent's po, dense in [0, size of the level above)),
  // then the parents' sizes stored; levels above past the LDS take device atomics
  for (uint32_t k = maxup; k >= 1; k--) {
    const uint32_t a = S.uoff[k], b = S.uoff[k + 1], pa = S.uoff[k - 1], mp = a - pa;
    if (mp <= LW) {
      for (uint32_t w = tid; w < mp; w += GB) lw[w] = 0;
      __syncthreads();
      for (uint32_t j0 = a + tid; j0 < b; j0 += GB * GU) {
        uint32_t i[GU], p[GU], sz[GU], po[GU];
#pragma unroll
        for (int q = 0; q < GU; q++) i[q] = j0 + q * GB < b ? S.ub[j0 + q * GB] : 0u;
#pragma unroll
        for (int q = 0; q < GU; q++) {
          p[q] = j0 + q * GB < b ? S.bp[i[q]] : 0u;
          sz[q] = j0 + q * GB < b ? S.S[i[q]] : 0u;
        }
#pragma unroll
        for (int q = 0; q < GU; q++) po[q] = j0 + q * GB < b ? S.po[p[q]] : 0u;
#pragma unroll
        for (int q = 0; q < GU; q++)
          if (j0 + q * GB < b) atomicAdd(&lw[po[q]], sz[q]);
      }
      __syncthreads();
      for (uint32_t j0 = pa + tid; j0 < a; j0 += GB * GU) {
        uint32_t i[GU], po[GU];
#pragma unroll
        for (int q = 0; q < GU; q++) i[q] = j0 + q * GB < a ? S.ub[j0 + q * GB] : 0u;
#pragma unroll
        for (int q = 0; q < GU; q++) po[q] = j0 + q * GB < a ? S.po[i[q]] : 0u;
#pragma unroll
        for (int q = 0; q < GU; q++)
          if (j0 + q * GB < a) S.S[i[q]] = 1u + lw[po[q]];
      }
      __syncthreads();
    } else {
      for (uint32_t j = a + tid; j < b; j += GB) {
        const uint32_t i = S.ub[j];
        atomicAdd(&S.S[S.bp[i]], S.S[i]);
      }
      __syncthreads();
    }
  }
  for (uint32_t i0 = tid; i0 < n; i0 += GB * GU) {
    uint32_t k[GU], po[GU], sz[GU], base[GU];
#pragma unroll
    for (int q = 0; q < GU; q++) {
      const bool in = i0 + q * GB < n;
      k[q] = in ? (uint32_t)S.up[i0 + q * GB] : 0u;
      po[q] = in ? S.po[i0 + q * GB] : 0u;
      sz[q] = in ? S.S[i0 + q * GB] : 0u;
    }
#pragma unroll
    for (int q = 0; q < GU; q++) base[q] = S.uoff[k[q]];
#pragma unroll
    for (int q = 0; q < GU; q++)
      if (i0 + q * GB < n) S.A[base[q] + po[q]] = sz[q];
  }
  __syncthreads();
  block_scan_inplace<GB, 16>(S.A, n, s_lds);
  for (uint32_t i0 = tid; i0 < n; i0 += GB * GU) {
    uint32_t k[GU], po[GU], fp[GU], base[GU], a1[GU], a0[GU];
#pragma unroll
    for (int q = 0; q < GU; q++) {
      const bool in = i0 + q * GB < n;
      k[q] = in ? (uint32_t)S.up[i0 + q * GB] : 0u;
      po[q] = in ? S.po[i0 + q * GB] : 0u;
      fp[q] = in ? S.fpos[i0 + q * GB] : 0u;
    }
#pragma unroll
    for (int q = 0; q < GU; q++) base[q] = S.uoff[k[q]];
#pragma unroll
    for (int q = 0; q < GU; q++) {
      a1[q] = S.A[base[q] + po[q]];
      a0[q] = S.A[base[q] + fp[q]];
    }
#pragma unroll
    for (int q = 0; q < GU; q++) {
      const uint32_t i = i0 + q * GB;
      if (i >= n) continue;
      va[i] = a1[q] - a0[q];
      if (k[q] == 0) hd[i] = i;
    }
  }
  __syncthreads();
  for (uint32_t k = 1; k <= maxup; k++) {
    for (uint32_t j0 = S.uoff[k] + tid; j0 < S.uoff[k + 1]; j0 += GB * GU) {
      uint32_t i[GU], p[GU], v[GU], vp[GU], hp[GU];
      const uint32_t b = S.uoff[k + 1];
#pragma unroll
      for (int q = 0; q < GU; q++) i[q] = j0 + q * GB < b ? S.ub[j0 + q * GB] : GNIL;
#pragma unroll
      for (int q = 0; q < GU; q++) {
        p[q] = i[q] != GNIL ? S.bp[i[q]] : 0u;
        v[q] = i[q] != GNIL ? va[i[q]] : 0u;
      }
#pragma unroll
      for (int q = 0; q < GU; q++) {
        vp[q] = i[q] != GNIL ? va[p[q]] : 0u;
        hp[q] = i[q] != GNIL ? hd[p[q]] : 0u;
      }
#pragma unroll
      for (int q = 0; q < GU; q++)
        if (i[q] != GNIL) {
          va[i[q]] = v[q] + vp[q];
          hd[i[q]] = hp[q];
        }
    }
    __syncthreads();
  }
  STAMP(6);
  GSTOP(6);
  // one representative per accepted path (the witness whose best parent does not continue into it)
  // (GU nodes per thread per round, each round's gathers in flight together)
  for (uint32_t i0 = 0; i0 < n; i0 += GB * GU) {
    uint32_t up[GU], bp[GU], nb[GU], h[GU], t[GU], dn[GU], ch[GU];
#pragma unroll
    for (int q = 0; q < GU; q++) {
      const uint32_t i = i0 + q * GB + tid;
      const bool in = i < n;
      up[q] = in ? (uint32_t)S.up[i] : 0u;
      bp[q] = in ? S.bp[i] : 0u;
      h[q] = in ? hd[i] : 0u;
      t[q] = in ? tl[i] : 0u;
      dn[q] = in ? (uint32_t)S.down[i] : 0u;
    }
#pragma unroll
    for (int q = 0; q < GU; q++) {
      nb[q] = up[q] ? S.nxt[bp[q]] : 0u;
      ch[q] = S.crank[h[q]];
    }
#pragma unroll
    for (int q = 0; q < GU; q++) {
      const uint32_t i = i0 + q * GB + tid;
      const bool rep = i < n && (up[q] == 0 || nb[q] != i);
      const uint64_t m = __ballot(rep);  // one LDS atomic per wave
      uint32_t b = 0;
      if (m && lane_id() == 0) b = atomicAdd(&s_nch, (uint32_t)__popcll(m));
      b = __builtin_amdgcn_readlane(b, 0);
      if (!rep) continue;
      uint32_t *r = tmp + 5 * (b + mbcnt(m));
      r[0] = h[q];
      r[1] = t[q];
      r[2] = up[q] + dn[q];
      r[3] = ch[q];
      r[4] = i;
    }
  }
  __threadfence_block();
  __syncthreads();
  const uint32_t nch = s_nch;
  STAMP(7);
  GSTOP(7);
  // ---- acceptance order (len desc, preorder asc) -------------------------------------
  // pre = va + up is the representative's preorder index (unique, < n): the chains
  // laid out by it are already in preorder; a stable LSD counting sort by
  // (maxlen - len), 4 bits a pass, each thread a contiguous chunk, then orders them
  // by length.  (A bitonic network over the padded key array made ~190 passes.)
  for (uint32_t i = tid; i < n; i += GB) S.grp[i] = GNIL;
  __syncthreads();
  for (uint32_t q0 = tid; q0 < nch; q0 += GB * GU) {  // chain of each preorder index
    uint32_t rp[GU], v[GU], u[GU];
#pragma unroll
    for (int q = 0; q < GU; q++) rp[q] = q0 + q * GB < nch ? tmp[5 * (q0 + q * GB) + 4] : 0u;
#pragma unroll
    for (int q = 0; q < GU; q++) {
      v[q] = va[rp[q]];
      u[q] = (uint32_t)S.up[rp[q]];
    }
#pragma unroll
    for (int q = 0; q < GU; q++)
      if (q0 + q * GB < nch) S.grp[v[q] + u[q]] = q0 + q * GB;
  }
  __syncthreads();
  unsigned long long *ka = S.key, *kb = S.key + nch;  // nch <= n <= V: both fit the 2V keys
  {
    uint32_t o = 0;
    for (uint32_t b0 = 0; b0 < n; b0 += GB * CP) {
      const uint32_t p0 = b0 + tid * CP;
      uint32_t qv[CP], cl = 0;
#pragma unroll
      for (int q = 0; q < CP; q++) {
        qv[q] = p0 + q < n ? S.grp[p0 + q] : GNIL;
        cl += qv[q] != GNIL ? 1u : 0u;
      }
      uint32_t tot;
      uint32_t i = block_exscan<GB>(cl, &tot, s_lds) + o;
#pragma unroll
      for (int q = 0; q < CP; q++)
        if (qv[q] != GNIL)
          ka[i++] = ((unsigned long long)(maxlen - tmp[5 * qv[q] + 2]) << 32) | (p0 + (uint32_t)q);
      o += tot;
    }
  }
  __syncthreads();
  static_assert(16 * 512 <= sizeof(GSweepLds) / 4, "per-thread digit counters fit the sweeps' LDS");
  const uint32_t kbits = 32u - (uint32_t)__clz((int)max(maxlen, 1u));
  for (uint32_t sh = 32; sh < 32 + kbits; sh += 4) {
    const uint32_t per = (nch + GB - 1) / GB, a = min(nch, tid * per), z = min(nch, a + per);
#pragma unroll
    for (int d = 0; d < 16; d++) lw[d * GB + tid] = 0;  // thread tid's column: no conflicts, no atomics
    for (uint32_t i = a; i < z; i++) lw[((uint32_t)(ka[i] >> sh) & 15u) * GB + tid]++;
    __syncthreads();
    block_scan_inplace<GB>(lw, 16 * GB, s_lds);  // digit-major: bases in (digit, thread) order
    for (uint32_t i = a; i < z; i++) {
      const unsigned long long x = ka[i];
      kb[lw[((uint32_t)(x >> sh) & 15u) * GB + tid]++] = x;
    }
    __syncthreads();
    unsigned long long *t = ka;
    ka = kb;
    kb = t;
  }
  STAMP(8);
  GSTOP(8);
  uint32_t *out = c.chain + 5 * gv.n0;
  for (uint32_t p0 = tid; p0 < nch; p0 += GB * GU) {
    uint32_t q[GU], h[GU], t[GU], l[GU], hh[GU], tt[GU];
#pragma unroll
    for (int k = 0; k < GU; k++) q[k] = p0 + k * GB < nch ? S.grp[(uint32_t)(ka[p0 + k * GB] & 0xFFFFFFFFu)] : 0u;
#pragma unroll
    for (int k = 0; k < GU; k++) {
      h[k] = tmp[5 * q[k]];
      t[k] = tmp[5 * q[k] + 1];
      l[k] = tmp[5 * q[k] + 2];
    }
#pragma unroll
    for (int k = 0; k < GU; k++) {
      hh[k] = hs[h[k]];
      tt[k] = hs[t[k]];
    }
#pragma unroll
    for (int k = 0; k < GU; k++) {
      if (p0 + k * GB >= nch) continue;
      uint32_t *w = out + 5 * (p0 + k * GB);
      w[0] = hh[k];
      w[1] = tt[k];
      w[2] = l[k];
      w[3] = gv.rank_of(hh[k]);
      w[4] = 0;
    }
  }
  STAMP(9);
  if (tid == 0) {
    c.nch[g] = nch;
    if (s_fail) c.err[g] = NEMO_ERR_INVALID;
  }
}

uint32_t glob_team_words() { return PT_TEAMS * PT_WORDS; }

void launch_chains_glob(const DevCorpus &c, hipStream_t s) {
  if (!c.gscratch) return;
  if (c.glob_prep) {
    launch_zero(c.team, PT_TEAMS * PT_WORDS * sizeof(uint32_t), s);
    // every member of a team must be resident at once (team barriers spin): the whole grid of
    // PT_B-thread workgroups must fit the device's CUs at the kernel's occupancy, which the
    // runtime reports; the grid never asks for more workgroups than that
    static int occ = -1;
    if (occ < 0) {
      int n = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_glob_prep, PT_B, 0) != hipSuccess) {
        (void)hipGetLastError();
        n = 1;
      }
      occ = std::max(1, n);
    }
    const uint32_t fit = (uint32_t)occ * c.n_cu / PT_TEAMS;  // members per team the device holds at once
    const uint32_t m = std::max(1u, std::min<uint32_t>({PT_M, c.n_cu / PT_TEAMS, fit}));
    hipLaunchKernelGGL(k_glob_prep, dim3(PT_TEAMS * m), dim3(PT_B), 0, s, c);
  }
  if (c.glob_block == 512)
    hipLaunchKernelGGL(k_chains_glob<512>, dim3(c.G), dim3(512), 0, s, c);
  else
    hipLaunchKernelGGL(k_chains_glob<256>, dim3(c.G), dim3(256), 0, s, c);
}

}  // namespace nemo
