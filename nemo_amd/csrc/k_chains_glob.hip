// k_chains_glob.hip — collapseNextChains' greedy chain cover
// (graphing/preprocessing.go:70-138) for deep graphs: the closed form of
// k_chains (accepted paths = {first(v) : v in H*}, acceptance order = length
// desc then the preorder of the representatives in the best-prefix forest)
// with every per-node array in a global scratch region, so it scales to
// chain subgraphs of hundreds of thousands of nodes and thousands of levels
// (1M-node graphs, EOT ~ 2000).  One 1024-thread workgroup per
// graph; long walks (chain heads and tails, ancestor sums) use pointer
// jumping, the final order a bitonic sort of 64-bit keys.  The graphs are the
// ones the host gave a scratch region (DevCorpus::gs_off, V >= glob_min_v);
// k_chains and k_chains_big skip them.
#include "device.h"
#include "internal.h"

namespace nemo {

#define GB 1024  // threads per workgroup
#define GNIL 0xFFFFFFFFu

// Scratch layout (u32 units) for a graph of V nodes and E edges.
struct GlobScratch {
  uint32_t *seg, *cur, *bm, *bmpre, *crank, *rule;
  uint32_t *ccoff, *pcoff, *ccur, *pcur, *child, *par;
  int32_t *up, *down;
  uint32_t *nxt, *bp, *po, *fpos, *ub, *uoff, *cnt, *grp;
  uint32_t *ha, *hb, *ta, *tb;  // pointer-jumping buffers (heads, tails)
  uint32_t *S, *A, *va, *vb, *pa, *pb;
  unsigned long long *key;      // up to 2V keys (power-of-two padded chain count)
};

uint64_t glob_words(uint64_t V, uint64_t E) {
  const uint64_t w = (V + 31) / 32 + 2;
  return 2 * (V + 1) + 2 * w + 4 * (V + 1) + 2 * E + 2 * (V + 2) + 20 * V + 4 * V + 64;
}

__device__ inline GlobScratch glob_carve(uint32_t *p, uint32_t V, uint32_t E) {
  GlobScratch s;
  const uint32_t w = (V + 31) / 32 + 2;
  auto take = [&](uint64_t n) {
    uint32_t *q = p;
    p += n;
    return q;
  };
  s.seg = take(V + 1);
  s.cur = take(V + 1);
  s.bm = take(w);
  s.bmpre = take(w);
  s.crank = take(V);
  s.rule = take(V);
  s.ccoff = take(V + 1);
  s.pcoff = take(V + 1);
  s.ccur = take(V + 1);
  s.pcur = take(V + 1);
  s.child = take(E);
  s.par = take(E);
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
  s.va = take(V);
  s.vb = take(V);
  s.pa = take(V);
  s.pb = take(V);
  p = (uint32_t *)(((uintptr_t)p + 7) & ~(uintptr_t)7);
  s.key = (unsigned long long *)p;
  return s;
}

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

__global__ __launch_bounds__(GB) void k_chains_glob(DevCorpus c) {
  __shared__ uint32_t s_lds[GB / 64];
  __shared__ uint32_t s_nch, s_fail;
  const uint32_t g = blockIdx.x, tid = threadIdx.x;
  if (c.err[g] || c.gs_off[g] == ~0ull) return;
  const GraphView gv = c.view(g);
  const uint32_t V = gv.V, E = gv.E, ns = gv.nlev;
  GlobScratch S = glob_carve(c.gscratch + c.gs_off[g], V, E);
  uint32_t *hs = c.s_a + gv.n0 + g;    // compact index -> graph-local node
  uint32_t *hidx = c.s_f + gv.n0 + g;  // graph-local node -> compact index
  uint32_t *tmp = c.chain_tmp + 5 * gv.n0;
  const uint8_t *f = gv.flags;
  const uint32_t *nlv = c.nlv + gv.n0;
  const uint32_t nw = (V + 31) / 32;
  if (tid == 0) {
    s_nch = 0;
    s_fail = 0;
  }
  STAMP(0);
  // ---- H* in level order, compact ID ranks ------------------------------------
  for (uint32_t l = tid; l <= ns; l += GB) S.seg[l] = 0;
  for (uint32_t w = tid; w < nw; w += GB) S.bm[w] = 0;
  __syncthreads();
  for (uint32_t x = tid; x < V; x += GB)
    if (f[x] & NEMO_F_DELETED) atomicAdd(&S.seg[nlv[x]], 1u);
  __syncthreads();
  const uint32_t n = block_scan_inplace<GB, 16>(S.seg, ns + 1, s_lds);
  if (n == 0) {
    if (tid == 0) c.nch[g] = 0;
    return;
  }
  for (uint32_t l = tid; l <= ns; l += GB) S.cur[l] = S.seg[l];
  __syncthreads();
  for (uint32_t x = tid; x < V; x += GB) {
    if (!(f[x] & NEMO_F_DELETED)) continue;
    const uint32_t i = atomicAdd(&S.cur[nlv[x]], 1u);
    hs[i] = x;
    hidx[x] = i;
    S.rule[i] = is_rule(gv.word[x]) ? 1u : 0u;
    const uint32_t r = gv.rank_of(x);
    S.crank[i] = r;
    atomicOr(&S.bm[r >> 5], 1u << (r & 31));
  }
  __syncthreads();
  for (uint32_t w = tid; w < nw; w += GB) S.bmpre[w] = __popc(S.bm[w]);
  __syncthreads();
  block_scan_inplace<GB, 16>(S.bmpre, nw, s_lds);
  for (uint32_t i = tid; i < n; i += GB) {
    const uint32_t r = S.crank[i];
    S.crank[i] = S.bmpre[r >> 5] + __popc(S.bm[r >> 5] & ((1u << (r & 31)) - 1u));
  }
  STAMP(1);
  // ---- H* adjacency (rows in any order: every consumer takes a max/min) ---------
  for (uint32_t i = tid; i <= n; i += GB) {
    S.ccoff[i] = 0;
    S.pcoff[i] = 0;
  }
  __syncthreads();
  const uint32_t *es = c.esrc + gv.e0, *ed = c.edst + gv.e0;
#define INH(v) ((f[v] & NEMO_F_DELETED) != 0)
  for (uint32_t e = tid; e < E; e += GB) {
    const uint32_t a = es[e], b = ed[e];
    if (!INH(a) || !INH(b)) continue;
    atomicAdd(&S.ccoff[hidx[a]], 1u);
    atomicAdd(&S.pcoff[hidx[b]], 1u);
  }
  __syncthreads();
  block_scan_inplace<GB, 16>(S.ccoff, n + 1, s_lds);
  block_scan_inplace<GB, 16>(S.pcoff, n + 1, s_lds);
  for (uint32_t i = tid; i < n; i += GB) {
    S.ccur[i] = S.ccoff[i];
    S.pcur[i] = S.pcoff[i];
  }
  __syncthreads();
  for (uint32_t e = tid; e < E; e += GB) {
    const uint32_t a = es[e], b = ed[e];
    if (!INH(a) || !INH(b)) continue;
    const uint32_t ia = hidx[a], ib = hidx[b];
    S.child[atomicAdd(&S.ccur[ia], 1u)] = ib;
    S.par[atomicAdd(&S.pcur[ib], 1u)] = ia;
  }
#undef INH
  __syncthreads();
  STAMP(2);
  // ---- up (forward) and down/nxt (backward), half the workgroup each -------------
  {
    constexpr uint32_t HALF = GB / 2;
    const bool upper = tid < HALF;
    const uint32_t ht = upper ? tid : tid - HALF;
    for (uint32_t s = 0; s < ns; s++) {
      if (upper) {
        for (uint32_t i = S.seg[s] + ht; i < S.seg[s + 1]; i += HALF) {
          int32_t d = S.rule[i] ? 0 : -1;
          for (uint32_t j = S.pcoff[i]; j < S.pcoff[i + 1]; j++) d = max(d, S.up[S.par[j]] + 1);
          S.up[i] = d;
        }
      } else {
        const uint32_t sd = ns - 1 - s;
        for (uint32_t i = S.seg[sd] + ht; i < S.seg[sd + 1]; i += HALF) {
          int32_t best = -1;
          uint32_t bc = GNIL, br = GNIL;
          for (uint32_t j = S.ccoff[i]; j < S.ccoff[i + 1]; j++) {
            const uint32_t w = S.child[j];
            const int32_t dw = S.down[w];
            const uint32_t rw = S.crank[w];
            if (dw > best || (dw == best && rw < br)) {
              best = dw;
              bc = w;
              br = rw;
            }
          }
          int32_t d = best >= 0 ? best + 1 : (S.rule[i] ? 0 : -1);
          if (S.rule[i] && d < 0) d = 0;
          if (d > 0 && best < 0) bc = GNIL;
          S.down[i] = d;
          S.nxt[i] = d > 0 ? bc : GNIL;
          if (d < 0) s_fail = 1;  // a goal without a chain continuation: impossible on H*
        }
      }
      __syncthreads();
    }
  }
  STAMP(3);
  uint32_t mu = 0, ml = 0;
  for (uint32_t i = tid; i < n; i += GB) {
    mu = max(mu, (uint32_t)max(S.up[i], 0));
    ml = max(ml, (uint32_t)max(S.up[i] + S.down[i], 0));
  }
  const uint32_t maxup = gmax_u32(mu, s_lds);
  const uint32_t maxlen = gmax_u32(ml, s_lds);
  // ---- bucket by up -----------------------------------------------------------------
  for (uint32_t k = tid; k <= maxup + 1; k += GB) S.uoff[k] = 0;
  __syncthreads();
  for (uint32_t i = tid; i < n; i += GB) atomicAdd(&S.uoff[S.up[i]], 1u);
  __syncthreads();
  block_scan_inplace<GB, 16>(S.uoff, maxup + 2, s_lds);
  for (uint32_t k = tid; k <= maxup + 1; k += GB) S.cnt[k] = S.uoff[k];
  __syncthreads();
  for (uint32_t i = tid; i < n; i += GB) S.ub[atomicAdd(&S.cnt[S.up[i]], 1u)] = i;
  // best parent fixed up front where only one parent has up == up(v) - 1
  constexpr uint32_t MULTI = 0xFFFFFFFEu;
  for (uint32_t i = tid; i < n; i += GB) {
    const int32_t k = S.up[i];
    uint32_t cand = GNIL, cn = 0;
    if (k > 0)
      for (uint32_t q = S.pcoff[i]; q < S.pcoff[i + 1]; q++)
        if (S.up[S.par[q]] == k - 1) {
          cn++;
          cand = S.par[q];
        }
    S.bp[i] = cn > 1 ? MULTI : cand;
  }
  __syncthreads();
  STAMP(4);
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
    for (uint32_t w = tid; w <= mp; w += GB) S.cnt[w] = 0;
    __syncthreads();
    for (uint32_t j = a + tid; j < b; j += GB) {
      const uint32_t i = S.ub[j];
      uint32_t bpi = S.bp[i];
      if (bpi == MULTI) {
        uint32_t bpo = GNIL;
        for (uint32_t q = S.pcoff[i]; q < S.pcoff[i + 1]; q++) {
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
  // ---- heads (roots of the bp forest) and tails (ends of nxt) by pointer jumping -----
  uint32_t *h0 = S.ha, *h1 = S.hb, *t0 = S.ta, *t1 = S.tb;
  for (uint32_t i = tid; i < n; i += GB) {
    h0[i] = S.up[i] > 0 ? S.bp[i] : i;
    t0[i] = S.nxt[i] != GNIL ? S.nxt[i] : i;
  }
  __syncthreads();
  for (uint32_t span = 1; span <= maxlen; span <<= 1) {
    for (uint32_t i = tid; i < n; i += GB) {
      h1[i] = h0[h0[i]];
      t1[i] = t0[t0[i]];
    }
    __syncthreads();
    uint32_t *x = h0;
    h0 = h1;
    h1 = x;
    x = t0;
    t0 = t1;
    t1 = x;
  }
  // one representative per accepted path (the witness whose best parent does not continue into it)
  for (uint32_t i = tid; i < n; i += GB) {
    const bool rep = S.up[i] == 0 || S.nxt[S.bp[i]] != i;
    if (!rep) continue;
    const uint32_t k = atomicAdd(&s_nch, 1u);
    uint32_t *r = tmp + 5 * k;
    r[0] = h0[i];
    r[1] = t0[i];
    r[2] = (uint32_t)(S.up[i] + S.down[i]);
    r[3] = S.crank[h0[i]];
    r[4] = i;
  }
  __threadfence_block();
  __syncthreads();
  const uint32_t nch = s_nch;
  STAMP(6);
  // ---- preorder of the representatives: pre(v) = up(v) + sum of off over v and its bp
  // ancestors, off = sizes of the earlier siblings (sizes laid out in (level, po) order)
  for (uint32_t i = tid; i < n; i += GB) S.S[i] = 1;
  __syncthreads();
  for (uint32_t k = maxup; k >= 1; k--) {
    for (uint32_t j = S.uoff[k] + tid; j < S.uoff[k + 1]; j += GB) {
      const uint32_t i = S.ub[j];
      atomicAdd(&S.S[S.bp[i]], S.S[i]);
    }
    __syncthreads();
  }
  for (uint32_t i = tid; i < n; i += GB) S.A[S.uoff[S.up[i]] + S.po[i]] = S.S[i];
  __syncthreads();
  block_scan_inplace<GB, 16>(S.A, n, s_lds);
  uint32_t *va = S.va, *vb = S.vb, *pa = S.pa, *pb = S.pb;
  for (uint32_t i = tid; i < n; i += GB) {
    const uint32_t k = S.up[i], base = S.uoff[k];
    va[i] = S.A[base + S.po[i]] - S.A[base + S.fpos[i]];
    pa[i] = k ? S.bp[i] : GNIL;
  }
  __syncthreads();
  for (uint32_t r = 1; r <= maxup; r <<= 1) {
    for (uint32_t i = tid; i < n; i += GB) {
      const uint32_t p = pa[i];
      if (p != GNIL) {
        vb[i] = va[i] + va[p];
        pb[i] = pa[p];
      } else {
        vb[i] = va[i];
        pb[i] = GNIL;
      }
    }
    __syncthreads();
    uint32_t *x = va;
    va = vb;
    vb = x;
    x = pa;
    pa = pb;
    pb = x;
  }
  STAMP(7);
  // ---- acceptance order: keys (len desc, preorder asc) are unique; bitonic sort -------
  uint32_t N2 = 1;
  while (N2 < nch) N2 <<= 1;
  for (uint32_t q = tid; q < N2; q += GB) {
    unsigned long long key = ~0ull;
    if (q < nch) {
      const uint32_t len = tmp[5 * q + 2], rep = tmp[5 * q + 4];
      key = ((unsigned long long)(0xFFFFFFFFu - len) << 32) | (va[rep] + (uint32_t)S.up[rep]);
    }
    S.key[q] = key;
  }
  // chain of each preorder index (grp is free again)
  for (uint32_t q = tid; q < nch; q += GB) {
    const uint32_t rep = tmp[5 * q + 4];
    S.grp[va[rep] + (uint32_t)S.up[rep]] = q;
  }
  __syncthreads();
  for (uint32_t k = 2; k <= N2; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = tid; i < N2; i += GB) {
        const uint32_t ixj = i ^ j;
        if (ixj > i) {
          const unsigned long long x = S.key[i], y = S.key[ixj];
          if ((x > y) == ((i & k) == 0)) {
            S.key[i] = y;
            S.key[ixj] = x;
          }
        }
      }
      __syncthreads();
    }
  }
  STAMP(8);
  uint32_t *out = c.chain + 5 * gv.n0;
  for (uint32_t pos = tid; pos < nch; pos += GB) {
    const uint32_t q = S.grp[(uint32_t)(S.key[pos] & 0xFFFFFFFFu)];
    uint32_t *w = out + 5 * pos;
    w[0] = hs[tmp[5 * q]];
    w[1] = hs[tmp[5 * q + 1]];
    w[2] = tmp[5 * q + 2];
    w[3] = gv.rank_of(w[0]);
    w[4] = 0;
  }
  STAMP(9);
  if (tid == 0) {
    c.nch[g] = nch;
    if (s_fail) c.err[g] = NEMO_ERR_INVALID;
  }
}

void launch_chains_glob(const DevCorpus &c, hipStream_t s) {
  if (!c.gscratch) return;
  hipLaunchKernelGGL(k_chains_glob, dim3(c.G), dim3(GB), 0, s, c);
}

}  // namespace nemo
