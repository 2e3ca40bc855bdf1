// k_load.hip — device side of loadProv (graphing/pre-post-prov.go:25-213):
// per-graph CSR build with the reference's edge validations, and Kahn levels.
#include "device.h"
#include "internal.h"

namespace nemo {

__device__ void sort_row(uint32_t *r, uint32_t n) {
  if (n <= 32) {
    for (uint32_t i = 1; i < n; i++) {
      uint32_t x = r[i], j = i;
      while (j > 0 && r[j - 1] > x) {
        r[j] = r[j - 1];
        j--;
      }
      r[j] = x;
    }
    return;
  }
  // heap sort for long rows
  auto sift = [&](uint32_t s, uint32_t end) {
    while (2 * s + 1 < end) {
      uint32_t ch = 2 * s + 1;
      if (ch + 1 < end && r[ch] < r[ch + 1]) ch++;
      if (r[s] >= r[ch]) return;
      uint32_t t = r[s];
      r[s] = r[ch];
      r[ch] = t;
      s = ch;
    }
  };
  for (uint32_t s = n / 2; s-- > 0;) sift(s, n);
  for (uint32_t end = n; end-- > 1;) {
    uint32_t t = r[0];
    r[0] = r[end];
    r[end] = t;
    sift(0, end);
  }
}

// CSR (forward + reverse) of every graph; rows sorted so that a merged
// duplicate DUETO edge is adjacent.  relationships-created counts edges that
// are neither duplicates nor goal->goal / rule->rule (pre-post-prov.go:150-210).
// Graphs with V < CSR_LDS count degrees, scan and hand out cursors in LDS;
// larger ones do the same with global atomics.
#define CSR_LDS 8192
__global__ __launch_bounds__(NEMO_BLOCK) void k_csr(DevCorpus c) {
  __shared__ uint32_t s_cnt[CSR_LDS];
  __shared__ uint32_t s_lds[NEMO_WAVES];
  __shared__ uint32_t s_bad, s_created;
  const uint32_t g = blockIdx.x;
  const uint64_t n0 = c.node_off[g], e0 = c.edge_off[g];
  const uint32_t V = (uint32_t)(c.node_off[g + 1] - n0), E = (uint32_t)(c.edge_off[g + 1] - e0);
  uint32_t *fp = c.fp + n0 + g, *rp = c.rp + n0 + g, *fc = c.fc + e0, *rc = c.rc + e0;
  const uint32_t *es = c.esrc + e0, *ed = c.edst + e0, *word = c.word + n0;
  if (threadIdx.x == 0) {
    s_bad = 0;
    s_created = 0;
  }
  for (uint32_t e = threadIdx.x; e < E; e += NEMO_BLOCK)
    if (es[e] >= V || ed[e] >= V) s_bad = 1;
  __syncthreads();
  if (s_bad) {
    if (threadIdx.x == 0) c.err[g] = NEMO_ERR_INVALID;
    return;
  }
  if (V < CSR_LDS) {
    for (int dir = 0; dir < 2; dir++) {
      const uint32_t *key = dir ? ed : es, *val = dir ? es : ed;
      uint32_t *ptr = dir ? rp : fp, *col = dir ? rc : fc;
      for (uint32_t v = threadIdx.x; v <= V; v += NEMO_BLOCK) s_cnt[v] = 0;
      __syncthreads();
      for (uint32_t e = threadIdx.x; e < E; e += NEMO_BLOCK) atomicAdd(&s_cnt[key[e]], 1u);
      __syncthreads();
      block_scan_inplace(s_cnt, V + 1, s_lds);
      for (uint32_t v = threadIdx.x; v <= V; v += NEMO_BLOCK) ptr[v] = s_cnt[v];
      __syncthreads();
      for (uint32_t e = threadIdx.x; e < E; e += NEMO_BLOCK) col[atomicAdd(&s_cnt[key[e]], 1u)] = val[e];
      __syncthreads();
    }
  } else {
    uint32_t *cf = c.s_a + n0 + g, *cr = c.s_b + n0 + g;
    for (uint32_t v = threadIdx.x; v <= V; v += NEMO_BLOCK) {
      fp[v] = 0;
      rp[v] = 0;
    }
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < E; e += NEMO_BLOCK) {
      atomicAdd(&fp[es[e]], 1u);
      atomicAdd(&rp[ed[e]], 1u);
    }
    __syncthreads();
    block_scan_inplace(fp, V + 1, s_lds);
    block_scan_inplace(rp, V + 1, s_lds);
    for (uint32_t v = threadIdx.x; v < V; v += NEMO_BLOCK) {
      cf[v] = fp[v];
      cr[v] = rp[v];
    }
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < E; e += NEMO_BLOCK) {
      const uint32_t s = es[e], d = ed[e];
      fc[atomicAdd(&cf[s], 1u)] = d;
      rc[atomicAdd(&cr[d], 1u)] = s;
    }
    __syncthreads();
  }
  __threadfence_block();
  uint32_t created = 0;
  for (uint32_t v = threadIdx.x; v < V; v += NEMO_BLOCK) {
    const uint32_t a = fp[v], b = fp[v + 1];
    sort_row(fc + a, b - a);
    sort_row(rc + rp[v], rp[v + 1] - rp[v]);
    const bool rv = is_rule(word[v]);
    for (uint32_t j = a; j < b; j++) {
      const uint32_t t = fc[j];
      const bool dup = j > a && fc[j - 1] == t;
      if (!dup && rv != is_rule(word[t])) created++;
    }
  }
  atomicAdd(&s_created, created);
  __syncthreads();
  if (threadIdx.x == 0) {
    c.created[g] = s_created;
    c.err[g] = (s_created == E) ? 0u : (uint32_t)NEMO_ERR_LOAD;
  }
}

// Kahn levels: topo[] lists the graph's nodes level by level, lvl[l]..lvl[l+1]
// is level l (longest path from a source).  A graph with a cycle is refused.
__global__ __launch_bounds__(NEMO_BLOCK) void k_topo(DevCorpus c) {
  __shared__ uint32_t s_tail;
  const uint32_t g = blockIdx.x;
  if (c.err[g]) return;
  const uint64_t n0 = c.node_off[g], e0 = c.edge_off[g];
  const uint32_t V = (uint32_t)(c.node_off[g + 1] - n0);
  const uint32_t *fp = c.fp + n0 + g, *rp = c.rp + n0 + g, *fc = c.fc + e0;
  uint32_t *topo = c.topo + n0, *lvl = c.lvl + n0 + g, *cnt = c.s_a + n0 + g;
  if (threadIdx.x == 0) s_tail = 0;
  for (uint32_t v = threadIdx.x; v < V; v += NEMO_BLOCK) cnt[v] = rp[v + 1] - rp[v];
  __syncthreads();
  for (uint32_t base = 0; base < V; base += NEMO_BLOCK) {
    const uint32_t v = base + threadIdx.x;
    wave_append(v < V && cnt[v] == 0u, v, topo, &s_tail);
  }
  __syncthreads();
  uint32_t lo = 0, hi = s_tail, nl = 0;
  if (threadIdx.x == 0) lvl[0] = 0;
  __syncthreads();
  while (lo < hi) {
    for (uint32_t base = lo; base < hi; base += NEMO_BLOCK) {
      const uint32_t i = base + threadIdx.x;
      uint32_t j = 0, je = 0;
      if (i < hi) {
        const uint32_t u = topo[i];
        j = fp[u];
        je = fp[u + 1];
      }
      while (__any(j < je)) {
        bool p = false;
        uint32_t ch = 0;
        if (j < je) {
          ch = fc[j++];
          p = atomicSub(&cnt[ch], 1u) == 1u;
        }
        wave_append(p, ch, topo, &s_tail);
      }
    }
    __syncthreads();
    nl++;
    lo = hi;  // level nl-1 is topo[lvl[nl-1] .. lo)
    hi = s_tail;
    if (threadIdx.x == 0) lvl[nl] = lo;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    c.nlev[g] = nl;
    if (hi != V) c.err[g] = NEMO_ERR_CYCLE;
  }
}

void launch_load(const DevCorpus &c, hipStream_t s) {
  hipLaunchKernelGGL(k_csr, dim3(c.G), dim3(NEMO_BLOCK), 0, s, c);
}
void launch_topo(const DevCorpus &c, hipStream_t s) {
  hipLaunchKernelGGL(k_topo, dim3(c.G), dim3(NEMO_BLOCK), 0, s, c);
}

}  // namespace nemo
