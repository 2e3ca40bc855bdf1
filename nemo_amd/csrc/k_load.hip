// k_load.hip — device side of loadProv (graphing/pre-post-prov.go:25-213):
// per-graph CSR build with the reference's edge validations, and Kahn levels.
#include <algorithm>

#include "device.h"
#include "internal.h"
#include "marksimp.h"

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

// Fused LDS tier of loadProv's device half for the bulk of a Molly corpus:
// reverse CSR, forward CSR and Kahn levels built in LDS, each output written
// once, coalesced.  The LDS image is sized per corpus (DevCorpus::bld_*): u16
// row pointers (counted and cursored with packed-u16 atomics), u16 columns,
// u8 in-degree counters (packed-u8 atomics) and a u16 level queue, so four
// workgroups share a CU.  A graph with an in-degree above 255 is flagged
// (redo) and rebuilt by k_csr + k_topo, which also take the graphs beyond
// the caps; both tiers produce the same outputs and validations.
#ifndef BLD_BLOCK
#define BLD_BLOCK 256  // k_build workgroup size (512: 3.91 ms against 3.66 at C3)
#endif
#define BLD_OCC(B) ((B) == 256 ? 4 : 6)  // waves per SIMD the register budget is cut for
#ifndef BLD_SQ
#define BLD_SQ 2    // rows per thread and round of the row sort (even; 4: no faster at C3, 128 VGPRs)
#endif
#ifndef BLD_KB
#define BLD_KB 4    // Kahn: children of a node processed per round
#endif


// 5-comparator sorting network for 4 keys
__device__ __forceinline__ void sort_net4(uint32_t *x) {
  constexpr int P[5][2] = {{0, 1}, {2, 3}, {0, 2}, {1, 3}, {1, 2}};
#pragma unroll
  for (int k = 0; k < 5; k++) {
    const uint32_t a = x[P[k][0]], b = x[P[k][1]];
    x[P[k][0]] = min(a, b);
    x[P[k][1]] = max(a, b);
  }
}

// 19-comparator sorting network for 8 keys (pads 0xFFFF sort last)
__device__ __forceinline__ void sort_net8(uint32_t *x) {
  constexpr int P[19][2] = {{0, 2}, {1, 3}, {4, 6}, {5, 7}, {0, 4}, {1, 5}, {2, 6}, {3, 7}, {0, 1}, {2, 3},
                            {4, 5}, {6, 7}, {2, 4}, {3, 5}, {1, 4}, {3, 6}, {1, 2}, {3, 4}, {5, 6}};
#pragma unroll
  for (int k = 0; k < 19; k++) {
    const uint32_t a = x[P[k][0]], b = x[P[k][1]];
    x[P[k][0]] = min(a, b);
    x[P[k][1]] = max(a, b);
  }
}

// 63-comparator odd-even merge network for 16 keys
__device__ __forceinline__ void sort_net16(uint32_t *x) {
  constexpr int P[63][2] = {
      {0, 1},   {2, 3},   {0, 2},   {1, 3},   {1, 2},   {4, 5},   {6, 7},   {4, 6},   {5, 7},   {5, 6},   {0, 4},
      {2, 6},   {2, 4},   {1, 5},   {3, 7},   {3, 5},   {1, 2},   {3, 4},   {5, 6},   {8, 9},   {10, 11}, {8, 10},
      {9, 11},  {9, 10},  {12, 13}, {14, 15}, {12, 14}, {13, 15}, {13, 14}, {8, 12},  {10, 14}, {10, 12}, {9, 13},
      {11, 15}, {11, 13}, {9, 10},  {11, 12}, {13, 14}, {0, 8},   {4, 12},  {4, 8},   {2, 10},  {6, 14},  {6, 10},
      {2, 4},   {6, 8},   {10, 12}, {1, 9},   {5, 13},  {5, 9},   {3, 11},  {7, 15},  {7, 11},  {3, 5},   {7, 9},
      {11, 13}, {1, 2},   {3, 4},   {5, 6},   {7, 8},   {9, 10},  {11, 12}, {13, 14}};
#pragma unroll
  for (int k = 0; k < 63; k++) {
    const uint32_t a = x[P[k][0]], b = x[P[k][1]];
    x[P[k][0]] = min(a, b);
    x[P[k][1]] = max(a, b);
  }
}

// k_build's row sort: rows v0 and v0 + B ([a, a + n) in col), both
// rows' LDS reads issued together and the entries sorted in registers (a row
// longer than RS: insertion sort in LDS); reverse rows (dir 0) also count the
// relationships created (pre-post-prov.go:150-210: distinct, goal<->rule).
template <int RS, int B, int NQ>
__device__ __forceinline__ uint32_t sort_row_pair(uint16_t *col, const uint32_t *s_rule, uint32_t E, uint32_t V,
                                                  int dir, uint32_t v0, const uint32_t *a, const uint32_t *n) {
  uint32_t x[NQ][RS], created = 0;
#pragma unroll
  for (int q = 0; q < NQ; q++)
#pragma unroll
    for (int i = 0; i < RS; i++) {
      const uint32_t y = col[min(a[q] + i, E - 1u)];  // clamped, unconditional: all reads in flight together
      x[q][i] = (uint32_t)i < n[q] ? y : 0xFFFFu;
    }
#pragma unroll
  for (int q = 0; q < NQ; q++) {
    const uint32_t v = v0 + q * B, b = a[q] + n[q];
    if (n[q] <= (uint32_t)RS) {
      if (n[q] >= 2) {
        if (RS == 4) sort_net4(x[q]);
        else if (RS == 8) sort_net8(x[q]);
        else sort_net16(x[q]);
#pragma unroll
        for (int i = 0; i < RS; i++)
          if ((uint32_t)i < n[q]) col[a[q] + i] = (uint16_t)x[q][i];
      }
      if (dir == 0 && n[q]) {
        const bool rv = (s_rule[v >> 5] >> (v & 31)) & 1u;
#pragma unroll
        for (int i = 0; i < RS; i++) {
          const uint32_t t = x[q][i], tw = min(t, V - 1u);
          const bool rt = (s_rule[tw >> 5] >> (tw & 31)) & 1u;
          created += (uint32_t)i < n[q] && !(i > 0 && x[q][i - 1] == t) && rv != rt;
        }
      }
      continue;
    }
    for (uint32_t i = a[q] + 1; i < b; i++) {  // long row: insertion sort in LDS
      const uint16_t y = col[i];
      uint32_t j = i;
      while (j > a[q] && col[j - 1] > y) {
        col[j] = col[j - 1];
        j--;
      }
      col[j] = y;
    }
    if (dir == 0) {
      const bool rv = (s_rule[v >> 5] >> (v & 31)) & 1u;
      for (uint32_t i = a[q]; i < b; i++) {
        const uint32_t t = col[i];
        const bool rt = (s_rule[t >> 5] >> (t & 31)) & 1u;
        if (!(i > a[q] && col[i - 1] == t) && rv != rt) created++;
      }
    }
  }
  return created;
}

__host__ __device__ uint32_t build_tier_bytes(uint32_t v, uint32_t e) {
  return lds_align(4u * ((v + 31u) / 32u)) + lds_align(2u * (v + 2u)) + lds_align(2u * e) + lds_align(v) +
         lds_align(2u * v);
}

// u16 LDS array -> u32 HBM array, four entries per thread and store (8-byte
// LDS read, 16-byte global store); src must be 8-byte aligned
template <int B>
__device__ __forceinline__ void lds16_to_hbm32(uint32_t *dst, const uint16_t *src, uint32_t n) {
  const uint32_t tid = threadIdx.x;
  for (uint32_t j = 4 * tid; j < n; j += 4 * B) {
    if (j + 3 < n) {
      const uint2 h = *(const uint2 *)(src + j);
      const uint4 w = make_uint4(h.x & 0xFFFFu, h.x >> 16, h.y & 0xFFFFu, h.y >> 16);
      __builtin_memcpy(dst + j, &w, 16);
    } else {
      for (uint32_t k = j; k < n; k++) dst[k] = src[k];
    }
  }
}

__device__ __forceinline__ bool build_fits(const DevCorpus &c, uint32_t V, uint32_t E) {
  return c.bld_bytes != 0u && V <= c.bld_v && E <= c.bld_e;
}

template <int B>
__global__ __launch_bounds__(B) __attribute__((amdgpu_waves_per_eu(BLD_OCC(B)))) void k_build(DevCorpus c) {
  constexpr int EPT = 8192 / B;  // edges per thread held in registers (bld_e <= 8192)
  extern __shared__ __align__(16) uint8_t dyn[];
  __shared__ uint32_t s_lds[B / 64];
  __shared__ uint32_t s_bad, s_created, s_tail, s_cnt[3];
  __shared__ uint32_t s_sink[64];  // per-lane no-op atomic targets (one bank each: no same-address serialisation)
  __shared__ uint32_t s_ms[3];
  const uint32_t g = blockIdx.x, tid = threadIdx.x;
  const uint64_t n0 = c.node_off[g], e0 = c.edge_off[g];
  const uint32_t V = (uint32_t)(c.node_off[g + 1] - n0), E = (uint32_t)(c.edge_off[g + 1] - e0);
  if (!build_fits(c, V, E)) return;
  uint8_t *p = dyn;
  uint32_t *s_rule = (uint32_t *)p;  // is_rule bitmap
  p += lds_align(4u * ((V + 31u) / 32u));
  uint16_t *ptr = (uint16_t *)p;  // counts -> row starts -> cursors (= row ends); u32-packed pairs
  uint32_t *ptr32 = (uint32_t *)p;
  p += lds_align(2u * (V + 2u));
  uint16_t *col = (uint16_t *)p;  // one direction's rows at a time
  p += lds_align(2u * E);
  uint8_t *cnt8 = p;  // in-degrees, u32-packed quads
  uint32_t *cnt32 = (uint32_t *)p;
  p += lds_align(V);
  uint16_t *q16 = (uint16_t *)p;  // Kahn order
  const uint32_t *es = c.esrc + e0, *ed = c.edst + e0, *word = c.word + n0;
  STAMP(10);
  // every load of the graph's input issued back to back: edge e = tid + q*BLOCK
  // as (src << 16 | dst), and the rule bits of the node words
  // (four consecutive edges per thread and 16-byte load; ~0u marks an empty
  // slot: a valid pair has src < 16384)
  uint32_t sd[EPT];
  bool bad = false;
#pragma unroll
  for (int g4 = 0; g4 < EPT / 4; g4++) {
    const uint32_t e0 = 4 * (g4 * B + tid);
    uint32_t xs[4], ys[4];
    if (e0 + 3 < E) {
      uint4 a4, b4;
      __builtin_memcpy(&a4, es + e0, 16);
      __builtin_memcpy(&b4, ed + e0, 16);
      xs[0] = a4.x, xs[1] = a4.y, xs[2] = a4.z, xs[3] = a4.w;
      ys[0] = b4.x, ys[1] = b4.y, ys[2] = b4.z, ys[3] = b4.w;
    } else {
#pragma unroll
      for (int b = 0; b < 4; b++) {
        xs[b] = e0 + b < E ? es[e0 + b] : 0u;
        ys[b] = e0 + b < E ? ed[e0 + b] : 0u;
      }
    }
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const bool in = e0 + b < E;
      bad |= in && (xs[b] >= V || ys[b] >= V);
      sd[4 * g4 + b] = in ? (xs[b] << 16) | (ys[b] & 0xFFFFu) : ~0u;
    }
  }
  for (uint32_t w = tid; w < (V + 31) / 32; w += B) s_rule[w] = 0;
  if (tid == 0) {
    s_bad = 0;
    s_created = 0;
    s_tail = 0;
    s_cnt[0] = 0;
    c.redo[g] = 0;
  }
  __syncthreads();
  // (four consecutive node words per thread and 16-byte load: eight lanes'
  // nibbles make one bitmap word)
  for (uint32_t base = 0; base < V; base += 8 * B) {
    uint32_t nib[2];
#pragma unroll
    for (int g4 = 0; g4 < 2; g4++) {
      const uint32_t v0 = base + 4 * (g4 * B + tid);
      uint32_t w[4];
      if (v0 + 3 < V) {
        uint4 w4;
        __builtin_memcpy(&w4, word + v0, 16);
        w[0] = w4.x, w[1] = w4.y, w[2] = w4.z, w[3] = w4.w;
      } else {
#pragma unroll
        for (int b = 0; b < 4; b++) w[b] = v0 + b < V ? word[v0 + b] : 0u;
      }
      nib[g4] = 0;
#pragma unroll
      for (int b = 0; b < 4; b++) nib[g4] |= (v0 + b < V && is_rule(w[b]) ? 1u : 0u) << b;
    }
#pragma unroll
    for (int g4 = 0; g4 < 2; g4++) {
      const uint32_t v0 = base + 4 * (g4 * B + tid);
      uint32_t x = nib[g4] << (4 * (tid & 7));
      x |= (uint32_t)__shfl_xor((int)x, 1);
      x |= (uint32_t)__shfl_xor((int)x, 2);
      x |= (uint32_t)__shfl_xor((int)x, 4);
      if ((tid & 7) == 0 && v0 < V && x) atomicOr(&s_rule[v0 >> 5], x);
    }
  }
  if (bad) s_bad = 1;
  __syncthreads();
  if (s_bad) {
    if (tid == 0) c.err[g] = NEMO_ERR_INVALID;
    return;
  }
  STAMP(11);
  uint32_t created = 0;
  for (int dir = 0; dir < 2; dir++) {  // 0: reverse rows (parents), 1: forward rows (children)
    const int ks = dir ? 16 : 0, vs = dir ? 0 : 16;  // key / value shifts in sd
    uint32_t *optr = dir ? c.fp + n0 + g : c.rp + n0 + g, *ocol = dir ? c.fc + e0 : c.rc + e0;
    for (uint32_t w = tid; w < (V + 2) / 2; w += B) ptr32[w] = 0;
    __syncthreads();
    if (dir == 0) STAMP(0);
#pragma unroll
    for (int q = 0; q < EPT; q++)
      if (sd[q] != ~0u) {
        const uint32_t k = (sd[q] >> ks) & 0xFFFFu;
        atomicAdd(&ptr32[k >> 1], 1u << (16 * (k & 1)));
      }
    __syncthreads();
    if (dir == 0) STAMP(1);
    if (dir == 0) {  // in-degrees; a graph beyond the u8 counters goes to the global tier
      bool heavy = false;
      for (uint32_t w = tid; 4 * w < V; w += B) {
        uint32_t x = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
          const uint32_t v = 4 * w + b, d = v < V ? ptr[v] : 0u;
          heavy |= d > 255u;
          x |= (d & 0xFFu) << (8 * b);
        }
        cnt32[w] = x;
      }
      if (heavy) s_bad = 1;
      __syncthreads();
      if (s_bad) {
        if (tid == 0) c.redo[g] = 1;
        return;
      }
    }
    if (dir == 0) STAMP(2);
    block_scan_inplace<B, 4, true>(ptr, V + 1, s_lds);
    if (dir == 0) STAMP(3);
    lds16_to_hbm32<B>(optr, ptr, V + 1);
    __syncthreads();
    if (dir == 0) STAMP(4);
#pragma unroll
    for (int q = 0; q < EPT; q++)
      if (sd[q] != ~0u) {
        const uint32_t k = (sd[q] >> ks) & 0xFFFFu, sh = 16 * (k & 1);
        col[(atomicAdd(&ptr32[k >> 1], 1u << sh) >> sh) & 0xFFFFu] = (uint16_t)((sd[q] >> vs) & 0xFFFFu);
      }
    __syncthreads();
    if (dir == 0) STAMP(5);
    // sort every row; two rows per thread at a time with all their LDS reads
    // issued together, the entries sorted in registers (a latency chain of a
    // few LDS round trips instead of one per entry)
    for (uint32_t v0 = tid; v0 < V; v0 += BLD_SQ * B) {
      uint32_t a[BLD_SQ], n[BLD_SQ];
#pragma unroll
      for (int q = 0; q < BLD_SQ; q++) {
        const uint32_t v = v0 + q * B;
        a[q] = v < V && v ? ptr[v - 1] : 0u;
        n[q] = v < V ? ptr[v] - a[q] : 0u;
      }
      uint32_t nmax = 0;
#pragma unroll
      for (int q = 0; q < BLD_SQ; q++) nmax = max(nmax, n[q]);
      // rows of at most four entries everywhere in the wave (most reverse rows,
      // goals' forward rows): the 4-key network over all BLD_SQ rows; else the
      // 8-key one two rows at a time
      if (!__any(nmax > 4u)) {
        created += sort_row_pair<4, B, BLD_SQ>(col, s_rule, E, V, dir, v0, a, n);
      } else {
#pragma unroll
        for (int h = 0; h < BLD_SQ; h += 2) {
          const uint32_t v = v0 + h * B;
          if (!__any(n[h] > 8u || n[h + 1] > 8u))
            created += sort_row_pair<8, B, 2>(col, s_rule, E, V, dir, v, a + h, n + h);
          else  // a row past eight entries in the wave: the 16-key network (an LDS insertion sort held the wave)
            created += sort_row_pair<16, B, 2>(col, s_rule, E, V, dir, v, a + h, n + h);
        }
      }
    }
    __syncthreads();
    if (dir == 0) STAMP(6);
    lds16_to_hbm32<B>(ocol, col, E);
    __syncthreads();
    STAMP(12 + dir);
  }
  atomicAdd(&s_created, created);
  uint32_t *nlv = c.nlv + n0;
  uint32_t *topo = c.topo + n0, *lvl = c.lvl + n0 + g;
  uint32_t hi = 0, nl = 0;
  // (round 6) Kahn levels by relaxation: lv(v) = max over v's parents of lv(u) + 1, swept over the
  // edges still in registers until a sweep changes nothing.  That is the longest path from a
  // source, the level Kahn's peeling gives; a sweep has no dependent chain (every edge's two LDS
  // reads are independent), where a peeled level is a chain of LDS round trips and a barrier.
  // Levels are u8 in cnt8's bytes (the in-degrees are recounted for the peeling below if the
  // sweeps give up), their histogram packed u16 in s_rule's bytes (the rule bitmap is done with):
  // a graph with more levels than either holds, or sweeps still changing after that many rounds
  // (a cycle, or lost updates: two lanes writing one node's byte), takes the peeling path.
  bool relaxed = false;
  if (c.bld_relax) {
    const uint32_t lcap = min(254u, lds_align(4u * ((V + 31u) / 32u)) / 2u - 1u);  // levels the histogram holds
    for (uint32_t w = tid; w < (V + 3) / 4; w += B) cnt32[w] = 0;
    if (tid < 3) s_cnt[tid] = 0;  // sweep r's "changed" flag is s_cnt[r % 3] (cleared two sweeps ahead)
    if (tid == 0) s_tail = 0;
    __syncthreads();
    bool gave_up = false;
    for (uint32_t r = 0;; r++) {
      if (tid == 0) s_cnt[(r + 1) % 3] = 0;  // its last readers passed the barrier of sweep r - 1
      bool ch = false;
#pragma unroll
      for (int q = 0; q < EPT; q++) {
        if (sd[q] != ~0u) {
          const uint32_t u = sd[q] >> 16, v = sd[q] & 0xFFFFu;
          const uint32_t lu = cnt8[u] + 1u;
          if (lu > cnt8[v]) {
            cnt8[v] = (uint8_t)min(lu, 255u);
            ch = true;
          }
        }
        if ((q & 7) == 7) __builtin_amdgcn_sched_barrier(0);  // eight edges' reads in flight at a time
      }
      if (__any(ch) && lane_id() == 0) s_cnt[r % 3] = 1;  // (not __syncthreads_or: its hidden LDS word
      __syncthreads();                                    // cost k_build a workgroup per CU)
      if (!s_cnt[r % 3]) break;
      if (r + 1 >= lcap) {  // uniform: every thread read the same flag
        gave_up = true;
        break;
      }
    }
    if (!gave_up) {  // a sweep can carry a level far along (edges in order): the levels are bounded, not the sweeps
      uint32_t mx = 0;
      for (uint32_t v = tid; v < V; v += B) mx = max(mx, (uint32_t)cnt8[v]);
      for (int d = 32; d >= 1; d >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, d));
      if (lane_id() == 0) atomicMax(&s_tail, mx);
      __syncthreads();
      gave_up = s_tail >= lcap;  // (a saturated byte, 255, is past lcap too)
    }
    if (!gave_up) {
      uint32_t *hist32 = s_rule;
      uint16_t *hist = (uint16_t *)s_rule;
      for (uint32_t i = tid; i < (lcap + 2) / 2; i += B) hist32[i] = 0;
      nl = V ? s_tail + 1u : 0u;
      __syncthreads();
      for (uint32_t v = tid; v < V; v += B) {  // coalesced
        const uint32_t l = cnt8[v];
        atomicAdd(&hist32[l >> 1], 1u << (16 * (l & 1)));
        nlv[v] = l;
      }
      __syncthreads();
      block_scan_inplace<B, 4, true>(hist, nl + 1, s_lds);  // level starts; hist[nl] = V
      for (uint32_t i = tid; i <= nl; i += B) lvl[i] = hist[i];
      for (uint32_t v = tid; v < V; v += B) {
        const uint32_t l = cnt8[v], sh = 16 * (l & 1);
        q16[(atomicAdd(&hist32[l >> 1], 1u << sh) >> sh) & 0xFFFFu] = (uint16_t)v;
      }
      hi = V;
      relaxed = true;
    } else {  // back to in-degree counters (and the append counters the flags used) for the peeling
      for (uint32_t w = tid; w < (V + 3) / 4; w += B) cnt32[w] = 0;
      if (tid < 3) s_cnt[tid] = 0;
      __syncthreads();
#pragma unroll
      for (int q = 0; q < EPT; q++)
        if (sd[q] != ~0u) {
          const uint32_t v = sd[q] & 0xFFFFu;
          atomicAdd(&cnt32[v >> 2], 1u << (8 * (v & 3)));
        }
    }
    __syncthreads();
  }
  // Kahn levels by peeling, over the forward rows still in LDS (ptr[v] = end of row v).
  // The sources in node order: each thread counts those of a contiguous run
  // of counter words (all its reads in flight together), one block scan
  // places them (no per-wave append chain)
  if (!relaxed) {
    constexpr int SW = 4;  // counter words (4 nodes each) per thread per round
    const uint32_t nw4 = (V + 3) / 4;
    uint32_t o = 0;
    for (uint32_t base = 0; base < nw4; base += SW * B) {
      const uint32_t w0 = base + tid * SW;
      uint32_t x[SW], n = 0;
#pragma unroll
      for (int k = 0; k < SW; k++) x[k] = cnt32[min(w0 + k, nw4 - 1u)];
#pragma unroll
      for (int k = 0; k < SW; k++)
#pragma unroll
        for (int b = 0; b < 4; b++) n += w0 + k < nw4 && 4 * (w0 + k) + b < V && ((x[k] >> (8 * b)) & 0xFFu) == 0u;
      uint32_t tot;
      uint32_t i = o + block_exscan<B, true>(n, &tot, s_lds);
#pragma unroll
      for (int k = 0; k < SW; k++)
#pragma unroll
        for (int b = 0; b < 4; b++) {
          const uint32_t v = 4 * (w0 + k) + b;
          if (w0 + k < nw4 && v < V && ((x[k] >> (8 * b)) & 0xFFu) == 0u) q16[i++] = (uint16_t)v;
        }
      o += tot;
    }
    if (tid == 0) s_tail = o;
    for (uint32_t v = tid; v < V; v += B)  // coalesced
      if (cnt8[v] == 0u) nlv[v] = 0;
  }
  __syncthreads();
  STAMP(14);
  // one barrier per level: level k appends behind the frontier through its
  // own counter s_cnt[k % 3]; the counter of level k + 1 is cleared during
  // level k (its last readers passed the barrier of level k - 1)
  uint32_t lo = 0;
  if (!relaxed) {
    hi = s_tail;
    if (tid == 0) lvl[0] = 0;
  }
  while (!relaxed && lo < hi) {
    uint32_t *cur = &s_cnt[nl % 3];
    if (tid == 0) s_cnt[(nl + 1) % 3] = 0;
    for (uint32_t base = lo; base < hi; base += B) {
      const uint32_t i = base + tid;
      // branch-free: reads and atomics at clamped / sink addresses, so the
      // BLD_KB slots' round trips overlap instead of waiting one by one
      const uint32_t u = q16[min(i, hi - 1u)];
      const uint32_t pu = ptr[u ? u - 1u : 0u], pe = ptr[u];
      uint32_t j = i < hi ? (u ? pu : 0u) : 0u, je = i < hi ? pe : 0u;
      // children BLD_KB at a time: their LDS reads and counter atomics are
      // independent, and the ready ones of all BLD_KB slots take one append
      // (ballots per slot, one counter atomic per wave)
      while (__any(j < je)) {
        uint32_t ch[BLD_KB], old[BLD_KB];
#pragma unroll
        for (int q = 0; q < BLD_KB; q++) {
          const uint32_t y = col[min(j + q, E - 1u)];
          ch[q] = j + q < je ? y : 0xFFFFu;
        }
#pragma unroll
        for (int q = 0; q < BLD_KB; q++) {
          const bool ok = ch[q] != 0xFFFFu;
          const uint32_t sh = 8 * (ch[q] & 3);
          const uint32_t r = atomicSub(ok ? &cnt32[ch[q] >> 2] : &s_sink[lane_id()], ok ? 1u << sh : 0u);
          old[q] = ok ? (r >> sh) & 0xFFu : 0u;
        }
        j = min(j + BLD_KB, je);
        uint64_t m[BLD_KB];
        uint32_t pre[BLD_KB], tot = 0;
#pragma unroll
        for (int q = 0; q < BLD_KB; q++) {
          m[q] = __ballot(old[q] == 1u);
          pre[q] = tot;
          tot += (uint32_t)__popcll(m[q]);
        }
        if (tot) {
          const int leader = __ffsll((long long)__ballot(1)) - 1;
          uint32_t b = 0;
          if ((int)lane_id() == leader) b = atomicAdd(cur, tot);
          b = hi + __builtin_amdgcn_readlane(b, leader);
#pragma unroll
          for (int q = 0; q < BLD_KB; q++)
            if (old[q] == 1u) {
              q16[b + pre[q] + mbcnt(m[q])] = (uint16_t)ch[q];
              nlv[ch[q]] = nl + 1;
            }
        }
      }
    }
    __syncthreads();
    nl++;
    lo = hi;
    hi += s_cnt[(nl - 1) % 3];  // after the barrier: plain LDS read
    if (tid == 0) lvl[nl] = lo;
  }
  STAMP(7);
  lds16_to_hbm32<B>(topo, q16, hi);
  if ((g & 1u) && hi == V) {
    // post graphs: the forward edges in source Kahn order for k_proto_lds (e2:
    // src << 16 | dst) and each Kahn position's first edge (posoff).  Every
    // thread copies the rows of a contiguous chunk of Kahn positions, four at a
    // time with their LDS reads issued together (rows past four entries loop).
    const uint32_t chunk = (V + B - 1) / B, i0 = min(V, tid * chunk), i1 = min(V, i0 + chunk);
    uint32_t sum = 0;
    for (uint32_t i = i0; i < i1; i += 4) {
      uint32_t u[4];
#pragma unroll
      for (int q = 0; q < 4; q++) u[q] = q16[min(i + q, i1 - 1u)];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t a = ptr[u[q] ? u[q] - 1u : 0u], b = ptr[u[q]];
        sum += i + q < i1 ? b - (u[q] ? a : 0u) : 0u;
      }
    }
    uint32_t tot;
    uint32_t off = block_exscan<B, true>(sum, &tot, s_lds);
    uint32_t *e2 = c.e2 + e0, *po = c.posoff + n0;
    for (uint32_t i = i0; i < i1; i += 4) {
      uint32_t u[4], a[4], n[4], y[4][4];
#pragma unroll
      for (int q = 0; q < 4; q++) u[q] = q16[min(i + q, i1 - 1u)];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t pa = ptr[u[q] ? u[q] - 1u : 0u], pb = ptr[u[q]];
        a[q] = u[q] ? pa : 0u;
        n[q] = i + q < i1 ? pb - a[q] : 0u;
      }
#pragma unroll
      for (int q = 0; q < 4; q++)
#pragma unroll
        for (int k = 0; k < 4; k++) y[q][k] = col[min(a[q] + k, E - 1u)];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        if (i + q < i1) po[i + q] = off;
#pragma unroll
        for (int k = 0; k < 4; k++)
          if ((uint32_t)k < n[q]) e2[off + k] = (u[q] << 16) | y[q][k];
        for (uint32_t k = 4; k < n[q]; k++) e2[off + k] = (u[q] << 16) | col[a[q] + k];
        off += n[q];
      }
    }
  }
  STAMP(15);
  uint32_t err = s_created == E ? 0u : (uint32_t)NEMO_ERR_LOAD;
  if (!err && hi != V) err = NEMO_ERR_CYCLE;
  if (tid == 0) {
    c.created[g] = s_created;
    c.nlev[g] = nl;
    c.err[g] = err;
  }
  // the deferred markConditionHolds + simplification of a well-formed graph
  // (k_marksimp's work, nemo_simplify then skips the graph): its edges are
  // still in sd, and the LDS image is free once the copies above have read it
  if (c.ms_fuse && !err && tier_fits(c.t_ms, V, E, nl)) {
    __syncthreads();
    marksimp_graph<B, EPT, true>(c, g, V, E, word, c.flags + n0, sd, true, [](uint32_t) {}, dyn, s_ms);
  }
}

// CSR (forward + reverse) of every graph; rows sorted so that a merged
// duplicate DUETO edge is adjacent.  relationships-created counts edges that
// are neither duplicates nor goal->goal / rule->rule (pre-post-prov.go:150-210).
// Graphs with V < CSR_LDS count degrees, scan and hand out cursors in LDS;
// larger ones do the same with global atomics.
#define CSR_LDS NEMO_CSR_BIG
template <int B>
__device__ __forceinline__ void csr_graph(const DevCorpus c, const uint32_t g) {
  __shared__ uint32_t s_cnt[CSR_LDS];
  __shared__ uint32_t s_lds[(B / 64)];
  __shared__ uint32_t s_created;
  const uint64_t n0 = c.node_off[g], e0 = c.edge_off[g];
  const uint32_t V = (uint32_t)(c.node_off[g + 1] - n0), E = (uint32_t)(c.edge_off[g + 1] - e0);
  if (build_fits(c, V, E) && !c.redo[g]) return;  // k_build's graph
  if (V >= CSR_LDS) return;                         // the multi-workgroup build (k_csrb_*)
  uint32_t *fp = c.fp + n0 + g, *rp = c.rp + n0 + g, *fc = c.fc + e0, *rc = c.rc + e0;
  const uint32_t *es = c.esrc + e0, *ed = c.edst + e0, *word = c.word + n0;
  if (threadIdx.x == 0) s_created = 0;  // first read after the barrier below
  bool bad = false;
  for (uint32_t e = threadIdx.x; e < E; e += B) bad |= es[e] >= V || ed[e] >= V;
  if (__syncthreads_or(bad)) {  // block-wide OR: no shared flag to reset racily
    if (threadIdx.x == 0) c.err[g] = NEMO_ERR_INVALID;
    return;
  }
  if (V < CSR_LDS) {
    for (int dir = 0; dir < 2; dir++) {
      const uint32_t *key = dir ? ed : es, *val = dir ? es : ed;
      uint32_t *ptr = dir ? rp : fp, *col = dir ? rc : fc;
      for (uint32_t v = threadIdx.x; v <= V; v += B) s_cnt[v] = 0;
      __syncthreads();
      for (uint32_t e = threadIdx.x; e < E; e += B) atomicAdd(&s_cnt[key[e]], 1u);
      __syncthreads();
      block_scan_inplace<B>(s_cnt, V + 1, s_lds);
      for (uint32_t v = threadIdx.x; v <= V; v += B) ptr[v] = s_cnt[v];
      __syncthreads();
      for (uint32_t e = threadIdx.x; e < E; e += B) col[atomicAdd(&s_cnt[key[e]], 1u)] = val[e];
      __syncthreads();
    }
  } else {
    uint32_t *cf = c.s_a + n0 + g, *cr = c.s_b + n0 + g;
    for (uint32_t v = threadIdx.x; v <= V; v += B) {
      fp[v] = 0;
      rp[v] = 0;
    }
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < E; e += B) {
      atomicAdd(&fp[es[e]], 1u);
      atomicAdd(&rp[ed[e]], 1u);
    }
    __syncthreads();
    block_scan_inplace<B, 16>(fp, V + 1, s_lds);
    block_scan_inplace<B, 16>(rp, V + 1, s_lds);
    for (uint32_t v = threadIdx.x; v < V; v += B) {
      cf[v] = fp[v];
      cr[v] = rp[v];
    }
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < E; e += B) {
      const uint32_t s = es[e], d = ed[e];
      fc[atomicAdd(&cf[s], 1u)] = d;
      rc[atomicAdd(&cr[d], 1u)] = s;
    }
    __syncthreads();
  }
  __threadfence_block();
  uint32_t created = 0;
  for (uint32_t v = threadIdx.x; v < V; v += B) {
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

// Graphs of CSR_LDS nodes or more (the deep corpora's 1M-node graphs): the
// same CSR build spread over many workgroups per graph.  A 2D grid takes the
// host's list of big graphs (y) and a chunk of each graph's edges or nodes
// (x); kernel boundaries replace the barriers between the phases (count ->
// per-graph scan -> scatter -> row sort + relationships-created).  Global
// atomics on the row counters and cursors; one workgroup per graph only for
// the scans.
#define CSRB_BLOCK 256
__device__ __forceinline__ bool csrb_take(const DevCorpus &c, uint32_t g, uint32_t V, uint32_t E) {
  return V >= CSR_LDS && !(build_fits(c, V, E) && !c.redo[g]);
}
__global__ __launch_bounds__(CSRB_BLOCK) void k_csrb_count(DevCorpus c) {
  for (uint32_t b = blockIdx.y; b < c.n_big; b += gridDim.y) {
    const uint32_t g = c.big[b];
    const uint64_t n0 = c.node_off[g], e0 = c.edge_off[g];
    const uint32_t V = (uint32_t)(c.node_off[g + 1] - n0), E = (uint32_t)(c.edge_off[g + 1] - e0);
    if (!csrb_take(c, g, V, E)) continue;
    uint32_t *fp = c.fp + n0 + g, *rp = c.rp + n0 + g;
    const uint32_t *es = c.esrc + e0, *ed = c.edst + e0;
    const uint32_t stride = gridDim.x * CSRB_BLOCK;
    bool bad = false;
    for (uint32_t e = blockIdx.x * CSRB_BLOCK + threadIdx.x; e < E; e += stride) {
      const uint32_t x = es[e], y = ed[e];
      if (x >= V || y >= V) {
        bad = true;
        continue;
      }
      atomicAdd(&fp[x], 1u);
      atomicAdd(&rp[y], 1u);
    }
    if (__any(bad) && lane_id() == 0) atomicMax(&c.err[g], (uint32_t)NEMO_ERR_INVALID);
  }
}
__global__ __launch_bounds__(CSRB_BLOCK) void k_csrb_zero(DevCorpus c) {
  for (uint32_t b = blockIdx.y; b < c.n_big; b += gridDim.y) {
    const uint32_t g = c.big[b];
    const uint64_t n0 = c.node_off[g];
    const uint32_t V = (uint32_t)(c.node_off[g + 1] - n0), E = (uint32_t)(c.edge_off[g + 1] - c.edge_off[g]);
    if (!csrb_take(c, g, V, E)) continue;
    uint32_t *fp = c.fp + n0 + g, *rp = c.rp + n0 + g;
    for (uint32_t v = blockIdx.x * CSRB_BLOCK + threadIdx.x; v <= V; v += gridDim.x * CSRB_BLOCK) {
      fp[v] = 0;
      rp[v] = 0;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) c.created[g] = 0;
  }
}
// one 1024-thread workgroup per big graph: row starts, and the scatter cursors
__global__ __launch_bounds__(1024) void k_csrb_scan(DevCorpus c) {
  __shared__ uint32_t s_lds[16];
  const uint32_t g = c.big[blockIdx.x];
  const uint64_t n0 = c.node_off[g];
  const uint32_t V = (uint32_t)(c.node_off[g + 1] - n0), E = (uint32_t)(c.edge_off[g + 1] - c.edge_off[g]);
  if (!csrb_take(c, g, V, E) || c.err[g]) return;
  uint32_t *fp = c.fp + n0 + g, *rp = c.rp + n0 + g, *cf = c.s_a + n0 + g, *cr = c.s_b + n0 + g;
  block_scan_inplace<1024, 16>(fp, V + 1, s_lds);
  block_scan_inplace<1024, 16>(rp, V + 1, s_lds);
  for (uint32_t v = threadIdx.x; v < V; v += 1024) {
    cf[v] = fp[v];
    cr[v] = rp[v];
  }
}
__global__ __launch_bounds__(CSRB_BLOCK) void k_csrb_scatter(DevCorpus c) {
  for (uint32_t b = blockIdx.y; b < c.n_big; b += gridDim.y) {
    const uint32_t g = c.big[b];
    const uint64_t n0 = c.node_off[g], e0 = c.edge_off[g];
    const uint32_t V = (uint32_t)(c.node_off[g + 1] - n0), E = (uint32_t)(c.edge_off[g + 1] - e0);
    if (!csrb_take(c, g, V, E) || c.err[g]) continue;
    uint32_t *fc = c.fc + e0, *rc = c.rc + e0, *cf = c.s_a + n0 + g, *cr = c.s_b + n0 + g;
    const uint32_t *es = c.esrc + e0, *ed = c.edst + e0;
    for (uint32_t e = blockIdx.x * CSRB_BLOCK + threadIdx.x; e < E; e += gridDim.x * CSRB_BLOCK) {
      const uint32_t x = es[e], y = ed[e];
      fc[atomicAdd(&cf[x], 1u)] = y;
      rc[atomicAdd(&cr[y], 1u)] = x;
    }
  }
}
// rows sorted (a merged duplicate DUETO edge is adjacent), relationships created
__global__ __launch_bounds__(CSRB_BLOCK) void k_csrb_rows(DevCorpus c) {
  __shared__ uint32_t s_cr;
  for (uint32_t b = blockIdx.y; b < c.n_big; b += gridDim.y) {
    const uint32_t g = c.big[b];
    const uint64_t n0 = c.node_off[g], e0 = c.edge_off[g];
    const uint32_t V = (uint32_t)(c.node_off[g + 1] - n0), E = (uint32_t)(c.edge_off[g + 1] - e0);
    if (!csrb_take(c, g, V, E) || c.err[g]) continue;
    const uint32_t *fp = c.fp + n0 + g, *rp = c.rp + n0 + g, *word = c.word + n0;
    uint32_t *fc = c.fc + e0, *rc = c.rc + e0;
    if (threadIdx.x == 0) s_cr = 0;
    __syncthreads();
    uint32_t created = 0;
    for (uint32_t v = blockIdx.x * CSRB_BLOCK + threadIdx.x; v < V; v += gridDim.x * CSRB_BLOCK) {
      const uint32_t a = fp[v], bb = fp[v + 1];
      sort_row(fc + a, bb - a);
      sort_row(rc + rp[v], rp[v + 1] - rp[v]);
      const bool rv = is_rule(word[v]);
      for (uint32_t j = a; j < bb; j++) {
        const uint32_t t = fc[j];
        if (!(j > a && fc[j - 1] == t) && rv != is_rule(word[t])) created++;
      }
    }
    for (int d = 32; d >= 1; d >>= 1) created += __shfl_xor(created, d);
    if (lane_id() == 0 && created) atomicAdd(&s_cr, created);
    __syncthreads();
    if (threadIdx.x == 0 && s_cr) atomicAdd(&c.created[g], s_cr);
    __syncthreads();
  }
}
__global__ __launch_bounds__(CSRB_BLOCK) void k_csrb_fin(DevCorpus c) {
  const uint32_t b = blockIdx.x * CSRB_BLOCK + threadIdx.x;
  if (b >= c.n_big) return;
  const uint32_t g = c.big[b];
  const uint32_t V = (uint32_t)(c.node_off[g + 1] - c.node_off[g]), E = (uint32_t)(c.edge_off[g + 1] - c.edge_off[g]);
  if (!csrb_take(c, g, V, E) || c.err[g]) return;
  c.err[g] = c.created[g] == E ? 0u : (uint32_t)NEMO_ERR_LOAD;
}

#define TOPO_BATCH 4
// Kahn levels: topo[] lists the graph's nodes level by level, lvl[l]..lvl[l+1]
// is level l (longest path from a source).  A graph with a cycle is refused.
template <int B>
__device__ __forceinline__ void topo_graph(const DevCorpus c, const uint32_t g) {
  __shared__ uint32_t s_tail;
  if (c.err[g]) return;
  const uint64_t n0 = c.node_off[g], e0 = c.edge_off[g];
  const uint32_t V = (uint32_t)(c.node_off[g + 1] - n0);
  if (build_fits(c, V, (uint32_t)(c.edge_off[g + 1] - e0)) && !c.redo[g]) return;  // k_build's graph
  if (V >= CSR_LDS) return;  // k_topo_deep's graph
  const uint32_t *fp = c.fp + n0 + g, *rp = c.rp + n0 + g, *fc = c.fc + e0;
  uint32_t *topo = c.topo + n0, *lvl = c.lvl + n0 + g, *cnt = c.s_a + n0 + g;
  if (threadIdx.x == 0) s_tail = 0;
  for (uint32_t v = threadIdx.x; v < V; v += B) cnt[v] = rp[v + 1] - rp[v];
  __syncthreads();
  for (uint32_t base = 0; base < V; base += B) {
    const uint32_t v = base + threadIdx.x;
    wave_append(v < V && cnt[v] == 0u, v, topo, &s_tail);
    if (v < V && cnt[v] == 0u) c.nlv[n0 + v] = 0;
  }
  __syncthreads();
  uint32_t lo = 0, hi = s_tail, nl = 0;
  if (threadIdx.x == 0) lvl[0] = 0;
  __syncthreads();
  while (lo < hi) {
    for (uint32_t base = lo; base < hi; base += B) {
      const uint32_t i = base + threadIdx.x;
      uint32_t j = 0, je = 0;
      if (i < hi) {
        const uint32_t u = topo[i];
        j = fp[u];
        je = fp[u + 1];
      }
      // children in batches of TOPO_BATCH: their loads and counter atomics are
      // independent, so a batch costs one round trip instead of one per child
      while (__any(j < je)) {
        uint32_t ch[TOPO_BATCH], old[TOPO_BATCH];
#pragma unroll
        for (int q = 0; q < TOPO_BATCH; q++) ch[q] = j + q < je ? fc[j + q] : NEMO_NONE;
#pragma unroll
        for (int q = 0; q < TOPO_BATCH; q++) old[q] = ch[q] != NEMO_NONE ? atomicSub(&cnt[ch[q]], 1u) : 0u;
        j = min(j + TOPO_BATCH, je);
#pragma unroll
        for (int q = 0; q < TOPO_BATCH; q++) {
          const bool p = old[q] == 1u;
          wave_append(p, ch[q], topo, &s_tail);
          if (p) c.nlv[n0 + ch[q]] = nl + 1;
        }
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

// The global-tier rebuild runs over a list of the graphs k_build did not take
// (past its LDS caps, or handed back): one early-exit workgroup per graph cost
// ~30 us per step at C3, where the list is empty.  k_csr and k_topo share it.
__global__ __launch_bounds__(NEMO_BLOCK) void k_load_sel(DevCorpus c) {
  const uint32_t g = blockIdx.x * NEMO_BLOCK + threadIdx.x;
  bool need = false;
  if (g < c.G) {
    const uint32_t V = (uint32_t)(c.node_off[g + 1] - c.node_off[g]);
    const uint32_t E = (uint32_t)(c.edge_off[g + 1] - c.edge_off[g]);
    need = !build_fits(c, V, E) || c.redo[g];
  }
  uint32_t *sel = c.sel + 2 * ((size_t)c.G + 1);
  wave_append(need, g, sel + 1, sel);
}
template <int B>
__global__ __launch_bounds__(B) void k_csr(DevCorpus c) {
  const uint32_t *sel = c.sel + 2 * ((size_t)c.G + 1);
  const uint32_t n = sel[0];
  for (uint32_t k = blockIdx.x; k < n; k += gridDim.x) {
    csr_graph<B>(c, sel[1 + k]);
    __syncthreads();  // LDS of this graph is done before the next one starts
  }
}
template <int B>
__global__ __launch_bounds__(B) void k_topo(DevCorpus c) {
  const uint32_t *sel = c.sel + 2 * ((size_t)c.G + 1);
  const uint32_t n = sel[0];
  for (uint32_t k = blockIdx.x; k < n; k += gridDim.x) {
    topo_graph<B>(c, sel[1 + k]);
    __syncthreads();
  }
}
// Kahn levels of the big graphs (V >= CSR_LDS: the deep corpora's 1M-node
// graphs, ~22k levels of a few dozen nodes).  A level is a chain of dependent
// HBM round trips (the frontier's row pointers, their children, the in-degree
// atomics), so the kernel is built to keep that chain short:
//   - the frontier lives in LDS (the level's nodes are not re-read from topo[]
//     unless the level outgrows TD_Q);
//   - edge-parallel: the frontier's rows are published with one block scan of
//     their degrees, and each thread takes edges (a binary search over the
//     row offsets in LDS), so a lane has ~one child load and one counter
//     atomic in flight.  A returning device-scope atomic costs ~3k cycles
//     under load; a lane queueing a whole row of them (one node per lane)
//     spent ~60 % of each level there (135 -> 115 -> 73 ms per C5 launch);
//   - ready children are appended with one wave scan and one LDS atomic per
//     wave; 256 threads, so the barriers of a level are four waves'.
#define TD_B 256
#define TD_Q 2048u
#ifndef TD_EPT
#define TD_EPT 4  // frontier edges per thread per round
#endif
// The LDS frontier holds each node's row (first edge, degree), not the node:
// a child's row bounds are loaded together with its in-degree atomic (for
// every child, ready or not), so a level starts from LDS instead of waiting on
// an HBM round trip for its rows.  Frontier entries past TD_Q are read back
// from topo[] and their rows loaded.
__device__ __forceinline__ bool topo_ell_takes(const DevCorpus &c, uint32_t g) {
  return c.topo_ell && c.gscratch && c.gs_off[g] != ~0ull;
}
__global__ __launch_bounds__(TD_B) void k_topo_deep(DevCorpus c) {
  __shared__ uint2 s_q[2][TD_Q];
  // appends of level L go to s_n[(L + 1) % 3]: read after the level's barrier,
  // reset during level L + 2, so one barrier per level orders everything
  __shared__ uint32_t s_n[3];
  __shared__ uint32_t s_eo[TD_B], s_j0[TD_B], s_red[TD_B / 64];
  const uint32_t g = c.big[blockIdx.x];
  if (c.err[g] || topo_ell_takes(c, g)) return;
  const uint64_t n0 = c.node_off[g], e0 = c.edge_off[g];
  const uint32_t V = (uint32_t)(c.node_off[g + 1] - n0), E = (uint32_t)(c.edge_off[g + 1] - e0);
  if ((build_fits(c, V, E) && !c.redo[g]) || V < CSR_LDS) return;
  const uint32_t *fp = c.fp + n0 + g, *rp = c.rp + n0 + g, *fc = c.fc + e0;
  uint32_t *topo = c.topo + n0, *lvl = c.lvl + n0 + g, *cnt = c.s_a + n0 + g, *nlv = c.nlv + n0;
  const uint32_t tid = threadIdx.x;
  if (tid < 3) s_n[tid] = 0;
  if (tid == 0) lvl[0] = 0;
  __syncthreads();
  // level 0: the sources
  for (uint32_t b = 0; b < V; b += TD_B) {
    const uint32_t v = b + tid;
    const uint32_t d = v < V ? rp[v + 1] - rp[v] : 1u;
    if (v < V) cnt[v] = d;
    const bool p = d == 0u;
    const uint64_t m = __ballot(p);
    if (m == 0) continue;
    uint32_t base = 0;
    if (lane_id() == 0) base = atomicAdd(&s_n[1], (uint32_t)__popcll(m));
    base = __builtin_amdgcn_readlane(base, 0);
    if (p) {
      const uint32_t i = base + mbcnt(m);
      topo[i] = v;
      nlv[v] = 0;
      if (i < TD_Q) {
        const uint32_t a = fp[v];
        s_q[0][i] = make_uint2(a, fp[v + 1] - a);
      }
    }
  }
  __syncthreads();
  uint32_t lo = 0, hi = s_n[1], nl = 0, cur = 0, k3 = 1;  // k3 = (nl + 1) % 3
  while (lo < hi) {
    const uint32_t n = hi - lo, kn = k3 == 2 ? 0u : k3 + 1u;  // this level's append counter
    if (tid == 0) s_n[kn == 2 ? 0u : kn + 1u] = 0;            // = (nl + 3) % 3: free since level nl - 1
    uint2 *qn = s_q[cur ^ 1];
    // edge-parallel: a chunk of TD_B frontier nodes publishes its rows (start,
    // exclusive degree offset); every thread then takes edges of the chunk, so
    // each lane has ~one child load and one counter atomic in flight instead of
    // a whole row's worth (a lane's 16 queued atomics were ~60 % of a level)
    for (uint32_t b = 0; b < n; b += TD_B) {
      const uint32_t i = b + tid, nc = min((uint32_t)TD_B, n - b);
      uint32_t j0 = 0, d = 0;
      if (i < n) {
        if (i < TD_Q) {
          const uint2 r = s_q[cur][i];
          j0 = r.x;
          d = r.y;
        } else {
          const uint32_t u = topo[lo + i];
          j0 = fp[u];
          d = fp[u + 1] - j0;
        }
      }
      uint32_t tot;
      const uint32_t eo = block_exscan<TD_B>(d, &tot, s_red);
      s_eo[tid] = eo;
      s_j0[tid] = j0;
      __syncthreads();
      for (uint32_t e0 = 0; e0 < tot; e0 += TD_B * TD_EPT) {
        uint32_t ch[TD_EPT], ra[TD_EPT], rb[TD_EPT];
        bool rdy[TD_EPT];
#pragma unroll
        for (int k = 0; k < TD_EPT; k++) {
          const uint32_t e = e0 + k * TD_B + tid;
          ch[k] = NEMO_NONE;
          if (e < tot) {
            uint32_t lo2 = 0, hi2 = nc;  // the last row starting at or before e
            while (hi2 - lo2 > 1) {
              const uint32_t mid = (lo2 + hi2) >> 1;
              if (s_eo[mid] <= e) lo2 = mid;
              else hi2 = mid;
            }
            ch[k] = fc[s_j0[lo2] + (e - s_eo[lo2])];
          }
        }
        uint32_t r = 0;
#pragma unroll
        for (int k = 0; k < TD_EPT; k++) {
          const bool ok = ch[k] != NEMO_NONE;
          const uint32_t cw = ok ? ch[k] : 0u;
          const uint32_t old = ok ? atomicSub(&cnt[cw], 1u) : 0u;
          ra[k] = fp[cw];  // the child's row, in flight with its atomic
          rb[k] = fp[cw + 1];
          rdy[k] = old == 1u;
          r += rdy[k] ? 1u : 0u;
        }
        uint32_t wt;
        const uint32_t ex = wave_exscan(r, &wt);
        if (wt) {
          uint32_t base = 0;
          if (lane_id() == 0) base = atomicAdd(&s_n[kn], wt);
          uint32_t at = __builtin_amdgcn_readlane(base, 0) + ex;
#pragma unroll
          for (int k = 0; k < TD_EPT; k++) {
            if (!rdy[k]) continue;
            topo[hi + at] = ch[k];
            nlv[ch[k]] = nl + 1;
            if (at < TD_Q) qn[at] = make_uint2(ra[k], rb[k] - ra[k]);
            at++;
          }
        }
      }
      __syncthreads();  // s_eo / s_j0 are rewritten by the next chunk
    }
    const uint32_t m = s_n[kn];
    nl++;
    lo = hi;
    hi += m;
    cur ^= 1;
    k3 = kn;
    if (tid == 0) lvl[nl] = lo;
  }
  if (tid == 0) {
    c.nlev[g] = nl;
    if (hi != V) c.err[g] = NEMO_ERR_CYCLE;
  }
}

// Kahn levels of the deep graphs, one HBM round trip per level (round 6).  k_topo_deep's level is
// two dependent round trips: the frontier's children (fc[] at the row starts it holds) and then
// their in-degree atomics.  Here every node has a child record of TE_K u32 in its graph's
// gscratch region (free at load time; k_chains_glob's until the next rebuild): its children
// (NEMO_NONE padded), or for a longer row TE_OVF, its row start and degree.  The frontier holds
// each node's record in LDS, so a level is: the frontier's children from the LDS records into an
// LDS edge list (a round trip to fc[] only for a level holding a row past TE_K) -> one edge per
// thread: its child's in-degree atomic and, in the same round trip, the child's record -> the
// ready children appended with their records.  Edge-parallel as k_topo_deep: a long row is
// spread over the lanes, not walked by one.
#define TE_K 16
#define TE_Q 256u    // LDS frontier records per buffer (2 x 256 x 64 B)
#define TE_EL 4096u  // LDS edge list of a chunk of TD_B frontier nodes (longer: several passes)
#define TE_OVF 0xFFFFFFFEu
__global__ __launch_bounds__(NEMO_BLOCK) void k_topo_ellprep(DevCorpus c) {
  const uint32_t g = c.big[blockIdx.y];
  if (c.err[g] || !topo_ell_takes(c, g)) return;
  const uint64_t n0 = c.node_off[g], e0 = c.edge_off[g];
  const uint32_t V = (uint32_t)(c.node_off[g + 1] - n0), E = (uint32_t)(c.edge_off[g + 1] - e0);
  if ((build_fits(c, V, E) && !c.redo[g]) || V < CSR_LDS) return;
  const uint32_t *fp = c.fp + n0 + g, *fc = c.fc + e0;
  uint4 *ell = reinterpret_cast<uint4 *>(c.gscratch + c.gs_off[g]);
  for (uint32_t v = blockIdx.x * NEMO_BLOCK + threadIdx.x; v < V; v += gridDim.x * NEMO_BLOCK) {
    const uint32_t a = fp[v], d = fp[v + 1] - a;
    uint32_t r[TE_K];
    if (d <= TE_K) {
#pragma unroll
      for (int k = 0; k < TE_K; k++) r[k] = (uint32_t)k < d ? fc[a + k] : NEMO_NONE;
    } else {
      r[0] = TE_OVF;
      r[1] = a;
      r[2] = d;
#pragma unroll
      for (int k = 3; k < TE_K; k++) r[k] = NEMO_NONE;
    }
#pragma unroll
    for (int q = 0; q < TE_K / 4; q++)
      ell[(TE_K / 4) * (size_t)v + q] = make_uint4(r[4 * q], r[4 * q + 1], r[4 * q + 2], r[4 * q + 3]);
  }
}

__global__ __launch_bounds__(NEMO_BLOCK) void k_topo_ell(DevCorpus c) {
  constexpr uint32_t RQ = TE_K / 4;  // uint4 per record
  __shared__ uint4 s_q[2][TE_Q][RQ];
  __shared__ uint32_t s_el[TE_EL];  // the chunk's children, by the exclusive degree offsets
  // appends of level L go to s_n[(L + 1) % 3]: read after the level's barrier, reset during
  // level L + 2, so one barrier per level orders everything (as k_topo_deep)
  __shared__ uint32_t s_n[3], s_red[NEMO_BLOCK / 64];
  const uint32_t g = c.big[blockIdx.x];
  if (c.err[g] || !topo_ell_takes(c, g)) return;
  const uint64_t n0 = c.node_off[g], e0 = c.edge_off[g];
  const uint32_t V = (uint32_t)(c.node_off[g + 1] - n0), E = (uint32_t)(c.edge_off[g + 1] - e0);
  if ((build_fits(c, V, E) && !c.redo[g]) || V < CSR_LDS) return;
  const uint32_t *rp = c.rp + n0 + g, *fc = c.fc + e0;
  const uint4 *ell = reinterpret_cast<const uint4 *>(c.gscratch + c.gs_off[g]);
  uint32_t *topo = c.topo + n0, *lvl = c.lvl + n0 + g, *cnt = c.s_a + n0 + g, *nlv = c.nlv + n0;
  const uint32_t tid = threadIdx.x;
  if (tid < 3) s_n[tid] = 0;
  if (tid == 0) lvl[0] = 0;
  __syncthreads();
  // level 0: the sources, with their records
  for (uint32_t b = 0; b < V; b += NEMO_BLOCK) {
    const uint32_t v = b + tid;
    const uint32_t d = v < V ? rp[v + 1] - rp[v] : 1u;
    if (v < V) cnt[v] = d;
    const bool p = d == 0u;
    const uint64_t m = __ballot(p);
    if (m == 0) continue;
    uint32_t base = 0;
    if (lane_id() == 0) base = atomicAdd(&s_n[1], (uint32_t)__popcll(m));
    base = __builtin_amdgcn_readlane(base, 0);
    if (p) {
      const uint32_t i = base + mbcnt(m);
      topo[i] = v;
      nlv[v] = 0;
      if (i < TE_Q)
#pragma unroll
        for (uint32_t q = 0; q < RQ; q++) s_q[0][i][q] = ell[RQ * (size_t)v + q];
    }
  }
  __syncthreads();
  uint32_t lo = 0, hi = s_n[1], nl = 0, cur = 0, k3 = 1;  // k3 = (nl + 1) % 3
  while (lo < hi) {
    const uint32_t n = hi - lo, kn = k3 == 2 ? 0u : k3 + 1u;  // this level's append counter
    if (tid == 0) s_n[kn == 2 ? 0u : kn + 1u] = 0;            // = (nl + 3) % 3: free since level nl - 1
    for (uint32_t b = 0; b < n; b += NEMO_BLOCK) {
      const uint32_t i = b + tid;
      uint32_t r[TE_K];
#pragma unroll
      for (int k = 0; k < TE_K; k++) r[k] = NEMO_NONE;
      if (i < n) {  // (no arrays of uint4: they were kept in scratch)
        const uint4 *src = i < TE_Q ? &s_q[cur][i][0] : nullptr;
        const uint32_t u = i < TE_Q ? 0u : topo[lo + i];  // past the LDS frontier: the record from HBM
#pragma unroll
        for (uint32_t t = 0; t < RQ; t++) {
          const uint4 x = src ? src[t] : ell[RQ * (size_t)u + t];
          r[4 * t] = x.x, r[4 * t + 1] = x.y, r[4 * t + 2] = x.z, r[4 * t + 3] = x.w;
        }
      }
      const bool ovf = r[0] == TE_OVF;
      uint32_t d = 0;
      if (!ovf) {
#pragma unroll
        for (int k = 0; k < TE_K; k++) d += r[k] != NEMO_NONE ? 1u : 0u;
      } else {
        d = r[2];
      }
      uint32_t tot;
      const uint32_t eo = block_exscan<NEMO_BLOCK>(d, &tot, s_red);
      // the chunk's children into the LDS edge list, TE_EL at a time (rows in order of eo)
      for (uint32_t p0 = 0; p0 < tot; p0 += TE_EL) {
        if (ovf) {  // a long row: its children from fc[] (every lane's loads in flight together)
          const uint32_t a = max(eo, p0), z = min(eo + d, p0 + TE_EL);
          for (uint32_t x = a; x < z; x += 8) {  // eight loads in flight, then their stores
            uint32_t y[8];
#pragma unroll
            for (int k = 0; k < 8; k++) y[k] = x + k < z ? fc[r[1] + (x + k - eo)] : 0u;
#pragma unroll
            for (int k = 0; k < 8; k++)
              if (x + k < z) s_el[x + k - p0] = y[k];
          }
        } else {
#pragma unroll
          for (int k = 0; k < TE_K; k++) {
            const uint32_t x = eo + k;
            if ((uint32_t)k < d && x >= p0 && x < p0 + TE_EL) s_el[x - p0] = r[k];
          }
        }
        __syncthreads();
        const uint32_t ne = min(tot - p0, TE_EL);
        // one edge per thread and round: the child's in-degree atomic and its record
        for (uint32_t e = tid; e < ne; e += NEMO_BLOCK) {
          const uint32_t ch = s_el[e];
          const uint32_t old = atomicSub(&cnt[ch], 1u);
          const uint4 c0 = ell[RQ * (size_t)ch], c1 = ell[RQ * (size_t)ch + 1];
          const uint4 c2 = ell[RQ * (size_t)ch + 2], c3 = ell[RQ * (size_t)ch + 3];
          static_assert(RQ == 4, "four uint4 per record");
          if (old == 1u) {  // ready: a slot by one LDS atomic (a level has a few dozen)
            const uint32_t at = atomicAdd(&s_n[kn], 1u);
            topo[hi + at] = ch;
            nlv[ch] = nl + 1;
            if (at < TE_Q) {
              s_q[cur ^ 1][at][0] = c0;
              s_q[cur ^ 1][at][1] = c1;
              s_q[cur ^ 1][at][2] = c2;
              s_q[cur ^ 1][at][3] = c3;
            }
          }
        }
        __syncthreads();  // s_el is rewritten by the next pass / chunk
      }
    }
    __syncthreads();
    const uint32_t m = s_n[kn];
    nl++;
    lo = hi;
    hi += m;
    cur ^= 1;
    k3 = kn;
    if (tid == 0) lvl[nl] = lo;
  }
  if (tid == 0) {
    c.nlev[g] = nl;
    if (hi != V) c.err[g] = NEMO_ERR_CYCLE;
  }
}

#define LOAD_GRID 2048u

void launch_build(const DevCorpus &c, hipStream_t s) {
  if (!c.bld_bytes) return;
#ifndef BLD_PAD
#define BLD_PAD 0  // diagnostic: extra LDS per workgroup (fewer workgroups per CU)
#endif
  hipFuncSetAttribute((const void *)k_build<BLD_BLOCK>, hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)(c.bld_bytes + BLD_PAD));
  hipLaunchKernelGGL(k_build<BLD_BLOCK>, dim3(c.G), dim3(BLD_BLOCK), c.bld_bytes + BLD_PAD, s, c);
}
void launch_load(const DevCorpus &c, hipStream_t s) {
  if (!c.G) return;
  launch_zero(c.sel + 2 * ((size_t)c.G + 1), sizeof(uint32_t), s);
  hipLaunchKernelGGL(k_load_sel, dim3((c.G + NEMO_BLOCK - 1) / NEMO_BLOCK), dim3(NEMO_BLOCK), 0, s, c);
  const uint32_t grid = std::min(c.G, LOAD_GRID);
  if (c.gblock == 1024)
    hipLaunchKernelGGL(k_csr<1024>, dim3(grid), dim3(1024), 0, s, c);
  else
    hipLaunchKernelGGL(k_csr<NEMO_BLOCK>, dim3(grid), dim3(NEMO_BLOCK), 0, s, c);
}
// Bucketed form of the same build (the default for big graphs): scattered
// global atomics on 1M-entry row counters run at the memory-side atomic rate
// (~20 G/s chip-wide, MI355X_MICROARCH.md "Global float atomics"), so the
// counting happens in LDS instead.  Per direction: (1) every CB_CHUNK-edge
// chunk histograms its keys by CB_NB-node bucket in LDS; (2) one workgroup per
// graph scans the (bucket, chunk) counts; (3) each chunk partitions its edges
// into their buckets' ranges (LDS cursors) as (key, value) pairs in HBM
// scratch; (4) one workgroup per bucket counts its nodes' degrees, writes
// their row pointers and scatters the values into their rows with LDS
// cursors, then sorts the rows (and, forward, counts relationships created).
// Every global write is then a streaming store into a contiguous range.
#ifndef CB_BLOCK
#define CB_BLOCK 1024
#endif
__global__ __launch_bounds__(CB_BLOCK) void k_cb_hist(DevCorpus c, int dir) {
  __shared__ uint32_t h[CB_MAXB];
  const uint32_t b = blockIdx.y, g = c.big[b];
  const uint64_t n0 = c.node_off[g], e0 = c.edge_off[g];
  const uint32_t V = (uint32_t)(c.node_off[g + 1] - n0), E = (uint32_t)(c.edge_off[g + 1] - e0);
  const uint32_t nbk = (V + CB_NB - 1) / CB_NB, nck = (E + CB_CHUNK - 1) / CB_CHUNK;
  if (blockIdx.x >= nck || !csrb_take(c, g, V, E)) return;
  for (uint32_t k = threadIdx.x; k < nbk; k += CB_BLOCK) h[k] = 0;
  __syncthreads();
  const uint32_t *key = (dir ? c.edst : c.esrc) + e0, *oth = (dir ? c.esrc : c.edst) + e0;
  const uint32_t a = blockIdx.x * CB_CHUNK, z = min(E, a + CB_CHUNK);
  bool bad = false;
  for (uint32_t e0 = a + 4 * threadIdx.x; e0 < z; e0 += 4 * CB_BLOCK) {  // four edges per thread and load
    uint32_t k[4], o[4];
    if (e0 + 3 < z) {
      uint4 k4, o4;
      __builtin_memcpy(&k4, key + e0, 16);
      __builtin_memcpy(&o4, oth + e0, 16);
      k[0] = k4.x, k[1] = k4.y, k[2] = k4.z, k[3] = k4.w;
      o[0] = o4.x, o[1] = o4.y, o[2] = o4.z, o[3] = o4.w;
    } else {
#pragma unroll
      for (int b = 0; b < 4; b++) {
        k[b] = e0 + b < z ? key[e0 + b] : 0u;
        o[b] = e0 + b < z ? oth[e0 + b] : 0u;
      }
    }
#pragma unroll
    for (int b = 0; b < 4; b++) {
      if (e0 + b >= z) continue;
      bad |= k[b] >= V || o[b] >= V;
      if (k[b] < V) atomicAdd(&h[k[b] / CB_NB], 1u);
    }
  }
  if (__any(bad) && lane_id() == 0) atomicMax(&c.err[g], (uint32_t)NEMO_ERR_INVALID);
  __syncthreads();
  uint32_t *out = c.cb_hist + c.cb_hoff[b];  // (bucket, chunk) counts, bucket-major
  for (uint32_t k = threadIdx.x; k < nbk; k += CB_BLOCK) out[(uint64_t)k * nck + blockIdx.x] = h[k];
}
__global__ __launch_bounds__(1024) void k_cb_scan(DevCorpus c) {
  __shared__ uint32_t s_lds[16];
  const uint32_t b = blockIdx.x, g = c.big[b];
  const uint32_t V = (uint32_t)(c.node_off[g + 1] - c.node_off[g]), E = (uint32_t)(c.edge_off[g + 1] - c.edge_off[g]);
  if (!csrb_take(c, g, V, E) || c.err[g]) return;
  const uint32_t nbk = (V + CB_NB - 1) / CB_NB, nck = (E + CB_CHUNK - 1) / CB_CHUNK;
  block_scan_inplace<1024, 16>(c.cb_hist + c.cb_hoff[b], nbk * nck, s_lds);
}
__global__ __launch_bounds__(CB_BLOCK) void k_cb_part(DevCorpus c, int dir) {
  __shared__ uint32_t cur[CB_MAXB];
  const uint32_t b = blockIdx.y, g = c.big[b];
  const uint64_t n0 = c.node_off[g], e0 = c.edge_off[g];
  const uint32_t V = (uint32_t)(c.node_off[g + 1] - n0), E = (uint32_t)(c.edge_off[g + 1] - e0);
  const uint32_t nbk = (V + CB_NB - 1) / CB_NB, nck = (E + CB_CHUNK - 1) / CB_CHUNK;
  if (blockIdx.x >= nck || !csrb_take(c, g, V, E) || c.err[g]) return;
  const uint32_t *off = c.cb_hist + c.cb_hoff[b];
  for (uint32_t k = threadIdx.x; k < nbk; k += CB_BLOCK) cur[k] = off[(uint64_t)k * nck + blockIdx.x];
  __syncthreads();
  const uint32_t *key = (dir ? c.edst : c.esrc) + e0, *oth = (dir ? c.esrc : c.edst) + e0;
  uint32_t *ok = c.cb_key + e0, *ov = c.cb_val + e0;
  const uint32_t a = blockIdx.x * CB_CHUNK, z = min(E, a + CB_CHUNK);
  for (uint32_t e0 = a + 4 * threadIdx.x; e0 < z; e0 += 4 * CB_BLOCK) {  // four edges per thread and load
    uint32_t k[4], o[4];
    if (e0 + 3 < z) {
      uint4 k4, o4;
      __builtin_memcpy(&k4, key + e0, 16);
      __builtin_memcpy(&o4, oth + e0, 16);
      k[0] = k4.x, k[1] = k4.y, k[2] = k4.z, k[3] = k4.w;
      o[0] = o4.x, o[1] = o4.y, o[2] = o4.z, o[3] = o4.w;
    } else {
#pragma unroll
      for (int b = 0; b < 4; b++) {
        k[b] = e0 + b < z ? key[e0 + b] : 0u;
        o[b] = e0 + b < z ? oth[e0 + b] : 0u;
      }
    }
#pragma unroll
    for (int b = 0; b < 4; b++) {
      if (e0 + b >= z) continue;
      const uint32_t pos = atomicAdd(&cur[k[b] / CB_NB], 1u);
      ok[pos] = k[b];
      ov[pos] = o[b];
    }
  }
}
// One bucket's rows built in LDS: degrees, row starts, the values scattered
// by LDS cursors and each row sorted there, then written out coalesced.  A
// bucket of more than CB_LDS_E edges (a hub-heavy one) sorts in HBM instead.
#ifndef CB_LDS_E
#define CB_LDS_E 14336u
#endif
#define CB_CB 4  // a bucket's edges per thread per batch (loads in flight together)
#define CB_WSORT_MIN 17u

// a row [a, a + n) of u32 entries (n <= RS) sorted in registers, its reads
// in flight together; returns a bit per duplicate entry (x[i-1] == x[i])
template <int RS>
__device__ __forceinline__ uint32_t cb_sort_row(uint32_t *rows, uint32_t a, uint32_t n, uint32_t (&x)[16]) {
  uint32_t dup = 0;
#pragma unroll
  for (int i = 0; i < RS; i++) x[i] = (uint32_t)i < n ? rows[a + i] : 0xFFFFFFFFu;
  if (n < 2) return 0;
  if (RS == 4) sort_net4(x);
  else if (RS == 8) sort_net8(x);
  else sort_net16(x);
#pragma unroll
  for (int i = 0; i < RS; i++)
    if ((uint32_t)i < n) rows[a + i] = x[i];
#pragma unroll
  for (int i = 1; i < RS; i++) dup |= ((uint32_t)i < n && x[i - 1] == x[i] ? 1u : 0u) << i;
  return dup;
}

// (<= 64 VGPRs: two 1024-thread workgroups per CU, as the LDS allows)
__global__ __launch_bounds__(CB_BLOCK) __attribute__((amdgpu_waves_per_eu(8))) void k_cb_bucket(DevCorpus c, int dir) {
  __shared__ uint32_t cnt[CB_NB + 1];
  __shared__ uint32_t s_long[CB_NB], s_nlong;
  __shared__ uint32_t rows[CB_LDS_E];
  __shared__ uint32_t s_lds[CB_BLOCK / 64];
  __shared__ uint32_t s_cr;
  const uint32_t b = blockIdx.y, g = c.big[b];
  const uint64_t n0 = c.node_off[g], e0 = c.edge_off[g];
  const uint32_t V = (uint32_t)(c.node_off[g + 1] - n0), E = (uint32_t)(c.edge_off[g + 1] - e0);
  const uint32_t nbk = (V + CB_NB - 1) / CB_NB, nck = (E + CB_CHUNK - 1) / CB_CHUNK;
  const uint32_t bk = blockIdx.x, tid = threadIdx.x;
  if (bk >= nbk || !csrb_take(c, g, V, E) || c.err[g]) return;
  const uint32_t *off = c.cb_hist + c.cb_hoff[b];
  const uint32_t lo = off[(uint64_t)bk * nck], hi = bk + 1 < nbk ? off[(uint64_t)(bk + 1) * nck] : E;
  const uint32_t v0 = bk * CB_NB, nv = min(V, v0 + CB_NB) - v0, ne = hi - lo;
  const uint32_t *ek = c.cb_key + e0 + lo, *ev = c.cb_val + e0 + lo;
  uint32_t *ptr = (dir ? c.rp : c.fp) + n0 + g, *col = (dir ? c.rc : c.fc) + e0 + lo;
  const uint32_t *word = c.word + n0;
  const bool lds = ne <= CB_LDS_E;
  uint32_t *dst = lds ? rows : col;  // where the rows are assembled and sorted
  // degrees; forward rows also check each edge's goal/rule kinds
  // (pre-post-prov.go:150-210 creates a relationship only between a goal and
  // a rule): the node words of both ends gathered with the batch's loads in
  // flight together, instead of a dependent load per row entry after the sort
  uint32_t created = 0;
  for (uint32_t i = tid; i <= nv; i += CB_BLOCK) cnt[i] = 0;
  if (tid == 0) s_cr = 0;
  __syncthreads();
  // (CB_CB consecutive edges per thread and 16-byte load)
  auto ld_kv = [&](uint32_t j0, uint32_t (&k)[CB_CB], uint32_t (&v)[CB_CB], bool want_v) {
    static_assert(CB_CB == 4, "one 16-byte load per array");
    if (j0 + 3 < ne) {
      uint4 k4, v4 = make_uint4(0, 0, 0, 0);
      __builtin_memcpy(&k4, ek + j0, 16);
      if (want_v) __builtin_memcpy(&v4, ev + j0, 16);
      k[0] = k4.x, k[1] = k4.y, k[2] = k4.z, k[3] = k4.w;
      v[0] = v4.x, v[1] = v4.y, v[2] = v4.z, v[3] = v4.w;
    } else {
#pragma unroll
      for (int q = 0; q < CB_CB; q++) {
        k[q] = j0 + q < ne ? ek[j0 + q] : v0;
        v[q] = j0 + q < ne && want_v ? ev[j0 + q] : 0u;
      }
    }
  };
  for (uint32_t j0 = CB_CB * tid; j0 < ne; j0 += CB_CB * CB_BLOCK) {
    uint32_t k[CB_CB], v[CB_CB];
    ld_kv(j0, k, v, dir == 0);
#pragma unroll
    for (int q = 0; q < CB_CB; q++)
      if (j0 + q < ne) atomicAdd(&cnt[k[q] - v0], 1u);
    if (dir == 0) {
      uint32_t wk[CB_CB], wv[CB_CB];
#pragma unroll
      for (int q = 0; q < CB_CB; q++) {
        wk[q] = word[k[q]];
        wv[q] = word[v[q]];
      }
#pragma unroll
      for (int q = 0; q < CB_CB; q++) created += j0 + q < ne && is_rule(wk[q]) != is_rule(wv[q]) ? 1u : 0u;
    }
  }
  __syncthreads();
  block_scan_inplace<CB_BLOCK>(cnt, nv + 1, s_lds);
  for (uint32_t i = tid; i < nv; i += CB_BLOCK) ptr[v0 + i] = lo + cnt[i];
  if (bk + 1 == nbk && tid == 0) ptr[V] = E;
  __syncthreads();
  for (uint32_t j0 = CB_CB * tid; j0 < ne; j0 += CB_CB * CB_BLOCK) {
    uint32_t k[CB_CB], v[CB_CB];
    ld_kv(j0, k, v, true);
#pragma unroll
    for (int q = 0; q < CB_CB; q++)
      if (j0 + q < ne) dst[atomicAdd(&cnt[k[q] - v0], 1u)] = v[q];
  }
  __threadfence_block();
  __syncthreads();  // cnt[i] = end of row i (local)
  // rows sorted (a merged duplicate DUETO edge is adjacent).  In LDS: rows of
  // up to 16 entries in registers (4-, 8- or 16-key networks, two rows per
  // thread), rows of CB_WSORT_MIN..64 entries by a whole wave (bitonic network
  // over shuffles), longer ones by their thread; in HBM: by their thread (one
  // thread heap-sorting a 60-entry row in LDS held the workgroup for most of
  // its time).  A duplicate's relationship is created once: forward rows take
  // it back out of the edge-parallel count above.
  if (tid == 0) s_nlong = 0;
  __syncthreads();
  if (lds) {
    static_assert(CB_NB == 2 * CB_BLOCK, "two rows per thread");
    uint32_t ra[2], rn[2];
#pragma unroll
    for (int q = 0; q < 2; q++) {
      const uint32_t i = tid + q * CB_BLOCK;
      ra[q] = i < nv && i ? cnt[i - 1] : 0u;
      rn[q] = i < nv ? cnt[i] - ra[q] : 0u;
    }
#pragma unroll
    for (int q = 0; q < 2; q++) {
      const uint32_t i = tid + q * CB_BLOCK;
      const bool wide = rn[q] >= CB_WSORT_MIN && rn[q] <= 64u;
      wave_append(wide, i, s_long, &s_nlong);
      if (rn[q] > 64u) sort_row(dst + ra[q], rn[q]);
    }
    // one row at a time (register budget); the network by the longest such row in the wave
#pragma unroll
    for (int q = 0; q < 2; q++) {
      const uint32_t sn = rn[q] <= 16u ? rn[q] : 0u;
      uint32_t x[16], dup;
      if (!__any(sn > 4u)) dup = cb_sort_row<4>(dst, ra[q], sn, x);
      else if (!__any(sn > 8u)) dup = cb_sort_row<8>(dst, ra[q], sn, x);
      else dup = cb_sort_row<16>(dst, ra[q], sn, x);
      if (dir == 0 && dup) {  // rare
        const bool rv = is_rule(word[v0 + tid + q * CB_BLOCK]);
#pragma unroll
        for (int i = 1; i < 16; i++)
          if ((dup >> i) & 1u) created -= rv != is_rule(word[x[i]]) ? 1u : 0u;
      }
    }
  } else {
    for (uint32_t i = tid; i < nv; i += CB_BLOCK) {
      const uint32_t a = i ? cnt[i - 1] : 0u, z = cnt[i], n = z - a;
      const bool wide = n >= CB_WSORT_MIN && n <= 64u;
      wave_append(wide, i, s_long, &s_nlong);
      if (!wide) sort_row(dst + a, n);
    }
  }
  __syncthreads();
  for (uint32_t q = tid >> 6; q < s_nlong; q += CB_BLOCK / 64) {
    const uint32_t i = s_long[q], a = i ? cnt[i - 1] : 0u, n = cnt[i] - a, l = lane_id();
    uint32_t x = l < n ? dst[a + l] : 0xFFFFFFFFu;
#pragma unroll
    for (uint32_t k = 2; k <= 64; k <<= 1)
#pragma unroll
      for (uint32_t j = k >> 1; j > 0; j >>= 1) {
        const uint32_t y = (uint32_t)__shfl_xor((int)x, (int)j);
        const bool up = (l & k) == 0, low = (l & j) == 0;
        x = (low == up) ? min(x, y) : max(x, y);
      }
    if (l < n) dst[a + l] = x;
  }
  __threadfence_block();
  __syncthreads();
  // forward rows: duplicates in the rows the register networks did not sort
  // (wide and long rows, and every row of a bucket sorted in HBM) are taken
  // back out of the edge-parallel count
  if (dir == 0) {
    for (uint32_t i = tid; i < nv; i += CB_BLOCK) {
      const uint32_t a = i ? cnt[i - 1] : 0u, z = cnt[i];
      if (lds && z - a <= 16u) continue;
      for (uint32_t j = a + 1; j < z; j++) {
        const uint32_t t = dst[j];
        if (dst[j - 1] == t && is_rule(word[v0 + i]) != is_rule(word[t])) created--;
      }
    }
  }
  __syncthreads();
  if (lds)
    for (uint32_t j = tid; j < ne; j += CB_BLOCK) col[j] = rows[j];
  for (int d = 32; d >= 1; d >>= 1) created += __shfl_xor(created, d);
  if (lane_id() == 0 && created) atomicAdd(&s_cr, created);
  __syncthreads();
  if (tid == 0 && s_cr) atomicAdd(&c.created[g], s_cr);
}
__global__ __launch_bounds__(CSRB_BLOCK) void k_cb_zero(DevCorpus c) {
  const uint32_t b = blockIdx.x * CSRB_BLOCK + threadIdx.x;
  if (b < c.n_big) c.created[c.big[b]] = 0;
}

void launch_csr_big(const DevCorpus &c, uint32_t chunks, hipStream_t s) {
  if (!c.n_big) return;
  if (c.cb_hist) {  // bucketed build (every big graph within CB_MAXB buckets)
    hipLaunchKernelGGL(k_cb_zero, dim3((c.n_big + CSRB_BLOCK - 1) / CSRB_BLOCK), dim3(CSRB_BLOCK), 0, s, c);
    for (int dir = 0; dir < 2; dir++) {
      const dim3 gc(c.cb_maxck, c.n_big), gb(c.cb_maxbk, c.n_big);
      hipLaunchKernelGGL(k_cb_hist, gc, dim3(CB_BLOCK), 0, s, c, dir);
      hipLaunchKernelGGL(k_cb_scan, dim3(c.n_big), dim3(1024), 0, s, c);
      hipLaunchKernelGGL(k_cb_part, gc, dim3(CB_BLOCK), 0, s, c, dir);
      hipLaunchKernelGGL(k_cb_bucket, gb, dim3(CB_BLOCK), 0, s, c, dir);
    }
    hipLaunchKernelGGL(k_csrb_fin, dim3((c.n_big + CSRB_BLOCK - 1) / CSRB_BLOCK), dim3(CSRB_BLOCK), 0, s, c);
    return;
  }
  if (!c.n_big) return;
  const dim3 grid(chunks, std::min(c.n_big, 65535u));
  hipLaunchKernelGGL(k_csrb_zero, grid, dim3(CSRB_BLOCK), 0, s, c);
  hipLaunchKernelGGL(k_csrb_count, grid, dim3(CSRB_BLOCK), 0, s, c);
  hipLaunchKernelGGL(k_csrb_scan, dim3(c.n_big), dim3(1024), 0, s, c);
  hipLaunchKernelGGL(k_csrb_scatter, grid, dim3(CSRB_BLOCK), 0, s, c);
  hipLaunchKernelGGL(k_csrb_rows, grid, dim3(CSRB_BLOCK), 0, s, c);
  hipLaunchKernelGGL(k_csrb_fin, dim3((c.n_big + CSRB_BLOCK - 1) / CSRB_BLOCK), dim3(CSRB_BLOCK), 0, s, c);
}
void launch_topo(const DevCorpus &c, hipStream_t s, bool list) {  // after launch_load: its list
  if (!c.G) return;
  const uint32_t grid = std::min(c.G, LOAD_GRID);
  if (!list) {  // the host knows the list is empty (api.hip tiers_known)
  } else if (c.gblock == 1024)
    hipLaunchKernelGGL(k_topo<1024>, dim3(grid), dim3(1024), 0, s, c);
  else
    hipLaunchKernelGGL(k_topo<NEMO_BLOCK>, dim3(grid), dim3(NEMO_BLOCK), 0, s, c);
  if (!c.n_big) return;
  hipLaunchKernelGGL(k_topo_deep, dim3(c.n_big), dim3(TD_B), 0, s, c);  // graphs without child records
  if (c.topo_ell && c.gscratch) {
    hipLaunchKernelGGL(k_topo_ellprep, dim3(256, c.n_big), dim3(NEMO_BLOCK), 0, s, c);
    hipLaunchKernelGGL(k_topo_ell, dim3(c.n_big), dim3(NEMO_BLOCK), 0, s, c);
  }
}

}  // namespace nemo
