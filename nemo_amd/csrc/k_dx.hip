// k_dx.hip — CreateNaiveDiffProv (differential-provenance.go:18-146) for many
// label sources at once.
//
// Every diff entry works on run 0's post graph g0 and differs only in its
// label source (failGoals = collect(failed.label), :22-24):
//   Good_u = goals of g0 whose label is not a post-goal label of source u
//   D_u    = Fwd*(Good_u) ∩ Bwd*(Good_u)                (:22-32, APOC export)
//   missing_u = D_u rules with a D_u-leaf goal child at maximal depth (:82-98)
// Reachability is the same sweep for every source, so one bit per source in a
// u64 word carries 64 sources through one reversed-Kahn-order walk (a
// "chunk").  The depth of a D rule is 1 + the longest path from a Good goal
// (k_dx_walk, MODE 2): per source, two or four sources per workgroup, one
// walking wave each, over the same staged graph windows; it needs neither D
// nor a Fwd* walk (its non-zero values are Fwd*), so it runs beside Bwd*.
//
// Kernels per call (launch_dx):
//   k_dx_label   present bitmaps: g0 positions whose label a source holds
//   k_dx_good    Good words per chunk (64 bitmaps transposed by ballots)
//   k_dx_walks   Bwd* per chunk (+ leaf candidates) and the longest paths per
//                source, one launch
//   k_dx_lp      D = Fwd* & Bwd*, LP rules, the longest LP path per source
//   k_dx_emit    missing rows (LP rules at that length)
//   k_dx_mask    D masks by node for every entry (entries -> sources)
// When g0 fits LDS whole (C3), k_dx_walks also does k_dx_lp's, k_dx_emit's and
// (one entry per source) k_dx_mask's work: the chunk's Bwd* workgroup computes
// the leaf candidates and, per rule, the OR of its children's, publishes them
// with Bwd* (agent-scope release + flag), and each longest-path workgroup, whose
// NE sources' values sit in its LDS over every position, waits for that flag and
// finishes its sources alone (LP rules, maxLen as an LDS maximum, missing rows,
// masks): label, good, walks per call.
// g0's Kahn-order relayout (k_dxp_*) is built with the CSR in every load /
// rebuild (launch_dx_prep), since it depends on the graph alone.
//
// The walk (k_dx_walk): positions in walk order (Kahn order, or reversed for
// Bwd*) are taken in windows.  All waves stage a window: its rows' links as a
// CSR of ring indices, the init value of every position (Good, or 0) written
// into its ring slot, the end of its Kahn level.  A link to a position older
// than the ring reads that position's final value from HBM and is folded into
// its owner's init at staging.  Then one wave per source walks the window's
// levels: each level is one step of independent lanes (no barrier, a wave's
// LDS operations complete in order), value = init op (ring values of links).
#include <atomic>

#include "device.h"
#include "internal.h"

namespace nemo {

// ---- device-wide exclusive scan (in place) --------------------------------------------
// tiles of DSC_TILE entries: tile sums, their scan (one workgroup), then each
// tile scanned with its offset
#define DSC_NT 1024
#define DSC_PER 4
#define DSC_TILE (DSC_NT * DSC_PER)
__global__ __launch_bounds__(DSC_NT) void k_scan_tiles(const uint32_t *a, uint32_t n, uint32_t *tsum) {
  __shared__ uint32_t s_red[DSC_NT / 64];
  const uint32_t i0 = blockIdx.x * DSC_TILE + threadIdx.x * DSC_PER;
  uint32_t x = 0;
#pragma unroll
  for (int q = 0; q < DSC_PER; q++) x += i0 + q < n ? a[i0 + q] : 0u;
  uint32_t tot;
  block_exscan<DSC_NT>(x, &tot, s_red);
  if (threadIdx.x == 0) tsum[blockIdx.x] = tot;
}
__global__ __launch_bounds__(DSC_NT) void k_scan_sums(uint32_t *tsum, uint32_t nt) {
  __shared__ uint32_t s_red[DSC_NT / 64];
  block_scan_inplace<DSC_NT, 4>(tsum, nt, s_red);
}
__global__ __launch_bounds__(DSC_NT) void k_scan_apply(uint32_t *a, uint32_t n, const uint32_t *tsum) {
  __shared__ uint32_t s_red[DSC_NT / 64];
  const uint32_t i0 = blockIdx.x * DSC_TILE + threadIdx.x * DSC_PER;
  uint32_t x[DSC_PER], sum = 0;
#pragma unroll
  for (int q = 0; q < DSC_PER; q++) {
    x[q] = i0 + q < n ? a[i0 + q] : 0u;
    sum += x[q];
  }
  uint32_t tot;
  uint32_t ex = block_exscan<DSC_NT>(sum, &tot, s_red) + tsum[blockIdx.x];
#pragma unroll
  for (int q = 0; q < DSC_PER; q++) {
    if (i0 + q < n) a[i0 + q] = ex;
    ex += x[q];
  }
}
uint32_t dx_scan_tiles(uint32_t n) { return (n + DSC_TILE - 1) / DSC_TILE + 1; }
void launch_scan(uint32_t *a, uint32_t n, uint32_t *tsum, hipStream_t s) {
  const uint32_t nt = (n + DSC_TILE - 1) / DSC_TILE;
  if (!nt) return;
  hipLaunchKernelGGL(k_scan_tiles, dim3(nt), dim3(DSC_NT), 0, s, a, n, tsum);
  hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(DSC_NT), 0, s, tsum, nt);
  hipLaunchKernelGGL(k_scan_apply, dim3(nt), dim3(DSC_NT), 0, s, a, n, tsum);
}

// ---- g0 relayout (launch_dx_prep) ---------------------------------------------------
// pass 1, one thread per position i: node -> position, row lengths (parents in
// Kahn order, children in reversed Kahn order), level bounds, rule bit
__global__ __launch_bounds__(NEMO_BLOCK) void k_dxp_a(DevCorpus c, DxPrep p) {
  if (*p.err0) return;  // g0 failed to load: its CSR and Kahn order may be partial
  const GraphView gv = c.view(p.g0);
  const uint32_t i = blockIdx.x * NEMO_BLOCK + threadIdx.x;
  if (i == 0) {
    p.rp[gv.V] = 0;
    p.fp[gv.V] = 0;
  }
  if (i >= gv.V) return;
  const uint32_t v = gv.topo[i];
  p.tpos[v] = i;
  p.pnode[i] = v;
  p.rp[i] = gv.rp[v + 1] - gv.rp[v];
  p.fp[gv.V - 1u - i] = gv.fp[v + 1] - gv.fp[v];
  const uint32_t l = c.nlv[gv.n0 + v];
  p.lbeg[i] = gv.lvl[l];
  p.lend[i] = gv.lvl[l + 1];
  p.info[i] = (l << 3) | (is_rule(gv.word[v]) ? DXI_RULE : 0u);
}
// pass 2 (launch_scan): row starts
// pass 3, one thread per position: rows as walk indices (parents as positions,
// children as reversed positions), label entries as positions
__global__ __launch_bounds__(NEMO_BLOCK) void k_dxp_b(DevCorpus c, DxPrep p) {
  if (*p.err0) return;  // g0 failed to load: its CSR and Kahn order may be partial
  const GraphView gv = c.view(p.g0);
  const uint32_t i = blockIdx.x * NEMO_BLOCK + threadIdx.x;
  if (i < p.n_r0lab) {
    const uint32_t pos = p.tpos[p.r0idx[i]], l = p.r0lab[i];
    p.r0pos[i] = pos;
    if (p.r0dense && (i == 0 || p.r0lab[i - 1] != l)) {  // the label's first entry: its dense entry
      uint32_t n = 1;
      while (n < 15u && i + n < p.n_r0lab && p.r0lab[i + n] == l) n++;
      p.r0dense[l] = n == 1u ? pos << 4 : (i << 4) | n;
    }
  }
  if (i >= gv.V) return;
  const uint32_t v = gv.topo[i], V = gv.V;
  uint32_t o = p.rp[i];
  for (uint32_t j = gv.rp[v]; j < gv.rp[v + 1]; j++) p.rc[o++] = p.tpos[gv.rc[j]];
  o = p.fp[V - 1u - i];
  for (uint32_t j = gv.fp[v]; j < gv.fp[v + 1]; j++) p.fc[o++] = V - 1u - p.tpos[gv.fc[j]];
}

void launch_dx_prep(const DevCorpus &c, const DxPrep &p, uint32_t *tsum, hipStream_t s) {
  const uint32_t nb = (std::max(p.V0, p.n_r0lab) + NEMO_BLOCK - 1) / NEMO_BLOCK;
  if (!nb) return;
  hipLaunchKernelGGL(k_dxp_a, dim3(nb), dim3(NEMO_BLOCK), 0, s, c, p);
  launch_scan(p.rp, p.V0 + 1, tsum, s);
  launch_scan(p.fp, p.V0 + 1, tsum, s);
  hipLaunchKernelGGL(k_dxp_b, dim3(nb), dim3(NEMO_BLOCK), 0, s, c, p);
}

// ---- walk images (launch_dx_img) -------------------------------------------------------
// windows: greedy in walk order, one workgroup per image; a window ends before
// W positions or before its links pass EC (every row fits: dx_max_row)
struct DxImgSet {
  DxImg m[2];
};
__global__ __launch_bounds__(1024) void k_dxi_bounds(DxPrep p, DxImgSet set) {
  if (*p.err0) return;  // g0 failed to load: its CSR and Kahn order may be partial
  __shared__ uint32_t s_best[3];
  const DxImg m = set.m[blockIdx.x];
  const uint32_t V = p.V0, tid = threadIdx.x, lane = lane_id();
  const uint32_t *rowp = m.rev ? p.fp : p.rp;
  if (tid < 3) s_best[tid] = 0;
  __syncthreads();
  uint32_t b = 0, k = 0;
  while (b < V) {  // workgroup-uniform
    const uint32_t nmax = min(m.W, V - b), base = rowp[b];
    uint32_t best = 0;
    for (uint32_t t = tid + 1; t <= nmax; t += 1024)
      if (rowp[b + t] - base <= m.EC) best = max(best, t);
    for (int d = 32; d >= 1; d >>= 1) best = max(best, (uint32_t)__shfl_xor(best, d));
    // three buffers: round k fills k % 3 and clears (k + 1) % 3, last read in round k - 2
    if (tid == 0) s_best[(k + 1) % 3] = 0;
    if (lane == 0) atomicMax(&s_best[k % 3], best);
    __syncthreads();
    const uint32_t n = max(s_best[k % 3], 1u);
    if (tid == 0) m.wb[k] = b;
    b += n;
    k++;
  }
  if (tid == 0) {
    m.wb[k] = V;
    m.nw[0] = k;
  }
}
// the window of walk index i: wb[k] <= i < wb[k + 1]
__device__ __forceinline__ uint32_t dxi_window(const DxImg &m, uint32_t nw, uint32_t i) {
  uint32_t lo = 0, hi = nw;  // wb[lo] <= i < wb[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (m.wb[mid] <= i) lo = mid;
    else hi = mid;
  }
  return lo;
}
// A link of window k to walk index x leaves the ring when x + R < end of window
// k + 1: the walk of window k then never reads a slot that the staging of
// window k + 1 (running beside it) writes, and with R >= 4 W such an x lies two
// windows back or more, whose values are in HBM by then.
__device__ __forceinline__ uint32_t dxi_far_end(const DxImg &m, uint32_t nw, uint32_t k) {
  return m.wb[min(k + 2u, nw)];
}
// per walk index: segment flag (the window's first position or a level's
// first), links that leave the ring
__global__ __launch_bounds__(NEMO_BLOCK) void k_dxi_count(DxPrep p, DxImg m, DxImgScratch t) {
  if (*p.err0) return;  // g0 failed to load: its CSR and Kahn order may be partial
  const uint32_t V = p.V0, i = blockIdx.x * NEMO_BLOCK + threadIdx.x;
  if (i > V) return;
  if (i == V) {
    t.fseg[V] = 0;
    m.moff[V] = 0;
    return;
  }
  const uint32_t nw = m.nw[0], k = dxi_window(m, nw, i), w0 = m.wb[k], fe = dxi_far_end(m, nw, k);
  const uint32_t *rowp = m.rev ? p.fp : p.rp, *col = m.rev ? p.fc : p.rc;
  const uint32_t pos = m.rev ? V - 1u - i : i;
  const uint32_t lstart = m.rev ? V - p.lend[pos] : p.lbeg[pos];
  t.fseg[i] = (i == w0 || lstart == i) ? 1u : 0u;
  uint32_t nm = 0;
  if (!m.whole)
    for (uint32_t j = rowp[i]; j < rowp[i + 1]; j++) nm += col[j] + m.R < fe ? 1u : 0u;
  m.moff[i] = nm;
}
// per walk index: its segment's first position, its links' records and misses
__global__ __launch_bounds__(NEMO_BLOCK) void k_dxi_fill(DxPrep p, DxImg m, DxImgScratch t) {
  if (*p.err0) return;  // g0 failed to load: its CSR and Kahn order may be partial
  const uint32_t V = p.V0, i = blockIdx.x * NEMO_BLOCK + threadIdx.x;
  if (i >= V) {
    if (i == V) t.segpos[t.fseg[V]] = V;
    return;
  }
  const uint32_t nw = m.nw[0], k = dxi_window(m, nw, i), fe = dxi_far_end(m, nw, k);
  const uint32_t *rowp = m.rev ? p.fp : p.rp, *col = m.rev ? p.fc : p.rc;
  if (t.fseg[i + 1] != t.fseg[i]) t.segpos[t.fseg[i]] = i;
  const uint32_t own = (m.whole ? i : (i & (m.R - 1u))) << 16;
  uint32_t o = m.moff[i];
  for (uint32_t j = rowp[i]; j < rowp[i + 1]; j++) {
    const uint32_t x = col[j];
    const bool far = !m.whole && x + m.R < fe;
    m.rec[j] = (far ? m.R : (m.whole ? x : (x & (m.R - 1u)))) | own;
    if (far) m.mx[o++] = x;
  }
}
// per segment: its walk steps (<= DX_STEP links each; a segment without links has none)
#define DX_STEP 256u
__global__ __launch_bounds__(NEMO_BLOCK) void k_dxi_stepcount(DxPrep p, DxImg m, DxImgScratch t) {
  if (*p.err0) return;  // g0 failed to load: its CSR and Kahn order may be partial
  const uint32_t V = p.V0, sg = blockIdx.x * NEMO_BLOCK + threadIdx.x, ns = t.fseg[V];
  if (sg > V) return;
  const uint32_t *rowp = m.rev ? p.fp : p.rp;
  t.fstep[sg] = sg < ns ? (rowp[t.segpos[sg + 1]] - rowp[t.segpos[sg]] + DX_STEP - 1u) / DX_STEP : 0u;
}
__global__ __launch_bounds__(NEMO_BLOCK) void k_dxi_steps(DxPrep p, DxImg m, DxImgScratch t) {
  if (*p.err0) return;  // g0 failed to load: its CSR and Kahn order may be partial
  const uint32_t V = p.V0, sg = blockIdx.x * NEMO_BLOCK + threadIdx.x, ns = t.fseg[V];
  if (sg >= ns) return;
  const uint32_t *rowp = m.rev ? p.fp : p.rp;
  const uint32_t nw = m.nw[0], a = t.segpos[sg], k = dxi_window(m, nw, a), w0 = m.wb[k];
  const uint32_t rel = rowp[a] - rowp[w0], cnt = rowp[t.segpos[sg + 1]] - rowp[a];
  uint32_t o = t.fstep[sg];
  if (a == w0) m.stepb[k] = o;
  if (sg == 0) m.stepb[nw] = t.fstep[ns];
  for (uint32_t r = 0; r * DX_STEP < cnt; r++) m.steps[o++] = (rel + r * DX_STEP) | (min(DX_STEP, cnt - r * DX_STEP) << 16);
}

void launch_dx_img(const DxPrep &p, DxImg img[2], const DxImgScratch &t, hipStream_t s) {
  const uint32_t V = p.V0;
  if (!V) return;
  DxImgSet set;
  for (int k = 0; k < 2; k++) set.m[k] = img[k];
  hipLaunchKernelGGL(k_dxi_bounds, dim3(2), dim3(1024), 0, s, p, set);
  const uint32_t nb = (V + 1 + NEMO_BLOCK - 1) / NEMO_BLOCK;
  for (int k = 0; k < 2; k++) {
    hipLaunchKernelGGL(k_dxi_count, dim3(nb), dim3(NEMO_BLOCK), 0, s, p, img[k], t);
    launch_scan(t.fseg, V + 1, t.tsum, s);
    launch_scan(img[k].moff, V + 1, t.tsum, s);
    hipLaunchKernelGGL(k_dxi_fill, dim3(nb), dim3(NEMO_BLOCK), 0, s, p, img[k], t);
    hipLaunchKernelGGL(k_dxi_stepcount, dim3(nb), dim3(NEMO_BLOCK), 0, s, p, img[k], t);
    launch_scan(t.fstep, V + 1, t.tsum, s);
    hipLaunchKernelGGL(k_dxi_steps, dim3(nb), dim3(NEMO_BLOCK), 0, s, p, img[k], t);
  }
}

// ---- present bitmaps ------------------------------------------------------------------
// Workgroup (x, u): source u's nodes [x * lab_per, ...).  Every goal label is
// looked up in g0's label table (open-addressed: key = label + 1) and each g0
// goal carrying it gets its position's bit.  Bitmaps of up to DXL_LDS words
// are gathered in LDS and stored whole (one workgroup per source) or ORed in
// by word; larger ones take global atomics.
#define DXL_LDS 4096u
#ifndef DXL_BATCH
#define DXL_BATCH 24  // source nodes per thread and round (all their loads in flight together)
#endif
__global__ __launch_bounds__(NEMO_BLOCK) void k_dx_label(DevCorpus c, DxArgs a) {
  __shared__ uint32_t bm[DXL_LDS];
  const uint32_t u = blockIdx.y, tid = threadIdx.x;
  const bool lds = a.w32 <= DXL_LDS;
  const uint32_t *lab, *word;
  uint32_t n;
  if (a.ref_labels) {
    lab = a.ref_labels + 1;
    word = nullptr;
    n = a.ref_labels[0];
  } else {
    const GraphView s = c.view(a.src[u]);
    lab = s.label;
    word = s.word;
    n = s.V;
  }
  uint32_t *pb = a.pb + (size_t)u * a.w32;
  STAMP2(10);
  if (blockIdx.x == 0 && tid == 0) {
    a.maxlen[u] = 0;  // k_dx_lp's maxima (two launches later)
    if (u < a.nch) a.wflag[u] = 0;  // the chunks' Bwd* flags (k_dx_walks)
  }
  if (lds) {
    for (uint32_t w = tid; w < a.w32; w += NEMO_BLOCK) bm[w] = 0;
    __syncthreads();
  }
  const uint32_t lo = blockIdx.x * a.lab_per, hi = min(n, lo + a.lab_per);
  auto mark = [&](uint32_t p) {
    if (lds) atomicOr(&bm[p >> 5], 1u << (p & 31u));
    else atomicOr(&pb[p >> 5], 1u << (p & 31u));
  };
  if (a.r0dense) {  // labels and node words together, one dense-table load per source goal
    // (four consecutive nodes per thread and 16-byte load when the slice allows; vectorising a
    // misaligned slice after a head of up to three nodes measured no faster)
    auto mark_dense = [&](uint32_t lbv, uint32_t dvv) {
      if (dvv == NEMO_NONE) return;
      if ((dvv & 15u) == 0u) {  // one run-0 goal carries the label
        mark(dvv >> 4);
        return;
      }
      const uint32_t i0 = dvv >> 4, cnt = dvv & 15u;
      for (uint32_t t = 0; t < cnt; t++) mark(a.p.r0pos[i0 + t]);
      if (cnt == 15u)  // 15 or more entries: the rest of the run
        for (uint32_t i = i0 + 15u; i < a.p.n_r0lab && a.r0lab[i] == lbv; i++) mark(a.p.r0pos[i]);
    };
    const bool vec = ((((uintptr_t)(lab + lo)) | (word ? (uintptr_t)(word + lo) : 0u)) & 15u) == 0u;
    for (uint32_t base = lo; base < hi; base += DXL_BATCH * NEMO_BLOCK) {
      uint32_t lb[DXL_BATCH], wd[DXL_BATCH], dv[DXL_BATCH];
      if (vec) {
#pragma unroll
        for (int g4 = 0; g4 < DXL_BATCH / 4; g4++) {
          const uint32_t x = base + 4 * (g4 * NEMO_BLOCK + tid);
          uint4 l4 = make_uint4(NEMO_NONE, NEMO_NONE, NEMO_NONE, NEMO_NONE), w4 = make_uint4(0, 0, 0, 0);
          if (x + 3 < hi) {
            l4 = *reinterpret_cast<const uint4 *>(lab + x);
            if (word) w4 = *reinterpret_cast<const uint4 *>(word + x);
          } else {
            if (x < hi) l4.x = lab[x], w4.x = word ? word[x] : 0u;
            if (x + 1 < hi) l4.y = lab[x + 1], w4.y = word ? word[x + 1] : 0u;
            if (x + 2 < hi) l4.z = lab[x + 2], w4.z = word ? word[x + 2] : 0u;
          }
          lb[4 * g4] = l4.x, lb[4 * g4 + 1] = l4.y, lb[4 * g4 + 2] = l4.z, lb[4 * g4 + 3] = l4.w;
          wd[4 * g4] = w4.x, wd[4 * g4 + 1] = w4.y, wd[4 * g4 + 2] = w4.z, wd[4 * g4 + 3] = w4.w;
        }
      } else {
#pragma unroll
        for (int q = 0; q < DXL_BATCH; q++) {
          const uint32_t x = base + q * NEMO_BLOCK + tid;
          lb[q] = x < hi ? lab[x] : NEMO_NONE;
          wd[q] = x < hi && word ? word[x] : 0u;
        }
      }
      STAMP2(11);
#pragma unroll
      for (int q = 0; q < DXL_BATCH; q++) dv[q] = lb[q] < a.nlab && !is_rule(wd[q]) ? a.r0dense[lb[q]] : NEMO_NONE;
      STAMP2(12);
#pragma unroll
      for (int q = 0; q < DXL_BATCH; q++) mark_dense(lb[q], dv[q]);
    }
  }
  for (uint32_t base = lo; base < hi && !a.r0dense; base += DXL_BATCH * NEMO_BLOCK) {
    uint32_t lb[DXL_BATCH], h[DXL_BATCH], pos[DXL_BATCH], live = 0;
#pragma unroll
    for (int q = 0; q < DXL_BATCH; q++) {
      const uint32_t x = base + q * NEMO_BLOCK + tid;
      const bool in = x < hi && (!word || !is_rule(word[x]));
      lb[q] = in ? lab[x] : 0u;
      h[q] = hash_label(lb[q]) & a.r0hmask;
      pos[q] = NEMO_NONE;
      live |= (in ? 1u : 0u) << q;
    }
    while (live) {
      uint32_t k[DXL_BATCH];
#pragma unroll
      for (int q = 0; q < DXL_BATCH; q++) k[q] = ((live >> q) & 1u) ? a.r0hkey[h[q]] : 0u;
#pragma unroll
      for (int q = 0; q < DXL_BATCH; q++) {
        if (!((live >> q) & 1u)) continue;
        if (k[q] == lb[q] + 1u) {
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
    for (int q = 0; q < DXL_BATCH; q++)
      if (pos[q] != NEMO_NONE) pos[q] = a.r0hval[pos[q]];
#pragma unroll
    for (int q = 0; q < DXL_BATCH; q++) {
      if (pos[q] == NEMO_NONE) continue;
      for (uint32_t i = pos[q]; i < a.p.n_r0lab && a.r0lab[i] == lb[q]; i++) mark(a.p.r0pos[i]);
    }
  }
  if (!lds) return;
  STAMP2(13);
  __syncthreads();
  for (uint32_t w = tid; w < a.w32; w += NEMO_BLOCK) {
    if (a.lab_split == 1) pb[w] = bm[w];
    else if (bm[w]) atomicOr(&pb[w], bm[w]);
  }
  STAMP2(14);
}

// ---- Good words: chunk c's 64 bitmaps transposed, one wave per 64 positions ----------
// lane e holds source 64c+e's bitmap words for the 64 positions; 64 ballots
// hand position p0+l's 64 source bits to lane l.
__global__ __launch_bounds__(NEMO_BLOCK) void k_dx_good(DxArgs a) {
  const uint32_t c = blockIdx.y, lane = lane_id(), V = a.p.V0;
  const uint32_t p0 = (blockIdx.x * (NEMO_BLOCK / 64) + (threadIdx.x >> 6)) * 64u;
  if (p0 >= V) return;  // wave-uniform
  const uint32_t u = c * 64u + lane;
  const bool valid = u < a.nu;
  const uint32_t *row = a.pb + (size_t)(valid ? u : 0u) * a.w32;
  const uint32_t wi = p0 >> 5;
  const uint32_t w0 = valid ? row[wi] : 0u;
  const uint32_t w1 = (valid && wi + 1 < a.w32) ? row[wi + 1] : 0u;
  uint64_t pres = 0;
#pragma unroll
  for (uint32_t b = 0; b < 32; b++) {
    const uint64_t m = __ballot((w0 >> b) & 1u);
    pres = lane == b ? m : pres;
  }
#pragma unroll
  for (uint32_t b = 0; b < 32; b++) {
    const uint64_t m = __ballot((w1 >> b) & 1u);
    pres = lane == 32u + b ? m : pres;
  }
  const uint64_t vm = __ballot(valid);
  const uint32_t pos = p0 + lane;
  if (pos < V) a.gw[(size_t)c * V + pos] = (a.p.info[pos] & DXI_RULE) ? 0ull : (~pres & vm);
}

// ---- the windowed walk ------------------------------------------------------------------
// MODE 0: Bwd* reachability, T = u64 (64 sources per bit column), one walker,
//         over children in reversed Kahn order (image m1); value = Good | OR(links).
//         When the walk is done the workgroup also writes the chunk's leaf
//         candidates LC(x) = B(x) & ~OR(B of x's children) for goals x.
// MODE 2: longest paths from Good, T = u32, NE walkers (sources NE·bx + e), Kahn
//         order over parents (image m0):
//           val(v) = max(Good(v), max over parents p of c(val(p))), c(x) = x + (x > 0)
//         so val(v) = 1 + the longest path from a Good goal to v, and 0 off
//         Fwd*(Good).  For v in D = Fwd* ∩ Bwd* this is depth(v) + 1, the reference's
//         depth (:82-98): every path from a Good goal to a D node stays in D, and a
//         D node without a D parent is a Good goal.  The walk needs no D and no Fwd*
//         walk: it runs beside the Bwd* walk (one launch, k_dx_walks).
// WHOLE: the graph is one window (ring = positions, no wrap, no misses).
//
// Windows are pipelined: while the walker waves walk window k, the other
// ("worker") waves finalize window k - 1 (values to HBM) and stage window k + 1
// (its link records and steps copied from the image into the other LDS buffer,
// every position's init value, with the values of its links that leave the
// ring folded in from HBM, into its ring slot); one barrier per window.  The
// image's ring misses make this safe (dxi_far_end).
//
// A walk step is <= 256 links of one level, lanes over links: read the linked
// values, apply them to the owners' slots with LDS atomics.  Lane l takes the
// step's links 4l..4l+3, one per atomic instruction: a row's consecutive links
// (one owner) go to different instructions, as lanes of one instruction on one
// slot would be applied one after another.  A step only reads
// slots of earlier levels and a wave's LDS operations complete in order, so
// no barrier separates steps; the next step's records are read during the
// step before, and step descriptors come 64 at a time (one LDS read per 64
// steps), so a step costs one LDS round trip.
template <typename T, int NE>
struct DxLds {
  T *ring0;          // NE rings of [R + 1 + 64] (stride rs): [R] the identity (sink), [R + 1 + lane] dump slots
  uint32_t rs;
  uint32_t *lk;      // [NB][EC] link records of a window
  uint32_t *st;      // [NB][64] its first 64 step descriptors (the rest is read from the image)
};
template <typename T, int NE>
__host__ __device__ inline uint32_t dx_lds_bytes(uint32_t W, uint32_t R, uint32_t EC, bool whole) {
  const uint32_t NB = whole ? 1u : 2u;
  (void)W;
  return NE * lds_align((uint32_t)sizeof(T) * (R + 65u)) + NB * lds_align(4u * EC) + NB * 256u;
}
// the fused Bwd* workgroup's extra LDS past its own image: leaf candidates (u64) and rule
// flags (u8), by reversed walk index
__host__ __device__ inline uint32_t dx_fuse_bytes(uint32_t V, uint32_t EC) {
  (void)EC;
  return lds_align(8u * V) + lds_align(V);
}
template <typename T, int NE>
__device__ __forceinline__ DxLds<T, NE> dx_carve(void *base, uint32_t R, uint32_t EC, bool whole) {
  const uint32_t NB = whole ? 1u : 2u;
  uint8_t *p = (uint8_t *)base;
  DxLds<T, NE> L;
  L.ring0 = (T *)p;
  L.rs = lds_align((uint32_t)sizeof(T) * (R + 65u)) / (uint32_t)sizeof(T);
  p += NE * lds_align((uint32_t)sizeof(T) * (R + 65u));
  L.lk = (uint32_t *)p;
  p += NB * lds_align(4u * EC);
  L.st = (uint32_t *)p;
  return L;
}
// (val <= the nodes on a path <= V0: u32 values never overflow)
#define DXP_B 256        // k_dx_lp: threads per workgroup
#define DXF_K 6          // positions per thread and round of the leaf-candidate and fused LP passes

template <int NE, int NT>
__device__ __forceinline__ void dx_lp_fused(const DevCorpus &c, const DxArgs &a, uint32_t chunk, uint32_t grp,
                                            const uint32_t *ring0, uint32_t rs, uint8_t *lpb);

// The fused walks' hand-off from a chunk's Bwd* workgroup to its longest-path workgroups
// (one writer, several readers, flag values 1 then 2 per call; k_dx_label zeroes the flags).
//   writer: payload stores by every wave; each wave drains them (s_waitcnt vmcnt(0)); a
//           workgroup barrier; then one lane stores the flag with an agent-scope RELEASE
//           (buffer_wbl2 sc1 + s_waitcnt: every store of this workgroup that L2 acknowledged
//           reaches memory before the flag does -- without the release, the write-through
//           payload and the flag go out through different L2 channels and the flag can land
//           first; that was round 5's r05aa D-mask mismatch, test_deep_shape, per-run mode).
//   reader: one lane polls the flag (relaxed, agent scope), then an agent-scope ACQUIRE fence
//           (buffer_inv sc1: the CU's L1 and this XCD's L2 drop stale lines), then a workgroup
//           barrier; the other waves' payload loads are ordered after it by the barrier.
// Forward progress: readers spin, so every writer must be dispatched while readers wait.  The
// writers are blocks [0, nch) of the launch and the hardware dispatches a grid's workgroups in
// blockIdx order, so a writer is resident before any reader of its chunk.  The spin is bounded
// all the same (DX_SPIN_MAX polls, seconds): past it the reader gives up, raises DX_ERR_HANDOFF in
// the call's row counter and the host fails the call (nemo_fetch_missing) instead of hanging.
#define DX_SPIN_MAX (1u << 21)
__device__ __forceinline__ void dx_publish(uint32_t *flag, uint32_t v) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

template <int MODE, int NE, bool WHOLE, int NT>
__device__ __forceinline__ void dx_walk(const DevCorpus &c, const DxArgs &a, const DxImg &m0, const DxImg &m1,
                                        uint32_t bx, uint8_t *dyn) {
  using T = typename std::conditional<MODE == 0, uint64_t, uint32_t>::type;
  const uint32_t tid = threadIdx.x, lane = lane_id(), wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr bool rev = MODE == 0;
  const DxImg &m = rev ? m1 : m0;
  const uint32_t V = a.p.V0, R = m.R, EC = m.EC;
  // MODE 2: workgroup bx takes sources 64 chunk + NE g + e (e < NE, NE g + e < 64) of its chunk
  constexpr uint32_t GPC = (64u + NE - 1u) / NE;  // workgroups per chunk
  const uint32_t chunk = MODE == 0 ? bx : bx / GPC, grp = MODE == 0 ? 0u : bx % GPC;
  DxLds<T, NE> L = dx_carve<T, NE>(dyn, R, EC, WHOLE);
  const uint32_t *rowp = rev ? a.p.fp : a.p.rp;
  // per walker e: its source (MODE 2), ring and value array, computed from e (a
  // dynamically indexed register array would live in scratch memory)
  auto srcu = [&](uint32_t e) -> uint32_t {  // NEMO_NONE: no source
    if (MODE == 0) return 0u;
    const uint32_t b = grp * NE + e, u = 64u * chunk + b;
    return b < 64u && u < a.nu ? u : NEMO_NONE;
  };
  auto ringp = [&](uint32_t e) -> T * { return L.ring0 + (size_t)e * L.rs; };
  uint64_t *const bwv = a.bw + (size_t)chunk * V;
  auto sval = [&](uint32_t e) -> uint32_t * {
    return a.sval + (size_t)min(64u * chunk + min(grp * NE + e, 63u), a.nu - 1u) * V;
  };
  // this workgroup's Fwd* byte plane (bit e: source 64 chunk + NE grp + e), MODE 2
  uint8_t *const fbp = a.fb + ((size_t)chunk * GPC + grp) * V;
  auto slot = [&](uint32_t i) -> uint32_t { return WHOLE ? i : (i & (R - 1u)); };
  if (tid < (uint32_t)NE) ringp(tid)[R] = (T)0;  // the sink reads as "no value": OR 0, max 0
  // ---- staging of window kw by threads [wt0, wt0 + nwt) (whole waves) ----
  auto stage = [&](uint32_t kw, uint32_t buf, uint32_t wt, uint32_t nwt) {
    const uint32_t w0 = m.wb[kw], w1 = m.wb[kw + 1], n = w1 - w0;
    const uint32_t base = rowp[w0], ne = rowp[w1] - base;
    const uint32_t st0 = m.stepb[kw], nst = m.stepb[kw + 1] - st0;
    uint32_t *lk = L.lk + buf * EC, *st = L.st + buf * 64u;
    // records, in 16-B chunks of the image
    const uint32_t c0 = base >> 2, c1 = (base + ne + 3u) >> 2;
    for (uint32_t cb = c0; cb < c1; cb += 2 * nwt) {
      uint4 v4[2];
#pragma unroll
      for (int q = 0; q < 2; q++) {
        const uint32_t ck = cb + q * nwt + wt;
        v4[q] = ck < c1 ? reinterpret_cast<const uint4 *>(m.rec)[ck] : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 2; q++) {
        const uint32_t ck = cb + q * nwt + wt;
        const uint32_t qs[4] = {v4[q].x, v4[q].y, v4[q].z, v4[q].w};
#pragma unroll
        for (int b = 0; b < 4; b++) {
          const uint32_t j = 4 * ck + b;
          if (ck < c1 && j >= base && j < base + ne) lk[j - base] = qs[b];
        }
      }
    }
    if (wt < 64u) st[wt] = wt < nst ? m.steps[st0 + wt] : 0u;
    // init values (Good) with the misses folded in
    for (uint32_t k0 = 0; k0 < n; k0 += nwt) {
      const uint32_t kk = k0 + wt;
      const bool in = kk < n;
      const uint32_t i = w0 + (in ? kk : 0u), pos = rev ? V - 1u - i : i;
      const uint32_t mo0 = !WHOLE && in ? m.moff[i] : 0u, mo1 = !WHOLE && in ? m.moff[i + 1] : 0u;
      const uint64_t gd = in ? a.gw[(size_t)chunk * V + pos] : 0ull;
      if (MODE == 0) {
        T v = (T)gd;
        for (uint32_t mm = mo0; mm < mo1; mm++)
          v |= __hip_atomic_load(bwv + m.mx[mm], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (in) ringp(0)[slot(i)] = v;
      } else {
        uint32_t r[NE];
#pragma unroll
        for (int e = 0; e < NE; e++) r[e] = grp * NE + e < 64u ? (uint32_t)((gd >> (grp * NE + e)) & 1ull) : 0u;
        for (uint32_t mm = mo0; mm < mo1; mm++) {
          const uint32_t x = m.mx[mm];
#pragma unroll
          for (int e = 0; e < NE; e++)
            if (srcu(e) != NEMO_NONE) {
              const uint32_t v = __hip_atomic_load(sval(e) + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              r[e] = max(r[e], v + (v ? 1u : 0u));
            }
        }
#pragma unroll
        for (int e = 0; e < NE; e++)
          if (in) ringp(e)[slot(i)] = r[e];
      }
    }
  };
  // ---- finalize of window kw: values to HBM ----
  auto finalize = [&](uint32_t kw, uint32_t wt, uint32_t nwt) {
    const uint32_t w0 = m.wb[kw], n = m.wb[kw + 1] - w0;
    for (uint32_t kk = wt; kk < n; kk += nwt) {
      const uint32_t i = w0 + kk, sl = slot(i);
      if (MODE == 0) {
        if (!WHOLE) bwv[i] = ringp(0)[sl];
      } else {
        uint32_t fbits = 0;
#pragma unroll
        for (int e = 0; e < NE; e++) {
          if (srcu(e) == NEMO_NONE) continue;
          const uint32_t v = (uint32_t)ringp(e)[sl];
          if (!WHOLE || !a.fuse) sval(e)[i] = v;  // fused: values stay in LDS
          fbits |= (v ? 1u : 0u) << e;
        }
        fbp[i] = (uint8_t)fbits;
      }
    }
  };
  // ---- the walk of window kw by wave e ----
  auto walk = [&](uint32_t kw, uint32_t buf, uint32_t e) {
    const uint32_t st0 = __builtin_amdgcn_readfirstlane(m.stepb[kw]);
    const uint32_t nst = __builtin_amdgcn_readfirstlane(m.stepb[kw + 1]) - st0;
    const uint32_t *lk = L.lk + buf * EC, *st = L.st + buf * 64u;
    T *ring = ringp(e);
    const uint32_t idle = R | ((R + 1u + lane) << 16);
    auto apply = [&](uint32_t rec, T x) {
      if (MODE == 0) atomicOr((unsigned long long *)&ring[rec >> 16], (unsigned long long)x);
      else atomicMax((uint32_t *)&ring[rec >> 16], (uint32_t)x + ((uint32_t)x ? 1u : 0u));
    };
    if (!nst) return;
    // step descriptors 64 at a time: the first 64 staged in LDS, the next
    // batches read from the image a batch ahead (in flight while 64 steps run)
    uint32_t bat = st[lane];
    const uint32_t d = __builtin_amdgcn_readlane(bat, 0);
    uint32_t rc[4];
#pragma unroll
    for (int q = 0; q < 4; q++) rc[q] = 4u * lane + q < (d >> 16) ? lk[(d & 0xFFFFu) + 4u * lane + q] : idle;
    // nothing in flight at the loop entry (the compiler's wait counting sees
    // this wait): a step then waits only for its own reads
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    for (uint32_t b0 = 0; b0 < nst; b0 += 64u) {
      const uint32_t nbat = b0 + 64u + lane < nst ? m.steps[st0 + b0 + 64u + lane] : 0u;
      const uint32_t ns = min(64u, nst - b0);
      for (uint32_t s = 0; s < ns; s++) {
        T x[4];
#pragma unroll
        for (int q = 0; q < 4; q++) x[q] = ring[rc[q] & 0xFFFFu];
        // the next step's records (0 past the last step)
        const uint32_t d1 = s + 1u < 64u ? __builtin_amdgcn_readlane(bat, s + 1u) : __builtin_amdgcn_readlane(nbat, 0);
        uint32_t rn[4];
#pragma unroll
        for (int q = 0; q < 4; q++) rn[q] = 4u * lane + q < (d1 >> 16) ? lk[(d1 & 0xFFFFu) + 4u * lane + q] : idle;
#pragma unroll
        for (int q = 0; q < 4; q++) apply(rc[q], x[q]);
#pragma unroll
        for (int q = 0; q < 4; q++) rc[q] = rn[q];
      }
      bat = nbat;
    }
  };
  bool any = MODE == 0;
  for (uint32_t e = 0; e < (uint32_t)NE; e++) any |= srcu(e) != NEMO_NONE;
  if (!any) return;  // workgroup-uniform
  const bool walker = wv < (uint32_t)NE && (MODE == 0 || srcu(wv) != NEMO_NONE);
  const bool worker = wv >= (uint32_t)NE;
  const uint32_t wt = tid - NE * 64u, nwt = NT - NE * 64u;
  const uint32_t nw = m.nw[0];
  STAMP(0);
  stage(0, 0, tid, NT);
  __syncthreads();
  // fused Bwd* workgroup: its spare LDS (the launch's LDS is sized for the longest-path
  // workgroups) takes the leaf candidates and the rule flags, by reversed walk index
  const uint32_t fz0 = dx_lds_bytes<T, NE>(m.W, R, EC, true);
  uint64_t *const lcl = (uint64_t *)(dyn + fz0);
  uint8_t *const rl = (uint8_t *)(dyn + fz0 + lds_align(8u * V));
  if (WHOLE) {
    STAMP(1);
    if (walker) {
      walk(0, 0, wv);
    } else if (MODE == 0 && a.fuse) {  // the idle waves fetch the rule flags while wave 0 walks
      for (uint32_t i = tid - 64u; i < V; i += NT - 64u) {
        rl[i] = (uint8_t)(a.p.info[V - 1u - i] & DXI_RULE);
        lcl[i] = 0;
      }
    }
    __syncthreads();
    STAMP(2);
    if (MODE == 0 || !a.fuse) finalize(0, tid, NT);  // fused: the values stay in LDS, D overwrites Fwd*
    STAMP(3);
    if (MODE == 2 && a.fuse) {  // the link records are dead: their LDS holds the LP bytes
      dx_lp_fused<NE, NT>(c, a, chunk, grp, (const uint32_t *)L.ring0, L.rs, (uint8_t *)L.lk);
      return;
    }
  } else {
    for (uint32_t k = 0; k < nw; k++) {
      if (walker) {
        walk(k, k & 1u, wv);
      } else if (worker) {
        if (k > 0) finalize(k - 1, wt, nwt);
        if (k + 1 < nw) stage(k + 1, (k + 1) & 1u, wt, nwt);
        // finalized values reach this XCD's L2 before a later staging reads them
        // back with L2-served loads (the stores' completion is all that is needed)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
    }
    finalize(nw - 1, tid, NT);
  }
  // leaf candidates of the chunk: goals in Bwd* none of whose children is (a D
  // goal's children are all in Fwd*, so its D children are its Bwd* children).
  // Whole graphs: from the ring, here; windowed walks: k_dx_lc over the grid (one
  // workgroup re-reading a 1M-node graph's rows from HBM was the walks' long pole)
  if (MODE != 0 || !WHOLE) return;
  __syncthreads();
  if (a.fuse) {
    // two hand-offs to the chunk's longest-path workgroups (write-through stores, a drain per
    // storing wave, an agent-scope flag): Bwd* right after the walk (flag 1: they form D and
    // the masks meanwhile), then the rules' leaf-child words (flag 2)
    for (uint32_t i = tid; i < V; i += NT)
      __hip_atomic_store(bwv + i, (uint64_t)ringp(0)[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    dx_publish(a.wflag + chunk, 1u);
    // leaf candidates LC(x) = B(x) & ~OR B(children) of goals, then per rule the OR of its
    // children's LC (the longest-path workgroups' LP test: a D rule with an LC child), all
    // from LDS; the rules' words go to HBM (lw by position)
    // over the links of the whole-graph image (still in LDS: owner's slot << 16 | child's
    // slot, slots = reversed walk indices) with LDS atomics, then per index
    uint64_t *const rw = (uint64_t *)ringp(0);
    const uint32_t *lk = L.lk, E0 = a.p.E0;
    for (uint32_t j = tid; j < E0; j += NT) {  // goals: the OR of their children's B
      const uint32_t rec = lk[j], o = rec >> 16, x = rec & 0xFFFFu;
      if (!rl[o]) {
        const uint64_t v = rw[x];
        if (v) atomicOr((unsigned long long *)&lcl[o], (unsigned long long)v);
      }
    }
    __syncthreads();
    for (uint32_t i = tid; i < V; i += NT) {  // LC; the ring is free after this
      const uint64_t b = rw[i];
      lcl[i] = rl[i] ? 0ull : b & ~lcl[i];
      rw[i] = 0;
    }
    __syncthreads();
    STAMP(4);
    for (uint32_t j = tid; j < E0; j += NT) {  // rules: the OR of their children's LC, in the ring
      const uint32_t rec = lk[j], o = rec >> 16, x = rec & 0xFFFFu;
      if (rl[o]) {
        const uint64_t v = lcl[x];
        if (v) atomicOr((unsigned long long *)&rw[o], (unsigned long long)v);
      }
    }
    __syncthreads();
    uint64_t *olw = a.lw + (size_t)chunk * V;
    for (uint32_t i = tid; i < V; i += NT)
      __hip_atomic_store(olw + (V - 1u - i), rw[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    dx_publish(a.wflag + chunk, 2u);
    STAMP(5);
    return;
  }
  uint64_t *lc = a.lw + (size_t)chunk * V;
  const T *rg = ringp(0);
  // DXF_K indices per thread and round, the rows' loads in flight together, then the
  // children's ring slots four children at a time
  for (uint32_t base = 0; base < V; base += DXF_K * NT) {
    uint32_t j0[DXF_K], j1[DXF_K];
    uint64_t b[DXF_K], ch[DXF_K];
    bool goal[DXF_K];
#pragma unroll
    for (int k = 0; k < DXF_K; k++) {  // i: reversed walk index, its row = the children
      const uint32_t i = base + k * NT + tid;
      const bool in = i < V;
      goal[k] = in && !(a.p.info[V - 1u - min(i, V - 1u)] & DXI_RULE);
      j0[k] = in ? rowp[i] : 0u;
      j1[k] = in ? rowp[i + 1] : 0u;
      b[k] = in ? (uint64_t)rg[i] : 0ull;
      ch[k] = 0;
      if (in) bwv[i] = b[k];
    }
#pragma unroll
    for (int k = 0; k < DXF_K; k++)
      if (!goal[k] || !b[k]) j1[k] = j0[k];
    for (;;) {
      bool more = false;
#pragma unroll
      for (int k = 0; k < DXF_K; k++) more |= j0[k] < j1[k];
      if (!more) break;
      uint32_t x[DXF_K][4];
#pragma unroll
      for (int k = 0; k < DXF_K; k++)
#pragma unroll
        for (int q = 0; q < 4; q++) x[k][q] = j0[k] + q < j1[k] ? a.p.fc[j0[k] + q] : R;  // R: the sink (0)
#pragma unroll
      for (int k = 0; k < DXF_K; k++) {
#pragma unroll
        for (int q = 0; q < 4; q++) ch[k] |= (uint64_t)rg[x[k][q]];
        j0[k] = min(j0[k] + 4u, j1[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < DXF_K; k++) {
      const uint32_t i = base + k * NT + tid;
      if (i < V) lc[V - 1u - i] = goal[k] ? b[k] & ~ch[k] : 0ull;
    }
  }
}

// Whole-graph walks, fused: a longest-path workgroup holds its NE sources' values over
// every position.  Once its chunk's Bwd* workgroup has published Bwd* (flag 1) it forms D
// and (one entry per source) writes the D masks; once the rules' leaf-child words follow
// (flag 2) it finds the sources' LP rules (D rules with a leaf-candidate child), maxLen (an
// LDS maximum: no other workgroup holds these sources) and the missing rows (LP rules with
// val == maxLen), in place of k_dx_lp, k_dx_emit and k_dx_mask.  Without its own masks its
// Fwd* byte plane is overwritten with D (k_dx_mask reads D there).
template <int NE, int NT>
__device__ __forceinline__ void dx_lp_fused(const DevCorpus &c, const DxArgs &a, uint32_t chunk, uint32_t grp,
                                            const uint32_t *ring0, uint32_t rs, uint8_t *lpb) {
  (void)c;
  __shared__ uint32_t s_max[NE];
  const uint32_t tid = threadIdx.x, V = a.p.V0, sh = grp * NE;
  constexpr uint32_t NM = (1u << NE) - 1u;
  uint32_t live = 0;  // this workgroup's sources (bit e: source 64 chunk + NE grp + e)
#pragma unroll
  for (int e = 0; e < NE; e++) live |= (sh + e < 64u && 64u * chunk + sh + e < a.nu ? 1u : 0u) << e;
  if (tid < (uint32_t)NE) s_max[tid] = 0;
  // the first round's static loads (rule flags, node positions) before the wait
  uint32_t pinf[DXF_K], ptp[DXF_K];
#pragma unroll
  for (int k = 0; k < DXF_K; k++) {
    const uint32_t p = min(k * NT + tid, V - 1u);
    pinf[k] = a.p.info[p];
    ptp[k] = a.own_mask ? a.p.tpos[p] : 0u;
  }
  // one lane polls the chunk's flag until it reaches `want` (bounded: dx_publish), then one
  // acquire for the workgroup
  auto wait_flag = [&](uint32_t want) {
    if (tid == 0) {
      uint32_t n = 0;
      while (__hip_atomic_load(a.wflag + chunk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
        if (++n == DX_SPIN_MAX) {
          atomicOr(a.n_missing, DX_ERR_HANDOFF);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  };
  wait_flag(1);  // Bwd*
  STAMP(4);
  // D by position, in LDS past the LP bytes (and over the Fwd* plane for k_dx_mask when the
  // masks are not written here)
  const bool own = a.own_mask != 0u;
  uint8_t *const dl = lpb + ((V + 15u) & ~15u);
  uint8_t *dpl = a.fb + ((size_t)chunk * ((64u + NE - 1u) / NE) + grp) * V;
  uint32_t mx[NE];
#pragma unroll
  for (int e = 0; e < NE; e++) mx[e] = 0;
  const uint64_t *bw = a.bw + (size_t)chunk * V, *lw = a.lw + (size_t)chunk * V;
  for (uint32_t base = 0; base < V; base += DXF_K * NT) {  // DXF_K positions per thread, loads together
    uint64_t b[DXF_K];
#pragma unroll
    for (int k = 0; k < DXF_K; k++) b[k] = bw[V - 1u - min(base + k * NT + tid, V - 1u)];
#pragma unroll
    for (int k = 0; k < DXF_K; k++) {
      const uint32_t pos = base + k * NT + tid;
      if (pos >= V) continue;
      uint32_t f = 0;
#pragma unroll
      for (int e = 0; e < NE; e++) {
        const uint32_t v = ring0[(size_t)e * rs + pos];
        f |= (v ? 1u : 0u) << e;
      }
      const uint32_t d = f & live & (uint32_t)(b[k] >> sh) & NM;
      dl[pos] = (uint8_t)d;
      if (!own) dpl[pos] = (uint8_t)d;
    }
  }
  __syncthreads();
  // one entry per source: the D masks by node, consecutive nodes per wave (coalesced bytes),
  // while the Bwd* workgroup computes the leaf candidates
  if (own) {
    uint32_t ent[NE];
#pragma unroll
    for (int e = 0; e < NE; e++) ent[e] = ((live >> e) & 1u) ? a.urep[64u * chunk + sh + e] : 0u;
    for (uint32_t base = 0; base < V; base += DXF_K * NT) {
      uint32_t tp[DXF_K];  // every position loaded before the byte stores (which may alias)
#pragma unroll
      for (int k = 0; k < DXF_K; k++) tp[k] = base == 0 ? ptp[k] : a.p.tpos[min(base + k * NT + tid, V - 1u)];
#pragma unroll
      for (int k = 0; k < DXF_K; k++) {
        const uint32_t v = base + k * NT + tid;
        if (v >= V) continue;
        const uint32_t d = dl[tp[k]];
#pragma unroll
        for (int e = 0; e < NE; e++)
          if ((live >> e) & 1u) a.mask[(size_t)ent[e] * V + v] = (uint8_t)((d >> e) & 1u);
      }
    }
  }
  wait_flag(2);  // the rules' leaf-child words
  // LP = D rules with a leaf-candidate child; their longest val per source
  for (uint32_t base = 0; base < V; base += DXF_K * NT) {
    uint32_t inf[DXF_K];
    uint64_t o[DXF_K];
#pragma unroll
    for (int k = 0; k < DXF_K; k++) {
      const uint32_t p = min(base + k * NT + tid, V - 1u);  // clamped, unconditional: all loads in flight
      inf[k] = base == 0 ? pinf[k] : a.p.info[p];
      o[k] = lw[p];
    }
#pragma unroll
    for (int k = 0; k < DXF_K; k++) {
      const uint32_t pos = base + k * NT + tid;
      if (pos >= V) continue;
      const uint32_t lp = (inf[k] & DXI_RULE) ? dl[pos] & (uint32_t)(o[k] >> sh) & NM : 0u;
#pragma unroll
      for (int e = 0; e < NE; e++)
        if ((lp >> e) & 1u) mx[e] = max(mx[e], ring0[(size_t)e * rs + pos]);
      lpb[pos] = (uint8_t)lp;
    }
  }
  // maxima: the wave's, then one LDS atomic per wave and source
#pragma unroll
  for (int e = 0; e < NE; e++) {
    uint32_t x = mx[e];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, o));
    if (lane_id() == 0 && x) atomicMax(&s_max[e], x);
  }
  __syncthreads();
  STAMP(5);
  if (tid < (uint32_t)NE && ((live >> tid) & 1u)) a.maxlen[64u * chunk + sh + tid] = s_max[tid];
  // the rows: counted per thread, one block scan and one global atomic per workgroup
  __shared__ uint32_t s_scan[NT / 64], s_base;
  auto hits = [&](uint32_t pos) -> uint32_t {
    const uint32_t lp = lpb[pos];
    uint32_t h = 0;
    if (lp) {
#pragma unroll
      for (int e = 0; e < NE; e++)
        if (((lp >> e) & 1u) && ring0[(size_t)e * rs + pos] == s_max[e]) h |= 1u << e;
    }
    return h;
  };
  uint32_t cnt = 0;
  for (uint32_t pos = tid; pos < V; pos += NT) cnt += (uint32_t)__popc(hits(pos));
  uint32_t tot;
  uint32_t q = block_exscan<NT>(cnt, &tot, s_scan);
  if (tid == 0 && tot) s_base = atomicAdd(a.n_missing, tot) & DX_ROWS;
  if (!tot) return;  // workgroup-uniform
  __syncthreads();
  q += s_base;
  for (uint32_t pos = tid; pos < V && cnt; pos += NT) {
    const uint32_t h = hits(pos);
    if (!h) continue;
    const uint32_t node = a.p.pnode[pos];
#pragma unroll
    for (int e = 0; e < NE; e++) {
      if (!((h >> e) & 1u)) continue;
      a.missing[2 * q] = 64u * chunk + sh + e;
      a.missing[2 * q + 1] = node;
      q++;
      cnt--;
    }
  }
  STAMP(6);
}

// leaf candidates after windowed walks: one thread per (position, chunk)
__global__ __launch_bounds__(NEMO_BLOCK) void k_dx_lc(DxArgs a) {
  const uint32_t c = blockIdx.y, V = a.p.V0;
  const uint32_t i = blockIdx.x * NEMO_BLOCK + threadIdx.x;  // reversed walk index: its row = the children
  if (i >= V) return;
  const uint32_t pos = V - 1u - i;
  const uint64_t *bw = a.bw + (size_t)c * V;
  uint64_t w = 0;
  if (!(a.p.info[pos] & DXI_RULE)) {
    const uint64_t b = bw[i];
    uint64_t ch = 0;
    if (b) {
      const uint32_t j0 = a.p.fp[i], j1 = a.p.fp[i + 1];
      for (uint32_t j = j0; j < j1; j += 4) {
        uint64_t v[4];
#pragma unroll
        for (int q = 0; q < 4; q++) v[q] = j + q < j1 ? bw[a.p.fc[j + q]] : 0ull;
#pragma unroll
        for (int q = 0; q < 4; q++) ch |= v[q];
      }
    }
    w = b & ~ch;
  }
  a.lw[(size_t)c * V + pos] = w;
}

// One launch for both walks: blocks [0, nch) walk Bwd* of their chunk, the rest
// the longest paths of NE sources each.
template <int NE, bool WHOLE, int NT>
__global__ __launch_bounds__(NT) void k_dx_walks(DevCorpus c, DxArgs a, DxImg m0, DxImg m1) {
  extern __shared__ __align__(16) uint8_t dyn[];
  if (blockIdx.x < a.nch) dx_walk<0, 1, WHOLE, NT>(c, a, m0, m1, blockIdx.x, dyn);
  else dx_walk<2, NE, WHOLE, NT>(c, a, m0, m1, blockIdx.x - a.nch, dyn);
}

// ---- D, LP rules and the longest LP path per source ----------------------------------
// D_u(v) = Fwd*_u(v) and Bwd*_u(v) (the walks' planes); LP rule r of source u: r in D_u
// with a D_u-leaf goal child (a leaf candidate child, k_dx_walk).  maxLen_u = max val_u
// over them (:82-98), reduced per workgroup in LDS before one global max per source.
// the values of up to 8 set bits of m at position pos, their loads in flight together
__device__ __forceinline__ uint32_t dx_vals8(const DxArgs &a, uint32_t c, uint32_t pos, uint64_t &m, uint32_t (&e)[8],
                                             uint32_t (&v)[8]) {
  uint32_t n = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    e[k] = m ? (uint32_t)__builtin_ctzll(m) : 64u;
    if (m) {
      m &= m - 1ull;
      n++;
    }
  }
#pragma unroll
  for (int k = 0; k < 8; k++) v[k] = e[k] < 64u ? a.sval[(size_t)(64u * c + e[k]) * a.p.V0 + pos] : 0u;
  return n;
}

template <int NE>
__global__ __launch_bounds__(DXP_B) void k_dx_lp(DxArgs a, uint32_t per) {
  __shared__ uint32_t s_max[64];
  const uint32_t c = blockIdx.y, V = a.p.V0, tid = threadIdx.x;
  if (tid < 64) s_max[tid] = 0;
  __syncthreads();
  for (uint32_t pos = blockIdx.x * DXP_B * per + tid; pos < min(V, (blockIdx.x + 1) * DXP_B * per); pos += DXP_B) {
    constexpr uint32_t GPC = (64u + NE - 1u) / NE;
    uint64_t f = 0;
    const uint8_t *fb = a.fb + (size_t)c * GPC * V + pos;
#pragma unroll
    for (uint32_t g = 0; g < GPC; g++) f |= (uint64_t)fb[(size_t)g * V] << (g * NE);
    const uint32_t r = V - 1u - pos;
    const uint64_t d = f & a.bw[(size_t)c * V + r];
    a.dw[(size_t)c * V + pos] = d;
    uint64_t lp = 0;
    if (d && (a.p.info[pos] & DXI_RULE)) {
      uint64_t ol = 0;
      for (uint32_t j = a.p.fp[r]; j < a.p.fp[r + 1]; j++) ol |= a.lw[(size_t)c * V + (V - 1u - a.p.fc[j])];
      lp = d & ol;
      for (uint64_t m = lp; m;) {
        uint32_t e[8], v[8];
        dx_vals8(a, c, pos, m, e, v);
#pragma unroll
        for (int k = 0; k < 8; k++)
          if (e[k] < 64u) atomicMax(&s_max[e[k]], v[k]);
      }
    }
    a.gw[(size_t)c * V + pos] = lp;
  }
  __syncthreads();
  if (tid < 64 && s_max[tid]) atomicMax(a.maxlen + 64u * c + tid, s_max[tid]);
}
// missing rows: LP rules at the maximal depth, val == maxLen.  Eight threads per
// position, eight sources each: one round of value loads per thread
__global__ __launch_bounds__(NEMO_BLOCK) void k_dx_emit(DxArgs a) {
  const uint32_t c = blockIdx.y, V = a.p.V0;
  const uint32_t t = blockIdx.x * NEMO_BLOCK + threadIdx.x, pos = t >> 3, sub = t & 7u;
  // (no early return: every lane takes part in the wave's append)
  uint64_t lp = pos < V ? a.gw[(size_t)c * V + pos] & (0xFFull << (8u * sub)) : 0ull;
  uint32_t e[8], v[8], ml[8], hit = 0;
  if (!__any(lp != 0ull)) return;  // wave-uniform
  dx_vals8(a, c, pos, lp, e, v);  // at most eight bits: one round
#pragma unroll
  for (int k = 0; k < 8; k++) ml[k] = e[k] < 64u ? a.maxlen[64u * c + e[k]] : 0u;
#pragma unroll
  for (int k = 0; k < 8; k++) hit |= (e[k] < 64u && v[k] == ml[k] ? 1u : 0u) << k;
  // one append per wave (a counter taking one atomic per row serialised the rows)
  uint32_t tot;
  const uint32_t ex = wave_exscan((uint32_t)__popc(hit), &tot);
  if (!tot) return;
  uint32_t base = 0;
  if (lane_id() == 0) base = atomicAdd(a.n_missing, tot);
  uint32_t q = ((__builtin_amdgcn_readfirstlane(base) & DX_ROWS) + ex);
  const uint32_t node = hit ? a.p.pnode[pos] : 0u;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    if (!((hit >> k) & 1u)) continue;
    a.missing[2 * q] = 64u * c + e[k];
    a.missing[2 * q + 1] = node;
    q++;
  }
}

// ---- D masks by node for every entry ------------------------------------------------
// thread: one node, DXM_E consecutive entries, all their loads in flight together.
// D: after fused walks the source's bit of its longest-path workgroup's D byte plane
// (dx_lp_fused), else its bit of the chunk's D word (k_dx_lp)
#define DXM_E 32
__global__ __launch_bounds__(NEMO_BLOCK) void k_dx_mask(DxArgs a) {
  const uint32_t V = a.p.V0, v = blockIdx.x * NEMO_BLOCK + threadIdx.x;
  if (v >= V) return;
  const uint32_t pos = a.p.tpos[v], gpc = (64u + a.ne - 1u) / a.ne;
  const uint32_t e0 = blockIdx.y * DXM_E, n = min(a.n_entries - e0, (uint32_t)DXM_E);
  uint32_t bit[DXM_E];
#pragma unroll
  for (int k = 0; k < DXM_E; k++) {
    const uint32_t u = (uint32_t)k < n ? a.map[e0 + k] : 0u, c = u >> 6, b = u & 63u;
    if (a.fuse) {
      const uint32_t g = b / a.ne;
      bit[k] = (uint32_t)a.fb[((size_t)c * gpc + g) * V + pos] >> (b - g * a.ne);
    } else {
      bit[k] = (uint32_t)(a.dw[(size_t)c * V + pos] >> b);
    }
  }
#pragma unroll
  for (int k = 0; k < DXM_E; k++)
    if ((uint32_t)k < n) a.mask[(size_t)(e0 + k) * V + v] = (uint8_t)(bit[k] & 1u);
}

// ---- launch -----------------------------------------------------------------------------
template <int NE, bool WHOLE, int NT>
static void walks_launch(const DevCorpus &c, const DxArgs &a, hipStream_t s) {
  const DxImg &m = a.img[0];
  const uint32_t bytes =
      std::max(dx_lds_bytes<uint64_t, 1>(m.W, m.R, m.EC, WHOLE), dx_lds_bytes<uint32_t, NE>(m.W, m.R, m.EC, WHOLE));
  // per instantiation and device: the attribute call (host time before the launch) only when
  // the size grows
  static std::atomic<uint32_t> set[64];
  int dev = 0;
  hipGetDevice(&dev);
  std::atomic<uint32_t> &st = set[dev & 63];
  if (bytes > st.load()) {
    hipFuncSetAttribute((const void *)k_dx_walks<NE, WHOLE, NT>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    st.store(bytes);
  }
  const dim3 grid(a.nch * (1u + (64u + NE - 1u) / NE));
  hipLaunchKernelGGL((k_dx_walks<NE, WHOLE, NT>), grid, dim3(NT), bytes, s, c, a, a.img[0], a.img[1]);
}

#define DX_LDS_MAX (160u * 1024u - 1024u)
// windowed configurations: W positions, R ring slots (power of two, >= 4 W), EC links.
// 1024 threads: the Bwd* walk one walker (u64 ring), the longest paths two or
// four (u32 rings; four when the whole graph's image fits LDS with them)
#define DX_NT 1024
struct DxCfg {
  uint32_t W, R, EC;
};
static const DxCfg kWin = {2048, 8192, 8192};
// test knob (window = 2): small windows and rings, so that many links leave them
static const DxCfg kTiny = {512, 2048, 8192};

// every row of g0 must fit one window's links (launch_dx's windowed configurations)
uint32_t dx_max_row() { return kWin.EC; }
uint32_t dx_max_row_tiny() { return kTiny.EC; }

// image 0: Kahn order (longest paths), 1: reversed (Bwd*); the whole graph in one
// window when its image fits LDS (ring slots and link offsets are u16)
void dx_img_configs(uint32_t V, uint32_t E, uint32_t window, DxImg out[2]) {
  const bool small = window == 0 && V + 64u <= 0xFFFFu && E <= 0xFFFFu;
  const uint32_t EC = std::max(E, 1u);
  const bool whole = small && dx_lds_bytes<uint64_t, 1>(V, V, EC, true) <= DX_LDS_MAX &&
                     dx_lds_bytes<uint32_t, 2>(V, V, EC, true) <= DX_LDS_MAX;
  const DxCfg g = window == 2 ? kTiny : kWin;
  for (int k = 0; k < 2; k++) {
    DxImg &m = out[k];
    m.W = whole ? V : g.W;
    m.R = whole ? V : g.R;
    m.EC = whole ? EC : g.EC;
    m.whole = whole ? 1u : 0u;
    m.rev = (uint32_t)k;
  }
}

void launch_dx(const DevCorpus &c, const DxArgs &a_in, hipStream_t s) {
  DxArgs a = a_in;
  const uint32_t V = a.p.V0;
  if (!V || !a.nu) return;
  const uint32_t nbv = (V + NEMO_BLOCK - 1) / NEMO_BLOCK;
  if (a.lab_split > 1 || a.w32 > DXL_LDS) launch_zero(a.pb, (uint64_t)a.nu * a.w32 * 4u, s);
  hipLaunchKernelGGL(k_dx_label, dim3(a.lab_split, a.nu), dim3(NEMO_BLOCK), 0, s, c, a);
  const DxImg &m = a.img[0];
  // positions per k_dx_lp thread: enough workgroups for the chip, few enough that the
  // per-workgroup maxima leave few global atomics per source
  const uint32_t per = std::max(1u, (uint32_t)(((uint64_t)V * a.nch + DXP_B * 2048ull - 1) / (DXP_B * 2048ull)));
  const dim3 glp((V + DXP_B * per - 1) / (DXP_B * per), a.nch);
  // the most longest-path walkers whose rings fit LDS (one round of workgroups over the CUs)
  // whole graphs: the longest-path workgroups finish the call's LP rules and missing rows
  // (their LP and D bytes over the dead link records), the Bwd* workgroup's rows and
  // leaf candidates in the LDS the longest-path workgroups' rings leave it
  const uint32_t ne = dx_lds_bytes<uint32_t, 6>(m.W, m.R, m.EC, true) <= DX_LDS_MAX   ? 6u
                      : dx_lds_bytes<uint32_t, 4>(m.W, m.R, m.EC, true) <= DX_LDS_MAX ? 4u
                                                                                       : 2u;
  const uint32_t bwd = dx_lds_bytes<uint64_t, 1>(m.W, m.R, m.EC, true);
  const uint32_t lds = std::max(bwd, ne == 6   ? dx_lds_bytes<uint32_t, 6>(m.W, m.R, m.EC, true)
                                     : ne == 4 ? dx_lds_bytes<uint32_t, 4>(m.W, m.R, m.EC, true)
                                               : dx_lds_bytes<uint32_t, 2>(m.W, m.R, m.EC, true));
  a.fuse = m.whole && 2u * ((V + 15u) & ~15u) <= 4u * m.EC && bwd + dx_fuse_bytes(V, m.EC) <= lds && !a.legacy_lp ? 1u : 0u;
  hipLaunchKernelGGL(k_dx_good, dim3((V + NEMO_BLOCK - 1) / NEMO_BLOCK, a.nch), dim3(NEMO_BLOCK), 0, s, a);
  if (m.whole && ne == 6) {
    a.ne = 6;
    walks_launch<6, true, DX_NT>(c, a, s);
    if (!a.fuse) hipLaunchKernelGGL(k_dx_lp<6>, glp, dim3(DXP_B), 0, s, a, per);
  } else if (m.whole && ne == 4) {
    a.ne = 4;
    walks_launch<4, true, DX_NT>(c, a, s);
    if (!a.fuse) hipLaunchKernelGGL(k_dx_lp<4>, glp, dim3(DXP_B), 0, s, a, per);
  } else {
    a.ne = 2;
    if (m.whole) {
      walks_launch<2, true, DX_NT>(c, a, s);
    } else {
      walks_launch<2, false, DX_NT>(c, a, s);
      hipLaunchKernelGGL(k_dx_lc, dim3(nbv, a.nch), dim3(NEMO_BLOCK), 0, s, a);
    }
    if (!a.fuse) hipLaunchKernelGGL(k_dx_lp<2>, glp, dim3(DXP_B), 0, s, a, per);
  }
  if (!a.fuse)
    hipLaunchKernelGGL(k_dx_emit, dim3((8 * V + NEMO_BLOCK - 1) / NEMO_BLOCK, a.nch), dim3(NEMO_BLOCK), 0, s, a);
  if (a.n_entries && !(a.fuse && a.own_mask))
    hipLaunchKernelGGL(k_dx_mask, dim3(nbv, (a.n_entries + DXM_E - 1) / DXM_E), dim3(NEMO_BLOCK), 0, s, a);
}

}  // namespace nemo
