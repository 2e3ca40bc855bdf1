// internal.h — host/device interface between the C ABI (api.hip) and the kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

struct DevCorpus;

namespace nemo {

struct DiffArgs {
  uint32_t g0;              // run 0's post graph
  const uint32_t *src;      // [entries] label-source graph per entry
  const uint32_t *ref_labels;  // label mode: [n, label...] used by every entry (NULL: src)
  const uint32_t *r0lab;    // sorted goal labels of g0
  const uint32_t *r0idx;    // local node of each sorted label
  uint32_t n_r0lab;
  const uint32_t *r0hkey;   // open-addressed label -> first sorted entry: key = label + 1 (0 empty)
  const uint32_t *r0hval;
  uint32_t r0hmask;         // table size - 1 (power of two)
  uint8_t *bits;            // [entries * V0] scratch
  int32_t *depth;           // [entries * V0] scratch
  // g0 in Kahn order for the global tier (k_dprep_*): node -> position,
  // parent / child rows as positions, level << 1 | rule, label nodes as positions
  uint32_t *tpos, *trp, *tfp, *trc, *tfc, *tinfo, *r0pos;
  uint8_t *mask;            // [entries * V0] D mask (output)
  uint32_t *missing;        // [2 * cap] (entry, rule)
  uint32_t *n_missing;      // counter
};

// Run 0's post graph g0 relaid in Kahn order (k_dx.hip k_dxp_*, built with the
// CSR in every load / rebuild): positions 0..V0-1 are the Kahn order; parents
// in Kahn order and children in reversed Kahn order ("walk order"), as walk
// indices, so that a window of consecutive positions reads one contiguous row range.
struct DxPrep {
  uint32_t g0, V0, E0;
  uint32_t *tpos;            // [V0] node -> position
  uint32_t *pnode;           // [V0] position -> node (the Kahn order the relayout was built from)
  uint32_t *info;            // [V0] level << 3 | DXI_RULE
  uint32_t *lbeg, *lend;     // [V0] first position of the position's Kahn level / of the next level
  uint32_t *rp, *rc;         // [V0 + 1], [E0 + 4] parents of position i, as positions
  uint32_t *fp, *fc;         // [V0 + 1], [E0 + 4] children of position V0-1-i, as reversed positions
  const uint32_t *r0idx;     // [n_r0lab] node of each sorted run-0 goal label
  uint32_t *r0pos;           // [n_r0lab] its position
  uint32_t n_r0lab;
  uint32_t *r0dense;         // the dense label table (DxArgs::r0dense; null: none): k_dxp_b writes
                             // the run-0 labels' entries, a single position as pos << 4
  const uint32_t *r0lab;     // [n_r0lab] sorted run-0 goal labels
  const uint32_t *err0;      // g0's load error flag (k_build / k_csr / k_topo): set, the CSR and Kahn
                             // order may be partial and every relayout kernel does nothing (the load fails)
};
#define DXI_RULE 1u   // the position is a rule

// A walk image of g0 (k_dx.hip k_dxi_*, built once per load and window
// configuration): the walk order cut into windows, and per window its links
// as ring records, its walk steps (<= 256 links of one level) and, per
// position, the links that leave the ring.  The walks stage a window by
// copying these ranges (no per-window derivation).  Image 0: Kahn order over
// parents (Fwd*, depth), 1: reversed Kahn order over children (Bwd*).
struct DxImg {
  uint32_t W, R, EC;         // positions, ring slots (power of two, >= 4 W; whole: V0), links per window
  uint32_t whole;            // 1: one window, ring = positions (no misses)
  uint32_t rev;              // 1: reversed walk order (children rows)
  uint32_t *nw;              // [1] windows
  uint32_t *wb;              // [V0 + 2] first walk index of window k; wb[nw] = V0
  uint32_t *stepb;           // [V0 + 2] first step of window k; [nw] = total
  uint32_t *steps;           // [2 V0 + E0 / 256 + 4] first link (in the window) | links << 16
  uint32_t *rec;             // [E0 + 4] per link (walk-order rows): linked ring slot (R: a miss) | owner's slot << 16
  uint32_t *moff;            // [V0 + 1] first miss of walk index i in mx
  uint32_t *mx;              // [E0 + 1] walk index linked by each miss
};
struct DxImgScratch {
  uint32_t *fseg;            // [V0 + 1] segment flags -> segment numbers
  uint32_t *segpos;          // [V0 + 2] first walk index of each segment
  uint32_t *fstep;           // [V0 + 1] steps per segment -> first step
  uint32_t *tsum;            // scan tiles
};

// the diff call's row counter (DxArgs::n_missing): rows in the low bits, bit 30 raised when a
// fused walk's hand-off wait gave up (k_dx.hip dx_publish)
#define DX_ROWS 0x3FFFFFFFu
#define DX_ERR_HANDOFF 0x40000000u

// One multi-entry CreateNaiveDiffProv call (k_dx.hip): nu distinct label
// sources in chunks of 64, one bit per source in every u64 word.
struct DxArgs {
  DxPrep p;
  uint32_t nu, nch;          // distinct label sources, 64-source chunks
  const uint32_t *src;       // [nu] label-source graph (post graph of the source run)
  const uint32_t *ref_labels;  // label mode: [n, label...] of the single source (src unused)
  const uint32_t *r0lab, *r0hkey, *r0hval;
  uint32_t r0hmask;
  // label -> its run-0 position << 4 when it labels one run-0 goal, else (first sorted run-0 goal
  // label entry << 4 | min(count, 15)); NEMO_NONE = not a run-0 post-goal label; labels >= nlab are
  // not either (null: the hash table above)
  const uint32_t *r0dense;
  uint32_t nlab;
  uint32_t *pb;              // [nu][w32] present bitmaps over positions
  uint32_t w32;              // ceil(V0 / 32)
  uint32_t lab_per;          // source nodes per k_dx_label workgroup
  uint32_t lab_split;        // workgroups per source (1: LDS bitmap stored whole)
  uint64_t *gw;              // [nch][V0] Good bits by position; after the walks: LP rules (k_dx_lp)
  uint64_t *bw;              // [nch][V0] Bwd*(Good) by REVERSED position (V0 - 1 - pos)
  uint64_t *dw;              // [nch][V0] D = Fwd* & Bwd* by position (k_dx_lp; k_dx_mask reads fb & bw)
  uint64_t *lw;              // [nch][V0] leaf candidates: Bwd* goals without a Bwd* child, by position
  uint8_t *fb;               // [nch][64 / NE][V0] Fwd* bits of the NE sources of longest-path workgroup g
  uint32_t *sval;            // [nu][V0] val = 1 + the longest path from Good (0 off Fwd*) by position
  uint32_t *maxlen;          // [nu] the longest LP val of each source (zeroed per call)
  uint32_t *wflag;           // [nch] Bwd* walk of the chunk done (whole-graph walks; zeroed per call)
  uint32_t ne;               // sources per longest-path workgroup of the walks launched (k_dx_mask)
  uint32_t fuse;             // 1: the longest-path workgroups also take LP rules, maxLen and the missing
                             // rows (whole-graph walks; k_dx_lp / k_dx_emit not launched)
  uint32_t legacy_lp;        // test knob (option diff_fuse 0): no fusion
  const uint32_t *urep;      // [nu] each source's first entry
  uint32_t own_mask;         // 1: one entry per source and fused walks: the longest-path workgroups
                             // write the D masks (k_dx_mask not launched)
  uint8_t *mask;             // [n_entries][V0] D masks by node (output)
  const uint32_t *map;       // [n_entries] entry -> source
  uint32_t n_entries;
  uint32_t *missing;         // [2 * cap] (source, rule node)
  uint32_t *n_missing;
  uint32_t window;           // test knob: 0 by size, 1 windowed walks, 2 tiny windows (ring misses)
  DxImg img[2];              // walk images: Kahn order (Fwd*, depth), reversed (Bwd*)
};

struct PullArgs {
  uint32_t which;           // 0 raw, 1 simplified, 2 diff
  uint32_t g0;              // graph of which == 2
  const uint8_t *mask;      // which == 2: D masks of the entries
  uint64_t mask_stride;     // bytes between two entries' masks
  const uint32_t *mask_row; // which == 2: slot -> the entry whose mask it takes (null: the slot's own)
  uint32_t *cnt;            // [slots] edges of the slot
  uint64_t *off;            // [slots] first edge of the slot in src/dst
  unsigned long long *cursor;  // region allocator (zeroed before the launch)
  uint64_t cap;             // capacity of src/dst
  uint32_t *src, *dst;      // output
  // big slots (graph of >= NEMO_CSR_BIG nodes): multi-workgroup pull over
  // MWP_CH-node chunks, [row slots][maxck] chunk counts -> offsets (null: none)
  uint32_t *ccnt;
  uint32_t maxck;
};

struct TrigArgs {
  uint32_t g_pre, g_post;
  uint32_t *counts;         // [3] pre rows, post rows, async rules
  uint32_t *pre, *post, *async_rules;
};

__host__ __device__ uint32_t build_tier_bytes(uint32_t v, uint32_t e);
void launch_build(const DevCorpus &c, hipStream_t s);
void launch_load(const DevCorpus &c, hipStream_t s);
void launch_topo(const DevCorpus &c, hipStream_t s, bool list = true);
void launch_csr_big(const DevCorpus &c, uint32_t chunks, hipStream_t s);
// per_graph false: no graph below NEMO_CSR_BIG is past the skipped tier (host count), so only the big-graph kernels run
void launch_mark(const DevCorpus &c, bool skip_tier, hipStream_t s, bool per_graph = true);
void launch_simplify(const DevCorpus &c, bool skip_tier, hipStream_t s, bool per_graph = true);
void launch_marksimp(const DevCorpus &c, hipStream_t s, bool skip_built);
void launch_chains(const DevCorpus &c, hipStream_t s, bool tiers = true);
void launch_chains_glob(const DevCorpus &c, hipStream_t s);
uint64_t glob_words(uint64_t V, uint64_t E);  // k_chains_glob scratch of one graph (u32)
uint32_t glob_team_words();                   // k_glob_prep's team scratch (u32)
void launch_proto(const DevCorpus &c, hipStream_t s, bool tiers = true);
void launch_reduce(const DevCorpus &c, const uint8_t *is_success, const uint8_t *owned, uint32_t first_run,
                   uint32_t *red, hipStream_t s);
void launch_diff(const DevCorpus &c, const DiffArgs &a, uint32_t n_entries, uint32_t V0, hipStream_t s);
// entry e's D mask = unique result map[e]'s ([n_entries][V0] from [n_uniq][V0])
void launch_diff_expand(uint8_t *mask, const uint8_t *umask, const uint32_t *map, uint64_t V0, uint32_t n_entries,
                        hipStream_t s);
void launch_dx_prep(const DevCorpus &c, const DxPrep &p, uint32_t *tsum, hipStream_t s);
void launch_dx(const DevCorpus &c, const DxArgs &a, hipStream_t s);
uint32_t dx_max_row();       // the longest row of g0 the multi-entry diff takes
uint32_t dx_max_row_tiny();  // the same under the tiny-window test knob
// window configurations of the two walk images for g0 (V0, E0) under the test knob `window`
void dx_img_configs(uint32_t V0, uint32_t E0, uint32_t window, DxImg out[2]);
void launch_dx_img(const DxPrep &p, DxImg img[2], const DxImgScratch &t, hipStream_t s);
uint32_t dx_scan_tiles(uint32_t n);  // tile sums launch_scan needs for n entries
void launch_scan(uint32_t *a, uint32_t n, uint32_t *tsum, hipStream_t s);  // in-place exclusive scan
// rest: graphs (which 0/1) or g0 (which 2) past k_pull_lds's LDS tier, counted on the host
void launch_pull(const DevCorpus &c, const PullArgs &a, uint32_t slots, uint32_t rest, hipStream_t s);
void launch_chain_pairs(const DevCorpus &c, const uint64_t *off, uint32_t *out, uint64_t cap, int wide,
                        hipStream_t s);
void launch_pack_state(const uint8_t *flags, uint32_t *out, uint64_t V, hipStream_t s);
void launch_chain_gather(const DevCorpus &c, uint64_t *off, uint32_t *out, hipStream_t s);
void launch_triggers(const DevCorpus &c, const TrigArgs &a, int phase, hipStream_t s);
void launch_goal_labels(const DevCorpus &c, uint32_t g, uint32_t *out, hipStream_t s);
void launch_to_host(void *dst, const void *src, uint64_t bytes, hipStream_t s, uint32_t max_blocks = 64);
struct HostCopy {
  uint8_t *dst;
  const uint8_t *src;
  uint64_t n;
};
struct HostCopies {  // up to four copies by one k_to_host_multi launch
  HostCopy seg[4];
  uint32_t n = 0;
  void add(void *d, const void *s, uint64_t bytes) {
    if (bytes) seg[n++] = {(uint8_t *)d, (const uint8_t *)s, bytes};
  }
};
void launch_to_host_multi(const HostCopies &h, hipStream_t s);
void launch_zero(void *dst, uint64_t bytes, hipStream_t s);

}  // namespace nemo
