#!/usr/bin/env python
"""bench.py — BASELINE.json's metric on its single-GPU config (C3), run-sharded over N GPUs.

Metric: fault-injection runs analyzed per second (whole job, all ranks) plus
edges traversed per second and the dominant kernel's fraction of the MI355X
HBM roofline.  Workload: a synthetic Molly-shaped corpus of
10k runs x (pre, post) provenance graphs of ~5k nodes per GPU (weak scaling:
every rank owns its own 10k runs; run 0 is replicated on every rank as the
good run of the differential provenance).

One step = the whole hot path over the rank's corpus, inputs resident in HBM:
  loadProv's device half (CSR + Kahn levels + validations)   nemo_rebuild
  markConditionHolds (all graphs)                            nemo_mark_holds
  SimplifyProv: cleanCopyProv + collapseNextChains           nemo_simplify
  CreatePrototypes: extractProtos partial -> RCCL all-reduce (N>1) -> finalize,
                    missingFrom for every failed run (table sets D2H)
  CreateNaiveDiffProv for every failed run (reference label set)  nemo_diffprov(_labels)
  GenerateCorrections/Extensions trigger patterns (rank owning run 0)
  PullPrePostProv + Q24 edge pulls (device compaction of simplified + diff graphs)
  D2H of every host-facing result: 2-bit node state (alive, holds) + chain (head,
    tail) pairs (pinned, async on a copy stream from right after SimplifyProv), D
    masks, missing events, table sets, trigger rows

Launched as `python bench.py` (N=1) or under torch.distributed.run for N>1
(RANK/LOCAL_RANK/WORLD_SIZE from the env, backend nccl = RCCL).
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, MI355X_MICROARCH.md "Chip-level parameters"
METRIC = "fault-injection runs analyzed/sec (whole node) + edges traversed/sec vs HBM roofline"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", choices=["c3", "c3_molly", "c4", "c5"], default="c3",
                    help="c3: 10k runs x ~5k-node graphs (E ~ 1.5 V) per GPU, the headline line (weak scaling); "
                         "c3_molly: the same at Molly's own 1-3-atom bodies (E ~ 1.18 V); c4: 100k runs in total, "
                         "LPT-sharded over the ranks (strong scaling); c5: deep provenance, ~1M-node graphs at EOT 2000")
    ap.add_argument("--runs-per-gpu", type=int, default=None)
    ap.add_argument("--nodes", type=int, default=None, help="target nodes per provenance graph")
    ap.add_argument("--eot", type=int, default=None)
    ap.add_argument("--diff-mode", choices=["per_run", "reference"], default="reference",
                    help="reference: differential-provenance.go:22-43's failedRuns[0] label set for every entry "
                         "(broadcast from its owner rank when N>1); per_run: each failed run's own labels")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="CPU time budget of each baseline leg")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--e2e-runs", type=int, default=2000,
                    help="end-to-end leg (rank 0, N=1): runs of the same shape written as a Molly directory, then "
                         "streaming native ingest -> H2D -> analysis -> host results, pipelined by chunk (0: off)")
    ap.add_argument("--e2e-chunk", type=int, default=500)
    ap.add_argument("--kernel-timing", choices=["dominant", "on", "off"], default="dominant",
                    help="dominant: every kernel group is timed with HIP events during the warmup steps, and the "
                         "timed steps time only the dominant group (the roofline's kernel; an event pair costs the "
                         "stream a few us per launch); on: every group in the timed steps too; off: the timed steps "
                         "run without events (two extra steps collect them)")
    ap.add_argument("--stage-blocks", type=int, default=0, help="bulk D2H staging by a k_to_host grid of this size (0: runtime copies)")
    ap.add_argument("--lanes", type=int, default=None,
                    help="N=1 only: the corpus run-sharded over this many libnemohip contexts on the one GPU, each "
                         "on its own stream, their phases issued in turn so that one lane's latency-bound level "
                         "sweeps overlap another's bandwidth-bound passes (default: the config's)")
    ap.add_argument("--set", action="append", default=[], metavar="NAME=VALUE",
                    help="a libnemohip option (nemo_set_option) before the load, e.g. chains_glob_block=512")
    ap.add_argument("--diff-at", choices=("mark", "protos"), default="mark",
                    help="where the step issues the diff: after mark (its kernels beside the simplification) or "
                         "after the protos, as main.go:146-160 orders CreatePrototypes and CreateNaiveDiffProv")
    ap.add_argument("--no-prefetch", action="store_true",
                    help="--runs-total passes: no load of the next pass's first batch beside the last analysis")
    ap.add_argument("--runs-total", type=int, default=None,
                    help="C5 at its configured size (BASELINE configs[4]: 1k runs): the runs in batches of "
                         "--batch-runs, each uploaded (H2D + CSR) on one of two contexts while the previous batch is "
                         "analysed on the other; value = runs/s of whole passes including the uploads")
    ap.add_argument("--batch-runs", type=int, default=0,
                    help="runs per batch of --runs-total (0: by the device's CUs, so that a batch's graphs, run 0's "
                         "included, are at most one per CU)")
    ap.add_argument("--diff-reps", type=int, default=5,
                    help="per_run differential-provenance leg after the timed steps (roofline_diff): this many "
                         "nemo_diffprov(failed, NEMO_DIFF_PER_RUN) calls over the resident corpus (0: off)")
    return ap.parse_args()


# workload per config (generator settings: tools/synth.py CONFIGS); cpu_runs: the bounded sample the CPU
# baseline times when a whole pass would take minutes
CONFIGS = {"c3": {"runs": 10000, "gen": "c3", "cpu_runs": None, "lanes": 1},
           "c3_molly": {"runs": 10000, "gen": "c3_molly", "cpu_runs": None, "lanes": 1},
           "c4": {"runs_total": 100000, "gen": "c3", "cpu_runs": 5000, "lanes": 1},
           # C5 (1k runs of 1M-node graphs) does not fit 288 GB at once: the bench keeps a batch of 320 runs
           # resident (~240 GB) and times passes over it.  The CPU oracle is superlinear in graph size on
           # C5's shape (~30 min per 1M-node graph), so its bounded sample is 4 runs of the same shape at
           # 50k-node graphs (EOT 100, same density)
           "c5": {"runs": 320, "gen": "c5", "cpu_runs": 4, "cpu_sample": {"target_nodes": 50_000, "eot": 100},
                  "lanes": 1}}


def cpu_info():
    """Host CPU facts for cpu_baseline: nproc, the cores this process may use, the model string."""
    model = None
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    # a cgroup CPU quota (cgroup v2 cpu.max "<quota> <period>") caps what all threads together can
    # run, whatever the affinity mask says: it, not OMP_NUM_THREADS, is the real limit when present
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    threads = usable if quota is None else max(1, min(usable, int(quota + 0.999)))
    return {"nproc": os.cpu_count(), "usable_cores": usable, "cgroup_cpu_quota": quota, "threads": threads,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"), "model": model}


def main():
    args = parse()
    cfg = CONFIGS[args.config]
    strong = "runs_total" in cfg
    import torch
    import torch.distributed as dist

    from nemo_amd.corpus import DIFF_PER_RUN, DIFF_REFERENCE
    from nemo_amd.engine import Engine
    from tools import synth

    gen = dict(synth.CONFIGS[cfg["gen"]])
    if args.nodes:
        gen["target_nodes"] = args.nodes
    if args.eot:
        gen["eot"] = args.eot
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    n_gpus = world
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    threads = cpu_info()["threads"]  # host generation / e2e ingest: every core the quota allows
    if args.runs_total:
        return runs_total_main(args, cfg, gen, threads, world, rank, local, torch, dist)
    t0 = time.time()
    if strong:  # C4: one fixed corpus, LPT-sharded by Σ(V+E) (nemo_partition_runs), run 0 replicated
        R_total = args.runs_per_gpu * world if args.runs_per_gpu else cfg["runs_total"]
        full, _ = synth.generate(R_total, threads=threads, **gen)
        if world > 1:
            from nemo_amd.shard import shard_layout
            runs, own = shard_layout(full, rank, world)
            corpus = full.subset(runs, own)
        else:
            corpus = full
        del full
    else:  # weak scaling: every rank its own block of runs (iterations rank*R ..), run 0 replicated
        R = args.runs_per_gpu or cfg["runs"]
        corpus, _ = synth.generate(R, run_base=rank * R, prepend_run0=True, threads=threads, **gen)
    gen_s = time.time() - t0
    owned = corpus.owned if corpus.owned is not None else np.ones(corpus.n_runs, np.uint8)
    status_ok = np.array([s == "success" for s in corpus.status])
    its = corpus.iteration
    # global GetSuccessRunsIters(): run 0 is the fault-free first run, so it leads the list
    success = [0] + [int(it) for it, ok, o in zip(its, status_ok, owned) if ok and o and it != 0]
    failed = [int(it) for it, ok, o in zip(its, status_ok, owned) if (not ok) and o]
    has_run0 = bool(owned[corpus.run_index(0)]) if 0 in set(its.tolist()) else False
    mode = DIFF_PER_RUN if args.diff_mode == "per_run" else DIFF_REFERENCE

    def new_engine():
        e = Engine(local)
        e.set_option("stage_blocks", args.stage_blocks)
        for kv in args.set:
            k, v = kv.split("=", 1)
            e.set_option(k, int(v))
        return e

    lanes_n = 1 if world > 1 else (args.lanes or cfg.get("lanes", 1))
    free0 = torch.cuda.mem_get_info()[0]
    if lanes_n > 1:
        lanes = make_lanes(corpus, lanes_n, new_engine, success, failed, mode)
        engines = [ln["eng"] for ln in lanes]
        eng = engines[0]
    else:
        eng = new_engine()
        eng.set_stream(torch.cuda.current_stream().cuda_stream)
        eng.load(corpus)
        engines = [eng]
    d_red = torch.zeros(eng.reduce_len(), dtype=torch.int32, device="cuda")
    V0 = corpus.graph_size(2 * corpus.run_index(0) + 1)

    # sharded reference mode: failedRuns[0] = the lowest failed iteration of the whole job; its owner
    # extracts the post-goal label set on the device and RCCL broadcasts it (differential-provenance.go:22-43)
    label_bcast = world > 1 and mode == DIFF_REFERENCE
    if label_bcast:
        t = torch.tensor([min(failed) if failed else 2 ** 62, int(np.diff(corpus.node_off.astype(np.int64)).max()) + 1],
                         dtype=torch.int64, device="cuda")
        dist.all_reduce(t[0:1], op=dist.ReduceOp.MIN)
        dist.all_reduce(t[1:2], op=dist.ReduceOp.MAX)
        f0, lab_cap = int(t[0].item()), int(t[1].item())
        o = torch.tensor([rank if f0 in set(failed) else world], dtype=torch.int64, device="cuda")
        dist.all_reduce(o, op=dist.ReduceOp.MIN)
        lab_owner = int(o.item())
        d_lab = torch.zeros(lab_cap, dtype=torch.int32, device="cuda")

    fidx = np.array([corpus.run_index(f) for f in failed], np.int64)  # failed runs' rows of the table sets

    def step():
        # every device phase is enqueued first; host-side retrieval (which syncs) comes last
        eng.rebuild()
        eng.mark()

        # CreateNaiveDiffProv reads only the raw run-0 graph and the label source
        # (differential-provenance.go:22-98): its kernels run on the library's second stream from the
        # point of the call on (beside the simplification, or beside the protos and pulls);
        # pull(2) and the mask views wait for them
        def diff():
            if label_bcast:
                if rank == lab_owner:
                    eng.goal_labels(f0, 1, d_lab.data_ptr(), lab_cap)
                dist.broadcast(d_lab, lab_owner)
                eng.diffprov_labels(failed, d_lab.data_ptr(), lab_cap)
            else:
                eng.diffprov(failed, mode)
        if args.diff_at == "mark":
            diff()
        eng.simplify()
        eng.protos_partial(success, d_red.data_ptr())
        if args.diff_at == "protos":
            diff()
        # flags + chain pairs -> pinned host on the copy stream, overlapping the pulls (queued
        # after k_proto_lds, the LDS-heaviest kernel, which a concurrent PCIe blit slows most)
        eng.stage_simplified()
        if world > 1:
            dist.all_reduce(d_red)
        eng.protos_stage(d_red.data_ptr())  # the vector's D2H queued behind the all-reduce
        if has_run0:
            eng.triggers()
        eng.pull(1)
        eng.pull(2)
        protos = eng.protos_finalize(d_red.data_ptr())
        tabs = eng.run_tables(1)
        if len(fidx):  # missingFrom (prototype.go:141-206) for every failed run: proto tables absent from its set
            tf = tabs[fidx]
            _ = table_mask(protos["inter"], tf.shape[1]) & ~tf
            _ = table_mask(protos["union"], tf.shape[1]) & ~tf
        if has_run0:
            eng.trigger_rows()
        masks = eng.diff_masks_view() if failed else None
        miss = eng.missing()
        state, chain_off, chain_ht = eng.simplified_view()
        return state, chain_off, chain_ht, masks, miss

    if lanes_n > 1:
        step = lambda: step_lanes(lanes, corpus, mode)  # noqa: E731

    def gather_timings():
        out = {}
        for e in engines:  # per-launch figures of every lane (a lane's launch overlaps the others')
            for k, v in e.timings().items():
                a = out.setdefault(k, {"launches": 0, "ms": 0.0, "bytes": 0.0, "edges": 0.0})
                for f in a:
                    a[f] += v[f]
        return out

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    hbm_used = free0 - torch.cuda.mem_get_info()[0]  # the resident corpus + every buffer a step grew
    warm = None
    if args.kernel_timing == "dominant" and args.warmup > 0:
        # one more untimed step, every group timed: picks the dominant group and gives the per-group
        # table (the first warmup step runs cold, so it is not the one measured)
        for e in engines:
            e.set_timing(True)
            e.reset_timings()
        step()
        torch.cuda.synchronize()
        warm = gather_timings()
    dom_group = max(warm.items(), key=lambda kv: kv[1]["ms"])[0] if warm else None
    for e in engines:
        e.set_timing(args.kernel_timing != "off")
        e.set_timing_groups([dom_group] if dom_group else [])
        e.reset_timings()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # the host's cyclic garbage collector runs outside the timed steps (a full collection of the
    # corpus' Python objects landed in a timed step and cost it ~15 ms)
    gc.collect()
    gc.disable()
    t_start = time.perf_counter()
    step_ends = []
    for _ in range(args.steps):
        step()
        step_ends.append(time.perf_counter())
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    gc.enable()
    step_ms = [round((b - a) * 1e3, 3) for a, b in zip([t_start] + step_ends[:-1], step_ends)]
    if args.kernel_timing == "off":
        for e in engines:
            e.set_timing(True)
        for _ in range(2):
            step()
        torch.cuda.synchronize()
    tim = gather_timings()
    for e in engines:
        e.set_timing(False)
        e.set_timing_groups([])
    # the per-group table and the traversed edges (algorithmic counts) come from the warmup steps when
    # the timed steps timed only the dominant group; the roofline from the timed steps' own events
    table, table_steps = (warm, 1) if dom_group else (tim, args.steps if args.kernel_timing != "off" else 2)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    owned_runs = int(owned.sum())
    total_runs = owned_runs
    if world > 1:
        t = torch.tensor([owned_runs], dtype=torch.int64, device="cuda")
        dist.all_reduce(t)
        total_runs = int(t.item())
    runs_per_s = total_runs * args.steps / elapsed
    edges = sum(v["edges"] for v in table.values()) * args.steps / max(table_steps, 1)
    if world > 1:
        t = torch.tensor([edges], dtype=torch.float64, device="cuda")
        dist.all_reduce(t)
        edges = float(t.item())
    # edges/s: edges examined by all traversal kernels of all ranks over the wall time
    edges_per_s = edges / elapsed
    dname = dom_group or max(tim.items(), key=lambda kv: kv[1]["ms"])[0]
    d = tim[dname]
    per_launch_bytes = d["bytes"] / d["launches"]
    avg_ms = d["ms"] / d["launches"]
    achieved = per_launch_bytes / (avg_ms * 1e-3) / 1e9
    traffic = pmc_traffic(dname, corpus)
    rdiff = None
    if args.diff_reps > 0 and lanes_n == 1:
        rdiff = diff_leg(args, eng, corpus, failed, world, torch, dist)
    e2e = None
    if rank == 0 and world == 1 and args.e2e_runs > 0 and not strong and args.config != "c5":
        for e in engines:
            e.close()
        eng = Engine(local)
        engines = [eng]
        e2e = e2e_leg(args, gen, eng, threads, mode)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, cfg, gen, corpus, success, failed, owned_runs, mode)
    E = int(corpus.edge_off[-1])
    Vn = int(corpus.node_off[-1])
    out = {
        "metric": METRIC,
        "value": round(runs_per_s, 2),
        "unit": "runs/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic",
        "config": {"workload": {"c3": "C3: synthetic Molly-shaped corpus, runs_per_gpu runs x (pre, post) provenance "
                                      "graphs of ~nodes_per_graph nodes, E ~ 1.5 V (SURVEY.md 8d), run 0 replicated",
                                "c3_molly": "C3 at Molly's own rule-body sizes (1-3 atoms, E ~ 1.18 V)",
                                "c4": "C4: synthetic Molly-shaped corpus of 100k runs in total, LPT-sharded over the "
                                      "ranks by nodes+edges, ~nodes_per_graph-node graphs, run 0 replicated",
                                "c5": "C5: synthetic deep-provenance corpus, runs_per_gpu runs x (pre, post) graphs of "
                                      "~nodes_per_graph nodes / ~4 edges per node at EOT eot (SURVEY.md 8d), run 0 "
                                      "replicated"}[args.config],
                   "runs_per_gpu": int(corpus.n_runs), "nodes_per_graph": gen["target_nodes"], "eot": gen["eot"],
                   "nodes_total_rank0": Vn, "edges_total_rank0": E, "edges_per_node": round(E / max(Vn, 1), 3),
                   "failed_runs_rank0": len(failed), "diff_mode": args.diff_mode,
                   "parallelism": f"run-sharded x{n_gpus}, RCCL all-reduce of the prototype vector"
                                  + (" + broadcast of failedRuns[0]'s label set" if label_bcast else "")
                                  + (f"; on the GPU, {lanes_n} lanes: the rank's runs LPT-sharded over {lanes_n} "
                                     "contexts, one stream each, phases issued in turn, vectors summed on the "
                                     "host" if lanes_n > 1 else ""),
                   "lib_options": args.set},
        "edges_traversed_per_s": round(edges_per_s, 1),
        "roofline": {"bound": "hbm", "kernel": dname, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "bytes_per_launch": per_launch_bytes, "avg_launch_ms": round(avg_ms, 4),
                     "bytes_formula": "DESIGN.md section 3 (HBM lower bound per launch)"},
        "cpu_baseline": cpu,
        "kernels": {k: {"launches": v["launches"], "ms_total": round(v["ms"], 3),
                        "gbs": round(v["bytes"] / (v["ms"] * 1e-3) / 1e9, 1) if v["ms"] > 0 else None}
                    for k, v in sorted(table.items(), key=lambda kv: -kv[1]["ms"])},
        "kernel_timing": {"mode": args.kernel_timing, "timed_steps_groups": [dom_group] if dom_group else "all",
                          "kernels_table_from": "one untimed step after the warmup" if dom_group else "the timed steps"},
        "step_host_ms_rank0": step_ms,
        "gen_seconds_rank0": round(gen_s, 2),
        "hbm_used_gb_rank0": round(hbm_used / 1e9, 2),
        "diff_dedupe": "entries sharing a label source share one computation (reference mode: failedRuns[0] "
                       "for every entry, differential-provenance.go:22-43)",
    }
    if e2e is not None:
        out["e2e_runs_per_s"] = e2e["runs_per_s"]
        out["e2e"] = e2e
    if "k_diff" in table:  # all entries of a diffprov call run concurrently: the launch time is each entry's latency
        out["k_diff_entry_latency_ms"] = round(table["k_diff"]["ms"] / table["k_diff"]["launches"], 4)
    if rdiff is not None:
        out["roofline_diff"] = rdiff
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as fh:
                fh.write(line + "\n")
    for e in engines:
        e.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def table_mask(tables, words):
    """u32 bitset of a table-id list (missingFrom's proto side, prototype.go:191-198)."""
    m = np.zeros(words, np.uint32)
    for t in tables:
        m[t >> 5] |= np.uint32(1 << (t & 31))
    return m


def runs_total_main(args, cfg, gen, threads, world, rank, local, torch, dist):
    """C5 at its configured size (BASELINE.json configs[4]: 1k runs of 1M-node graphs), which does not fit
    one MI355X's 288 GB at once.  The rank's runs are generated up front (host memory) in batches of
    --batch-runs, each a corpus of its own with run 0 replicated, not owned, after the first.  A pass is
    nemo_amd/batched.py's BatchedPasses.run_pass (tests/test_gpu_batched.py checks the same code against the
    oracle): batch i+1 loaded (H2D + CSR + Kahn levels) on one of two contexts from a second host thread while
    batch i is analysed on the other, the batches' proto vectors summed on the host (prototype.go:79-130).
    The last batch's analysis overlaps the load of the next pass's first batch (BatchedPasses prefetch;
    --no-prefetch: each pass starts with its own first load): every timed pass does one load and one analysis
    per batch, and the clock stops only after the load the last pass started is done.
    value = runs of a pass / its wall time, uploads included; generation and the one-time page-locking of the
    batches are not timed (they stand in for reading Molly output; the pin time is reported)."""
    from nemo_amd.batched import BatchedPasses, split_even
    from nemo_amd.corpus import DIFF_PER_RUN, DIFF_REFERENCE
    from tools import synth
    mode = DIFF_PER_RUN if args.diff_mode == "per_run" else DIFF_REFERENCE
    R = args.runs_total // world
    base = rank * R
    # the deep graphs' per-graph kernels (k_topo_deep, k_glob_prep / k_chains_glob) run one workgroup per
    # graph and are latency-bound: a batch of at most one graph per CU gives each its own CU (1000 runs:
    # eight batches of 125 + run 0 = 252 graphs on 256 CUs, 447.5 runs/s, against seven of 143 + run 0 =
    # 288 graphs, 408.7, on one box, gpurun_out r06ab)
    batch = args.batch_runs
    if batch <= 0:
        n_cu = torch.cuda.get_device_properties(local).multi_processor_count
        batch = max(1, n_cu // 2 - 1)
    sizes = split_even(R, batch)
    t0 = time.time()
    batches, a = [], 0
    for n in sizes:
        c, _ = synth.generate(n, run_base=base + a, prepend_run0=True, threads=threads, **gen)
        batches.append(c)
        a += n
    gen_s = time.time() - t0
    opts = [tuple(kv.split("=", 1)) for kv in args.set]
    bp = BatchedPasses(batches, mode=mode, device=local, options=[(k, int(v)) for k, v in opts],
                       prefetch=not args.no_prefetch)
    phase = {}
    try:
        for _ in range(args.warmup):
            bp.run_pass()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t_start = time.perf_counter()
        for _ in range(args.steps):
            phase = bp.run_pass().phases
        bp.drain()  # the next pass's first load, started inside the timed passes, is timed too
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t_start
    finally:
        bp.close()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    runs = sum(int((c.owned if c.owned is not None else np.ones(c.n_runs, np.uint8)).sum()) for c in batches)
    total = runs * world
    Vn = sum(int(c.node_off[-1]) for c in batches)
    E_ = sum(int(c.edge_off[-1]) for c in batches)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and cfg.get("cpu_runs"):
        cpu = cpu_baseline(args, cfg, gen, None, None, None, None, mode)  # its bounded sample of the same shape
        # the sample's graphs are ~20x smaller than this line's: state the baseline per node too, and scaled
        # to this line's nodes per run (linear scaling: the oracle is superlinear in graph size, so the
        # scaled figure overstates the CPU)
        nodes_per_run = Vn / max(sum(c.n_runs for c in batches), 1)
        cpu["value_nodes_per_s"] = round(cpu["value"] * cpu["sample_nodes_per_run"], 1)
        cpu["value_scaled_to_line"] = round(cpu["value_nodes_per_s"] / nodes_per_run, 4)
        cpu["scaling_note"] = (f"value is runs/s of the sample's {cpu['sample_nodes_per_run']:.0f}-node runs; "
                               f"value_scaled_to_line = nodes/s / this line's {nodes_per_run:.0f} nodes per run "
                               "(linear in nodes: an upper bound for the CPU)")
    out = {"metric": METRIC, "value": round(total * args.steps / elapsed, 2), "unit": "runs/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
           "config": {"workload": "C5 at its configured size: runs_total runs x (pre, post) graphs of ~nodes_per_graph "
                                  "nodes / ~4 edges per node at EOT eot (BASELINE configs[4]); a step is one pass "
                                  "over every run, batches of batch_runs uploaded on one context while the previous "
                                  "batch is analysed on another, uploads included",
                      "runs_total": total, "runs_per_gpu": runs, "batch_runs": max(sizes), "batch_sizes": sizes,
                      "batches_per_gpu": len(batches),
                      "nodes_per_graph": gen["target_nodes"], "eot": gen["eot"], "nodes_total_rank0": Vn,
                      "edges_total_rank0": E_, "edges_per_node": round(E_ / max(Vn, 1), 3),
                      "failed_runs_rank0": len(bp.failed), "diff_mode": args.diff_mode,
                      "parallelism": f"run-sharded x{world}; two contexts per GPU (upload / analysis overlapped"
                                     f"{'' if args.no_prefetch else ', the next pass first batch loaded beside the last analysis'}"
                                     f"); batches page-locked once (nemo_host_register)",
                      "lib_options": args.set},
           "roofline": None, "cpu_baseline": cpu, "gen_seconds_rank0": round(gen_s, 2),
           "pass_phases_rank0": dict(phase), "pin_s_rank0": round(bp.pin_s, 3), "pin_failed_arrays": bp.pin_failed,
           "note": "no per-kernel roofline on this line: the resident-batch line (--config c5) carries it; the "
                   "one-time page-locking (pin_s_rank0) is outside the timed passes"}
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as fh:
                fh.write(line + "\n")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def pmc_traffic(group, corpus):
    """HBM bytes per launch of a timed group from profiles/pmc_summary.json (tools/pmc_summary.py: 2 x
    FETCH_SIZE + WRITE_SIZE of the group's kernels), keyed by the workload's node count; None if absent."""
    pmc = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(pmc):
        return None
    try:
        return json.load(open(pmc)).get(group, {}).get(str(int(corpus.node_off[-1])), {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def diff_leg(args, eng, corpus, failed, world, torch, dist):
    """roofline_diff: CreateNaiveDiffProv (differential-provenance.go:22-146) in the per-run label mode, every
    distinct failed run computed, over the corpus already resident in HBM.  Each rep is one
    nemo_diffprov(failed, NEMO_DIFF_PER_RUN) call plus its host hand-over (D masks, missing events).  The
    library's k_diff group is timed with HIP events on the stream its kernels run on; its bytes are the HBM
    lower bound DESIGN.md section 3 gives (run 0's post graph once, every label source, every D mask)."""
    from nemo_amd.corpus import DIFF_PER_RUN
    t_all = torch.tensor([0.0, 0.0, 0.0, float(len(failed))], dtype=torch.float64, device="cuda")
    if failed:
        eng.set_timing(True)
        eng.reset_timings()
        walls = []
        for _ in range(args.diff_reps):
            torch.cuda.synchronize()
            t = time.perf_counter()
            eng.diffprov(failed, DIFF_PER_RUN)
            eng.diff_masks_view()
            eng.missing()
            walls.append(time.perf_counter() - t)
        k = eng.timings().get("k_diff")
        eng.set_timing(False)
        t_all[0] = k["ms"] / k["launches"]
        t_all[1] = k["bytes"] / k["launches"]
        t_all[2] = k["edges"] / k["launches"]
        wall_ms = float(np.median(walls)) * 1e3
    else:
        wall_ms = 0.0
    if world > 1:  # every rank's leg runs at once: the slowest rank's launch, the ranks' bytes and entries summed
        mx = t_all[0:1].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(t_all)
        t_all[0] = mx[0]
    ms, nbytes, edges, entries = (float(x) for x in t_all.tolist())
    if ms <= 0:
        return None
    gbs = nbytes / (ms * 1e-3) / 1e9
    r0 = corpus.run_index(0)
    g0 = 2 * r0 + 1
    return {"bound": "hbm", "kernel": "k_diff", "mode": "per_run", "entries": int(entries),
            "distinct_label_sources": int(entries), "v0": int(corpus.graph_size(g0)),
            "e0": int(corpus.edge_off[g0 + 1] - corpus.edge_off[g0]),
            "bytes_per_launch": nbytes, "avg_launch_ms": round(ms, 4), "achieved": round(gbs, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
            "traffic": pmc_traffic("k_diff_per_run", corpus),
            "edges_traversed_per_s": round(edges / (ms * 1e-3), 1),
            "wall_ms_per_call": round(wall_ms, 3), "reps": args.diff_reps,
            "bytes_formula": "8 E0 + 16 V0 (run 0's post graph) + 8 V per label source + V0 per D mask "
                             "(DESIGN.md section 3, k_diff row)",
            "edges_formula": "3 E0 per distinct label source (Fwd*, Bwd*, longest path)"}


def make_lanes(corpus, n, new_engine, success, failed, mode):
    """The N=1 corpus run-sharded over n contexts on the one GPU (nemo_partition_runs' LPT shards, run 0
    replicated, not owned, in every lane).  Each lane loads its runs; the reference diff mode's label
    source (failedRuns[0]'s post-goal labels, differential-provenance.go:22-43) is handed to every lane
    as a host label set (nemo_diffprov_host_labels)."""
    from nemo_amd.corpus import DIFF_REFERENCE, NODE_RULE
    from nemo_amd.shard import partition_runs, shard_layout
    parts = partition_runs(corpus, n)
    f0_labels = None
    if failed and mode == DIFF_REFERENCE:
        g = 2 * corpus.run_index(failed[0]) + 1
        a, b = int(corpus.node_off[g]), int(corpus.node_off[g + 1])
        f0_labels = corpus.label[a:b][(corpus.node_word[a:b] & NODE_RULE) == 0].copy()
    fset = set(failed)
    lanes = []
    for k in range(n):
        runs, own = shard_layout(corpus, k, n, parts)
        sub = corpus.subset(runs, own)
        o = sub.owned if sub.owned is not None else np.ones(sub.n_runs, np.uint8)
        its = [int(x) for x in sub.iteration]
        e = new_engine()
        e.load(sub)
        lf = [it for it, ok in zip(its, o) if ok and it in fset]
        has0 = 0 in its and bool(o[its.index(0)])
        lanes.append({"eng": e, "corpus": sub, "failed": lf, "has0": has0, "success": success,
                      "fidx": np.array([sub.run_index(f) for f in lf], np.int64), "labels": f0_labels})
    return lanes


def step_lanes(lanes, corpus, mode):
    """One step over every lane: each phase is issued on every lane's stream before the next phase, so
    the lanes' kernels run side by side; then the host-side retrieval, as the single-context step."""
    from nemo_amd import engine as E
    from nemo_amd.corpus import DIFF_PER_RUN
    for ln in lanes:
        ln["eng"].rebuild()
    for ln in lanes:
        ln["eng"].mark()
    for ln in lanes:
        if ln["labels"] is not None:
            ln["eng"].diffprov_host_labels(ln["failed"], ln["labels"])
        else:
            ln["eng"].diffprov(ln["failed"], DIFF_PER_RUN)
    for ln in lanes:
        ln["eng"].simplify()
    for ln in lanes:
        ln["eng"].protos_partial(ln["success"], 0)
    for ln in lanes:
        ln["eng"].stage_simplified()
    for ln in lanes:
        if ln["has0"]:
            ln["eng"].triggers()
    for ln in lanes:
        ln["eng"].pull(1)
    for ln in lanes:
        ln["eng"].pull(2)
    vec = sum(ln["eng"].reduce_vector().astype(np.int64) for ln in lanes)  # the vectors summed (prototype.go:79-130)
    T = corpus.n_tables
    _, inter, uni = E.reduce_interpret(vec.astype(np.uint32), T, corpus.table_post)
    inter, uni = np.asarray(inter, np.int64), np.asarray(uni, np.int64)
    out = []
    for ln in lanes:
        e = ln["eng"]
        tabs = e.run_tables(1)
        if len(ln["fidx"]):  # missingFrom (prototype.go:141-206) for every failed run
            _ = (tabs[ln["fidx"]][:, inter >> 5] >> (inter & 31).astype(np.uint32)) & 1 if len(inter) else None
            _ = (tabs[ln["fidx"]][:, uni >> 5] >> (uni & 31).astype(np.uint32)) & 1 if len(uni) else None
        if ln["has0"]:
            e.trigger_rows()
        masks = e.diff_masks_view() if ln["failed"] else None
        out.append((e.simplified_view(), masks, e.missing()))
    return out


def e2e_leg(args, gen, eng, threads, mode):
    """SURVEY.md 8d metric 1, second half: runs/s from a Molly-format directory on disk to host results.
    nemo_amd/pipeline.py streams the directory through nemo_ingest_next (native JSON decode + interning,
    `threads` threads) in chunks; chunk i is uploaded (nemo_load_corpus: H2D + CSR) and analysed while
    chunk i+1 is decoded.  Best of 2 passes (the first also warms the page cache, as a re-analysis would)."""
    import shutil
    import tempfile

    from nemo_amd import pipeline
    from nemo_amd.ingest import load_molly_native
    from tools import synth
    corpus, info = synth.generate(args.e2e_runs, threads=threads, **gen)
    d = tempfile.mkdtemp(prefix="nemo_e2e_")
    try:
        synth.write_molly(corpus, info, d, threads=threads)
        del corpus
        size = sum(os.path.getsize(os.path.join(d, x)) for x in os.listdir(d))
        best = None
        for _ in range(2):
            r = pipeline.run(d, eng, chunk=args.e2e_chunk, threads=threads, diff_mode=mode, keep=False)
            if best is None or r.timings["total_s"] < best.timings["total_s"]:
                best = r
        t = time.perf_counter()  # the decode alone, one shot (its rate bounds the pipeline)
        c = load_molly_native(d, threads=threads)
        t_ingest = time.perf_counter() - t
        del c
    finally:
        shutil.rmtree(d, ignore_errors=True)
    tot = best.timings["total_s"]
    return {"runs_per_s": round(args.e2e_runs / tot, 1), "runs": args.e2e_runs, "json_gb": round(size / 1e9, 3),
            "chunk": args.e2e_chunk, "ingest_threads": threads, "total_s": round(tot, 3),
            "device_and_handover_s": round(best.timings["device_s"], 3),
            "ingest_only_s": round(t_ingest, 3), "ingest_gb_per_s": round(size / t_ingest / 1e9, 3),
            "note": "JSON decode bound: the pipeline overlaps device work with the next chunk's decode"}


def cpu_baseline(args, cfg, gen, corpus, success, failed, owned_runs, mode):
    """oracle/nemo_oracle.c timed on the host (rank 0, N=1): OpenMP over graphs on every usable core
    (or the cgroup quota's worth when one is set) and on one core, each leg for about --cpu-seconds of a
    bounded sample."""
    from oracle import oracle as O
    from tools import synth
    info = cpu_info()
    threads = info["threads"]
    sample, s_succ, s_fail, s_runs = corpus, success, failed, owned_runs
    desc = f"the same {s_runs}-run {args.config.upper()} corpus"
    if cfg["cpu_runs"]:  # deep graphs / huge corpora: a bounded sample of the same shape
        g = dict(gen)
        g.update(cfg.get("cpu_sample", {}))
        sample, _ = synth.generate(cfg["cpu_runs"], threads=threads, **g)
        s_succ, s_fail, s_runs = sample.success_iters(), sample.failed_iters(), sample.n_runs
        desc = f"{s_runs} runs of the same shape" + (f" at {g['target_nodes']}-node graphs (EOT {g['eot']})"
                                                    if "cpu_sample" in cfg else "")

    def leg(n_threads, smp, su, fa, runs):
        reps, t = 0, 0.0
        while t < args.cpu_seconds or reps == 0:
            tc = time.perf_counter()
            O.analyze(smp, su, fa, diff_mode=mode, threads=n_threads, skip_pulls=False)
            t += time.perf_counter() - tc
            reps += 1
        return runs * reps / t, reps, t

    v_all, reps, t_all = leg(threads, sample, s_succ, s_fail, s_runs)
    # one core: the first 500 runs (run 0 included) of the sample
    n1 = min(sample.n_runs, 500)
    one = sample.subset(np.arange(n1)) if n1 < sample.n_runs else sample
    own1 = one.owned if one.owned is not None else np.ones(one.n_runs, np.uint8)
    su1 = [x for x in s_succ if x in set(one.iteration.tolist())]
    fa1 = [x for x in s_fail if x in set(one.iteration.tolist())]
    v_one, reps1, t_one = leg(1, one, su1, fa1, int(own1.sum()))
    return {"value": round(v_all, 4), "unit": "runs/s", "cores": threads, "kind": "port",
            "sample_nodes_per_run": round(int(sample.node_off[-1]) / max(sample.n_runs, 1), 1),
            "value_1core": round(v_one, 4), "nproc": info["nproc"], "usable_cores": info["usable_cores"],
            "cgroup_cpu_quota": info["cgroup_cpu_quota"], "omp_num_threads_env": info["omp_num_threads_env"],
            "cores_rule": "every usable core, or the cgroup cpu.max quota when one is set (OMP_NUM_THREADS "
                          "is not a cap)",
            "cpu_model": info["model"],
            "sample": f"oracle/nemo_oracle.c (OpenMP over graphs, {threads} threads) on {desc}, {reps} full pass(es) "
                      f"in {t_all:.1f}s, the same phases incl. the edge-list materialisation; 1-core leg: the "
                      f"first {n1} runs of it, {reps1} pass(es) in {t_one:.1f}s"}


if __name__ == "__main__":
    main()
