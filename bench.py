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
  CreateNaiveDiffProv for every failed run (per-run label sets)  nemo_diffprov
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
    ap.add_argument("--config", choices=["c3", "c4", "c5"], default="c3",
                    help="c3: 10k runs x ~5k-node graphs per GPU (the headline line, weak scaling); c4: 100k runs "
                         "in total sharded over the ranks (strong scaling); c5: deep provenance, ~1M-node graphs "
                         "at EOT 2000")
    ap.add_argument("--runs-per-gpu", type=int, default=None)
    ap.add_argument("--nodes", type=int, default=None, help="target nodes per provenance graph")
    ap.add_argument("--eot", type=int, default=None)
    ap.add_argument("--diff-mode", choices=["per_run", "reference"], default="per_run")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--kernel-timing", choices=["on", "off"], default="on",
                    help="off: the timed steps run without per-launch HIP events (two extra steps collect them)")
    ap.add_argument("--stage-blocks", type=int, default=0, help="bulk D2H staging by a k_to_host grid of this size (0: runtime copies)")
    return ap.parse_args()


CONFIGS = {"c3": {"runs": 10000, "nodes": 5000, "eot": 10, "cpu_runs": None},
           "c4": {"runs_total": 100000, "nodes": 5000, "eot": 10, "cpu_runs": 5000},
           # C5 "1M-node / 4M-edge graphs": rule bodies of 1-3 atoms plus 0..12 extra ones over a key space
           # small enough to share body goals (~0.95M nodes, ~4.0M edges per graph at EOT 2000)
           # the CPU oracle is superlinear in graph size on this shape (>15 min per 1M-node run), so its
           # bounded sample is 4 runs of the same shape at 50k-node graphs (EOT 100, same density)
           "c5": {"runs": 128, "nodes": 1_000_000, "eot": 2000, "cpu_runs": 4,
                  "gen": {"body_extra": 6, "nval": 3, "nloc": 4}, "cpu_sample": {"nodes": 50_000, "eot": 100}}}


def main():
    args = parse()
    cfg = CONFIGS[args.config]
    strong = "runs_total" in cfg
    args.nodes = args.nodes or cfg["nodes"]
    args.eot = args.eot or cfg["eot"]
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    n_gpus = world
    if strong:  # C4: a fixed corpus split over the ranks
        args.runs_per_gpu = args.runs_per_gpu or (cfg["runs_total"] + world - 1) // world
    else:
        args.runs_per_gpu = args.runs_per_gpu or cfg["runs"]
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from nemo_amd.corpus import DIFF_PER_RUN, DIFF_REFERENCE
    from nemo_amd.engine import Engine
    from tools import synth

    R = args.runs_per_gpu
    if strong:
        R = max(0, min(R, cfg["runs_total"] - rank * R))
    t0 = time.time()
    gen = cfg.get("gen", {})
    corpus, info = synth.generate(R, target_nodes=args.nodes, eot=args.eot, run_base=rank * R,
                                  prepend_run0=True, threads=min(16, os.cpu_count() or 1), **gen)
    gen_s = time.time() - t0
    owned = corpus.owned if corpus.owned is not None else np.ones(corpus.n_runs, np.uint8)
    status_ok = np.array([s == "success" for s in corpus.status])
    its = corpus.iteration
    # global GetSuccessRunsIters(): run 0 is the fault-free first run, so it leads the list
    success = [0] + [int(it) for it, ok, o in zip(its, status_ok, owned) if ok and o and it != 0]
    failed = [int(it) for it, ok, o in zip(its, status_ok, owned) if (not ok) and o]
    has_run0 = bool(owned[corpus.run_index(0)]) if 0 in set(its.tolist()) else False
    mode = DIFF_PER_RUN if args.diff_mode == "per_run" else DIFF_REFERENCE

    eng = Engine(local)
    eng.set_option("stage_blocks", args.stage_blocks)
    stream = torch.cuda.current_stream()
    eng.set_stream(stream.cuda_stream)
    eng.load(corpus)
    d_red = torch.zeros(eng.reduce_len(), dtype=torch.int32, device="cuda")
    T = corpus.n_tables
    W = (T + 31) // 32
    g0 = 2 * corpus.run_index(0) + 1
    V0 = corpus.graph_size(g0)

    fidx = np.array([corpus.run_index(f) for f in failed], np.int64)  # failed runs' rows of the table sets

    def step():
        # every device phase is enqueued first; host-side retrieval (which syncs) comes last
        eng.rebuild()
        eng.mark()
        eng.simplify()
        eng.stage_simplified()  # flags + chain pairs -> pinned host, overlapping the rest
        eng.protos_partial(success, d_red.data_ptr())
        if world > 1:
            dist.all_reduce(d_red)
        eng.diffprov(failed, mode)
        if has_run0:
            eng.triggers()
        eng.pull(1)
        eng.pull(2)
        protos = eng.protos_finalize(d_red.data_ptr())
        tabs = eng.run_tables(1)
        inter = np.asarray(protos["inter"], np.int64)
        uni = np.asarray(protos["union"], np.int64)
        if len(fidx):
            have_i = (tabs[fidx][:, inter >> 5] >> (inter & 31).astype(np.uint32)) & 1 if len(inter) else None
            have_u = (tabs[fidx][:, uni >> 5] >> (uni & 31).astype(np.uint32)) & 1 if len(uni) else None
        if has_run0:
            eng.trigger_rows()
        masks = eng.diff_masks_view() if failed else None
        miss = eng.missing()
        state, chain_off, chain_ht = eng.simplified_view()
        return state, chain_off, chain_ht, masks, miss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    eng.set_timing(args.kernel_timing == "on")
    eng.reset_timings()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    if args.kernel_timing == "off":
        eng.set_timing(True)
        for _ in range(2):
            step()
        torch.cuda.synchronize()
    tim = eng.timings()
    eng.set_timing(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    owned_runs = int(owned.sum())
    total_runs = owned_runs * world if world > 1 else owned_runs
    if world > 1:
        t = torch.tensor([owned_runs], dtype=torch.int64, device="cuda")
        dist.all_reduce(t)
        total_runs = int(t.item())
    runs_per_s = total_runs * args.steps / elapsed
    kern_ms = sum(v["ms"] for v in tim.values())
    edges = sum(v["edges"] for v in tim.values())
    if world > 1:
        t = torch.tensor([edges, kern_ms], dtype=torch.float64, device="cuda")
        dist.all_reduce(t)
        edges, kern_ms_sum = float(t[0].item()), float(t[1].item())
    # edges/s: edges examined by all traversal kernels of all ranks over the wall time
    edges_per_s = edges / elapsed
    dom = max(tim.items(), key=lambda kv: kv[1]["ms"])
    dname, d = dom
    per_launch_bytes = d["bytes"] / d["launches"]
    avg_ms = d["ms"] / d["launches"]
    achieved = per_launch_bytes / (avg_ms * 1e-3) / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", f"pmc_{dname}.json")
    if os.path.exists(pmc):
        try:
            pj = json.load(open(pmc))
            if pj.get("workload_nodes") == int(corpus.node_off[-1]):
                traffic = pj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as O
        threads = min(16, os.cpu_count() or 1)
        sample, s_succ, s_fail, s_runs = corpus, success, failed, owned_runs
        if cfg["cpu_runs"]:  # deep graphs: the oracle needs seconds per graph, time a bounded sample
            cs = cfg.get("cpu_sample", {"nodes": args.nodes, "eot": args.eot})
            sample, _ = synth.generate(cfg["cpu_runs"], target_nodes=cs["nodes"], eot=cs["eot"], threads=threads, **gen)
            s_succ, s_fail, s_runs = sample.success_iters(), sample.failed_iters(), sample.n_runs
        reps, t_cpu = 0, 0.0
        while t_cpu < args.cpu_seconds:
            tc = time.perf_counter()
            O.analyze(sample, s_succ, s_fail, diff_mode=mode, threads=threads, skip_pulls=True)
            t_cpu += time.perf_counter() - tc
            reps += 1
        cpu = {"value": round(s_runs * reps / t_cpu, 4), "unit": "runs/s", "cores": threads, "kind": "port",
               "sample": f"oracle/nemo_oracle.c (OpenMP over graphs, {threads} threads) on "
                         f"{'the same ' + str(s_runs) + '-run ' + args.config.upper() + ' corpus' if sample is corpus else str(s_runs) + ' runs of the same shape'}"
                         f"{' at ' + str(cfg['cpu_sample']['nodes']) + '-node graphs (EOT ' + str(cfg['cpu_sample']['eot']) + ')' if 'cpu_sample' in cfg else ''}"
                         f", {reps} full pass(es) in {t_cpu:.1f}s; same phases except the D2H/edge-list "
                         f"materialisation"}
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
                                      "graphs of ~nodes_per_graph nodes (SURVEY.md 8d), run 0 replicated",
                                "c4": "C4: synthetic Molly-shaped corpus of 100k runs in total, run-sharded over the "
                                      "ranks (runs_per_gpu each), ~nodes_per_graph-node graphs, run 0 replicated",
                                "c5": "C5: synthetic deep-provenance corpus, runs_per_gpu runs x (pre, post) graphs of "
                                      "~nodes_per_graph nodes / ~4 edges per node at EOT eot (SURVEY.md 8d), run 0 "
                                      "replicated"}[args.config],
                   "runs_per_gpu": R, "nodes_per_graph": args.nodes, "eot": args.eot,
                   "nodes_total_rank0": int(corpus.node_off[-1]), "edges_total_rank0": int(corpus.edge_off[-1]),
                   "failed_runs_rank0": len(failed), "diff_mode": args.diff_mode,
                   "parallelism": f"run-sharded x{n_gpus}, RCCL all-reduce of the prototype vector"},
        "edges_traversed_per_s": round(edges_per_s, 1),
        "roofline": {"bound": "hbm", "kernel": dname, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "bytes_per_launch": per_launch_bytes, "avg_launch_ms": round(avg_ms, 4)},
        "cpu_baseline": cpu,
        "kernels": {k: {"launches": v["launches"], "ms_total": round(v["ms"], 3),
                        "gbs": round(v["bytes"] / (v["ms"] * 1e-3) / 1e9, 1) if v["ms"] > 0 else None}
                    for k, v in sorted(tim.items(), key=lambda kv: -kv[1]["ms"])},
        "gen_seconds_rank0": round(gen_s, 2),
    }
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as fh:
                fh.write(line + "\n")
    eng.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
