"""Diagnostic: CreateNaiveDiffProv alone (nemo_diffprov) on a corpus of the C3 or C5 shape, for rocprofv3
kernel traces of the diff kernels without the rest of the step.

usage: python tools/diff_probe.py [--config c3|c5] [--runs N] [--p-fault P] [--reps K] [--mode per_run|reference]
                                  [--set name=value ...]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--runs", type=int, default=None)
    ap.add_argument("--p-fault", type=float, default=None)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--mode", default="per_run")
    ap.add_argument("--set", action="append", default=[])
    args = ap.parse_args()
    import torch  # noqa: F401  (the engine binds torch's HIP runtime first)
    from nemo_amd.corpus import DIFF_PER_RUN, DIFF_REFERENCE
    from nemo_amd.engine import Engine
    from tools import synth
    gen = dict(synth.CONFIGS[args.config])
    runs = args.runs or (10000 if args.config == "c3" else 64)
    pf = args.p_fault if args.p_fault is not None else (0.15 if args.config == "c3" else 0.6)
    corpus, _ = synth.generate(runs, p_fault=pf, prepend_run0=True, **gen)
    f = corpus.failed_iters()
    eng = Engine(0)
    for kv in args.set:
        k, v = kv.split("=", 1)
        eng.set_option(k, int(v))
    eng.load(corpus)
    eng.mark()
    mode = DIFF_PER_RUN if args.mode == "per_run" else DIFF_REFERENCE
    eng.diffprov(f, mode)
    eng.diff_masks_view()
    eng.set_timing(True)
    eng.reset_timings()
    walls = []
    for _ in range(args.reps):
        t = time.perf_counter()
        eng.diffprov(f, mode)
        eng.diff_masks_view()
        walls.append(time.perf_counter() - t)
    tim = eng.timings()
    k = tim.get("k_diff", {})
    print(json.dumps({"config": args.config, "runs": runs, "failed": len(f), "mode": args.mode, "set": args.set,
                      "k_diff_ms": k.get("ms", 0) / max(1, k.get("launches", 1)),
                      "wall_ms": float(np.median(walls)) * 1e3, "v0": corpus.graph_size(2 * corpus.run_index(0) + 1)}),
          flush=True)
    eng.close()


if __name__ == "__main__":
    main()
