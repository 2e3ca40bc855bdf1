"""End-to-end throughput (SURVEY.md §8d metric 1, "end-to-end incl. host
interning, H2D"): a synthetic Molly-format directory on disk -> native ingest
(nemo_ingest_molly) -> nemo_load_corpus (H2D + CSR) -> the analysis pass of
bench.py -> results on the host.  The device-resident number is bench.py's
`value`; this is the number beside it.

usage: python tools/e2e_bench.py [--runs N] [--nodes V] [--threads T] [--dir D] [--py-sample K] [--no-gpu]
Writes the corpus once (not timed), then times REPS end-to-end passes.
"""
import argparse
import json
import os
import shutil
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from nemo_amd.corpus import DIFF_PER_RUN, load_molly  # noqa: E402
from nemo_amd.ingest import load_molly_native  # noqa: E402
from tools import synth  # noqa: E402


def analysis(eng, corpus):
    s, f = corpus.success_iters(), corpus.failed_iters()
    eng.load(corpus)
    eng.mark()
    eng.simplify()
    eng.stage_simplified()
    eng.protos_partial(s, 0)
    red = eng.protos_finalize(0)
    eng.diffprov(f, DIFF_PER_RUN)
    eng.triggers()
    eng.pull(1)
    state, off, ht = eng.simplified_view()
    masks = eng.diff_masks_view()
    return red, len(ht), masks.shape


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=1000)
    ap.add_argument("--nodes", type=int, default=5000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dir", default="/tmp/nemo_e2e")
    ap.add_argument("--py-sample", type=int, default=20, help="runs timed through the Python loader")
    ap.add_argument("--no-gpu", action="store_true")
    a = ap.parse_args()
    t = time.time()
    corpus, info = synth.generate(a.runs, target_nodes=a.nodes, eot=10)
    shutil.rmtree(a.dir, ignore_errors=True)
    synth.to_molly(corpus, info, a.dir)
    size = sum(os.path.getsize(os.path.join(a.dir, x)) for x in os.listdir(a.dir))
    print(f"wrote {a.runs} runs ({int(corpus.node_off[-1])} nodes, {size / 1e9:.2f} GB JSON) in "
          f"{time.time() - t:.1f}s", flush=True)
    out = {"runs": a.runs, "nodes": int(corpus.node_off[-1]), "json_bytes": size, "threads": a.threads}
    del corpus
    best = None
    eng = None
    if not a.no_gpu:
        from nemo_amd import engine as E
        eng = E.Engine(0)
    for rep in range(a.reps):
        t0 = time.time()
        c = load_molly_native(a.dir, threads=a.threads)
        t1 = time.time()
        if eng is not None:
            analysis(eng, c)
            eng.synchronize()
        t2 = time.time()
        print(f"rep {rep}: ingest {t1 - t0:.2f}s, load+analysis {t2 - t1:.2f}s", flush=True)
        if best is None or t2 - t0 < best[0]:
            best = (t2 - t0, t1 - t0, t2 - t1)
        del c
    out.update({"ingest_s": round(best[1], 3), "device_s": round(best[2], 3), "total_s": round(best[0], 3),
                "ingest_gb_per_s": round(size / best[1] / 1e9, 3),
                "e2e_runs_per_s": round(a.runs / best[0], 1) if eng is not None else None,
                "ingest_runs_per_s": round(a.runs / best[1], 1)})
    if a.py_sample:
        # the sequential decoder (what Go's encoding/json + per-element interning does), on a sample
        sample = a.dir + "_sample"
        shutil.rmtree(sample, ignore_errors=True)
        os.makedirs(sample)
        runs = json.load(open(os.path.join(a.dir, "runs.json")))[:a.py_sample]
        for i in range(len(runs)):
            for cond in ("pre", "post"):
                shutil.copy(os.path.join(a.dir, f"run_{i}_{cond}_provenance.json"), sample)
        json.dump(runs, open(os.path.join(sample, "runs.json"), "w"))
        t = time.time()
        load_molly(sample)
        tp = time.time() - t
        t = time.time()
        load_molly_native(sample, threads=1)
        tn1 = time.time() - t
        out.update({"py_loader_runs_per_s": round(len(runs) / tp, 1),
                    "native_1thread_runs_per_s": round(len(runs) / tn1, 1), "py_sample_runs": len(runs)})
        shutil.rmtree(sample, ignore_errors=True)
    if eng is not None:
        eng.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
