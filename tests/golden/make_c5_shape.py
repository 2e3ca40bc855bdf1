"""Generate tests/golden/c5_shape/digest.json: the CPU oracle (oracle/nemo_oracle.c) on four runs of the
bench's own C5 corpus, reduced to a digest the GPU test compares against.

The bench's C5 corpus (bench.py --config c5) is synth.generate(128, prepend_run0=True,
**synth.CONFIGS["c5"]): ~1M-node / ~4.2M-edge graphs at EOT 2000.  Its 1M-node graphs take the oracle's
greedy @next-chain cover (preprocessing.go:108-138) ~15 min each, so the oracle runs once, here, in the
build container, and tests/test_gpu_c5_shape.py (-m gpu) re-generates the same corpus on the GPU box,
runs it through libnemohip and compares with this digest.

Runs in the digest: run 0 (the good run of every diff, differential-provenance.go:26), the next success
run, and the corpus' first two failed runs (failedRuns[0] is the reference diff mode's label source,
differential-provenance.go:22-43).  Per graph: sha256 of the node flags, the accepted chains (count +
sha256 of (k, head, tail, len)), the simplified graph's edges (count + sha256 of the sorted
src<<32|dst keys); per run: the proto table bits (success runs) and the simplified-graph table set;
per failed run in the per-run diff mode: sha256 + popcount of the D mask over run 0's post graph and
the missing rules.  The reference mode's entries all equal failedRuns[0]'s per-run entry.

Two additions pin the digest further (round 4):
  --diff-all   the per-run diff of EVERY failed run of the 128-run corpus (the oracle's diff-only mode:
               run 0's post graph and each failed run's post-goal labels), under "diff_per_run_all";
  --rescan     the oracle's literal greedy rescan (NEMO_ORACLE_RESCAN=1, preprocessing.go:108-138 as the
               queries read) on the digest's four runs, its flags and chains compared with the digest's
               (which come from greedy_incremental), recorded as "rescan_equal".

Usage: python tests/golden/make_c5_shape.py [--diff-all | --rescan]  (writes tests/golden/c5_shape/digest.json)
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

BENCH_RUNS = 128  # the first 128 runs of bench.py --config c5 (each run's graphs depend only on its own seed)
OUT = os.path.join(ROOT, "tests", "golden", "c5_shape", "digest.json")


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def edge_digest(src, dst):
    k = (np.asarray(src, np.uint64) << np.uint64(32)) | np.asarray(dst, np.uint64)
    k.sort()
    return {"n": int(len(k)), "sha256": sha(k)}


def chain_digest(rows):
    """rows: (k, head, tail, len) in k order."""
    return {"n": int(len(rows)), "sha256": sha(np.asarray(rows, np.uint32).reshape(-1, 4))}


def bench_corpus(threads=None):
    from tools import synth
    corpus, _ = synth.generate(BENCH_RUNS, prepend_run0=True, threads=threads, **synth.CONFIGS["c5"])
    return corpus


def pick_runs(corpus):
    """Run indices of the digest: run 0, the next success run, the first two failed runs."""
    ok = [s == "success" for s in corpus.status]
    its = [int(x) for x in corpus.iteration]
    r0 = its.index(0)
    succ = next(r for r in range(corpus.n_runs) if ok[r] and r != r0)
    failed = [r for r in range(corpus.n_runs) if not ok[r]][:2]
    assert len(failed) == 2, "the C5 bench corpus has fewer than two failed runs"
    return sorted({r0, succ, *failed}), [its[r] for r in failed]


def main():
    from oracle import oracle as O
    t0 = time.time()
    full = bench_corpus(threads=min(16, os.cpu_count() or 1))
    runs, f_its = pick_runs(full)
    sub = full.subset(runs)
    del full
    print(f"runs {runs} (failed iterations {f_its}), {int(sub.node_off[-1])} nodes, "
          f"{int(sub.edge_off[-1])} edges; generated in {time.time() - t0:.0f}s", flush=True)
    s = [0] + [x for x in sub.success_iters() if x != 0]
    t = time.time()
    orc = O.analyze(sub, s, f_its, diff_mode=1, threads=min(8, os.cpu_count() or 1), skip_pulls=False)
    print(f"oracle {time.time() - t:.0f}s, {len(orc.chains)} chains", flush=True)
    W = (sub.n_tables + 31) // 32
    dig = {"bench_runs": BENCH_RUNS, "config": "c5", "runs": [], "failed_iters": f_its,
           "n_tables": int(sub.n_tables), "words": W,
           "generator": "tools/synth.py CONFIGS['c5'], synth.generate(128, prepend_run0=True)",
           "oracle_seconds": round(time.time() - t, 1)}
    po = orc.pulled_off.astype(np.int64)
    for i, r in enumerate(runs):
        it = int(sub.iteration[i])
        ent = {"run": int(r), "iteration": it, "status": sub.status[i], "graphs": []}
        for k in (0, 1):
            g = 2 * i + k
            a, b = int(sub.node_off[g]), int(sub.node_off[g + 1])
            ch = orc.chains[orc.chains[:, 0] == g][:, 1:5]
            ent["graphs"].append({"nodes": b - a, "edges": int(sub.edge_off[g + 1] - sub.edge_off[g]),
                                  "flags_sha256": sha(orc.flags[a:b]), "chains": chain_digest(ch),
                                  "pulled": edge_digest(orc.pulled_src[po[g]:po[g + 1]],
                                                        orc.pulled_dst[po[g]:po[g + 1]])})
        ent["graph_tables"] = [int(x) for x in orc.graph_tables[i]]
        if sub.status[i] == "success":
            ent["proto_bits"] = [int(x) for x in orc.proto_bits[i]]
        if it in f_its:
            e = f_its.index(it)
            m = orc.diff_mask[e]
            ent["diff_per_run"] = {"mask_sha256": sha(m), "mask_popcount": int(np.count_nonzero(m)),
                                   "missing": sorted(int(x) for x in orc.missing[orc.missing[:, 0] == e][:, 1])}
        dig["runs"].append(ent)
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "w") as fh:
        json.dump(dig, fh, indent=1)
    print("wrote", OUT, f"total {time.time() - t0:.0f}s")


def diff_all():
    """Per-run D masks and missing rules of every failed run of the corpus (oracle diff-only mode)."""
    from oracle import oracle as O
    t0 = time.time()
    full = bench_corpus(threads=min(16, os.cpu_count() or 1))
    ok = [st == "success" for st in full.status]
    its = [int(x) for x in full.iteration]
    r0 = its.index(0)
    frs = [r for r in range(full.n_runs) if not ok[r]]
    sub = full.subset([r0] + frs)
    del full
    f_its = [its[r] for r in frs]
    t = time.time()
    orc = O.analyze(sub, [0], f_its, diff_mode=1, threads=min(8, os.cpu_count() or 1), diff_only=True)
    dig = json.load(open(OUT))
    ent = {}
    for e, it in enumerate(f_its):
        m = orc.diff_mask[e]
        ent[str(it)] = {"mask_sha256": sha(m), "mask_popcount": int(np.count_nonzero(m)),
                        "missing": sorted(int(x) for x in orc.missing[orc.missing[:, 0] == e][:, 1])}
    dig["diff_per_run_all"] = {"failed_iters": f_its, "entries": ent, "oracle_seconds": round(time.time() - t, 1),
                               "how": "oracle diff-only mode (run 0's post graph + each failed run's post-goal "
                                      "labels), per-run label mode"}
    for r in dig["runs"]:  # the four-run digest's own entries must agree
        if "diff_per_run" in r:
            assert r["diff_per_run"] == ent[str(r["iteration"])], r["iteration"]
    with open(OUT, "w") as fh:
        json.dump(dig, fh, indent=1)
    print(f"{len(f_its)} failed runs, wrote {OUT}, total {time.time() - t0:.0f}s")


def rescan():
    """The literal greedy rescan on the digest's runs: flags and chains must equal the digest's."""
    from oracle import oracle as O
    t0 = time.time()
    full = bench_corpus(threads=min(16, os.cpu_count() or 1))
    runs, f_its = pick_runs(full)
    sub = full.subset(runs)
    del full
    dig = json.load(open(OUT))
    os.environ["NEMO_ORACLE_RESCAN"] = "1"
    t = time.time()
    s = [0] + [x for x in sub.success_iters() if x != 0]
    orc = O.analyze(sub, s, f_its, diff_mode=1, threads=min(8, os.cpu_count() or 1), skip_pulls=True)
    del os.environ["NEMO_ORACLE_RESCAN"]
    secs = time.time() - t
    same = True
    for i, r in enumerate(dig["runs"]):
        assert int(sub.iteration[i]) == r["iteration"]
        for k in (0, 1):
            g = 2 * i + k
            a, b = int(sub.node_off[g]), int(sub.node_off[g + 1])
            ch = orc.chains[orc.chains[:, 0] == g][:, 1:5]
            want = r["graphs"][k]
            ok = sha(orc.flags[a:b]) == want["flags_sha256"] and chain_digest(ch) == want["chains"]
            print(f"run {r['iteration']} graph {k}: {'equal' if ok else 'DIFFERENT'}", flush=True)
            same &= ok
    dig["rescan_equal"] = {"equal": bool(same), "graphs": 2 * len(dig["runs"]), "oracle_seconds": round(secs, 1),
                           "how": "NEMO_ORACLE_RESCAN=1 (greedy_rescan, the literal recompute after every "
                                  "accepted chain) on the digest's runs: flags and chains vs the digest"}
    with open(OUT, "w") as fh:
        json.dump(dig, fh, indent=1)
    print(f"rescan equal={same}, wrote {OUT}, total {time.time() - t0:.0f}s")


if __name__ == "__main__":
    if "--diff-all" in sys.argv:
        diff_all()
    elif "--rescan" in sys.argv:
        rescan()
    else:
        main()
