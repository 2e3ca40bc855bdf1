"""Deep-graph probe (SURVEY §8d C5 shape: ~1M-node graphs, EOT 2000) on one GPU.

usage: python tools/deep_probe.py RUNS [NODES] [EOT] [--check] [--dense]
--dense: bench.py's C5 generator settings (~4 edges per node).
Prints per-kernel HIP-event times of one analysis pass; --check compares every
device result with the CPU oracle (slow: the oracle needs seconds per graph).
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nemo_amd import engine as E  # noqa: E402
from nemo_amd.corpus import DIFF_PER_RUN  # noqa: E402
from tools import synth  # noqa: E402

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 4
nodes = int(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("-") else 1_000_000
eot = int(sys.argv[3]) if len(sys.argv) > 3 and not sys.argv[3].startswith("-") else 2000
check = "--check" in sys.argv
gen = dict(body_extra=6, nval=3, nloc=4) if "--dense" in sys.argv else {}
t = time.time()
corpus, _ = synth.generate(runs, target_nodes=nodes, eot=eot, threads=16, **gen)
print(f"generated {runs} runs, {int(corpus.node_off[-1])} nodes, {int(corpus.edge_off[-1])} edges "
      f"in {time.time() - t:.1f}s", flush=True)
s, f = corpus.success_iters(), corpus.failed_iters()
eng = E.Engine(0)
t = time.time()
eng.load(corpus)
eng.synchronize()
print(f"load {time.time() - t:.2f}s", flush=True)
for rep in range(2):
    eng.set_timing(True)
    eng.reset_timings()
    t = time.time()
    eng.rebuild()
    eng.mark()
    eng.simplify()
    eng.prototypes(s)
    eng.diffprov(f, DIFF_PER_RUN)
    eng.triggers()
    eng.pull(1)
    eng.pull(2)
    eng.synchronize()
    wall = time.time() - t
    tim = eng.timings()
    eng.set_timing(False)
    print(f"pass {rep}: {wall * 1e3:.1f} ms wall, {runs / wall:.1f} runs/s", flush=True)
    for k, v in sorted(tim.items(), key=lambda kv: -kv[1]["ms"]):
        if v["ms"] > 0.05:
            print(f"  {k:16s} {v['ms']:10.2f} ms", flush=True)
if check:
    from oracle import oracle as O
    from tests.compare import assert_same
    import threading
    t = time.time()
    box = {}
    th = threading.Thread(target=lambda: box.setdefault("orc", O.analyze(corpus, s, f, diff_mode=DIFF_PER_RUN,
                                                                          threads=16)))
    th.start()
    while th.is_alive():  # heartbeat: the oracle needs minutes on dense 1M-node graphs
        th.join(30)
        if th.is_alive():
            print(f"  oracle running {time.time() - t:.0f}s", flush=True)
    orc = box["orc"]
    print(f"oracle {time.time() - t:.1f}s", flush=True)
    res = E.analyze(corpus, s, f, diff_mode=DIFF_PER_RUN, engine=eng, pulls=True)
    assert_same(corpus, res, orc, len(f))
    print("parity OK", flush=True)
eng.close()
