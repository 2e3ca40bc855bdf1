"""Host-side timeline of bench.py's C3 step (no extra syncs): the time each API call of the step returns,
relative to the step start, averaged over steps.  Shows where the host blocks (syncs) and where it computes.
usage: python tools/step_host.py [runs] [steps]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nemo_amd.corpus import DIFF_REFERENCE  # noqa: E402
from nemo_amd.engine import Engine  # noqa: E402
from tools import synth  # noqa: E402
from bench import table_mask  # noqa: E402

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
corpus, _ = synth.generate(runs, prepend_run0=True, threads=16, **synth.CONFIGS["c3"])
success, failed = corpus.success_iters(), corpus.failed_iters()
if success[0] != 0:
    success = [0] + [s for s in success if s != 0]
eng = Engine(0)
eng.set_stream(torch.cuda.current_stream().cuda_stream)
if os.environ.get("NEMO_STAGE_SDMA") == "1":
    eng.set_option("stage_sdma", 1)
eng.load(corpus)
d_red = torch.zeros(eng.reduce_len(), dtype=torch.int32, device="cuda")
fidx = np.array([corpus.run_index(f) for f in failed], np.int64)
marks = {}
STAGE_FIRST = os.environ.get("STAGE_FIRST") == "1"


def step(rec):
    t0 = time.perf_counter()

    def m(name):
        if rec:
            marks.setdefault(name, []).append((time.perf_counter() - t0) * 1e6)
    eng.rebuild(); m("rebuild")
    eng.mark(); m("mark")
    eng.diffprov(failed, DIFF_REFERENCE); m("diffprov")
    eng.simplify(); m("simplify")
    if STAGE_FIRST:
        eng.stage_simplified(); m("stage")
    eng.protos_partial(success, d_red.data_ptr()); m("protos_partial")
    eng.protos_stage(d_red.data_ptr())
    if not STAGE_FIRST:
        eng.stage_simplified(); m("stage")
    eng.triggers(); m("triggers")
    eng.pull(1); m("pull1")
    eng.pull(2); m("pull2")
    protos = eng.protos_finalize(d_red.data_ptr()); m("protos_finalize")
    tabs = eng.run_tables(1); m("run_tables")
    tf = tabs[fidx]
    _ = table_mask(protos["inter"], tf.shape[1]) & ~tf
    _ = table_mask(protos["union"], tf.shape[1]) & ~tf
    m("missingFrom(host)")
    eng.trigger_rows(); m("trigger_rows")
    eng.diff_masks_view(); m("diff_masks_view")
    eng.missing(); m("missing")
    eng.simplified_view(); m("simplified_view")


for _ in range(2):
    step(False)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(steps):
    step(True)
torch.cuda.synchronize()
print(f"{(time.perf_counter() - t) / steps * 1e3:.3f} ms per step")
prev = 0.0
for k, v in marks.items():
    a = float(np.mean(v))
    print(f"{k:>20} {a:9.1f} us  (+{a - prev:7.1f})")
    prev = a
