"""The oracle's incremental greedy @next-chain cover (greedy_incremental) against its literal form
(greedy_rescan: recompute every length of the component after each accepted chain), which is itself
checked against the path enumerator in test_oracle_literal.py.  Reference: preprocessing.go:70-138
(Q13's paths, longest first, accepted while they hold an unseen node).  CPU only."""
import os

import numpy as np
import pytest

from oracle import oracle as O
from tools import synth

CASES = {
    "c3_shape": dict(n=60, target_nodes=1500, body_extra=4),
    "dense": dict(n=12, target_nodes=5000, body_extra=6, nval=3, nloc=4),
    "molly": dict(n=40, target_nodes=2000),
    "deep_20k": dict(n=2, target_nodes=20000, eot=60, body_extra=6, nval=3, nloc=4),
}


def _run(c, rescan):
    if rescan:
        os.environ["NEMO_ORACLE_RESCAN"] = "1"
    try:
        return O.analyze(c, c.success_iters(), c.failed_iters(), threads=4, skip_pulls=True)
    finally:
        os.environ.pop("NEMO_ORACLE_RESCAN", None)


@pytest.mark.parametrize("name", sorted(CASES))
def test_incremental_equals_rescan(name):
    kw = dict(CASES[name])
    c, _ = synth.generate(kw.pop("n"), p_fault=0.3, **kw)
    a, b = _run(c, False), _run(c, True)
    assert len(a.chains) > 0
    assert np.array_equal(a.chains, b.chains)
    assert np.array_equal(a.flags, b.flags)


def test_c5_digest_pinned_by_rescan():
    """The C5-shape digest (tests/golden/c5_shape/digest.json, whose chains come from greedy_incremental) was
    recomputed once with greedy_rescan on its eight 1M-node graphs (make_c5_shape.py --rescan): identical
    flags and chains.  Its per-run diff entries cover every failed run of the 128-run corpus."""
    import json
    d = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c5_shape", "digest.json")))
    assert d["rescan_equal"]["equal"] is True and d["rescan_equal"]["graphs"] == 2 * len(d["runs"])
    alld = d["diff_per_run_all"]
    assert len(alld["failed_iters"]) == len(alld["entries"]) == 16
