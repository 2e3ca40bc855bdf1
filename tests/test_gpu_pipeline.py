"""GPU parity of the pipelined end-to-end path (nemo_amd/pipeline.py, SURVEY.md
§8f-4): a Molly-format directory parsed chunk by chunk (nemo_ingest_next) and
analysed chunk by chunk on the device equals the oracle on the whole
directory ingested at once.  Cross-chunk steps under test: the summed
prototype vectors (prototype.go:79-130), run 0 replicated into every later
chunk (differential-provenance.go:26), and the reference diff mode's
failedRuns[0] label set carried from its chunk to the others
(differential-provenance.go:22-43, nemo_diffprov_host_labels).
"""
import numpy as np
import pytest

from nemo_amd import engine as E
from nemo_amd import pipeline as P
from nemo_amd.corpus import DIFF_PER_RUN, DIFF_REFERENCE
from nemo_amd.ingest import load_molly_native
from oracle import oracle as O
from tools import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    e = E.Engine(0)
    yield e
    e.close()


@pytest.fixture(scope="module")
def molly_dir(tmp_path_factory):
    corpus, info = synth.generate(300, target_nodes=900, body_extra=3, p_fault=0.3)
    d = str(tmp_path_factory.mktemp("pipe") / "molly")
    synth.write_molly(corpus, info, d)
    return d


def _names(ids, tables):
    return sorted(tables[int(i)] for i in ids)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("chunk,mode", [(64, DIFF_REFERENCE), (300, DIFF_REFERENCE), (37, DIFF_PER_RUN)])
def test_pipeline_matches_oracle(eng, molly_dir, chunk, mode):
    one = load_molly_native(molly_dir, threads=8)
    s, f = one.success_iters(), one.failed_iters()
    assert len(f) > 20
    orc = O.analyze(one, s, f, diff_mode=mode, threads=8, skip_pulls=True)
    res = P.run(molly_dir, eng, chunk=chunk, threads=8, diff_mode=mode, keep=True)
    assert res.n_runs == one.n_runs
    for g in range(one.n_graphs):
        a, b = int(one.node_off[g]), int(one.node_off[g + 1])
        assert np.array_equal(res.flags[g], orc.flags[a:b]), f"flags of graph {g}"
    ch = np.concatenate(res.chains) if res.chains else np.zeros((0, 5), np.uint32)
    ch = ch[np.lexsort((ch[:, 1], ch[:, 0]))]
    assert np.array_equal(ch, orc.chains)
    assert res.achieved == orc.achieved
    # table ids may be numbered differently when a chunk after the first interns a new table
    assert _names(res.inter, res.tables) == _names(orc.inter, one.tables)
    assert _names(res.union, res.tables) == _names(orc.union, one.tables)
    if res.tables == one.tables:
        for r in range(one.n_runs):
            if one.status[r] == "success":
                assert np.array_equal(res.run_tables[r][0], orc.proto_bits[r]), f"proto list of run {r}"
            assert np.array_equal(res.run_tables[r][1], orc.graph_tables[r]), f"table set of run {r}"
    for e, it in enumerate(f):
        assert np.array_equal(res.diff_mask[it], orc.diff_mask[e]), f"D mask of failed run {it}"
        assert np.array_equal(res.missing[it], np.sort(orc.missing[orc.missing[:, 0] == e][:, 1])), it
    pre, post, asy = res.triggers
    assert np.array_equal(pre, orc.pre_rows) and np.array_equal(post, orc.post_rows)
    assert np.array_equal(np.sort(asy), np.sort(orc.async_rules))


@pytest.mark.timeout(300)
def test_pipeline_run0_not_first(eng, tmp_path):
    """runs.json lists run 0 in the middle: the stream parses it first, so the chunks before its old
    position still have the good run for their diffs (differential-provenance.go:26)."""
    from tests.test_ingest import rotate_dir
    corpus, info = synth.generate(120, target_nodes=700, body_extra=3, p_fault=0.3)
    d = str(tmp_path / "molly")
    synth.write_molly(corpus, info, d)
    rotate_dir(d, 50)
    one = load_molly_native(d, threads=8)
    assert int(one.iteration[0]) == 50
    s = [0] + [x for x in one.success_iters() if x != 0]
    f = one.failed_iters()
    assert f and min(one.run_index(x) for x in f) < one.run_index(0)
    orc = O.analyze(one, s, f, diff_mode=DIFF_REFERENCE, threads=8, skip_pulls=True)
    res = P.run(d, eng, chunk=32, threads=8, diff_mode=DIFF_REFERENCE, keep=True)
    for g in range(one.n_graphs):
        a, b = int(one.node_off[g]), int(one.node_off[g + 1])
        assert np.array_equal(res.flags[g], orc.flags[a:b]), f"flags of graph {g}"
    assert _names(res.inter, res.tables) == _names(orc.inter, one.tables)
    for e, it in enumerate(f):
        assert np.array_equal(res.diff_mask[it], orc.diff_mask[e]), f"D mask of failed run {it}"
        assert np.array_equal(res.missing[it], np.sort(orc.missing[orc.missing[:, 0] == e][:, 1])), it


@pytest.mark.timeout(300)
@pytest.mark.parametrize("chunk", [2, 32])
def test_pipeline_run0_failed_not_first(eng, tmp_path, chunk):
    """Run 0 itself failed and runs.json lists another failed run before it: failedRuns[0] (the reference
    diff's label source, differential-provenance.go:22-43) is not run 0, and the stream parses it right
    after run 0, so the first chunk holds both."""
    import json
    import os
    from tests.test_ingest import rotate_dir
    corpus, info = synth.generate(90, target_nodes=700, body_extra=3, p_fault=0.3)
    d = str(tmp_path / "molly")
    synth.write_molly(corpus, info, d)
    rotate_dir(d, 40)
    runs = json.load(open(os.path.join(d, "runs.json")))
    for r in runs:
        if int(r["iteration"]) == 0:
            r["status"] = "failure"
    json.dump(runs, open(os.path.join(d, "runs.json"), "w"))
    one = load_molly_native(d, threads=8)
    s, f = one.success_iters(), one.failed_iters()
    assert 0 in f and f[0] != 0 and one.run_index(f[0]) < one.run_index(0)
    orc = O.analyze(one, s, f, diff_mode=DIFF_REFERENCE, threads=8, skip_pulls=True)
    res = P.run(d, eng, chunk=chunk, threads=8, diff_mode=DIFF_REFERENCE, keep=True)
    assert _names(res.inter, res.tables) == _names(orc.inter, one.tables)
    for e, it in enumerate(f):
        assert np.array_equal(res.diff_mask[it], orc.diff_mask[e]), f"D mask of failed run {it}"
        assert np.array_equal(res.missing[it], np.sort(orc.missing[orc.missing[:, 0] == e][:, 1])), it
