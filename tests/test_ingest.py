"""Native Molly ingest (nemo_ingest_molly) against the Python
loader (nemo_amd/corpus.load_molly): identical arrays, strings and errors.
Host only: runs without a GPU."""
import json
import os
import random

import numpy as np
import pytest

from nemo_amd.corpus import LoadError, load_molly
from nemo_amd.ingest import STR_LABEL, STR_TABLE, load_molly_native
from tests.small import random_prov

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIXTURES = sorted(d for d in os.listdir(HERE) if os.path.isfile(os.path.join(HERE, d, "runs.json")))


def assert_same(a, b):
    for k in ("iteration", "node_off", "edge_off", "node_word", "label", "edge_src", "edge_dst", "id_rank"):
        assert np.array_equal(np.asarray(getattr(a, k)), np.asarray(getattr(b, k))), k
    assert (a.n_tables, a.table_pre, a.table_post) == (b.n_tables, b.table_pre, b.table_post)
    assert a.tables == b.tables and a.labels == b.labels and a.status == b.status
    V = int(a.node_off[-1])
    assert list(a.node_ids[:V]) == list(b.node_ids[:V])
    assert list(a.node_types[:V]) == list(b.node_types[:V])
    assert list(a.node_times[:V]) == list(b.node_times[:V])


@pytest.mark.parametrize("name", FIXTURES)
def test_fixture_ingest_matches_python(name):
    d = os.path.join(HERE, name)
    assert_same(load_molly_native(d, threads=4), load_molly(d))


def write_dir(d, runs):
    os.makedirs(d, exist_ok=True)
    meta = []
    for i, (it, st, pre, post) in enumerate(runs):
        meta.append({"iteration": it, "status": st})
        json.dump(pre, open(os.path.join(d, f"run_{i}_pre_provenance.json"), "w"))
        json.dump(post, open(os.path.join(d, f"run_{i}_post_provenance.json"), "w"))
    json.dump(meta, open(os.path.join(d, "runs.json"), "w"))


@pytest.mark.parametrize("seed", range(8))
def test_random_ingest_matches_python(tmp_path, seed):
    rng = random.Random(seed)
    runs = []
    for it in range(rng.randint(1, 6)):
        runs.append((it, "success" if it == 0 or rng.random() < 0.6 else "fail",
                     random_prov(rng, "pre", 30), random_prov(rng, "post", 30)))
    # clock goals, escapes and non-ASCII labels
    runs[0][2]["goals"].append({"id": "goalc", "label": "clock(a, b, 3, 4)", "table": "clock", "time": "9"})
    runs[0][2]["goals"].append({"id": "goalw", "label": "clock(a, a, 2, __WILDCARD__)", "table": "clock"})
    runs[0][3]["goals"].append({"id": "goalu", "label": "café(\"q\", \\, \U0001F600)", "table": "té"})
    # the two-number match wins over an earlier wildcard one; an escaped label (decoded copy)
    runs[0][2]["goals"].append({"id": "goalx", "label": "clock(a, 1, __WILDCARD__) clock(b, 7, 8)", "table": "clock"})
    runs[0][2]["goals"].append({"id": "goale", "label": "clock(\"q\", r, 11, 12)", "table": "clock"})
    write_dir(str(tmp_path), runs)
    n1 = load_molly_native(str(tmp_path), threads=1)
    n4 = load_molly_native(str(tmp_path), threads=4)
    py = load_molly(str(tmp_path))
    assert_same(n1, py)
    assert_same(n4, py)
    r0 = n1.graph_nodes(0)
    times = {n1.node_ids[i]: n1.node_times[i] for i in r0}
    assert times["run_0_pre_goalc"] == "3" and times["run_0_pre_goalw"] == "2"
    assert times["run_0_pre_goalx"] == "7" and times["run_0_pre_goale"] == "11"


@pytest.mark.parametrize("case", ["dangling", "dup_goal", "dup_edge", "bad_json", "missing"])
def test_ingest_errors_match_python(tmp_path, case):
    pre = {"goals": [{"id": "goal0", "label": "pre(a)", "table": "pre", "time": "1"}],
           "rules": [{"id": "rule1", "label": "pre", "table": "pre", "type": "single"}],
           "edges": [{"from": "goal0", "to": "rule1"}]}
    post = json.loads(json.dumps(pre))
    if case == "dangling":
        post["edges"].append({"from": "rule1", "to": "goal9"})
    elif case == "dup_goal":
        post["goals"].append(dict(post["goals"][0]))
    elif case == "dup_edge":
        post["edges"].append({"from": "goal0", "to": "rule1"})
    write_dir(str(tmp_path), [(0, "success", pre, post)])
    if case == "bad_json":
        open(os.path.join(str(tmp_path), "run_0_post_provenance.json"), "w").write('{"goals": [')
    if case == "missing":
        os.remove(os.path.join(str(tmp_path), "run_0_post_provenance.json"))
    with pytest.raises(LoadError) as native:
        load_molly_native(str(tmp_path))
    if case in ("dangling", "dup_goal", "dup_edge"):
        with pytest.raises(LoadError) as py:
            load_molly(str(tmp_path))
        assert str(native.value) == str(py.value)


def test_null_and_empty_sections(tmp_path):
    write_dir(str(tmp_path), [(0, "success", {"goals": None, "rules": [], "edges": None}, {})])
    c = load_molly_native(str(tmp_path))
    assert int(c.node_off[-1]) == 0 and c.tables == ["pre", "post"]


def _synth_dir(tmp_path, n_runs=40, nodes=300, body_extra=2):
    from tools import synth
    corpus, info = synth.generate(n_runs, target_nodes=nodes, body_extra=body_extra)
    d = str(tmp_path / "molly")
    synth.write_molly(corpus, info, d, threads=4)
    return corpus, info, d


def test_c_writer_matches_python_writer(tmp_path):
    """synth.write_molly (C) writes the same files, byte for byte, as synth.to_molly."""
    from tools import synth
    corpus, info, d = _synth_dir(tmp_path, n_runs=6, nodes=200)
    p = str(tmp_path / "py")
    synth.to_molly(corpus, info, p)
    names = sorted(os.listdir(p))
    assert names == sorted(os.listdir(d))
    for n in names:
        assert open(os.path.join(p, n), "rb").read() == open(os.path.join(d, n), "rb").read(), n


def _named(c, tables, labels, g):
    """Graph g of corpus c with interned ids replaced by their strings: (words with the table name,
    label names, id ranks, edges).  Stream and one-shot interning assign ids in different orders."""
    from nemo_amd.corpus import TABLE_MASK
    n0, n1 = int(c.node_off[g]), int(c.node_off[g + 1])
    e0, e1 = int(c.edge_off[g]), int(c.edge_off[g + 1])
    w = np.asarray(c.node_word)[n0:n1]
    return ([(int(x) & ~TABLE_MASK, tables[int(x) & TABLE_MASK]) for x in w],
            [labels[int(x)] for x in np.asarray(c.label)[n0:n1]], np.asarray(c.id_rank)[n0:n1].tolist(),
            np.asarray(c.edge_src)[e0:e1].tolist(), np.asarray(c.edge_dst)[e0:e1].tolist())


def _stream_runs(st, chunk, one):
    """Every owned run of the stream as (iteration, pre graph, post graph) by name, plus the chunks'
    checks: every chunk after the one holding run 0 starts with run 0, replicated and not owned."""
    out, seen0 = [], False
    while True:
        c = st.next(chunk)  # valid until the call after next: read it now
        if c is None:
            break
        tables, labels = st.strings(STR_TABLE), st.strings(STR_LABEL)  # ids interned so far
        own = c.owned if c.owned is not None else np.ones(c.n_runs, np.uint8)
        if seen0:
            assert int(c.iteration[0]) == 0 and own[0] == 0
        for lr in range(c.n_runs):
            if own[lr]:
                out.append((int(c.iteration[lr]), _named(c, tables, labels, 2 * lr),
                            _named(c, tables, labels, 2 * lr + 1)))
        seen0 = seen0 or 0 in set(int(x) for x in c.iteration)
        assert tables[c.table_pre] == "pre" and tables[c.table_post] == "post"
    return out, st.strings(STR_TABLE), st.strings(STR_LABEL)


def _expected_order(one):
    """Parse order: run 0, failedRuns[0] (first non-success run in runs.json order), the rest."""
    its = [int(x) for x in one.iteration]
    f0 = next((it for it, s in zip(its, one.status) if s != "success"), None)
    head = [0] if 0 in its else []
    if f0 is not None and f0 != 0:
        head.append(f0)
    return head + [it for it in its if it not in head]


@pytest.mark.parametrize("chunk", [1, 7, 16, 40, 100])
def test_stream_chunks_match_one_shot(tmp_path, chunk):
    """nemo_ingest_next's chunks, owned runs concatenated, hold nemo_ingest_molly's runs in parse order
    (run 0, failedRuns[0], the rest), each equal by name to the one-shot ingest's; every chunk after the
    one holding run 0 starts with run 0 replicated (not owned)."""
    from nemo_amd.pipeline import IngestStream
    _, _, d = _synth_dir(tmp_path)
    one = load_molly_native(d, threads=4)
    assert any(s != "success" for s in one.status)
    st = IngestStream(d, threads=3)
    runs, tables, labels = _stream_runs(st, chunk, one)
    assert [it for it, _, _ in runs] == _expected_order(one)
    for it, pre, post in runs:
        r = one.run_index(it)
        assert pre == _named(one, one.tables, one.labels, 2 * r), it
        assert post == _named(one, one.tables, one.labels, 2 * r + 1), it
    assert sorted(tables) == sorted(one.tables) and sorted(labels) == sorted(one.labels)
    st.close()


def test_stream_error_and_end(tmp_path):
    from nemo_amd.pipeline import IngestStream
    _, _, d = _synth_dir(tmp_path, n_runs=5, nodes=100)
    open(os.path.join(d, "run_3_post_provenance.json"), "w").write('{"goals": [')
    st = IngestStream(d)
    assert st.next(3) is not None
    with pytest.raises(LoadError):
        st.next(3)
    st.close()


def rotate_dir(d, k):
    """Rewrite a Molly directory so that runs.json lists its runs rotated by k (run 0 no longer first);
    provenance files follow their run's new index (molly.go:59-60 names them by index)."""
    runs = json.load(open(os.path.join(d, "runs.json")))
    R = len(runs)
    tmp = {}
    for j in range(R):
        old = (j + k) % R
        for cond in ("pre", "post"):
            tmp[(j, cond)] = open(os.path.join(d, f"run_{old}_{cond}_provenance.json"), "rb").read()
    for (j, cond), data in tmp.items():
        open(os.path.join(d, f"run_{j}_{cond}_provenance.json"), "wb").write(data)
    json.dump(runs[k:] + runs[:k], open(os.path.join(d, "runs.json"), "w"))


@pytest.mark.parametrize("chunk", [2, 4, 11])
def test_stream_parses_run0_first(tmp_path, chunk):
    """runs.json with run 0 in the middle and a failed run listed before it: the stream parses run 0 and
    then failedRuns[0] into the first chunk (run 0 owned there) and replicates run 0 into every later
    chunk, so each chunk with a failed run holds the good run and the reference diff's label source is
    known from the first chunk on; every run equals the one-shot ingest's for the same iteration."""
    from nemo_amd.pipeline import IngestStream
    _, _, d = _synth_dir(tmp_path, n_runs=30, nodes=200)
    rotate_dir(d, 17)
    one = load_molly_native(d, threads=4)
    assert int(one.iteration[0]) == 17 and int(one.iteration[13]) == 0
    order = _expected_order(one)
    f0 = order[1]
    assert one.run_index(f0) < one.run_index(0), "the fixture must list failedRuns[0] before run 0"
    st = IngestStream(d, threads=2)
    c = st.next(chunk)
    assert [int(x) for x in c.iteration[:2]] == [0, f0]
    st.close()
    st = IngestStream(d, threads=2)
    runs, _, _ = _stream_runs(st, chunk, one)
    assert [it for it, _, _ in runs] == order
    for it, pre, post in runs:
        r = one.run_index(it)
        assert pre == _named(one, one.tables, one.labels, 2 * r), it
        assert post == _named(one, one.tables, one.labels, 2 * r + 1), it
    st.close()


def test_map_limit_falls_back_to_read(tmp_path):
    """Every graph keeps its provenance file mapped while it lives, so a one-shot ingest of many runs would
    pass vm.max_map_count; past a limit the files are read into heap buffers instead.  With the limit
    lowered to 5 live mappings (NEMO_INGEST_MAP_LIMIT, read once per process: a child process), a 40-run
    directory (80 files) must ingest to the same arrays and strings as the mapped path."""
    import subprocess
    import sys
    _, _, d = _synth_dir(tmp_path, n_runs=40, nodes=300)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    arrays = ("iteration", "node_off", "edge_off", "node_word", "label", "edge_src", "edge_dst", "id_rank")
    strings = ("tables", "labels", "status", "node_ids", "node_types", "node_times")
    out = str(tmp_path / "limited")
    code = (f"import sys, json, numpy as np; sys.path.insert(0, {root!r})\n"
            f"from nemo_amd.ingest import load_molly_native\n"
            f"c = load_molly_native({d!r}, threads=4)\n"
            f"np.savez({out + '.npz'!r}, **{{k: np.asarray(getattr(c, k)) for k in {arrays!r}}})\n"
            f"json.dump({{k: list(getattr(c, k)) for k in {strings!r}}}, open({out + '.json'!r}, 'w'))\n")
    env = dict(os.environ, NEMO_INGEST_MAP_LIMIT="5")
    subprocess.run([sys.executable, "-c", code], check=True, env=env, timeout=300)
    lim = np.load(out + ".npz")
    lstr = json.load(open(out + ".json"))
    ref = load_molly_native(d, threads=4)
    for k in arrays:
        assert np.array_equal(np.asarray(getattr(ref, k)), lim[k]), k
    V = int(ref.node_off[-1])
    for k in strings:
        want = list(getattr(ref, k))
        got = lstr[k]
        if k.startswith("node_"):
            want, got = want[:V], got[:V]
        assert want == got, k
