"""Run-sharded multi-process protocol on CPU (gloo, world_size 2).

Each rank owns its LPT shard of the runs (nemo_partition_runs) plus a
replicated, not-owned run 0, computes its partial cross-run reduction vector
(the oracle stands in for libnemohip here: no GPU), all-reduces it with SUM,
and interprets it with the library's own host-only nemo_reduce_interpret.
The reference diff mode's failedRuns[0] label set is broadcast from the rank
that owns that run.  Every rank's results must equal the single-process
analysis of the whole corpus.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard(rank, world, n_runs, nodes=800):
    """This rank's LPT shard (nemo_partition_runs, run 0 replicated) of the global corpus, with the
    global success / failed lists restricted to what it owns."""
    from nemo_amd.shard import shard_layout
    from tools import synth
    full, _ = synth.generate(n_runs, target_nodes=nodes, threads=2, p_fault=0.4)
    runs, owned = shard_layout(full, rank, world)
    shard = full.subset(runs, owned)
    own = shard.owned if shard.owned is not None else np.ones(shard.n_runs, np.uint8)
    ok = [st == "success" for st in shard.status]
    success = [0] + [int(it) for it, o, s in zip(shard.iteration, own, ok) if o and s and it != 0]
    failed = [int(it) for it, o, s in zip(shard.iteration, own, ok) if o and not s]
    return full, shard, success, failed


def _broadcast_labels(labels, owner):
    """failedRuns[0]'s post-goal label set from the rank that owns that run (size, then the set)."""
    n = torch.tensor([len(labels) if labels is not None else 0], dtype=torch.int64)
    dist.broadcast(n, owner)
    buf = torch.from_numpy(np.asarray(labels, np.int64)) if labels is not None else torch.zeros(int(n), dtype=torch.int64)
    dist.broadcast(buf, owner)
    return buf.numpy().astype(np.uint32)


def _owner_of(value: bool):
    """Lowest rank for which `value` holds (MIN all-reduce)."""
    t = torch.tensor([dist.get_rank() if value else 1 << 30], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t)


def _worker(rank, world, port, n_runs, q):
    # the sharded protocol on CPU, with the oracle standing in for the device pass
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nemo_amd.corpus import DIFF_PER_RUN
        from nemo_amd.engine import reduce_interpret
        from oracle import oracle as O
        full, shard, success, failed = _shard(rank, world, n_runs)
        f0 = full.failed_iters()[0]
        owner = _owner_of(f0 in failed)
        labels = None
        if rank == owner:  # the owner's post-goal labels of failedRuns[0]
            g = 2 * shard.run_index(f0) + 1
            n0, n1 = int(shard.node_off[g]), int(shard.node_off[g + 1])
            labels = shard.label[n0:n1][(shard.node_word[n0:n1] & 0x80000000) == 0]
        labels = _broadcast_labels(labels, owner)
        res = O.analyze(shard, success, failed, threads=2, skip_pulls=True, diff_labels=labels)
        per_run = O.analyze(shard, success, failed, diff_mode=DIFF_PER_RUN, threads=2, skip_pulls=True)
        vec = torch.from_numpy(res.reduce.astype(np.int64))
        dist.all_reduce(vec)
        T = shard.n_tables
        achieved, inter, union = reduce_interpret(vec.numpy().astype(np.uint32), T, shard.table_post)
        q.put((rank, {"achieved": achieved, "inter": inter, "union": union, "pre_holds": int(vec[2 * T + 2]),
                      "n_runs": int(vec[2 * T + 3]), "failed": failed, "ref": res.diff_mask, "per_run": per_run.diff_mask,
                      "missing": res.missing}))
    finally:
        dist.destroy_process_group()


def _expect(n_runs):
    from nemo_amd.corpus import DIFF_PER_RUN, DIFF_REFERENCE
    from nemo_amd.engine import reduce_interpret
    from oracle import oracle as O
    from tools import synth
    corpus, _ = synth.generate(n_runs, target_nodes=800, threads=2, p_fault=0.4)
    s, f = corpus.success_iters(), corpus.failed_iters()
    full = O.analyze(corpus, s, f, diff_mode=DIFF_REFERENCE, threads=2, skip_pulls=True)
    per_run = O.analyze(corpus, s, f, diff_mode=DIFF_PER_RUN, threads=2, skip_pulls=True)
    T = corpus.n_tables
    a, inter, union = reduce_interpret(full.reduce, T, corpus.table_post)
    assert a == full.achieved and inter == [int(x) for x in full.inter]
    return corpus, f, full, per_run, (a, inter, union)


def _check_ranks(got, n_runs):
    corpus, f, full, per_run, (a, inter, union) = _expect(n_runs)
    T = corpus.n_tables
    seen = []
    for r, g in sorted(got.items()):
        assert g["achieved"] == a and g["inter"] == inter and g["union"] == union
        assert g["pre_holds"] == int(full.reduce[2 * T + 2]) and g["n_runs"] == corpus.n_runs
        idx = [f.index(it) for it in g["failed"]]
        seen += g["failed"]
        # reference mode (differential-provenance.go:22-43): failedRuns[0]'s labels for every entry,
        # though that run lives on one rank only
        assert np.array_equal(np.asarray(g["ref"]).reshape(len(idx), -1), full.diff_mask[idx]), f"rank {r}"
        assert np.array_equal(np.asarray(g["per_run"]).reshape(len(idx), -1), per_run.diff_mask[idx]), f"rank {r}"
        if "missing" in g:
            m = np.asarray(g["missing"]).reshape(-1, 2)
            want = full.missing[np.isin(full.missing[:, 0], idx)].copy()
            remap = {e: i for i, e in enumerate(idx)}
            want[:, 0] = [remap[int(e)] for e in want[:, 0]]
            assert np.array_equal(m, want), f"rank {r} missing events"
    assert sorted(seen) == sorted(f)
    return f


def _spawn(target, world, n_runs, timeout):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, n_runs, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=timeout) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


@pytest.mark.parametrize("world", [2])
def test_sharded_reduction_matches_single_process(world):
    n_runs = 24
    got = _spawn(_worker, world, n_runs, 300)
    f = _check_ranks(got, n_runs)
    # failedRuns[0] must not sit on every rank, or the broadcast would prove nothing
    from nemo_amd.shard import partition_runs
    from tools import synth
    corpus, _ = synth.generate(n_runs, target_nodes=800, threads=2, p_fault=0.4)
    parts = partition_runs(corpus, world)
    assert len(set(int(parts[corpus.run_index(it)]) for it in f)) == world


def _gpu_worker(rank, world, port, n_runs, q):
    # bench.py's rank flow on the device: LPT shard + replicated run 0, the
    # whole device pass, nemo_protos_partial into a device vector, all-reduce
    # (gloo over a host copy here: the box has one GPU, so two ranks share it
    # and RCCL refuses a duplicate device; bench.py all-reduces the device
    # vector with RCCL), nemo_protos_finalize; reference-mode diffs through
    # nemo_goal_labels on the owner of failedRuns[0] -> broadcast ->
    # nemo_diffprov_labels on every rank; per-run diffs
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nemo_amd.corpus import DIFF_PER_RUN
        from nemo_amd.engine import Engine
        full, shard, success, failed = _shard(rank, world, n_runs)
        f0 = full.failed_iters()[0]
        owner = _owner_of(f0 in failed)
        cap = int(np.max(np.diff(full.node_off.astype(np.int64)))) + 1
        eng = Engine(0)
        eng.load(shard)
        eng.rebuild()
        eng.mark()
        eng.simplify()
        d_red = torch.zeros(eng.reduce_len(), dtype=torch.int32, device="cuda:0")
        eng.protos_partial(success, d_red.data_ptr())
        d_lab = torch.zeros(cap, dtype=torch.int32, device="cuda:0")
        if rank == owner:
            eng.goal_labels(f0, 1, d_lab.data_ptr(), cap)
        eng.synchronize()
        h = d_lab.cpu()
        dist.broadcast(h, owner)
        d_lab.copy_(h)
        torch.cuda.synchronize()
        eng.diffprov_labels(failed, d_lab.data_ptr(), cap)
        ref = eng.diff_masks(len(failed)) if failed else np.zeros((0, 0), np.uint8)
        miss = eng.missing()
        eng.diffprov(failed, DIFF_PER_RUN)
        per_run = eng.diff_masks(len(failed)) if failed else np.zeros((0, 0), np.uint8)
        vec = d_red.cpu().to(torch.int64)
        dist.all_reduce(vec)
        d_red.copy_(vec.to(torch.int32))
        torch.cuda.synchronize()
        got = eng.protos_finalize(d_red.data_ptr())
        eng.close()
        got.update({"failed": failed, "ref": ref, "per_run": per_run, "missing": miss})
        q.put((rank, got))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_device_pass_matches_single_process():
    world, n_runs = 2, 24
    got = _spawn(_gpu_worker, world, n_runs, 110)
    _check_ranks(got, n_runs)


def test_reduce_interpret_first_list_empty():
    # prototype.go:80-103: `longest` is only updated inside the loop over list0,
    # so an empty first list empties both inter and union (Q-PROTO-FIRST)
    from nemo_amd.engine import reduce_interpret
    T = 4
    vec = np.zeros(2 * T + 4, np.uint32)
    vec[0:T] = [2, 1, 0, 2]       # counts over non-empty lists
    vec[2 * T] = 2                # achvdCond
    vec[2 * T + 1] = 0            # first list empty
    assert reduce_interpret(vec, T, 3) == (2, [], [])
    vec[T:2 * T] = [1, 1, 0, 1]
    vec[2 * T + 1] = 1
    # table 3 is "post": excluded from both (prototype.go:106,120)
    assert reduce_interpret(vec, T, 3) == (2, [0], [0, 1])
