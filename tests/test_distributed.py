"""Run-sharded multi-process protocol on CPU (gloo, world_size 2).

Each rank owns a contiguous block of runs plus a replicated, not-owned run 0
(bench.py's layout), computes its partial cross-run reduction vector (the
oracle stands in for libnemohip here: no GPU), all-reduces it with SUM, and
interprets it with the library's own host-only nemo_reduce_interpret.  The
result must equal the single-process analysis of the whole corpus.
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


def _worker(rank, world, port, runs_per_rank, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nemo_amd.engine import reduce_interpret
        from oracle import oracle as O
        from tools import synth
        corpus, _ = synth.generate(runs_per_rank, target_nodes=800, run_base=rank * runs_per_rank,
                                   prepend_run0=True, threads=2)
        owned = corpus.owned if corpus.owned is not None else np.ones(corpus.n_runs, np.uint8)
        ok = [s == "success" for s in corpus.status]
        success = [0] + [int(it) for it, o, s in zip(corpus.iteration, owned, ok) if o and s and it != 0]
        failed = [int(it) for it, o, s in zip(corpus.iteration, owned, ok) if o and not s]
        res = O.analyze(corpus, success, failed, threads=2, skip_pulls=True)
        vec = torch.from_numpy(res.reduce.astype(np.int64))
        dist.all_reduce(vec)
        T = corpus.n_tables
        achieved, inter, union = reduce_interpret(vec.numpy().astype(np.uint32), T, corpus.table_post)
        if rank == 0:
            q.put({"achieved": achieved, "inter": inter, "union": union, "pre_holds": int(vec[2 * T + 2]),
                   "n_runs": int(vec[2 * T + 3])})
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_reduction_matches_single_process(world):
    from nemo_amd.engine import reduce_interpret
    from oracle import oracle as O
    from tools import synth
    runs_per_rank = 12
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, runs_per_rank, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    corpus, _ = synth.generate(world * runs_per_rank, target_nodes=800, threads=2)
    full = O.analyze(corpus, corpus.success_iters(), corpus.failed_iters(), threads=2, skip_pulls=True)
    T = corpus.n_tables
    a, inter, union = reduce_interpret(full.reduce, T, corpus.table_post)
    assert got["achieved"] == a == full.achieved
    assert got["inter"] == inter == [int(x) for x in full.inter]
    assert got["union"] == union == [int(x) for x in full.union]
    assert got["pre_holds"] == int(full.reduce[2 * T + 2])
    assert got["n_runs"] == corpus.n_runs


def _gpu_worker(rank, world, port, runs_per_rank, q):
    # bench.py's rank flow on the device: shard + replicated run 0, the whole
    # device pass, nemo_protos_partial into a device vector, all-reduce (gloo
    # over a host copy here: the box has one GPU; bench.py uses RCCL on the
    # device vector), nemo_protos_finalize; plus every owned failed run's diff
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nemo_amd.corpus import DIFF_PER_RUN
        from nemo_amd.engine import Engine
        from oracle import oracle as O
        from tools import synth
        corpus, _ = synth.generate(runs_per_rank, target_nodes=800, run_base=rank * runs_per_rank,
                                   prepend_run0=True, threads=2)
        owned = corpus.owned if corpus.owned is not None else np.ones(corpus.n_runs, np.uint8)
        ok = [s == "success" for s in corpus.status]
        success = [0] + [int(it) for it, o, s in zip(corpus.iteration, owned, ok) if o and s and it != 0]
        failed = [int(it) for it, o, s in zip(corpus.iteration, owned, ok) if o and not s]
        eng = Engine(0)
        eng.load(corpus)
        eng.rebuild()
        eng.mark()
        eng.simplify()
        d_red = torch.zeros(eng.reduce_len(), dtype=torch.int32, device="cuda:0")
        eng.protos_partial(success, d_red.data_ptr())
        eng.diffprov(failed, DIFF_PER_RUN)
        eng.synchronize()
        vec = d_red.cpu().to(torch.int64)
        dist.all_reduce(vec)
        d_red.copy_(vec.to(torch.int32))
        torch.cuda.synchronize()
        got = eng.protos_finalize(d_red.data_ptr())
        orc = O.analyze(corpus, success, failed, diff_mode=DIFF_PER_RUN, threads=2, skip_pulls=True)
        masks = eng.diff_masks_view() if failed else None
        diff_ok = masks is None or np.array_equal(np.asarray(masks).reshape(-1), np.asarray(orc.diff_mask).reshape(-1))
        eng.close()
        q.put((rank, got, bool(diff_ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_device_pass_matches_single_process():
    from nemo_amd.engine import reduce_interpret
    from oracle import oracle as O
    from tools import synth
    world, runs_per_rank = 2, 12
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, world, port, runs_per_rank, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (g, d)) for r, g, d in (q.get(timeout=110) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    corpus, _ = synth.generate(world * runs_per_rank, target_nodes=800, threads=2)
    full = O.analyze(corpus, corpus.success_iters(), corpus.failed_iters(), threads=2, skip_pulls=True)
    T = corpus.n_tables
    a, inter, union = reduce_interpret(full.reduce, T, corpus.table_post)
    for r in range(world):
        g, diff_ok = got[r]
        assert diff_ok, f"rank {r}: diff masks differ from the oracle"
        assert g["achieved"] == a == full.achieved
        assert g["inter"] == inter and g["union"] == union
        assert g["pre_holds"] == int(full.reduce[2 * T + 2])
        assert g["n_runs"] == corpus.n_runs


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
