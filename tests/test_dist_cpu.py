"""Multi-rank rehearsal of the clause-sharded protocol on CPU (gloo, world_size 2 and 3).

Mirrors alll_runtime.cpp's enqueue_iteration for world > 1 with the oracle as the compute:
each rank evaluates only its clause shard (alll_shard_plan, the product's partitioning),
the violated-bitmask pieces are all-gathered, every rank computes the LFMIS of the global
violated set and resamples with Philox (replicated, "allgather" exchange) or resamples only
its own shard's MIS clauses into a bit-packed XOR delta that is all-reduced with SUM (disjoint
bits: SUM = OR; "allreduce" exchange, the north_star form).  Every rank must end with the
serial oracle's assignment and statistics, bit for bit.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, spec, mode, out_q):
    import sys

    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as o
    from alllsatisfiabilitysolver_amd import shard_plan

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, m, k, kind, seed, K = spec
    offs, lits = o.generate_ksat(1, n, m, k, kind)
    cb, ce, wpr = shard_plan(m, world, rank)
    A = o.init_assignment(seed, n)
    stats = dict(n_iterations=0, n_resamples=0, sum_mis=0)
    own_res = 0
    for it in range(K):
        stats["n_iterations"] += 1
        piece = np.zeros(wpr, np.uint64)
        if ce > cb:
            sub_offs = (offs[cb:ce + 1] - offs[cb]).astype(np.uint64)
            sub_lits = lits[int(offs[cb]):int(offs[ce])]
            _, vm = o.eval_mask(sub_offs, sub_lits, A)
            piece[: vm.size] = vm
        parts = [torch.zeros(wpr, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(parts, torch.from_numpy(piece.view(np.int64)))
        full = np.concatenate([p.numpy().view(np.uint64) for p in parts])[: (m + 63) // 64]
        U = o.mask_to_list(m, full)
        if U.size == 0:
            break
        M = o.lfmis(n, offs, lits, U)
        stats["sum_mis"] += M.size
        stats["n_resamples"] += int(np.sum(offs[M.astype(np.int64) + 1] - offs[M.astype(np.int64)]))
        if mode == "allgather":
            o.resample_words(A, seed, it, o.clause_vars(offs, lits, M))
        else:
            mine = M[(M >= cb) & (M < ce)]
            own_res += int(np.sum(offs[mine.astype(np.int64) + 1] - offs[mine.astype(np.int64)]))
            newA = o.resample_words(A.copy(), seed, it, o.clause_vars(offs, lits, mine))
            delta = torch.from_numpy((newA ^ A).astype(np.int64))
            dist.all_reduce(delta, op=dist.ReduceOp.SUM)
            A ^= delta.numpy().astype(np.uint32)
    out_q.put((rank, A.tolist(), stats, own_res))
    dist.barrier()
    dist.destroy_process_group()


def run_world(world, spec, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, spec, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res)


@pytest.mark.parametrize("world,mode", [(2, "allgather"), (2, "allreduce"), (3, "allgather"),
                                        (3, "allreduce")])
def test_sharded_protocol_equals_serial(oracle_mod, world, mode):
    o = oracle_mod
    n, m, k, kind, seed, K = spec = (3000, 12000, 3, 0, 21, 15)  # 3 tiles -> uneven shards at world 2
    offs, lits = o.generate_ksat(1, n, m, k, kind)
    # K resample rounds = a serial solve capped at K+1 eval passes
    st, A_ref, rows = o.solve(n, offs, lits, seed, max_iters=K + 1, trace=True)
    res = run_world(world, spec, mode)
    for rank, A, stats, own in res:
        np.testing.assert_array_equal(np.array(A, np.uint32), A_ref)
        assert stats["n_resamples"] == st["n_resamples"]
        assert stats["sum_mis"] == st["sum_mis_size"]
    if mode == "allreduce":  # per-rank shares add up to the total
        assert sum(r[3] for r in res) == st["n_resamples"]


def test_shard_plan_covers_clauses_in_order(native):
    from alllsatisfiabilitysolver_amd import shard_plan

    for m in (0, 1, 4095, 4096, 4097, 12000, 10_000_000, 128_000_000):
        for world in (1, 2, 3, 4, 8):
            prev = 0
            for r in range(world):
                b, e, w = shard_plan(m, world, r)
                assert b == prev and e >= b and w % 64 == 0
                assert b % 4096 == 0 or b == m
                assert (e - b) <= w * 64
                prev = e
            assert prev == m
