"""Clause-sharded multi-rank path on the GPU: world 2 and 3 ranks (one process each) share the
one visible MI355X and exchange through the host-staged hook (alll_set_host_exchange over
gloo) instead of RCCL, which cannot put two ranks on one device.  Everything else is the
production multi-GPU path: eval of the own shard only, all-gather of the violated bitmask,
collect of the other shards' lists, replicated LFMIS + Philox resample ("allgather") or
own-shard resample + all-reduce of the assignment XOR delta ("allreduce").  Every rank must
reproduce the serial oracle trajectory bit for bit, with per-GPU resample shares that add up.
"""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (spawned ranks import this module first: the library's ROCm runtime before torch's)
sys.path.insert(0, ROOT)
from alllsatisfiabilitysolver_amd import _native as _alll_native  # noqa: E402

try:
    _alll_native.lib()
except Exception:
    pass
torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402



def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, spec, flags, out_q):
    import sys

    sys.path.insert(0, ROOT)
    from alllsatisfiabilitysolver_amd import Solver, generate_ksat, gloo_exchange

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, m, k, kind, seed, K = spec[:6]
    T = spec[6] if len(spec) > 6 else 1
    offs, lits = make_instance(n, m, k, kind)
    try:
        with Solver(n, offs, lits, seed=seed, device=0, rank=rank, world=world, flags=flags,
                    exchange=gloo_exchange(), n_threads=T) as s:
            traj = []
            for _ in range(K):
                s.run(1)
                traj.append(s.assignment_words().tolist())
            st = s.stats()
            mis = s.mis().tolist()
            # a standalone evaluation after the loop: the count summed over the ranks and the
            # clause-order mask refreshed from it (own shard + all-gathered pieces)
            st["verify"] = s.verify()
            st["mask"] = s.violated_mask().tolist()
        out_q.put((rank, traj, st, mis, None))
    except Exception as e:  # surfaced by the parent
        out_q.put((rank, None, None, None, repr(e)))
    dist.barrier()
    dist.destroy_process_group()


def make_instance(n, m, k, kind):
    if isinstance(k, tuple):  # mixed widths (the ragged evaluation layout)
        from alllsatisfiabilitysolver_amd import generate_mixed

        return generate_mixed(1, n, m, *k)
    from alllsatisfiabilitysolver_amd import generate_ksat

    return generate_ksat(1, n, m, k, kind)


def run_world(world, spec, flags, env=None):
    for key, v in (env or {}).items():  # (inherited by the spawned ranks)
        os.environ[key] = v
    try:
        return _run_world(world, spec, flags)
    finally:
        for key in env or {}:
            del os.environ[key]


def _run_world(world, spec, flags):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, spec, flags, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=600) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
    return sorted(res, key=lambda r: r[0])


SPECS = {
    # 7 tiles of 4096 clauses -> uneven shards; fixed-k hybrid eval path
    "small": (7000, 28000, 3, 0, 5, 8),
    # more variables than one LDS window holds: windowed evaluation order inside every shard
    "windows": (1_600_000, 40000, 3, 0, 5, 4),
    # 300 iterations: the 8-bit cover stamps wrap once (the reduce clears them at iteration 255)
    "long": (3000, 12000, 3, 0, 6, 300),
    # BASELINE config C2 at full size (1M variables, 4M clauses = 977 tiles, 489 per rank):
    # two iterations, bit-exact on both ranks
    "c2": (1_000_000, 4_000_000, 3, 0, 1, 2),
    # BASELINE config C5 at full size (power-law 3-SAT, 2.5M variables / 10M clauses: hot
    # variables, vmix owner slots, 7 grid rounds), the 8-GPU config's sharded path at world 2
    "c5": (2_500_000, 10_000_000, 3, 1, 1, 2),
    # the round robin of T = 4 / 7 sets (the fixpoint passes) on every rank of the sharded loop
    "small_rr4": (7000, 28000, 3, 0, 5, 8, 4),
    "c2_rr7": (1_000_000, 4_000_000, 3, 0, 1, 2, 7),
    # clause ids not packed into the literals (evaluation positions + perm on the own shard)
    "small_positions": (7000, 28000, 3, 0, 5, 8),
    # mixed widths 2-12: the ragged evaluation layout (own shard), CSR LFMIS
    "ragged": (5000, 20000, (2, 12), 0, 5, 6),
    # 8-SAT: the wide fixed-width entries
    "k8": (40000, 60000, 8, 0, 3, 4),
    # the 8-way split of the BASELINE 8-GPU configs (C4, C5) at a small size: 16 tiles, two per
    # rank; and 9 tiles over 8 ranks (two per rank: ranks 5-7 own no clause)
    "small8": (16000, 64000, 3, 0, 5, 6),
    "uneven8": (9000, 36000, 3, 0, 5, 6),
}
ENV = {"small_positions": {"ALLL_PACKED_IDS": "0"}}


@pytest.mark.parametrize("world,mode,spec_name", [(2, "allgather", "small"), (2, "allreduce", "small"),
                                                  (3, "allgather", "small"), (3, "allreduce", "small"),
                                                  (2, "allgather", "windows"), (2, "allgather", "long"),
                                                  (2, "allreduce", "long"), (2, "allgather", "c2"),
                                                  (2, "allreduce", "c2"), (2, "allgather", "c5"),
                                                  (2, "allgather", "small_rr4"),
                                                  (3, "allreduce", "small_rr4"), (2, "allgather", "c2_rr7"),
                                                  (3, "allgather", "small_positions"), (2, "allgather", "ragged"),
                                                  (3, "allreduce", "ragged"), (2, "allgather", "k8"),
                                                  (8, "allgather", "small8"), (8, "allreduce", "small8"),
                                                  (8, "allgather", "uneven8")])
def test_sharded_solver_matches_oracle(oracle_mod, native, world, mode, spec_name):
    """Every rank lays out its own shard only; the other shards' violated lists come from the
    all-gathered clause-order mask and the AoS literals (k_cmark / k_collect)."""
    o = oracle_mod
    spec = SPECS[spec_name]
    n, m, k, kind, seed, K = spec[:6]
    T = spec[6] if len(spec) > 6 else 1
    flags = native.FLAG_EXCHANGE_ALLREDUCE if mode == "allreduce" else 0
    offs, lits = make_instance(n, m, k, kind)
    st_o, A_o, rows = o.solve(n, offs, lits, seed, max_iters=K + 1, trace=True, T=T)
    res = run_world(world, spec, flags, ENV.get(spec_name))
    for rank, traj, st, mis, err in res:
        assert err is None, f"rank {rank}: {err}"
        for i, (it, nu, nm, dres, A_after) in enumerate(rows):
            np.testing.assert_array_equal(np.array(traj[i], np.uint32), A_after, err_msg=f"rank {rank} iter {it}")
        assert st["n_resamples"] == st_o["n_resamples"]
        assert st["sum_mis_size"] == st_o["sum_mis_size"]
        assert st["n_gpus"] == world
        assert sum(st["gpu_resamples"]) == st["n_resamples"]
        # verify + get_violated_mask after the loop describe the final assignment
        nv_o, vm_o = o.eval_mask(offs, lits, np.array(traj[-1], np.uint32))
        assert st["verify"] == (nv_o == 0, nv_o), f"rank {rank}"
        np.testing.assert_array_equal(np.array(st["mask"], np.uint64), vm_o, err_msg=f"rank {rank} mask")
    # all ranks agree on the last MIS
    assert all(r[3] == res[0][3] for r in res)


@pytest.mark.parametrize("mode,spec_name", [("allgather", "small"), ("allreduce", "small"),
                                            ("allgather", "windows")])
def test_rccl_one_rank_matches_oracle(oracle_mod, native, mode, spec_name):
    """The multi-GPU exchange path over a real RCCL communicator of one rank: the all-gather of
    the violated bitmask (and the all-reduce of the XOR delta) run inside the captured hipGraphs
    of 1 and 8 iterations, the other-shard collect runs, and the trajectory stays the oracle's."""
    from alllsatisfiabilitysolver_amd import Solver, comm_unique_id

    o = oracle_mod
    n, m, k, kind, seed, K = SPECS[spec_name]
    K = max(K, 12)
    flags = native.FLAG_EXCHANGE_ALLREDUCE if mode == "allreduce" else 0
    offs, lits = o.generate_ksat(1, n, m, k, kind)
    st_o, A_o, rows = o.solve(n, offs, lits, seed, max_iters=K + 1, trace=True)
    def at(i):  # assignment after iteration i (a converged run keeps its last one)
        return rows[min(i, len(rows) - 1)][4]

    with Solver(n, offs, lits, seed=seed, device=0, rank=0, world=1, comm_id=comm_unique_id(), flags=flags) as s:
        assert s.comm_size() == 1
        for i in range(3):  # single-iteration graphs
            s.run(1)
            np.testing.assert_array_equal(s.assignment_words(), at(i), err_msg=f"iter {i}")
        s.run(8)  # the 8-iteration graph
        np.testing.assert_array_equal(s.assignment_words(), at(10), err_msg="iter 10")
        s.run(K - 11)
        np.testing.assert_array_equal(s.assignment_words(), at(K - 1), err_msg=f"iter {K - 1}")
        st = s.stats()
    assert st["n_resamples"] == sum(r[3] for r in rows[:K])
    assert st["n_gpus"] == 1


def _bench_stdout(args, env_extra=None):
    import json
    import subprocess
    import sys

    env = dict(os.environ, **(env_extra or {}))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=400, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, f"stdout must be one JSON line, got {len(lines)}: {r.stdout[:500]!r}"
    return json.loads(lines[0])


@pytest.mark.parametrize("mode", ["rccl_self", "host_n2", "host_n2_shard", "host_n2_watchdog"])
def test_bench_prints_one_json_line(mode):
    """The driver reads one JSON line from bench.py's stdout: RCCL's banner at communicator
    init and the rank processes' output must not reach it (N=1 over a one-rank RCCL
    communicator; N=2 self-launched ranks over the host exchange on this one GPU).  With N=2 the
    planner replicates C2 and the sharded path runs as the checked secondary
    line; --plan shard makes the sharded path the headline."""
    common = ["--config", "C2", "--steps", "4", "--warmup", "1", "--no-cpu-baseline", "--event-iters", "0"]
    if mode == "rccl_self":
        d = _bench_stdout(common + ["--rccl-self"])
        assert d["n_gpus"] == 1 and d["config"]["exchange"] == "allgather/rccl-self"
    else:
        extra = (["--plan", "shard"] if mode == "host_n2_shard" else
                 ["--shard-line-timeout", "0.01"] if mode == "host_n2_watchdog" else [])
        d = _bench_stdout(common + ["--gpus", "2", "--exchange-impl", "host"] + extra, {"ALLL_BENCH_SAME_DEVICE": "1"})
        assert d["n_gpus"] == 2 and d["ranks_seen"] == 2
        mp = d["multi_gpu_plan"]
        assert mp["plan"] == "replicate" and mp["requested"] == ("shard" if mode == "host_n2_shard" else "auto")
        if mode == "host_n2_shard":
            assert mp["chosen"] == "shard" and d["config"]["parallelism"] == "clause-shard x2"
            assert "shard_line" not in d
        elif mode == "host_n2_watchdog":
            # the sharded run cannot finish in 10 ms: the headline is written without it
            assert mp["chosen"] == "replicate" and "did not finish" in d["shard_line"]["error"]
        else:
            assert mp["chosen"] == "replicate" and d["config"]["parallelism"] == "replicated x2"
            sl = d["shard_line"]
            assert sl["n_comm"] == 2 and sl["steps"] == 20 and sl["value"] > 0
            assert sl["trajectory_check"]["match"] is True, sl["trajectory_check"]
        assert d["trajectory_check"]["match"] is True, d["trajectory_check"]
    assert d["steps_done"] == 4 and d["value"] > 0
