"""N>1 path on the CPU: two gloo ranks run bench.py's sharding and timing
helpers (juicefs_amd/shard.py) with the CPU oracle as the per-rank step.

Checks the contract bench.py keeps for `--gpus N` (barrier + sync around
exactly K steps, MAX of the wall time over ranks, MIN of the verification
flag, disjoint block sets per rank, whole-job value) and the round-robin deal
of the batch ABI (capi.hip `batch_common`).  No GPU, no RCCL.
"""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from juicefs_amd import shard as S  # noqa: E402

ORACLE_SO = os.path.join(ROOT, "oracle", "_build", "liboracle.so")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, q, slow_rank, bad_rank):
    import time

    import torch
    import torch.distributed as dist

    from juicefs_amd.blockgen import gen_block
    from tests.oracle_ctypes import Oracle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        env = S.rank_env()
        assert (env.world, env.rank) == (world, rank)
        nblk, U = 3, 1 << 14
        seeds = list(range(S.seed_base(rank, nblk), S.seed_base(rank, nblk) + nblk))
        orc = Oracle(ORACLE_SO)
        raw = [gen_block("T", sd, U) for sd in seeds]
        comp = [orc.lz4_compress(b)[1] for b in raw]
        ok = [True]

        def step():
            for c, b in zip(comp, raw):
                n, out = orc.lz4_decompress(c, U)
                ok[0] &= (n == U and out == b)
            if rank == slow_rank:
                time.sleep(0.05)

        mine = S.timed_steps(step, 4, 1, lambda: None, world)
        el = S.max_over_ranks(mine, world, torch.device("cpu"))
        good = S.all_ranks_ok(ok[0] and rank != bad_rank, world, torch.device("cpu"))
        q.put((rank, seeds, mine, el, good, S.whole_job_gib_s(world, nblk, U, 4, el)))
    finally:
        dist.destroy_process_group()


def _run(world, slow_rank=-1, bad_rank=-1):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, world, port, q, slow_rank, bad_rank)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=120)
        res[r[0]] = r
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.skipif(not os.path.exists(ORACLE_SO), reason="oracle not built (run build())")
def test_two_ranks_max_time_and_disjoint_blocks():
    res = _run(2, slow_rank=1)
    (_, s0, m0, e0, g0, v0), (_, s1, m1, e1, g1, v1) = res[0], res[1]
    assert not set(s0) & set(s1), "ranks must decode disjoint block sets"
    assert e0 == e1 == max(m0, m1), "elapsed is the max over ranks on every rank"
    assert m1 >= 4 * 0.05, "rank 1 slept in each of exactly 4 timed steps"
    assert g0 and g1
    assert v0 == v1 == pytest.approx(2 * 3 * (1 << 14) * 4 / e0 / 2**30)


@pytest.mark.skipif(not os.path.exists(ORACLE_SO), reason="oracle not built (run build())")
def test_one_bad_rank_fails_every_rank():
    res = _run(2, bad_rank=0)
    assert not res[0][4] and not res[1][4]


def test_round_robin_deal():
    d = S.deal_round_robin(10, 4)
    assert d == [[0, 4, 8], [1, 5, 9], [2, 6], [3, 7]]
    assert sorted(sum(d, [])) == list(range(10))
    assert S.deal_round_robin(2, 8)[:2] == [[0], [1]]
    assert S.shard_sizes([5, 6, 7], 2) == [12, 6]
    with pytest.raises(ValueError):
        S.deal_round_robin(3, 0)


def test_single_process_defaults(monkeypatch):
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    e = S.rank_env()
    assert (e.world, e.rank, e.local) == (1, 0, 0)
    calls = []
    t = S.timed_steps(lambda: calls.append(1), 5, 2, lambda: None, 1)
    assert len(calls) == 7 and t >= 0
