"""bench.py's multi-GPU plumbing on the CPU (no GPU, no RCCL): what the driver's
8-GPU run goes through before any kernel runs.

* `--gpus 8` without a torchrun environment re-launches itself under
  torch.distributed.run with 8 processes on 127.0.0.1 (_spawn_ranks), and a
  WORLD_SIZE that disagrees with --gpus stops the run.
* ranked_host_path (configs[0] on every rank, device_mask = 1 << local_rank)
  with WORLD_SIZE 8 over gloo, the batch ABI replaced by the CPU oracle: every
  rank passes its own mask, the timing is the max over ranks, the value is the
  whole job's bytes; a rank whose blocks report another device fails every
  rank loudly.
* the dealer leg's spread check refuses a deal that used fewer GPUs than the job.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

ORACLE_SO = os.path.join(ROOT, "oracle", "_build", "liboracle.so")


def test_spawn_ranks_command(monkeypatch):
    seen = {}

    class R:
        returncode = 7

    def fake_run(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return R()
    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "3", "--warmup", "1"])
    assert bench._spawn_ranks(8) == 7
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1].isdigit()
    assert os.path.samefile(cmd[cmd.index("--master-port") + 2], os.path.join(ROOT, "bench.py"))
    assert cmd[-6:] == ["--gpus", "8", "--steps", "3", "--warmup", "1"]


def test_main_spawns_when_not_under_torchrun(monkeypatch):
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8"])
    monkeypatch.setattr(bench, "_spawn_ranks", lambda n: 40 + n)
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 48


def test_main_rejects_world_size_mismatch(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("LOCAL_RANK", "0")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert "WORLD_SIZE=4" in str(e.value.code)


def test_check_spread():
    assert bench.check_spread({0: 5, 1: 5, 2: 4}, 3, 14) == [0, 1, 2]
    assert bench.check_spread({0: 2, 1: 0}, 2, 1) == [0]  # one block: one device
    with pytest.raises(RuntimeError):
        bench.check_spread({0: 14}, 8, 14)
    with pytest.raises(RuntimeError):
        bench.check_spread({0: 7, 3: 7}, 8, 14)


class CpuHostOps:
    """bench.GpuHostOps' methods on the CPU oracle; the 'device' a batch ran on
    is the one its mask names (or `lie`, to test the loud failure)."""

    def __init__(self, lie=None):
        from tests.oracle_ctypes import Oracle
        self.o = Oracle(ORACLE_SO)
        self.lie = lie
        self.blocks = {}
        self.masks = set()

    def gen(self, nblk, U, seed):
        from juicefs_amd.blockgen import gen_block
        return np.frombuffer(b"".join(gen_block("T", seed + i, U) for i in range(nblk)), dtype=np.uint8)

    def bound(self, U):
        return self.o.lz4_bound(U)

    def _count(self, n, mask):
        self.masks.add(mask)
        d = self.lie if self.lie is not None else mask.bit_length() - 1
        self.blocks[d] = self.blocks.get(d, 0) + n

    def compress(self, pairs, mask):
        self._count(len(pairs), mask)
        res = []
        for dst, src in pairs:
            n, c = self.o.lz4_compress(src.tobytes(), len(dst))
            dst[:n] = np.frombuffer(c, dtype=np.uint8)
            res.append((n, None if n > 0 else "fail"))
        return res

    def decompress(self, pairs, mask):
        self._count(len(pairs), mask)
        res = []
        for dst, src in pairs:
            n, d = self.o.lz4_decompress(src.tobytes(), len(dst))
            dst[:max(n, 0)] = np.frombuffer(d, dtype=np.uint8)
            res.append((n, None if n >= 0 else "fail"))
        return res

    def reset_stats(self):
        self.blocks = {}

    def device_blocks(self):
        return dict(self.blocks)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, q, liar):
    import torch
    import torch.distributed as dist

    from juicefs_amd import shard as S
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        env = S.rank_env()
        ops = CpuHostOps(lie=0 if rank == liar else None)
        try:
            r = bench.ranked_host_path(S, env.world, env.rank, env.local, torch.device("cpu"), 3, 1 << 14, ops=ops)
            q.put((rank, "ok", r["value"], r["decompress"]["s"], r["compress"]["s"], r["n_gpus"],
                   r["each_rank_used_only_its_gpu"], sorted(ops.masks), r["rank0_device_blocks"]))
        except RuntimeError as e:
            q.put((rank, "error", str(e)))
    finally:
        dist.destroy_process_group()


def _run(world, liar=-1):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, world, port, q, liar)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=180)
        res[r[0]] = r
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.skipif(not os.path.exists(ORACLE_SO), reason="oracle not built (run build())")
def test_ranked_host_path_world_size_8_gloo():
    res = _run(8)
    assert all(res[r][1] == "ok" for r in range(8)), res
    vals = {res[r][2] for r in range(8)}
    assert len(vals) == 1, "every rank reports the same whole-job value"
    td = res[0][3]
    assert all(res[r][3] == td for r in range(8)), "decode time is the max over ranks on every rank"
    assert vals.pop() == pytest.approx(8 * 3 * (1 << 14) / td / 2**30)
    for r in range(8):
        assert res[r][5] == 8 and res[r][6] is True
        assert res[r][7] == [1 << r], f"rank {r} must pass device_mask 1 << local_rank only"
        assert set(res[r][8]) == {r}  # blocks counted on its own device only


@pytest.mark.skipif(not os.path.exists(ORACLE_SO), reason="oracle not built (run build())")
def test_ranked_host_path_wrong_device_fails_every_rank():
    res = _run(8, liar=5)
    assert all(res[r][1] == "error" for r in range(8)), res
    assert "rank 5" in res[5][2]
