"""The framework communicator is created on every rank or on none (parallel/comm.py
``rccl_or_fallback``): 2 gloo ranks on the CPU with stand-in create/fallback callables, so the
agreement logic runs without a GPU (a failure on one rank only must not strand the
other inside RCCL's collective init)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Fake:
    kind = "rccl"

    def __init__(self, out, rank):
        self.out, self.rank = out, rank

    def destroy(self):
        with open(os.path.join(self.out, f"destroyed{self.rank}"), "w") as f:
            f.write("1")

    def abort(self):
        with open(os.path.join(self.out, f"aborted{self.rank}"), "w") as f:
            f.write("1")


def _worker(rank, ws, port, out, case):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if case == "preinit" and rank == 1:
        os.environ["DPT_TEST_FAIL_COMM_INIT_RANK"] = "1"
    import datetime
    import time
    pg_timeout = 8
    dist.init_process_group("gloo", rank=rank, world_size=ws, timeout=datetime.timedelta(seconds=pg_timeout))
    from distributed_pytorch_training_amd.parallel import comm as comm_mod
    from distributed_pytorch_training_amd.parallel.comm import init_timeout_for, rccl_or_fallback

    calls = []

    def new_uid():
        if case == "uid":
            raise RuntimeError("no unique id")
        return b"x" * 128

    def create(uid):
        calls.append("create")
        assert uid == b"x" * 128
        if case in ("init", "init-blocks") and rank == 1:
            raise RuntimeError("init failed here")
        if case == "init-blocks" and rank == 0:
            # what RcclComm does when its peer died inside the collective init: wait for the
            # init timeout derived from the process-group timeout, then give up
            time.sleep(init_timeout_for(pg_timeout))
            raise RuntimeError("ncclCommInitRank did not complete")
        return _Fake(out, rank)

    res = rccl_or_fallback(new_uid, create, lambda: "fallback", rank, ws, torch.device("cpu"))
    with open(os.path.join(out, f"r{rank}"), "w") as f:
        f.write(f"{'fake' if isinstance(res, _Fake) else res}|{','.join(calls)}|{comm_mod.LAST_FALLBACK_REASON or ''}")
    dist.destroy_process_group()


@pytest.mark.parametrize("case,want,created", [
    ("ok", "fake", True),            # both ranks build it
    ("uid", "fallback", False),      # rank 0 has no unique id: nobody enters RCCL
    ("preinit", "fallback", False),  # rank 1 not ready: nobody enters RCCL
    ("init", "fallback", True),      # rank 1's init throws: rank 0 aborts its communicator
    ("init-blocks", "fallback", True),  # rank 1 throws, rank 0 blocks until its init timeout
])
def test_every_rank_takes_the_same_branch(tmp_path, case, want, created):
    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path), case), nprocs=2, start_method="spawn")
    for r in range(2):
        got, calls, reason = (tmp_path / f"r{r}").read_text().split("|")
        assert got == want, (case, r, got)
        assert (calls == "create") == created, (case, r, calls)
        assert bool(reason) == (want == "fallback"), (case, r, reason)
    if case == "init":
        # a half-agreed communicator is aborted (ncclCommAbort), never destroyed (could block)
        assert (tmp_path / "aborted0").exists() and not (tmp_path / "destroyed0").exists()


def test_init_timeout_follows_the_process_group_timeout():
    from distributed_pytorch_training_amd.parallel.comm import MAX_INIT_TIMEOUT_S, init_timeout_for
    assert init_timeout_for(20) == 10.0
    assert init_timeout_for(1800) == MAX_INIT_TIMEOUT_S
    assert init_timeout_for(None) == MAX_INIT_TIMEOUT_S
