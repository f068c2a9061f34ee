"""Hang-proof bootstrap of the native RCCL communicator (parallel/comm.py
``_bootstrap_native``), exercised on CPU with a fake engine class.

The fake stands in for the C++ ``gk::RcclComm`` and injects a failure on ONE
rank at one bootstrap step: the unique id on rank 0, init that raises, init
that never completes (deadline -> abort), a self-test that raises or returns
wrong data.  Every rank must end on the non-native path, every communicator
that was built must be aborted, and nothing may hang.  Without a fault, every
rank gets ONE communicator shared by all its Exchangers (one init per
process, reference dist_trainer.py:125-126 calls hvd.init() once).

Two worlds: the in-process loopback world (4 virtual ranks, fast) and real
gloo processes (4 ranks, ``Exchanger.kind == "torch"`` after a fault)."""
import os
import socket
import tempfile
import threading

import pytest
import torch
import torch.multiprocessing as mp

from gaussiank_sgd_amd.parallel import comm

STEPS = ["uid", "init_raise", "init_hang", "init_error", "selftest_raise", "selftest_wrong"]


def make_fake(step: str, bad: int):
    """Engine class whose rank ``bad`` fails at ``step`` (``none``: no fault)."""
    lock = threading.Lock()

    class Fake:
        inits = 0
        aborts = 0
        destroys = 0

        @staticmethod
        def unique_id():
            if step == "uid":
                raise RuntimeError("injected: ncclGetUniqueId failed")
            return torch.arange(128, dtype=torch.uint8)

        def __init__(self):
            self.rank = None
            self.world = None
            self.live = False

        def init_async(self, uid, rank, world, device):
            assert uid.numel() == 128 and int(uid[5]) == 5
            self.rank, self.world = rank, world
            if step == "init_raise" and rank == bad:
                raise RuntimeError("injected: ncclCommInitRankConfig failed")
            self.live = True
            with lock:
                Fake.inits += 1

        def init_poll(self):
            if step == "init_hang" and self.rank == bad:
                return 1                      # never completes: the deadline must fire
            if step == "init_error" and self.rank == bad:
                self.abort()                  # the C++ engine aborts before it throws
                raise RuntimeError("injected: asynchronous init error")
            return 0

        def abort(self):
            if self.live:
                with lock:
                    Fake.aborts += 1
            self.live = False

        def allgather(self, inp, out):
            assert self.live
            if step == "selftest_raise" and self.rank == bad:
                raise RuntimeError("injected: ncclAllGather failed")
            if step == "selftest_wrong" and self.rank == bad:
                return                        # output stays -1
            n = inp.numel()
            for r in range(self.world):
                out[r * n:(r + 1) * n] = r

        def start_watchdog(self, timeout_s, poll_ms):
            pass

        def stop_watchdog(self):
            pass

        def destroy(self):
            with lock:
                Fake.destroys += 1
            self.live = False

    return Fake


def _loopback_run(Fake, P=4):
    def fn(r):
        ex1 = comm.Exchanger(torch.device("cpu"), engine_cls=Fake)
        ex2 = comm.Exchanger(torch.device("cpu"), engine_cls=Fake)
        return ex1.kind, ex2.kind, (ex1.native is ex2.native and ex1.native is not None)
    return comm.loopback_world(P, fn, timeout_s=60)


def test_bootstrap_success_builds_one_shared_communicator():
    Fake = make_fake("none", -1)
    res = _loopback_run(Fake)
    assert all(k1 == "rccl-native" and k2 == "rccl-native" and shared for k1, k2, shared in res), res
    assert Fake.inits == 4 and Fake.aborts == 0      # one init per rank for two Exchangers


@pytest.mark.parametrize("step", STEPS)
@pytest.mark.parametrize("bad", [0, 2])
def test_bootstrap_fault_on_one_rank_sends_every_rank_to_fallback(step, bad, monkeypatch):
    monkeypatch.setenv("GKSGD_RCCL_INIT_TIMEOUT_S", "0.3")
    Fake = make_fake(step, bad)
    res = _loopback_run(Fake)
    assert all(k1 == "loopback" and k2 == "loopback" and not shared for k1, k2, shared in res), res
    # every communicator that was built was released again (abort, never a blocking destroy)
    assert Fake.aborts == Fake.inits, (Fake.inits, Fake.aborts)
    if step == "uid":
        assert Fake.inits == 0


def test_exchanger_close_keeps_the_shared_communicator():
    Fake = make_fake("none", -1)

    def fn(r):
        ex1 = comm.Exchanger(torch.device("cpu"), engine_cls=Fake)
        nat = ex1.native
        ex1.close()
        ex2 = comm.Exchanger(torch.device("cpu"), engine_cls=Fake)
        return ex1.kind, ex2.kind, ex2.native is nat
    res = comm.loopback_world(2, fn)
    assert res == [("loopback", "rccl-native", True)] * 2
    assert Fake.inits == 2 and Fake.destroys == 0


# ---------------------------------------------------------------------------
# real processes (gloo): the agreement runs over the process group
# ---------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, P, port, step, bad, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(P),
                      LOCAL_RANK=str(rank), GKSGD_RCCL_INIT_TIMEOUT_S="0.5")
    from gaussiank_sgd_amd.parallel import comm as c
    c.init(device="cpu")
    Fake = make_fake(step, bad)
    ex1 = c.Exchanger(torch.device("cpu"), engine_cls=Fake)
    ex2 = c.Exchanger(torch.device("cpu"), engine_cls=Fake)
    with open(os.path.join(outdir, "r%d" % rank), "w") as f:
        f.write("%s %s %d %d %d" % (ex1.kind, ex2.kind, Fake.inits, Fake.aborts, int(ex1.native is ex2.native)))
    c.shutdown()


@pytest.mark.parametrize("step,bad", [("none", -1), ("init_hang", 3), ("selftest_wrong", 1), ("uid", 0)])
def test_gloo_world4_bootstrap(step, bad):
    P = 4
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(P, _free_port(), step, bad, d), nprocs=P, join=True)
        got = [open(os.path.join(d, "r%d" % r)).read().split() for r in range(P)]
    for r, (k1, k2, inits, aborts, shared) in enumerate(got):
        if step == "none":
            assert (k1, k2, inits, aborts, shared) == ("rccl-native", "rccl-native", "1", "0", "1"), (r, got)
        else:
            assert (k1, k2) == ("torch", "torch"), (r, got)
            assert inits == aborts, (r, got)      # a built communicator was aborted, not leaked
