"""Multi-rank checkpoint / resume (2 processes, gloo, CPU).

A run of 4 steps that saves (every rank its own file), resumed in FRESH
processes for 4 more steps, must end bit-identical to an uninterrupted 8-step
run -- weights, momentum, every rank's residuals and DGC velocities -- and
the two replicas must agree.  The run uses momentum SGD (or DGC momentum
correction) and the density warm-up, whose epoch boundary (0.004 -> 0.001,
a different record size) falls exactly at the resume point.

Reference resume (dist_trainer.py:26-33,57; dl_trainer.py:232-233,285-290,
649-661): rank 0 loads {iter, epoch, state}, which is broadcast -- lossy
(momentum and residuals are not saved) but consistent.  Here the per-rank
state is restored from each rank's own file and the replicated state
(momentum, schedule position) is broadcast from rank 0.

Also: a rank whose density-schedule position disagrees with the others
raises before the first exchange instead of entering a mismatched
all-gather."""
import glob
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

BS = 16
SAMPLES = 64          # 2 ranks x bs 16 -> 2 iterations per epoch


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, outdir, max_epochs, pretrain, mc, save_final, tag, bad_epoch):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK=str(rank))
    from gaussiank_sgd_amd.parallel import distributed_optimizer as hvd
    from gaussiank_sgd_amd.train.dist_trainer import ssgd
    hvd.init(device="cpu")
    try:
        if bad_epoch and rank == 1:
            # rank 1 alone believes it is two schedule epochs further on
            from gaussiank_sgd_amd.parallel import distributed_optimizer as dopt
            orig = dopt._DistributedOptimizer.broadcast_state

            def skewed(self, root_rank=0):
                orig(self, root_rank)
                self.train_epoch += 2
            dopt._DistributedOptimizer.broadcast_state = skewed
        err = None
        try:
            trainer, opt = ssgd("fcn5net", "mnist", os.path.join(outdir, "nodata"), 2, 0.1, BS, 1, max_epochs, 1,
                                pretrain, 35, "gaussian", 0.001, 524288000, saved_dir=outdir,
                                momentum_correction=mc, train_samples=SAMPLES, checkpoint_every=2,
                                save_final=save_final, metrics_dir=outdir)
        except RuntimeError as e:
            err = str(e)
        if bad_epoch:
            torch.save({"err": err or ""}, os.path.join(outdir, "%s-err-rank%d.pt" % (tag, rank)))
            return
        a = opt.arena
        res = {"w": a.weights.clone(), "iter": torch.tensor([opt.train_iter, opt.train_epoch,
                                                              trainer.train_iter, trainer.train_epoch])}
        if a.momentum is not None:
            res["m"] = a.momentum.clone()
        if a.residuals is not None:
            res["r"] = a.residuals.clone()
        if getattr(a, "velocity", None) is not None:
            res["u"] = a.velocity.clone()
        torch.save(res, os.path.join(outdir, "%s-rank%d.pt" % (tag, rank)))
    finally:
        hvd.comm.shutdown()


def _run(outdir, max_epochs, pretrain, mc, save_final, tag, bad_epoch=False):
    mp.spawn(_worker, args=(_free_port(), outdir, max_epochs, pretrain, mc, save_final, tag, bad_epoch), nprocs=2,
             join=True)


def _load(outdir, tag, r):
    return torch.load(os.path.join(outdir, "%s-rank%d.pt" % (tag, r)), weights_only=True)


@pytest.mark.parametrize("mc", [False, True], ids=["momentum", "momentum_correction"])
def test_resume_two_ranks_equals_uninterrupted(tmp_path, mc):
    full = str(tmp_path / "full")
    part = str(tmp_path / "part")
    os.makedirs(full)
    os.makedirs(part)
    _run(full, 4, None, mc, False, "full")            # 8 steps, epochs 0-3
    _run(part, 2, None, mc, True, "first")            # 4 steps, then every rank saves
    cks = sorted(glob.glob(os.path.join(part, "weights", "**", "*-rank*-epoch*.pth"), recursive=True))
    r0 = [c for c in cks if "-rank0-" in os.path.basename(c)]
    assert r0 and any("-rank1-" in os.path.basename(c) for c in cks), cks
    _run(part, 4, r0[-1], mc, False, "resumed")       # fresh processes: 4 more steps
    for r in range(2):
        a, b = _load(full, "full", r), _load(part, "resumed", r)
        assert a["iter"].tolist() == b["iter"].tolist() == [8, 4, 8, 3], (a["iter"], b["iter"])
        assert set(a) == set(b)
        for key in a:
            assert torch.equal(a[key], b[key]), "rank %d: %s differs after resume" % (r, key)
        if mc:
            assert "u" in a and float(a["u"].abs().sum()) > 0
        else:
            assert "m" in a and float(a["m"].abs().sum()) > 0
    w0, w1 = _load(part, "resumed", 0)["w"], _load(part, "resumed", 1)["w"]
    assert torch.equal(w0, w1), "replicas diverged after resume"
    # the residuals are per rank (not broadcast): they differ between ranks
    assert not torch.equal(_load(part, "resumed", 0)["r"], _load(part, "resumed", 1)["r"])


def test_schedule_mismatch_raises_instead_of_exchanging(tmp_path):
    d = str(tmp_path)
    _run(d, 1, None, False, False, "bad", bad_epoch=True)
    for r in range(2):
        err = torch.load(os.path.join(d, "bad-err-rank%d.pt" % r), weights_only=True)["err"]
        assert "disagree on the exchange plan" in err, err
