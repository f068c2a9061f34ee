"""Cross-rank order of the overlapped bucket exchanges (2 processes, gloo).

Buckets launch strictly in bucket-index order (DistributedOptimizer.
_launch_in_order): one rank whose gradient hooks fire in a DIFFERENT order
(here: all deferred to the end of backward and replayed in reverse) still
issues the same collective sequence as the others, so the result equals the
unperturbed run.  With the strict order bypassed, ``GKSGD_CHECK_ORDER=1``
turns the mismatched exchange into an error on every rank instead of a hang
or a wrong aggregate.

Reference: Horovod negotiates readiness by tensor name through its
coordinator (distributed_optimizer.py:426-427,461-463 rely on it)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

STEPS = 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, outdir, mode, check_order):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK=str(rank))
    if check_order:
        os.environ["GKSGD_CHECK_ORDER"] = "1"
    from gaussiank_sgd_amd.compression import compressors
    from gaussiank_sgd_amd.parallel import distributed_optimizer as hvd
    from gaussiank_sgd_amd.train import DLTrainer
    hvd.init(device="cpu")
    torch.manual_seed(0)
    t = DLTrainer(rank, 2, dnn="fcn5net", dataset="mnist", batch_size=32, lr=0.5, nworkers=2, device="cpu",
                  learnable_data=True, seed=rank)
    # threshold 0: one bucket per tensor (6 buckets, 6 all-gathers per step)
    opt = hvd.DistributedOptimizer(t.optimizer, named_parameters=t.net.named_parameters(),
                                   compression=compressors["gaussian"], is_sparse=True, density=0.01,
                                   threshold=0, density_warmup=False)
    assert len(opt.arena.buckets) == 6 and opt._overlap
    hvd.broadcast_parameters(t.net.state_dict(), root_rank=0)
    t.update_optimizer(opt)
    pending = []
    if mode != "plain" and rank == 1:
        for h in opt._grad_accs:
            h.remove()
        for p in opt._requires_update:
            fn = opt._make_hook(p)
            p.register_post_accumulate_grad_hook(lambda param, fn=fn: pending.append((fn, param)))
        if mode == "unordered":
            # the pre-fix behaviour: a bucket launches as soon as it completes
            def eager(self=opt):
                for b in self._arena.buckets:
                    if not b.launched and b.ready == len(b.params):
                        self._launch_bucket(b)
            opt._launch_in_order = eager
    err = ""
    try:
        for _ in range(STEPS):
            opt.zero_grad()
            t.train(1)
            for fn, param in reversed(pending):
                fn(param)
            pending.clear()
            t.update_model()
    except RuntimeError as e:
        err = str(e)
    torch.save({"w": opt.arena.weights.clone(), "err": err}, os.path.join(outdir, "%s-rank%d.pt" % (mode, rank)))
    hvd.comm.shutdown()


def _run(d, mode, check_order=False):
    mp.spawn(_worker, args=(_free_port(), d, mode, check_order), nprocs=2, join=True)
    return [torch.load(os.path.join(d, "%s-rank%d.pt" % (mode, r)), weights_only=True) for r in range(2)]


def test_perturbed_hook_order_gives_the_same_result(tmp_path):
    d = str(tmp_path)
    plain = _run(d, "plain")
    pert = _run(d, "reversed")
    for r in range(2):
        assert plain[r]["err"] == "" and pert[r]["err"] == ""
        assert torch.equal(plain[r]["w"], pert[r]["w"]), "rank %d: hook order changed the result" % r
    assert torch.equal(pert[0]["w"], pert[1]["w"])


def test_order_check_turns_a_mismatch_into_an_error(tmp_path):
    res = _run(str(tmp_path), "unordered", check_order=True)
    for r in range(2):
        assert "exchange order mismatch" in res[r]["err"], res[r]["err"]
