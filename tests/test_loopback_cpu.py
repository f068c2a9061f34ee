"""In-process loopback world (parallel/comm.py ``loopback_world``): P virtual
ranks as threads of one process with real collective semantics, so the whole
DistributedOptimizer path (hooks -> buckets -> compress -> exchange ->
decompress -> step) runs for any P without processes (SURVEY section 4.2 item 3;
the reference has no such harness, its Horovod data plane is external)."""
import pytest
import torch

from gaussiank_sgd_amd.parallel import comm


def test_loopback_collectives_world3():
    def body(r):
        assert comm.size() == 3 and comm.rank() == r and comm.backend() == "loopback"
        t = torch.full((4,), float(r + 1))
        comm.allreduce_(t, average=True)
        s = torch.full((2,), float(r + 1))
        comm.allreduce_(s, average=False)
        g = comm.allgather(torch.arange(r + 1, dtype=torch.int32) + 10 * r)   # unequal first dims
        out = torch.empty(3 * 2)
        comm.allgather_into_(out, torch.tensor([r, -r], dtype=torch.float32))
        b = torch.full((3,), float(r))
        comm.broadcast_(b, root_rank=2)
        obj = comm.broadcast_object({"rank": r}, root=1)
        comm.barrier()
        return t, s, g, out, b, obj

    res = comm.loopback_world(3, body)
    for t, s, g, out, b, obj in res:
        assert torch.equal(t, torch.full((4,), 2.0))
        assert torch.equal(s, torch.full((2,), 6.0))
        assert g.tolist() == [0, 10, 11, 20, 21, 22]
        assert out.tolist() == [0.0, 0.0, 1.0, -1.0, 2.0, -2.0]
        assert torch.equal(b, torch.full((3,), 2.0))
        assert obj == {"rank": 1}
    assert comm.size() == 1 and comm.backend() is None    # the caller's world is untouched


def test_loopback_error_propagates():
    def body(r):
        if r == 1:
            raise ValueError("rank 1 failed")
        comm.barrier()          # rank 0 would wait forever without the barrier abort

    with pytest.raises(ValueError, match="rank 1 failed"):
        comm.loopback_world(2, body, timeout_s=30)


def _train(P, comp, density, steps, **opt_kw):
    from gaussiank_sgd_amd.compression import compressors
    from gaussiank_sgd_amd.parallel import distributed_optimizer as hvd
    from gaussiank_sgd_amd.train import DLTrainer
    compressors[comp].clear()   # class-level residual state (reference API) starts empty
    trainers = []
    for r in range(P):          # built serially: model init draws from the global RNG
        torch.manual_seed(0)
        trainers.append(DLTrainer(r, P, dnn="fcn5net", dataset="mnist", batch_size=32, lr=0.5, nworkers=P,
                                  device="cpu", learnable_data=True, seed=r))

    def body(r):
        t = trainers[r]
        opt = hvd.DistributedOptimizer(t.optimizer, named_parameters=t.net.named_parameters(),
                                       compression=compressors[comp], is_sparse=comp not in ("none", "bucket"),
                                       density=density, density_warmup=False, **opt_kw)
        hvd.broadcast_parameters(t.net.state_dict(), root_rank=0)
        t.update_optimizer(opt)
        t.base_lr = 0.5
        sent = []
        for _ in range(steps):
            opt.zero_grad()
            t.train(1)
            t.update_model()
            b = opt.arena.buckets[0]
            if b.bufs is not None:
                rec = b.bufs.record
                sent.append(rec[4:4 + int(rec[0])].clone())
        st = {k: v.detach().clone() for k, v in t.net.state_dict().items()}
        st["__sent__"] = sent
        return st

    return comm.loopback_world(P, body)


@pytest.mark.parametrize("comp,density", [("gaussian", 0.01), ("topk", 0.01)])
def test_loopback_optimizer_matches_reference_aggregation(comp, density):
    """Two loopback ranks through the real DistributedOptimizer == the
    hand-rolled two-rank simulation of tests/test_dist_gloo.py (reference
    aggregation g = 1/P sum_r scatter(idx_r, val_r))."""
    from test_dist_gloo import STEPS, _loopback
    states = _train(2, comp, density, STEPS)
    for s in states:
        s.pop("__sent__")
    for k in states[0]:
        assert torch.equal(states[0][k], states[1][k]), "ranks diverged at %s" % k
    ref = _loopback(comp, density)
    for k in states[0]:
        assert torch.allclose(states[0][k], ref[0][k], atol=1e-6, rtol=1e-5), k


@pytest.mark.parametrize("P", [4, 8])
def test_loopback_world_ranks_agree(P):
    states = _train(P, "gaussian", 0.01, 3)
    for s in states[1:]:
        for k in s:
            if k != "__sent__":
                assert torch.equal(s[k], states[0][k]), k


@pytest.mark.parametrize("comp", ["randomksame", "randomksameec"])
def test_loopback_randomksame_ranks_pick_same_indices(comp):
    """*same variants: every rank sends the SAME index set each step (seed is a
    function of the iteration and bucket, not of a shared class counter)."""
    states = _train(4, comp, 0.01, 3)
    for s in states[1:]:
        for a, b in zip(s["__sent__"], states[0]["__sent__"]):
            assert torch.equal(a, b)
        for k in s:
            if k != "__sent__":
                assert torch.equal(s[k], states[0][k]), k
    # and different indices in different steps
    assert not torch.equal(states[0]["__sent__"][0], states[0]["__sent__"][1])


@pytest.mark.parametrize("comp", ["randomk", "dgcsampling", "topk_legacy", "bucketized_topk", "gaussian_cal"])
def test_loopback_reproducible_and_ranks_agree(comp):
    """Rank-dependent selectors: replicas agree, and two runs give the same result
    (no seed or residual state leaks between the virtual ranks)."""
    a = _train(3, comp, 0.01, 3)
    b = _train(3, comp, 0.01, 3)
    for s in a[1:]:
        for k in s:
            if k != "__sent__":
                assert torch.equal(s[k], a[0][k]), (comp, k)
    for k in a[0]:
        if k != "__sent__":
            assert torch.equal(a[0][k], b[0][k]), (comp, k)
    if comp == "randomk":       # independent draws per rank
        assert not torch.equal(a[0]["__sent__"][0], a[1]["__sent__"][0])


def test_loopback_momentum_correction_sparse_apply_matches_dense():
    """DGC momentum correction: the sparse SGD apply straight from the gathered
    records == scatter into the gradient arena + dense fused SGD."""
    sp = _train(4, "gaussian", 0.01, 4, momentum_correction=True, sparse_apply=True)
    dn = _train(4, "gaussian", 0.01, 4, momentum_correction=True, sparse_apply=False)
    for s in sp[1:]:
        for k in s:
            if k != "__sent__":
                assert torch.equal(s[k], sp[0][k]), k
    for k in sp[0]:
        if k != "__sent__":
            assert torch.allclose(sp[0][k], dn[0][k], atol=1e-6, rtol=1e-5), k




@pytest.mark.parametrize("kind", ["sgd", "lars", "plain"])
def test_broadcast_state_replicates_momentum_and_schedule_position(kind):
    """DistributedOptimizer.broadcast_state (multi-rank resume): rank 0 holds
    momentum (or LARS acceleration) and a later schedule position; after the
    broadcast every rank holds rank 0's buffers and train_epoch / train_iter,
    and one more identical step keeps the replicas identical."""
    from gaussiank_sgd_amd.compression import compressors
    from gaussiank_sgd_amd.optim.lars import LARS
    from gaussiank_sgd_amd.parallel.distributed_optimizer import DistributedOptimizer

    def body(r):
        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))
        if kind == "lars":
            base = LARS(net.parameters(), lr=0.1, momentum=0.9)
        else:
            base = torch.optim.SGD(net.parameters(), lr=0.1, momentum=0.9)
        opt = DistributedOptimizer(base, named_parameters=net.named_parameters(), compression=compressors["none"],
                                   is_sparse=False, density=1.0, threshold=10 ** 9, density_warmup=False,
                                   fused_optimizer=kind != "plain")
        if r == 0:
            # rank 0 "resumed": two local steps of state and a later position
            g = torch.Generator().manual_seed(7)
            for _ in range(2):
                opt.zero_grad()
                net(torch.randn(8, 16, generator=g)).pow(2).mean().backward()
                opt.local = True     # no exchange: rank 0 alone
                opt.step()
                opt.local = False
            opt.train_epoch, opt.train_iter = 3, 57
        opt.broadcast_state(0)
        comm.broadcast_parameters(net.state_dict(), root_rank=0)
        key = "acceleration" if kind == "lars" else "momentum_buffer"
        bufs = [opt.state[p][key].detach().clone() for p in net.parameters()]
        x = torch.randn(8, 16, generator=torch.Generator().manual_seed(11))
        opt.zero_grad()
        net(x).pow(2).mean().backward()
        opt.step()
        return (opt.train_epoch, opt.train_iter), bufs, [p.detach().clone() for p in net.parameters()]

    res = comm.loopback_world(2, body)
    (pos0, b0, w0), (pos1, b1, w1) = res
    assert pos0[0] == pos1[0] == 3
    assert pos0[1] == pos1[1]
    for a, b in zip(b0, b1):
        assert torch.equal(a, b)
    assert any(float(a.abs().sum()) > 0 for a in b0)
    for a, b in zip(w0, w1):
        assert torch.equal(a, b)
