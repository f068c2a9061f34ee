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


def _train(P, comp, density, steps):
    from gaussiank_sgd_amd.compression import compressors
    from gaussiank_sgd_amd.parallel import distributed_optimizer as hvd
    from gaussiank_sgd_amd.train import DLTrainer
    trainers = []
    for r in range(P):          # built serially: model init draws from the global RNG
        torch.manual_seed(0)
        trainers.append(DLTrainer(r, P, dnn="fcn5net", dataset="mnist", batch_size=32, lr=0.5, nworkers=P,
                                  device="cpu", learnable_data=True, seed=r))

    def body(r):
        t = trainers[r]
        opt = hvd.DistributedOptimizer(t.optimizer, named_parameters=t.net.named_parameters(),
                                       compression=compressors[comp], is_sparse=comp not in ("none", "bucket"),
                                       density=density, density_warmup=False)
        hvd.broadcast_parameters(t.net.state_dict(), root_rank=0)
        t.update_optimizer(opt)
        t.base_lr = 0.5
        for _ in range(steps):
            opt.zero_grad()
            t.train(1)
            t.update_model()
        return {k: v.detach().clone() for k, v in t.net.state_dict().items()}

    return comm.loopback_world(P, body)


@pytest.mark.parametrize("comp,density", [("gaussian", 0.01), ("topk", 0.01)])
def test_loopback_optimizer_matches_reference_aggregation(comp, density):
    """Two loopback ranks through the real DistributedOptimizer == the
    hand-rolled two-rank simulation of tests/test_dist_gloo.py (reference
    aggregation g = 1/P sum_r scatter(idx_r, val_r))."""
    from test_dist_gloo import STEPS, _loopback
    states = _train(2, comp, density, STEPS)
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
            assert torch.equal(s[k], states[0][k]), k


@pytest.mark.gpu
def test_loopback_world4_on_one_gpu():
    """Four virtual ranks sharing one MI355X: the HIP compress / scatter-add /
    fused-SGD path with a real P = 4 aggregation, ranks bit-identical, and
    equal (to fp32 rounding) to the same world on the CPU mirror ops."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from gaussiank_sgd_amd import ops
    assert ops.load(), ops._load_error
    from gaussiank_sgd_amd.compression import compressors
    from gaussiank_sgd_amd.parallel import distributed_optimizer as hvd
    from gaussiank_sgd_amd.train import DLTrainer

    def run(device):
        trainers = []
        for r in range(4):
            torch.manual_seed(0)
            trainers.append(DLTrainer(r, 4, dnn="fcn5net", dataset="mnist", batch_size=32, lr=0.5, nworkers=4,
                                      device=device, learnable_data=True, seed=r))

        def body(r):
            if device == "cuda":
                torch.cuda.set_device(0)
            t = trainers[r]
            opt = hvd.DistributedOptimizer(t.optimizer, named_parameters=t.net.named_parameters(),
                                           compression=compressors["gaussian"], is_sparse=True, density=0.01,
                                           density_warmup=False)
            hvd.broadcast_parameters(t.net.state_dict(), root_rank=0)
            t.update_optimizer(opt)
            t.base_lr = 0.5
            for _ in range(3):
                opt.zero_grad()
                t.train(1)
                t.update_model()
            if device == "cuda":
                torch.cuda.synchronize()
            return {k: v.detach().cpu().clone() for k, v in t.net.state_dict().items()}

        return comm.loopback_world(4, body)

    g = run("cuda")
    for s in g[1:]:
        for k in s:
            assert torch.equal(s[k], g[0][k]), k
    c = run("cpu")
    for k in g[0]:
        assert torch.allclose(g[0][k], c[0][k], atol=1e-5, rtol=1e-4), k
