"""Multi-process data parallelism on CPU (gloo, world_size 2): BASELINE config 1
(3-layer MLP on MNIST-shaped synthetic data, Gaussian-k at k = 1%).

The result of the real 2-process run is compared with an in-process
loopback simulation of the same two ranks (fake comm backend: each virtual
rank compresses with the CPU mirror, records are aggregated by the reference
formula g = 1/P sum_r scatter(idx_r, val_r))."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

STEPS = 6


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _make(rank, comp, density):
    from gaussiank_sgd_amd.train import DLTrainer
    torch.manual_seed(0)
    t = DLTrainer(rank, 2, dnn="fcn5net", dataset="mnist", batch_size=32, lr=0.5, nworkers=2, device="cpu",
                  learnable_data=True, seed=rank)
    return t


def _worker(rank, port, comp, density, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK=str(rank))
    from gaussiank_sgd_amd.compression import compressors
    from gaussiank_sgd_amd.parallel import distributed_optimizer as hvd
    hvd.init(device="cpu")
    t = _make(rank, comp, density)
    opt = hvd.DistributedOptimizer(t.optimizer, named_parameters=t.net.named_parameters(),
                                   compression=compressors[comp], is_sparse=comp not in ("none", "bucket"),
                                   density=density, density_warmup=False)
    hvd.broadcast_parameters(t.net.state_dict(), root_rank=0)
    t.update_optimizer(opt)
    t.base_lr = 0.5
    for _ in range(STEPS):
        opt.zero_grad()
        t.train(1)
        t.update_model()
    torch.save({k: v.detach().clone() for k, v in t.net.state_dict().items()},
               os.path.join(outdir, "rank%d.pt" % rank))
    hvd.comm.shutdown()


def _loopback(comp, density):
    """Two virtual ranks in one process with the same math as the real run."""
    from gaussiank_sgd_amd import ops
    from gaussiank_sgd_amd.compression import compressors
    from gaussiank_sgd_amd.parallel.buckets import GradArena, group_with_threshold
    c = compressors[comp]
    trainers = [_make(r, comp, density) for r in range(2)]
    trainers[1].net.load_state_dict(trainers[0].net.state_dict())
    arenas = []
    for t in trainers:
        named = list(t.net.named_parameters())
        keys = [k for k, _ in named]
        groups = group_with_threshold(keys, {k: p.numel() for k, p in named}, 0)
        arenas.append(GradArena(named, groups))
    opts = [torch.optim.SGD(t.optimizer.param_groups, lr=0.5) for t in trainers]
    for t in trainers:
        t.base_lr = 0.5
    for it in range(STEPS):
        for t in trainers:
            for g in t.optimizer.param_groups:
                pass
            t.net.zero_grad(set_to_none=False)
            t.train(1)
        for bi in range(len(arenas[0].buckets)):
            recs = []
            for r, a in enumerate(arenas):
                b = a.buckets[bi]
                k = c.k_of(b.numel, density)
                k_cap = c.k_cap_for(k, b.numel)
                bufs = ops.CompressBuffers(k_cap, "cpu")
                ops.compress_(b.slice(a.grads), b.slice(a.residuals), bufs, c.mode, ec=c.ec, zero_g=True,
                              loops=c.loops, z=c.z_for(density), k=k, k_cap=k_cap, n_stats=b.numel)
                recs.append(bufs.record)
            allrec = torch.stack(recs)
            for a in arenas:
                ops.scatter_add_records_(a.buckets[bi].slice(a.grads), allrec, 2, recs[0].numel() // 2 - 2, 0.5)
        for t, o in zip(trainers, opts):
            for g in o.param_groups:
                g["lr"] = t.lr
            o.step()
    return [{k: v.detach().clone() for k, v in t.net.state_dict().items()} for t in trainers]


@pytest.mark.parametrize("comp,density", [("gaussian", 0.01), ("topk", 0.01), ("none", 1.0)])
def test_gloo_world2_matches_loopback(comp, density):
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(port, comp, density, d), nprocs=2, join=True)
        s0 = torch.load(os.path.join(d, "rank0.pt"), weights_only=True)
        s1 = torch.load(os.path.join(d, "rank1.pt"), weights_only=True)
    for k in s0:
        assert torch.equal(s0[k], s1[k]), "ranks diverged at %s" % k
    if comp == "none":
        return
    ref = _loopback(comp, density)
    for k in s0:
        assert torch.allclose(s0[k], ref[0][k], atol=1e-6, rtol=1e-5), k
