"""Two ranks on the GPU (both on cuda:0, gloo transport): the multi-rank path
of the DistributedOptimizer -- per-rank fused HIP compression, packed record
all-gather, HIP scatter-add averaging, fused update -- against the CPU
loopback simulation of tests/test_dist_gloo.py.

RCCL refuses two ranks on one device ("Duplicate GPU detected"), so the
exchange here goes through torch.distributed/gloo (native_rccl=False); the
native engine itself is exercised at world size 1 in test_kernels_gpu.py and
by the driver's multi-GPU bench.
"""
import os
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

from gaussiank_sgd_amd.parallel import comm

from test_dist_gloo import STEPS, _free_port, _loopback

pytestmark = pytest.mark.gpu


def _worker(rank, port, comp, density, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    from gaussiank_sgd_amd.compression import compressors
    from gaussiank_sgd_amd.parallel import distributed_optimizer as hvd
    from gaussiank_sgd_amd.train import DLTrainer
    torch.cuda.set_device(0)
    hvd.comm.init(backend="gloo")
    torch.manual_seed(0)
    t = DLTrainer(rank, 2, dnn="fcn5net", dataset="mnist", batch_size=32, lr=0.5, nworkers=2, device="cpu",
                  learnable_data=True, seed=rank)
    # identical CPU-generated data/init as the loopback, then move to the GPU
    t.net.cuda()
    t.device = torch.device("cuda", 0)
    t.is_cuda = True
    opt = hvd.DistributedOptimizer(t.optimizer, named_parameters=t.net.named_parameters(),
                                   compression=compressors[comp], is_sparse=True, density=density,
                                   density_warmup=False, native_rccl=False)
    hvd.broadcast_parameters(t.net.state_dict(), root_rank=0)
    t.update_optimizer(opt)
    t.base_lr = 0.5
    for _ in range(STEPS):
        opt.zero_grad()
        t.train(1)
        t.update_model()
    torch.cuda.synchronize()
    torch.save({k: v.detach().cpu().clone() for k, v in t.net.state_dict().items()},
               os.path.join(outdir, "rank%d.pt" % rank))
    hvd.comm.shutdown()


@pytest.mark.parametrize("comp,density", [("gaussian", 0.01), ("topk", 0.01)])
def test_two_ranks_on_gpu_match_loopback(cuda, comp, density):
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(port, comp, density, d), nprocs=2, join=True)
        s0 = torch.load(os.path.join(d, "rank0.pt"), weights_only=True)
        s1 = torch.load(os.path.join(d, "rank1.pt"), weights_only=True)
    for k in s0:
        assert torch.equal(s0[k], s1[k]), "ranks diverged at %s" % k
    ref = _loopback(comp, density)
    for k in s0:
        assert torch.allclose(s0[k], ref[0][k], atol=2e-4, rtol=1e-3), (k, float((s0[k] - ref[0][k]).abs().max()))


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
