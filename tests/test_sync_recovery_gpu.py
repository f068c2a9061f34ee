"""Recovery from an expired grid-barrier spin of the fused compression decide
(compress.hip decide_fb_kernel): DistributedOptimizer.check_compress_sync()
(run at every epoch boundary) notices a new sticky sync_timeouts count,
returns the bucket's workspace to its at-rest state (every arrival counter /
flag zero) and switches the bucket to in-grid hand-offs, which do not use
that grid; training continues and stays correct."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_sync_timeout_resets_workspace_and_switches_handoff(cuda):
    from gaussiank_sgd_amd import ops
    from gaussiank_sgd_amd.compression import compressors
    from gaussiank_sgd_amd.parallel import comm
    from gaussiank_sgd_amd.parallel.distributed_optimizer import DistributedOptimizer
    comm.init()
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(512, 1024), torch.nn.ReLU(), torch.nn.Linear(1024, 10)).to(cuda)
    opt = DistributedOptimizer(torch.optim.SGD(net.parameters(), lr=0.05, momentum=0.9),
                               named_parameters=net.named_parameters(), compression=compressors["gaussian"],
                               is_sparse=True, density=0.01, compress_single_rank=True, density_warmup=False,
                               threshold=10 ** 9)
    x = torch.randn(64, 512, device=cuda)
    y = torch.randint(0, 10, (64,), device=cuda)

    def step():
        opt.zero_grad()
        torch.nn.functional.cross_entropy(net(x), y).backward()
        opt.step()

    step()
    torch.cuda.synchronize()
    b = opt.arena.buckets[0]
    assert opt.check_compress_sync() == 0 and "handoff" not in b.extra
    # simulate a grid that was not co-resident: a bumped sticky counter and
    # half-counted barrier words in the workspace
    ctrl_u32 = b.bufs.ctrl.view(torch.int32)
    ctrl_u32[ops.CTRL_SYNC_TIMEOUTS_U32] += 3
    b.bufs.ws.view(torch.int32)[-4096:] = 7
    assert opt.check_compress_sync() == 3
    assert b.extra["handoff"] == 1
    assert int(b.bufs.ws.abs().sum()) == 0
    assert opt.check_compress_sync() == 0     # already seen
    w0 = opt.arena.weights.clone()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    assert ops.sync_timeouts(b.bufs) == 3
    assert not torch.equal(w0, opt.arena.weights)
    assert int(b.bufs.record[0]) > 0
