"""Whole-step HIP-graph capture (train/graph.py): replays train (weights move,
loss on a fixed batch falls) and the host lr schedule reaches the captured
fused update through the device multiplier."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(bs=16):
    from gaussiank_sgd_amd.compression import compressors
    from gaussiank_sgd_amd.parallel import comm, install_bf16_shadow
    from gaussiank_sgd_amd.parallel.distributed_optimizer import DistributedOptimizer
    from gaussiank_sgd_amd.train import DLTrainer
    comm.init()
    t = DLTrainer(0, 1, dnn="resnet20", dataset="cifar10", batch_size=bs, lr=0.05, device="cuda", amp="bf16",
                  channels_last=True, data_pool=1, seed=0)
    opt = DistributedOptimizer(t.optimizer, named_parameters=t.net.named_parameters(),
                               compression=compressors["gaussian"], is_sparse=True, density=0.01,
                               compress_single_rank=True, density_warmup=False)
    install_bf16_shadow(t.net, opt)
    t.update_optimizer(opt)
    t.display = 10 ** 9
    return t, opt


def test_graph_replay_trains():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from gaussiank_sgd_amd.train.graph import GraphedStep
    t, opt = _setup()
    step = GraphedStep(t, opt)
    step()                                  # warm-up + capture + first replay
    assert step.captures == 1
    losses = []
    w_prev = opt.arena.weights.clone()
    for _ in range(6):
        step()
        torch.cuda.synchronize()
        losses.append(t.current_loss())
        w = opt.arena.weights
        assert (w - w_prev).abs().max().item() > 0, "a replay did not update the weights"
        w_prev = w.clone()
    assert step.captures == 1, "unexpected re-capture"
    assert all(l == l for l in losses)
    assert losses[-1] < losses[0] + 0.5


def test_graph_lr_multiplier_scales_update():
    """Replays with lr x0 leave the weights unchanged (the captured update
    reads the device multiplier)."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from gaussiank_sgd_amd.train.graph import GraphedStep
    t, opt = _setup()
    step = GraphedStep(t, opt)
    step()
    torch.cuda.synchronize()
    step.mult.fill_(0.0)
    w0 = opt.arena.weights.clone()
    step.graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(opt.arena.weights, w0)
