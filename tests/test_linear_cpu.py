"""FastLinear (ops/linear.py) on the CPU: the stock nn.Linear (+ GELU) path,
the PyTorch fallbacks of the fused column passes, and BERT-tiny / the PTB
LSTM stepping through the compressed optimizer with FastLinear layers."""
import torch
import torch.nn.functional as F

from gaussiank_sgd_amd.ops.linear import FastLinear, bias_grad_acc_, gelu_backward_


def test_fastlinear_cpu_is_nn_linear():
    torch.manual_seed(0)
    m = FastLinear(64, 128)
    ref = torch.nn.Linear(64, 128)
    ref.load_state_dict(m.state_dict())
    assert list(m.state_dict()) == ["weight", "bias"]
    x = torch.randn(5, 7, 64)
    assert torch.equal(m(x), ref(x))
    assert torch.equal(m(x, act="gelu"), F.gelu(ref(x)))


def test_column_pass_fallbacks():
    torch.manual_seed(1)
    dy = torch.randn(33, 24)
    db = torch.ones(24)
    bias_grad_acc_(db, dy)
    assert torch.allclose(db, 1 + dy.sum(0), atol=1e-5)
    pre = torch.randn(33, 24) * 2
    x = pre.clone().requires_grad_(True)
    F.gelu(x).backward(dy)
    db2 = torch.zeros(24)
    dpre = gelu_backward_(dy, pre, db2)
    assert torch.allclose(dpre, x.grad, atol=1e-6)
    assert torch.allclose(db2, x.grad.sum(0), atol=1e-5)


def _step(dnn, dataset, bs):
    from gaussiank_sgd_amd.compression import compressors
    from gaussiank_sgd_amd.parallel import comm
    from gaussiank_sgd_amd.parallel.distributed_optimizer import DistributedOptimizer
    from gaussiank_sgd_amd.train import DLTrainer
    torch.manual_seed(0)
    comm.init()
    t = DLTrainer(0, 1, dnn=dnn, dataset=dataset, batch_size=bs, lr=0.05, device="cpu", learnable_data=True,
                  data_pool=1)
    opt = DistributedOptimizer(t.optimizer, named_parameters=t.net.named_parameters(),
                               compression=compressors["gaussian"], is_sparse=True, density=0.01,
                               compress_single_rank=True, density_warmup=False)
    t.update_optimizer(opt)
    w0 = opt.arena.weights.clone()
    hidden = None
    for _ in range(2):
        opt.zero_grad()
        if dnn == "lstm":
            _, hidden = t.train(1, hidden=hidden)
        else:
            t.train(1)
        t.update_model()
    assert t.current_loss() == t.current_loss()
    assert float((opt.arena.weights - w0).abs().sum()) > 0
    return t


def test_bert_tiny_cpu_step():
    t = _step("bert_tiny", "wikipedia", 2)
    assert any(isinstance(m, FastLinear) for m in t.net.modules())


def test_split_heads_matches_permute_unbind():
    """models/bert.py _SplitHeads == view/permute/unbind, forward and backward."""
    from gaussiank_sgd_amd.models.bert import _SplitHeads
    torch.manual_seed(2)
    B, T, h, d = 2, 5, 3, 4
    y = torch.randn(B, T, 3 * h * d, requires_grad=True)
    y2 = y.detach().clone().requires_grad_(True)
    outs = _SplitHeads.apply(y, h)
    ref = y2.view(B, T, 3, h, d).permute(2, 0, 3, 1, 4).unbind(0)
    gs = [torch.randn(B, h, T, d) for _ in range(3)]
    for o, r in zip(outs, ref):
        assert torch.equal(o, r)
    sum((o * g).sum() for o, g in zip(outs, gs)).backward()
    sum((r * g).sum() for r, g in zip(ref, gs)).backward()
    assert torch.equal(y.grad, y2.grad)


def test_pad2_cache_shares_one_padded_copy():
    """ops/linear.py _pad2: with a backward-scoped cache the grad-input and
    grad-weight GEMMs get the SAME zero-padded copy (one fill + copy instead of
    two); without it every call pads afresh; values match F.pad."""
    import torch
    import torch.nn.functional as F
    from gaussiank_sgd_amd.ops.linear import _pad2
    t = torch.randn(7, 10)
    cache = {}
    a = _pad2(t, 8, 64, cache)
    b = _pad2(t, 8, 64, cache)
    assert a is b and len(cache) == 1
    assert torch.equal(a, F.pad(t, (0, 54, 0, 1)))
    assert _pad2(t, 8, 128, cache) is not a and len(cache) == 2   # another target shape
    assert _pad2(t, 8, 64) is not _pad2(t, 8, 64)                  # no cache: fresh copies
    assert _pad2(a, 8, 64, cache) is a                             # already padded + contiguous
