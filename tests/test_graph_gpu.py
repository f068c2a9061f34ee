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


def test_graph_randomk_indices_change_per_replay():
    """random-k under whole-step capture: the compressor seed is read from a
    device word refreshed before every replay, so two replays send different
    index sets (a seed baked in at capture would repeat them)."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from gaussiank_sgd_amd.compression import compressors
    from gaussiank_sgd_amd.parallel import comm
    from gaussiank_sgd_amd.parallel.distributed_optimizer import DistributedOptimizer
    from gaussiank_sgd_amd.train import DLTrainer
    from gaussiank_sgd_amd.train.graph import GraphedStep
    from gaussiank_sgd_amd import ops
    comm.init()
    t = DLTrainer(0, 1, dnn="resnet20", dataset="cifar10", batch_size=16, lr=0.05, device="cuda",
                  channels_last=True, data_pool=1, seed=0)
    opt = DistributedOptimizer(t.optimizer, named_parameters=t.net.named_parameters(),
                               compression=compressors["randomkec"], is_sparse=True, density=0.01,
                               compress_single_rank=True, density_warmup=False)
    t.update_optimizer(opt)
    t.display = 10 ** 9
    step = GraphedStep(t, opt)
    step()
    sets = []
    for _ in range(3):
        step()
        torch.cuda.synchronize()
        b = opt.arena.buckets[0]
        rec = b.bufs.record.cpu()
        sent = int(rec[0])
        assert sent > 0
        sets.append(frozenset(rec[ops.REC_HDR:ops.REC_HDR + sent].tolist()))
    assert step.captures == 1
    assert sets[0] != sets[1] and sets[1] != sets[2]


def test_graph_attention_dropout_changes_per_replay():
    """The fused attention's dropout mask under capture: the kernels mix the
    per-device replay word into their seed, so one input replayed twice gives
    two different outputs; without dropout the replays agree bit for bit."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from gaussiank_sgd_amd import ops
    from gaussiank_sgd_amd.ops.attention import fused_available, self_attention
    qkv = (torch.randn(2, 128, 3 * 2 * 64, device="cuda") * 0.5).to(torch.bfloat16)
    if not fused_available(qkv, 2):
        pytest.skip("fused attention unavailable")
    outs = {}
    for p in (0.0, 0.1):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self_attention(qkv, 2, p)          # warm-up outside the capture
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(g):
            o = self_attention(qkv, 2, p)
        res = []
        for r in range(2):
            ops.set_graph_seed(qkv.device, 1000 + r)
            g.replay()
            torch.cuda.synchronize()
            res.append(o.clone())
        outs[p] = res
    assert torch.equal(outs[0.0][0], outs[0.0][1])
    assert not torch.equal(outs[0.1][0], outs[0.1][1])


def test_dist_trainer_hip_graph_cli(tmp_path):
    """``dist_trainer --hip-graph`` (one GPU process): the whole step replays
    as a HIP graph -- the execution bench.py times for its reference-batch
    phases -- through an epoch boundary of the density warm-up (recapture)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root)
    cmd = [sys.executable, "-m", "gaussiank_sgd_amd.train.dist_trainer", "--dnn", "resnet20", "--dataset", "cifar10",
           "--batch-size", "32", "--density", "0.001", "--compressor", "gaussian", "--max-epochs", "2",
           "--train-samples", "640", "--compress-single-rank", "--hip-graph", "--logdir-root", str(tmp_path / "logs"),
           "--saved-dir", str(tmp_path), "--data-dir", str(tmp_path / "nodata")]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Speed:" in r.stderr
    assert "running eagerly" not in r.stderr
    assert "Average number of selected gradients" in r.stderr


def test_graph_lstm_carries_hidden_state():
    """The PTB LSTM (BASELINE config 4) replays as a HIP graph: its hidden
    state lives in static buffers the captured step reads and rewrites, so
    consecutive replays continue the sequence; reset_hidden() zeroes it."""
    from gaussiank_sgd_amd.compression import compressors
    from gaussiank_sgd_amd.parallel import comm
    from gaussiank_sgd_amd.parallel.distributed_optimizer import DistributedOptimizer
    from gaussiank_sgd_amd.train import DLTrainer
    from gaussiank_sgd_amd.train.graph import GraphedStep
    comm.init()
    torch.manual_seed(0)
    t = DLTrainer(0, 1, dnn="lstm", dataset="ptb", batch_size=8, lr=1.0, device="cuda:0", data_pool=4)
    opt = DistributedOptimizer(t.optimizer, named_parameters=t.net.named_parameters(),
                               compression=compressors["gaussian"], is_sparse=True, density=0.01,
                               compress_single_rank=True, density_warmup=False, threshold=524288000)
    from gaussiank_sgd_amd.parallel import install_direct_grads
    install_direct_grads(t.net, opt)
    t.update_optimizer(opt)
    # eager steps first, the caller keeping the returned state (as bench.py's
    # warm-up does): no autograd graph of theirs may survive into the capture
    hidden = None
    for _ in range(2):
        opt.zero_grad()
        _, hidden = t.train(1, hidden=hidden)
        t.update_model()
    assert hidden[0].grad_fn is None
    g = GraphedStep(t, opt, clip=0.25)
    assert g.hidden is not None
    w0 = opt.arena.weights.clone()
    g()
    h1 = [v.clone() for v in g.hidden]
    g()
    torch.cuda.synchronize()
    assert g.captures == 1 and g.replays == 2
    assert not torch.equal(h1[0], g.hidden[0]), "the replay did not advance the hidden state"
    assert float(h1[0].abs().sum()) > 0
    assert not torch.equal(w0, opt.arena.weights)
    assert t.current_loss() == t.current_loss()
    g.reset_hidden()
    assert all(float(v.abs().sum()) == 0 for v in g.hidden)
    g()
    torch.cuda.synchronize()
    assert float(g.hidden[0].abs().sum()) > 0
