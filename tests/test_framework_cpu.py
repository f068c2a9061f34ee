"""CPU tests of the framework plumbing: buckets/arena, planners, schedules,
density warm-up, checkpoint/resume (with residuals + momentum), the CLI entry
point, layer-wise profiler, evaluation and the log-parsing plot tool."""
import os
import subprocess
import sys

import pytest
import torch

from gaussiank_sgd_amd.compression import compressors
from gaussiank_sgd_amd.parallel import distributed_optimizer as hvd
from gaussiank_sgd_amd.parallel.buckets import GradArena, group_with_threshold
from gaussiank_sgd_amd.parallel.planner import models_for, plan_mgs, plan_mgwfbp
from gaussiank_sgd_amd.train import DLTrainer
from gaussiank_sgd_amd.train import schedules

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_group_with_threshold_reference_rule():
    keys = ["a", "b", "c", "d"]
    sizes = {"a": 10, "b": 20, "c": 30, "d": 40}
    assert group_with_threshold(keys, sizes, 0) == [["d"], ["c"], ["b"], ["a"]]
    assert group_with_threshold(keys, sizes, 65) == [["d", "c"], ["b", "a"]]
    assert group_with_threshold(keys, sizes, 524288000) == [["d", "c", "b", "a"]]


def test_arena_views_and_alignment():
    net = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.Linear(5, 3))
    named = list(net.named_parameters())
    keys = [k for k, _ in named]
    arena = GradArena(named, group_with_threshold(keys, {k: p.numel() for k, p in named}, 10 ** 9))
    for k, p in named:
        assert p.data.data_ptr() == arena.weight_views[k].data_ptr()
        assert p.grad.data_ptr() == arena.grad_views[k].data_ptr()
        assert (p.data.data_ptr() - arena.weights.data_ptr()) % 256 == 0
    x = torch.randn(4, 7)
    net(x).sum().backward()
    assert float(arena.grads.abs().sum()) > 0
    b = arena.buckets[0]
    assert b.numel == sum(p.numel() for _, p in named)
    assert b.span % 64 == 0


def test_planners_produce_partitions():
    names = ["l%d" % i for i in range(8)]
    sizes = [1000, 200000, 5000, 300000, 100, 4000000, 10, 25000]
    times = [1e-4, 3e-4, 1e-4, 5e-4, 1e-5, 2e-3, 1e-5, 2e-4]
    for P in (2, 8):
        ar, alpha, ct, ag = models_for(P, 0.001, "mi355x")
        g1, _ = plan_mgwfbp(names, times, sizes, ar, alpha)
        g2, _ = plan_mgs(names, times, sizes, ct, ag)
        for groups in (g1, g2):
            flat = [k for g in groups for k in g]
            assert sorted(flat) == sorted(names) and len(flat) == len(names)
            assert flat[0] == "l7"  # backward order
        ar, alpha, ct, ag = models_for(P, 0.001, "reference")
        g3, _ = plan_mgs(names, times, sizes, ct, ag)
        assert sorted(k for g in g3 for k in g) == sorted(names)


def test_lr_schedules():
    assert schedules.general_lr(0.1, 10, 0, 100, "cifar10", warmup=False) == 0.1
    assert abs(schedules.general_lr(0.1, 90, 0, 100, "cifar10", warmup=False) - 0.01) < 1e-12
    assert abs(schedules.general_lr(0.1, 35, 0, 100, "imagenet", warmup=False) - 0.01) < 1e-12
    w0 = schedules.general_lr(0.1, 0, 0, 100, "cifar10", warmup=True)
    w1 = schedules.general_lr(0.1, 2, 250, 100, "cifar10", warmup=True)
    assert w0 == pytest.approx(0.1 / 500) and w0 < w1 < 0.1
    assert schedules.lstm_ptb_lr(22.0, 70) == pytest.approx(22.0 * 0.01)
    s = schedules.AN4Schedule(1.0)
    assert s(0) == 1.0 and s(1) == pytest.approx(1 / 1.01)


def _trainer(tmp, comp="gaussian", density=0.01, **kw):
    torch.manual_seed(0)
    hvd.init()
    t = DLTrainer(0, 1, dnn="fcn5net", dataset="mnist", batch_size=16, lr=0.1, device="cpu", learnable_data=True,
                  weights_dir=str(tmp), **kw)
    opt = hvd.DistributedOptimizer(t.optimizer, named_parameters=t.net.named_parameters(),
                                   compression=compressors[comp], is_sparse=True, density=density,
                                   compress_single_rank=True)
    t.update_optimizer(opt)
    return t, opt


def test_density_warmup_schedule(tmp_path):
    t, opt = _trainer(tmp_path)
    assert opt.get_current_density() == 0.015625
    opt.increase_one_epoch()
    assert opt.get_current_density() == 0.004
    opt.increase_one_epoch()
    opt.increase_one_epoch()
    assert opt.get_current_density() == 0.001


def test_gradient_accumulation_local_steps(tmp_path):
    t, opt = _trainer(tmp_path)
    w0 = opt.arena.weights.clone()
    opt.zero_grad()
    opt.local = True
    t.train(1)
    assert all(b.ready == 0 for b in opt.arena.buckets)  # no exchange on local steps
    opt.local = False
    t.train(1)
    t.update_model()
    assert not torch.equal(w0, opt.arena.weights)


def test_checkpoint_resume_roundtrip(tmp_path):
    t, opt = _trainer(tmp_path)
    for _ in range(3):
        opt.zero_grad()
        t.train(1)
        t.update_model()
    st = t.checkpoint_state()
    fn = os.path.join(str(tmp_path), "ck.pth")
    t.save_checkpoint(st, fn)
    res0 = opt.arena.residuals.clone()
    mom0 = opt.arena.momentum.clone()
    w0 = opt.arena.weights.clone()
    t2, opt2 = _trainer(tmp_path)
    t2.load_model_from_file(fn)
    assert torch.equal(opt2.arena.weights, w0)
    assert torch.equal(opt2.arena.momentum, mom0)
    assert torch.equal(opt2.arena.residuals, res0)
    assert t2.train_iter == t.train_iter
    # both continue identically
    for tt, oo in ((t, opt), (t2, opt2)):
        oo.zero_grad()
        tt.train(1, data=t.data.test_batches(1)[0])
        tt.update_model()
    assert torch.allclose(opt.arena.weights, opt2.arena.weights, atol=1e-7)
    ck = torch.load(fn, weights_only=True)
    assert {"iter", "epoch", "state"} <= set(ck)


def test_layerwise_profiler(tmp_path):
    from gaussiank_sgd_amd.utils.profiler import benchmark
    t, _ = _trainer(tmp_path)
    keys, times, sizes = benchmark(t, warmup=1, iterations=3)
    assert keys == [k for k, _ in t.net.named_parameters()]
    assert len(times) == len(keys) and all(x >= 0 for x in times)
    assert sizes == [p.numel() for p in t.net.parameters()]


def test_dist_trainer_cli_and_plot(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "gaussiank_sgd_amd.train.dist_trainer", "--dnn", "fcn5net", "--dataset", "mnist",
           "--batch-size", "32", "--density", "0.01", "--compressor", "gaussian", "--max-epochs", "1",
           "--max-iters", "45", "--compress-single-rank", "--logdir-root", str(tmp_path / "logs"),
           "--saved-dir", str(tmp_path)]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Speed:" in r.stderr
    logs = []
    for d, _, fs in os.walk(tmp_path / "logs"):
        logs += [os.path.join(d, f) for f in fs if f.endswith(".log")]
    assert logs
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import plot
    data = plot.read_log(logs[0])
    assert data["speed"] and data["selected"]
    jl = []
    for d, _, fs in os.walk(tmp_path / "logs"):
        jl += [os.path.join(d, f) for f in fs if f.endswith(".jsonl")]
    assert jl
    import json
    rows = [json.loads(line) for line in open(jl[0])]
    assert rows and rows[-1]["samples_per_s"] > 0 and rows[-1]["compression_ratio"] > 1


def test_evaluate_checkpoints(tmp_path):
    from gaussiank_sgd_amd.train.evaluate import evaluate
    t, _ = _trainer(tmp_path)
    d = t.checkpoint_dir()
    for e in (1, 2):
        t.train_epoch = e
        t.save_checkpoint(t.checkpoint_state(), os.path.join(d, "fcn5net-rank0-epoch%d.pth" % e))
    best, ep, res = evaluate(d, "fcn5net", "mnist", data_dir=None, nepochs=3, batch_size=16, device="cpu",
                             num_batches=1)
    assert set(res) == {1, 2} and ep in (1, 2)


def test_post_accumulate_hook_fires_for_direct_grads():
    """The bf16 shadow / fused-BN direct paths return None for the fp32
    parameter and rely on its post-accumulate hook still firing (readiness)."""
    from gaussiank_sgd_amd.parallel.shadow import _ShadowWeight
    p = torch.nn.Parameter(torch.ones(4))
    fired = []
    p.register_post_accumulate_grad_hook(lambda q: fired.append(q.grad))
    sink_got = []
    y = _ShadowWeight.apply(p, torch.full((4,), 2.0), sink_got.append)
    (y * 3).sum().backward()
    assert len(fired) == 1 and fired[0] is None
    assert torch.equal(sink_got[0], torch.full((4,), 3.0))


def test_shadow_matches_autocast_cpu():
    """bf16 shadow weights + direct arena grads == plain bf16 autocast (CPU)."""
    from gaussiank_sgd_amd.models import resnet18
    from gaussiank_sgd_amd.parallel import install_bf16_shadow

    def run(shadow):
        torch.manual_seed(0)
        net = resnet18(num_classes=10)
        opt = hvd.DistributedOptimizer(torch.optim.SGD(net.parameters(), lr=0.01, momentum=0.9),
                                       named_parameters=net.named_parameters(), compression=compressors["none"])
        n = install_bf16_shadow(net, opt) if shadow else 0
        g = torch.Generator().manual_seed(1)
        losses = []
        for _ in range(2):
            x = torch.randn(4, 3, 32, 32, generator=g)
            y = torch.randint(0, 10, (4,), generator=g)
            opt.zero_grad()
            with torch.autocast("cpu", dtype=torch.bfloat16):
                loss = torch.nn.functional.cross_entropy(net(x), y)
            loss.backward()
            grads = opt.arena.grads.clone()
            opt.step()
            losses.append(float(loss))
        return n, losses, grads, opt

    _, la, ga, oa = run(False)
    n, lb, gb, ob = run(True)
    assert n == sum(1 for _ in resnet18(num_classes=10).parameters())  # conv/fc via shadow, BN direct
    assert la == lb
    assert torch.equal(ga, gb)
    assert torch.equal(oa.arena.weights, ob.arena.weights)
    assert torch.equal(ob.arena.shadow, ob.arena.weights.to(torch.bfloat16))


def test_momentum_correction_matches_dgc_formula():
    """DGC momentum correction (u = mu*u + g + wd*w; sparsify u + residual;
    mask u at the sent indices; plain SGD on the aggregate) vs a hand-written
    single-rank oracle (CPU fallbacks of the same ops)."""
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.ReLU(), torch.nn.Linear(64, 8))
    ref = [p.detach().clone() for p in net.parameters()]
    mu, wd, lr, density = 0.9, 1e-4, 0.1, 0.05
    base = torch.optim.SGD(net.parameters(), lr=lr, momentum=mu, weight_decay=wd)
    opt = hvd.DistributedOptimizer(base, named_parameters=net.named_parameters(), compression=compressors["topk"],
                                   is_sparse=True, density=density, compress_single_rank=True, density_warmup=False,
                                   momentum_correction=True, threshold=10 ** 9)
    arena = opt.arena
    b = arena.buckets[0]
    n_flat = b.span
    u = torch.zeros(n_flat)
    v = torch.zeros(n_flat)
    w = torch.zeros(n_flat)
    for k, o in zip(b.keys, b.offsets):
        w[o:o + arena.named[k].numel()] = arena.named[k].detach().view(-1)
    g = torch.Generator().manual_seed(3)
    for step in range(4):
        x = torch.randn(16, 32, generator=g)
        raw = torch.autograd.grad(net(x).pow(2).mean(), [arena.named[k] for k in b.keys])
        grad = torch.zeros(n_flat)
        for gr, o in zip(raw, b.offsets):
            grad[o:o + gr.numel()] = gr.reshape(-1)
        opt.zero_grad()
        net(x).pow(2).mean().backward()
        opt.step()
        # oracle
        u = mu * u + grad + wd * w
        acc = v + u
        k = max(int(b.numel * density), 1)
        idx = torch.topk(acc.abs(), k).indices
        upd = torch.zeros_like(acc)
        upd[idx] = acc[idx]
        v = acc.clone()
        v[idx] = 0
        u[idx] = 0
        w = w - lr * upd
        got = b.slice(arena.weights)
        assert torch.allclose(got, w, atol=1e-6), step
        assert torch.allclose(b.slice(arena.velocity), u, atol=1e-6)


def test_watchdog_reports_stall(caplog):
    import time as _t
    from gaussiank_sgd_amd.utils.watchdog import Watchdog
    wd = Watchdog(0.2, lambda: "bucket 0: 3/5 params ready")
    try:
        _t.sleep(0.8)
        assert wd.stalls == 1
        wd.kick()
        _t.sleep(0.05)
        assert wd.stalls == 1
    finally:
        wd.stop()


def test_dense_and_order_helpers():
    from gaussiank_sgd_amd import ops
    a = torch.zeros(4, 3, 2, 2).to(memory_format=torch.channels_last)
    b = torch.zeros(4, 3, 2, 2)
    assert ops._dense(a) and ops._dense(b) and not ops._dense(b[:, :, :1, :])
    assert ops._same_order(a, a) and not ops._same_order(a, b)
    w1 = torch.zeros(8, 4, 1, 1).to(memory_format=torch.channels_last)
    assert ops._same_order(w1, torch.zeros(8, 4, 1, 1))   # 1x1: size-1 dims ignored
    dst = torch.zeros(8, 4, 1, 1)
    ops.accum_grad_(dst, torch.ones(8, 4, 1, 1, dtype=torch.bfloat16))
    assert float(dst.sum()) == 32


def test_resnet20_selected_count_schedule():
    """exact top-k on ResNet-20 (269,722 params, one merged
    bucket) selects 4214 / 1078 / 269 gradients in epochs 0 / 1 / 2+ of the
    density warm-up, as in logs/results/SGD_1024_0.0001_topk:9,16,22."""
    from gaussiank_sgd_amd.models import create_net
    torch.manual_seed(0)
    net, _ = create_net(10, "resnet20")
    assert sum(p.numel() for p in net.parameters()) == 269_722
    opt = hvd.DistributedOptimizer(torch.optim.SGD(net.parameters(), lr=0.1, momentum=0.9),
                                   named_parameters=net.named_parameters(), compression=compressors["topk"],
                                   is_sparse=True, density=0.001, threshold=10 ** 9, compress_single_rank=True)
    assert len(opt.arena.buckets) == 1
    got = []
    losses = []
    g = torch.Generator().manual_seed(0)
    x = torch.randn(16, 3, 32, 32, generator=g)
    y = torch.randint(0, 10, (16,), generator=g)
    for epoch in range(3):
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(net(x), y)
        loss.backward()
        opt.step()
        losses.append(float(loss))
        got.append(opt._collect_selected())
        opt.increase_one_epoch()
    assert got == [[4214], [1078], [269]]


def test_global_avg_pool_cl():
    from gaussiank_sgd_amd.ops.bn import global_avg_pool
    x = torch.randn(2, 8, 5, 3).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    y = global_avg_pool(x)
    ref = torch.nn.functional.adaptive_avg_pool2d(x, 1).flatten(1)
    assert torch.allclose(y, ref, atol=1e-6)
    g = torch.randn(2, 8)
    (gx,) = torch.autograd.grad(y, x, g)
    (gr,) = torch.autograd.grad(ref, x, g)
    assert gx.is_contiguous(memory_format=torch.channels_last) and torch.allclose(gx, gr, atol=1e-6)


def test_winograd_candidate_filter_checks_every_operand():
    """Grad-input with C > K: dy [N, K, H, W] fits a 32-bit buffer descriptor
    but dx and the BN-backward epilogue's h / dy2 / mask ([N, C, H, W]) do not;
    the Winograd candidate must be refused (verdict r3 item 7)."""
    import torch
    from gaussiank_sgd_amd.ops import conv1x1 as cv
    N, H, W, C, K = 256, 56, 56, 1024, 64
    assert N * H * W * K * 4 < (1 << 31) <= N * H * W * C * 4
    assert not cv._wino_shape_fits(N, H, W, C, K)
    assert not cv._wino_shape_fits(N, H, W, K, C)      # forward / grad-weight, C < K
    key = cv._dgrad_key(N, C, H, W, K, 3, 1, torch.float32)
    assert "wino" not in key
    # below the limit in every operand: offered
    assert cv._wino_shape_fits(32, 56, 56, 256, 64)
    assert "wino" in cv._dgrad_key(32, 64, 56, 56, 64, 3, 1, torch.float32)


def test_splitk_candidates_only_for_underfilled_deep_gemms():
    """fp32 split-K configs (cfg + 10000 S) are offered only when the output
    is small (<= 4 M elements) and K splits into >= 128-deep, 64-aligned
    planes; bf16 never gets them (partial planes are fp32)."""
    import torch
    from gaussiank_sgd_amd.ops import conv1x1 as cv
    prev = cv.set_f32_matmul("native")     # the S digit alone (bf16x6 adds the 100000 digit)
    try:
        _splitk_checks(cv, torch)
        cv.set_f32_matmul("bf16x6")
        x6 = cv._splitk_cfgs(torch.float32, 1568, 512, 2048)
        assert {(x % cv.X6) // 10000 for x in x6} == {2, 4, 8} and any(x >= cv.X6 for x in x6)
    finally:
        cv.set_f32_matmul(prev)


def _splitk_checks(cv, torch):
    c = cv._splitk_cfgs(torch.float32, 1568, 512, 2048)          # stage-4 1x1 at bs32
    assert c and all(x >= 20000 for x in c)
    S = sorted({x // 10000 for x in c})
    assert S == [2, 4, 8]
    assert all(2048 % (64 * s) == 0 and 2048 // s >= 128 for s in S)
    assert {x % 10000 for x in c} == set(cv._SPLITK_BASE)
    assert cv._splitk_cfgs(torch.bfloat16, 1568, 512, 2048) == []
    assert cv._splitk_cfgs(torch.float32, 25088 * 16, 512, 2048) == []   # bs512: the output fills the chip
    assert {x // 10000 for x in cv._splitk_cfgs(torch.float32, 1568, 512, 256)} == {2}   # 256 / 4 < 128
    assert cv._splitk_cfgs(torch.float32, 1568, 512, 192) == []           # 192 % 128 != 0
    # implicit-GEMM convolutions split over their tap x channel depth (3x3 x 512)
    assert {x // 10000 for x in cv._splitk_cfgs(torch.float32, 1568, 512, 9 * 512)} == {2, 4, 8}


def test_winograd_split_candidates_small_grids_only():
    """Input-channel splits of the Winograd kernel are offered when the
    64-tile x 64-channel block grid is below one block per CU (bs32 stages
    3-4), never for the bs512 shapes."""
    import torch
    from gaussiank_sgd_amd.ops import conv1x1 as cv

    def tags(N, C, H, K):
        x = torch.empty(N, C, H, H, device="meta")
        w = torch.empty(K, C, 3, 3, device="meta")
        y = torch.empty(N, K, H, H, device="meta")
        return [t for t, _ in cv._wino_cands(x, w, y, False)]
    small = tags(32, 512, 7, 512)          # 512 tiles -> 8 x 8 = 64 blocks
    assert ("wino", 2, 0) in small and ("wino", 4, 0) in small
    big = tags(512, 512, 7, 512)           # 8192 tiles -> 128 x 8 blocks
    assert all(t[1] == 0 for t in big)
    odd = tags(32, 24, 7, 64)              # Ci = 24: 8 x 3 channel stages -> no 2- or 4-way split
    assert all(t[1] == 0 for t in odd)


def test_wgrad_side_stream_policy(monkeypatch):
    """ops/streams.py: the grad-weight side stream is on by default, off with
    GKSGD_WGRAD_STREAM=0 (any value other than 1, including round 4's
    removed "auto", is off), never for a CPU tensor and never while a HIP
    graph is being captured."""
    import torch
    from gaussiank_sgd_amd.ops import streams
    dev = torch.device("cuda")
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: False)
    monkeypatch.delenv("GKSGD_WGRAD_STREAM", raising=False)
    assert streams.enabled(dev)
    monkeypatch.setenv("GKSGD_WGRAD_STREAM", "auto")
    assert not streams.enabled(dev)
    monkeypatch.setenv("GKSGD_WGRAD_STREAM", "1")
    assert streams.enabled(dev)
    assert not streams.enabled(torch.device("cpu"))
    monkeypatch.setenv("GKSGD_WGRAD_STREAM", "0")
    assert not streams.enabled(dev)
    monkeypatch.setenv("GKSGD_WGRAD_STREAM", "1")
    # size gate: ResNet-50 grad-weights fork at bs512 (>= 13 GFLOP), not at bs32 (<= 7.4)
    monkeypatch.delenv("GKSGD_WGRAD_STREAM_MIN_GFLOP", raising=False)
    assert streams.worth(dev, 13.2e9) and not streams.worth(dev, 7.4e9)
    assert not streams.worth(torch.device("cpu"), 1e12)
    monkeypatch.setenv("GKSGD_WGRAD_STREAM_MIN_GFLOP", "0")
    assert streams.worth(dev, 1.0)
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: True)
    assert not streams.enabled(dev)
    assert not streams.worth(dev, 1e12)


def test_cal_accuracy_top1_argmax_matches_topk():
    """DLTrainer.cal_accuracy: the k = 1 argmax path scores exactly what the
    sorted top-k path scores (untied logits), alone and beside a top-5."""
    import torch
    from gaussiank_sgd_amd.train.trainer import DLTrainer
    g = torch.Generator().manual_seed(3)
    out = torch.randn(257, 1000, generator=g)
    tgt = torch.randint(0, 1000, (257,), generator=g)
    tgt[:40] = out[:40].argmax(1)            # some hits
    _, p = out.topk(5, 1, True, True)
    ref1 = float(p[:, :1].eq(tgt.view(-1, 1)).sum()) * 100.0 / 257
    ref5 = float(p.eq(tgt.view(-1, 1)).sum()) * 100.0 / 257
    a1, = DLTrainer.cal_accuracy(None, out, tgt, topk=(1,))
    b1, b5 = DLTrainer.cal_accuracy(None, out, tgt, topk=(1, 5))
    assert abs(float(a1) - ref1) < 1e-4 and abs(float(b1) - ref1) < 1e-4 and abs(float(b5) - ref5) < 1e-4


def test_tied_weight_sinks_never_fork():
    """parallel/shadow.py: a parameter held by two modules (tied weights) gets
    its direct-gradient sink flagged ``shared`` by both installers, so its
    grad-weight is never forked onto the side stream (it would race the other
    module's accumulation into the same arena view); untied sinks are not."""
    import torch
    import torch.nn as nn
    from gaussiank_sgd_amd.ops.linear import FastLinear
    from gaussiank_sgd_amd.parallel import comm, install_bf16_shadow, install_direct_grads
    from gaussiank_sgd_amd.parallel.distributed_optimizer import DistributedOptimizer

    comm.init()
    for install in (install_direct_grads, install_bf16_shadow):
        torch.manual_seed(0)
        enc, dec, mid = FastLinear(16, 16), FastLinear(16, 16), FastLinear(16, 16)
        dec.weight = enc.weight                      # tied
        net = nn.Sequential(enc, mid, dec)
        opt = DistributedOptimizer(torch.optim.SGD(net.parameters(), lr=0.1),
                                   named_parameters=net.named_parameters(), compression=None)
        assert install(net, opt) > 0
        table = lambda m: getattr(m, "_gk_direct_grads", None) or getattr(m, "_gk_shadow")  # noqa: E731
        sink = lambda e: e[1] if isinstance(e, tuple) else e  # noqa: E731
        assert sink(table(enc)["weight"]).shared and sink(table(dec)["weight"]).shared
        assert not sink(table(mid)["weight"]).shared and not sink(table(enc)["bias"]).shared
