"""Single-GPU entry (reference dl_trainer.py:879-927 ``train_with_single`` and
its ``__main__``): the CLI trains without communication, logs the reference's
throughput line into ``logs/singlegpu-<PREFIX>/<dnn>-n1-bs<B>-lr<lr>-ns<n>/
<host>.log``, and the fused arena update matches torch.optim.SGD."""
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_single_cli_logs_like_the_reference(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "gaussiank_sgd_amd.train.trainer", "--dnn", "fcn5net", "--dataset", "mnist",
           "--batch-size", "32", "--lr", "0.05", "--max-epochs", "1", "--max-iters", "6", "--train-samples", "192",
           "--logdir-root", str(tmp_path / "logs")]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-2000:]
    from gaussiank_sgd_amd import settings
    d = tmp_path / "logs" / ("singlegpu-%s" % settings.PREFIX) / "fcn5net-n1-bs32-lr0.0500-ns1"
    logs = list(d.glob("*.log"))
    assert logs, list((tmp_path / "logs").rglob("*"))
    text = logs[0].read_text()
    assert "Configurations:" in text
    assert "Time per iteration including communication:" in text and "Speed:" in text


def test_fused_single_update_matches_torch_sgd():
    from gaussiank_sgd_amd.train.single import train_with_single
    torch.manual_seed(0)
    a = train_with_single("fcn5net", "mnist", "/nonexistent", 1, 0.05, 16, 1, 1, max_iters=4, train_samples=64,
                          fused=True)
    torch.manual_seed(0)
    b = train_with_single("fcn5net", "mnist", "/nonexistent", 1, 0.05, 16, 1, 1, max_iters=4, train_samples=64,
                          fused=False)
    for (k, x), (_, y) in zip(a.net.state_dict().items(), b.net.state_dict().items()):
        assert torch.allclose(x, y, rtol=1e-5, atol=1e-6), k
    assert a.train_iter == b.train_iter == 4
