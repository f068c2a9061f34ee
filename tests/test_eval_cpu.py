"""Evaluation parity (reference dl_trainer.py:742-824, evaluate.py:20-73).

* ``DLTrainer.test()`` walks the WHOLE real test split once -- every sample
  exactly once, storage order, ragged last batch included -- like the
  reference's ``testloader`` loop; synthetic data keeps sampled batches.
* ``evaluate.py`` takes the reference's flags (``--model-path --dnn --dataset
  --data-dir --nepochs``), parses bs / lr from the directory name and logs to
  ``<model-path>/evaluate.log``.
* lstman4: greedy CTC decode + word error rate (reference :778-797,817-819).
"""
import os

import numpy as np
import torch

from gaussiank_sgd_amd.data.real import MNIST_MEAN, MNIST_STD


def _mnist_dir(tmp_path, n_test=70, n_train=64):
    d = tmp_path / "data"
    d.mkdir()
    rng = np.random.default_rng(0)
    for split, n in (("train", n_train), ("test", n_test)):
        x = rng.integers(0, 256, size=(n, 1, 28, 28), dtype=np.uint8)
        x[:, 0, 0, 0] = np.arange(n) % 256          # sample id in the first pixel
        y = rng.integers(0, 10, size=n).astype(np.int64)
        np.savez(d / ("mnist_%s.npz" % split), x=x, y=y)
    return str(d)


def test_test_visits_every_sample_once(tmp_path):
    from gaussiank_sgd_amd.train import DLTrainer
    data_dir = _mnist_dir(tmp_path)
    t = DLTrainer(0, 1, dnn="fcn5net", dataset="mnist", batch_size=32, lr=0.1, device="cpu", data_dir=data_dir)
    seen = []
    h = t.net.register_forward_pre_hook(lambda m, inp: seen.append(inp[0].detach().clone()))
    acc = t.test(1)
    h.remove()
    assert [s.shape[0] for s in seen] == [32, 32, 6]           # ragged last batch included
    got = torch.cat(seen).reshape(70, -1)[:, 0]
    ids = torch.round((got * MNIST_STD[0] + MNIST_MEAN[0]) * 255.0).long()
    assert torch.equal(ids, torch.arange(70))                  # each sample once, in order
    assert 0.0 <= acc <= 100.0
    # a second evaluation is the same pass (independent of the training stream)
    seen.clear()
    h = t.net.register_forward_pre_hook(lambda m, inp: seen.append(inp[0].detach().clone()))
    assert t.test(2) == acc
    h.remove()
    assert sum(s.shape[0] for s in seen) == 70


def test_synthetic_data_keeps_sampled_batches():
    from gaussiank_sgd_amd.train import DLTrainer
    t = DLTrainer(0, 1, dnn="fcn5net", dataset="mnist", batch_size=16, lr=0.1, device="cpu", data_dir=None)
    n = []
    h = t.net.register_forward_pre_hook(lambda m, inp: n.append(inp[0].shape[0]))
    t.test(1)
    t.test(1, num_batches=3)
    h.remove()
    assert n == [16, 16, 16, 16, 16]


def test_evaluate_cli_reference_flags(tmp_path):
    from gaussiank_sgd_amd.train import DLTrainer
    from gaussiank_sgd_amd.train.evaluate import main, parse_model_path
    data_dir = _mnist_dir(tmp_path)
    model_dir = tmp_path / "weights" / "fcn5net-n2-bs32-lr0.1000"
    model_dir.mkdir(parents=True)
    assert parse_model_path(str(model_dir)) == ("fcn5net", 32, 0.1)
    t = DLTrainer(0, 1, dnn="fcn5net", dataset="mnist", batch_size=32, lr=0.1, device="cpu", data_dir=data_dir)
    for e in (1, 2):
        t.train(1)
        t.optimizer.step()
        t.train_epoch = e
        t.save_checkpoint(t.checkpoint_state(), str(model_dir / ("fcn5net-rank0-epoch%d.pth" % e)))
    best, ep, res = main(["--model-path", str(model_dir), "--dnn", "resnet20", "--dataset", "mnist",
                          "--data-dir", data_dir, "--nepochs", "3"])
    assert set(res) == {1, 2} and best == max(res.values()) and ep in (1, 2)   # dnn came from the path
    log = open(model_dir / "evaluate.log").read()
    assert "Best validation accuracy or perprexity" in log and "val top-1 acc" in log


def test_ctc_greedy_decode_and_wer():
    from gaussiank_sgd_amd.train.trainer import AN4_LABELS_STR, ctc_greedy_decode, word_errors
    # frames: A A _ B B _ space C -> "AB C"
    A, B, C, SP = 2, 3, 4, 28
    seq = [A, A, 0, B, B, 0, SP, C, C, 0]
    out = torch.full((1, len(seq), 29), -5.0)
    for i, s in enumerate(seq):
        out[0, i, s] = 5.0
    dec = ctc_greedy_decode(out, torch.tensor([len(seq)]))
    assert AN4_LABELS_STR(dec[0]) == "AB C"
    assert ctc_greedy_decode(out, torch.tensor([3]))[0] == [A]
    assert word_errors("AB C", "AB C") == 0
    assert word_errors("AB", "AB C") == 1 and word_errors("X Y Z", "AB C") == 3


def test_lstman4_test_reports_wer():
    from gaussiank_sgd_amd.train import DLTrainer
    t = DLTrainer(0, 1, dnn="lstman4", dataset="an4", batch_size=2, lr=0.1, device="cpu", data_dir=None)
    wer = t.test(1, num_batches=1)
    assert 0.0 <= wer and np.isfinite(wer)
