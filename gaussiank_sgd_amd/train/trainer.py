"""DLTrainer: model + data + loss + local optimizer + LR schedule + eval + checkpoints.

Parity: reference ``dl_trainer.DLTrainer`` (dl_trainer.py:123-877): same
constructor arguments and methods (``train(num_of_iters, data, hidden)``,
``test(epoch)``, ``update_model()``, ``update_optimizer()``,
``get_num_of_training_samples()``, ``data_iter()``, ``load_model_from_file``,
``save_checkpoint``), the same per-dataset momentum / weight decay
(:197-228), the LR schedule called every iteration (:631) and the same log
lines (``Epoch``, ``val loss:``, ``top-5 acc:``) that tools/plot.py parses.

MI355X differences: synthetic on-device data by default; bf16 autocast and
channels_last options; the loss is NOT pulled to the host every iteration
(the reference's ``loss.item()`` is a device sync per step) -- it is
accumulated on the device and read every ``display`` iterations.
Checkpoints add momentum (optimizer state) and per-rank compression
residuals to the reference's ``{iter, epoch, state}``.
"""
from __future__ import annotations

import contextlib
import math
import os
import time
from typing import Optional

import numpy as np
import torch
import torch.nn as nn

from .. import settings
from ..data import DATASETS, SyntheticData
from ..models import MaskedLMLoss, create_net, repackage_hidden
from ..ops import xent
from ..optim import sgd_param_groups
from ..settings import logger
from ..utils import trace
from . import schedules

_support_datasets = ["imagenet", "cifar10", "an4", "ptb", "mnist", "mnist32", "wikipedia"]
_support_dnns = ["resnet50", "googlenet", "inceptionv4", "inceptionv3", "vgg16i", "alexnet", "resnet20", "resnet56",
                 "resnet110", "vgg19", "vgg16", "lstman4", "lstm", "mnistnet", "fcn5net", "lenet", "lr", "bert",
                 "bert_tiny", "resnet18", "resnet34", "resnet101", "resnet152", "densenet100", "resnext29"]


# AN4 character set (the reference's labels.json): index 0 is the CTC blank
AN4_LABELS = "_'ABCDEFGHIJKLMNOPQRSTUVWXYZ "


def AN4_LABELS_STR(ids) -> str:
    return "".join(AN4_LABELS[int(i)] for i in ids if 0 < int(i) < len(AN4_LABELS))


def ctc_greedy_decode(outputs: torch.Tensor, out_lens: torch.Tensor):
    """Best-path CTC decode of [N, T, C] scores: per-frame argmax, repeats
    collapsed, blanks (0) dropped; one id list per utterance."""
    best = outputs.argmax(-1).cpu()
    lens = out_lens.cpu().tolist()
    res = []
    for n in range(best.shape[0]):
        seq, prev = [], -1
        for t in best[n, : int(lens[n])].tolist():
            if t != prev and t != 0:
                seq.append(t)
            prev = t
        res.append(seq)
    return res


def split_targets(targets: torch.Tensor, tgt_lens: torch.Tensor):
    """Concatenated CTC targets -> one id list per utterance."""
    out, o = [], 0
    flat = targets.reshape(-1).cpu().tolist()
    for n in tgt_lens.cpu().tolist():
        out.append(flat[o:o + int(n)])
        o += int(n)
    return out


def word_errors(hyp: str, ref: str) -> int:
    """Word-level Levenshtein distance (the WER numerator)."""
    h, r = hyp.split(), ref.split()
    prev = list(range(len(h) + 1))
    for i in range(1, len(r) + 1):
        cur = [i] + [0] * len(h)
        for j in range(1, len(h) + 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (r[i - 1] != h[j - 1]))
        prev = cur
    return prev[-1]


def rank_checkpoint_path(path: str, rank: int) -> Optional[str]:
    """``.../<dnn>-rank0-epoch<e>.pth`` -> the same checkpoint of ``rank``
    (every rank saves its own residuals / velocity, save_epoch_checkpoint);
    None when the file name carries no ``-rank<r>-`` tag."""
    import re
    d, base = os.path.split(path)
    new, n = re.subn(r"-rank\d+-", "-rank%d-" % int(rank), base, count=1)
    return os.path.join(d, new) if n else None


class DLTrainer:
    def __init__(self, rank, size, master="gpu10", dist=True, ngpus=1, batch_size=32, is_weak_scaling=True,
                 data_dir="./data", dataset="cifar10", dnn="resnet20", lr=0.04, nworkers=1, prefix=None,
                 sparsity=0.95, pretrain=None, num_steps=35, tb_writer=None, amp_handle=None, device=None,
                 amp: Optional[str] = None, channels_last: bool = False, learnable_data: bool = False,
                 seed: int = 0, data_pool: int = 4, weights_dir: str = "./weights", seq_len: Optional[int] = None,
                 train_samples: Optional[int] = None, checkpoint_every: int = 2):
        # data_dir: real datasets (data/real.py: CIFAR-10 binary, MNIST idx, PTB text, .npz / .npy
        # arrays), sharded by (rank, nworkers); absent or unrecognised -> synthetic, shape-exact
        self.size = size
        self.rank = rank
        self.pretrain = pretrain
        self.dataset = dataset
        self.prefix = prefix
        self.num_steps = num_steps
        self.ngpus = ngpus
        self.writer = tb_writer
        self.amp_handle = amp_handle
        self.weights_dir = weights_dir
        self.train_samples = train_samples
        # save a checkpoint every N trainer epochs (reference: 2, dl_trainer.py:660)
        self.checkpoint_every = max(1, int(checkpoint_every))
        if device is None:
            device = "cuda" if (ngpus > 0 and torch.cuda.is_available()) else "cpu"
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.is_cuda = self.device.type == "cuda"
        self.batch_size = batch_size * max(1, ngpus) if (is_weak_scaling and ngpus > 1) else batch_size
        self.num_batches_per_epoch = -1
        spec = DATASETS.get(dataset)
        self.num_classes = spec.num_classes if spec is not None and spec.kind == "image" else 10
        if dataset == "an4":
            self.num_classes = 29
        self.nworkers = nworkers
        self.data_dir = data_dir
        self.amp = amp if amp is not None else ("bf16" if settings.USE_BF16 else None)
        self.channels_last = channels_last
        self.seed = seed
        torch.manual_seed(seed)
        if isinstance(dnn, nn.Module):
            self.net = dnn
            self.dnn = getattr(dnn, "name", "custom")
        else:
            self.dnn = dnn
            kw = {}
            if dnn == "lstm":
                kw = dict(vocab_size=10000, batch_size=self.batch_size, num_steps=num_steps)
            self.net, self.ext = create_net(self.num_classes, dnn, **kw)
        self.ext = getattr(self, "ext", None)
        self.net.to(self.device)
        if self.channels_last and self.is_cuda:
            self.net = self.net.to(memory_format=torch.channels_last)
        self.lr = lr
        self.base_lr = lr
        self.accuracy = 0
        self.loss = 0.0
        self._loss_acc = None
        self.train_iter = 0
        self.recved_counter = 0
        self.master = master
        self.average_iter = 0
        if self.dnn.startswith("bert"):
            self.criterion = MaskedLMLoss()
        elif self.dnn == "lstman4":
            self.criterion = nn.CTCLoss(blank=0, reduction="sum", zero_infinity=True)
        else:
            self.criterion = nn.CrossEntropyLoss()
        weight_decay = 1e-4
        self.m = 0.9
        if dataset == "an4":
            self.lstman4_sched = schedules.AN4Schedule(lr)
        elif dataset == "ptb":
            self.m = 0
            weight_decay = 0
        elif dataset == "imagenet":
            self.m = 0.875
            weight_decay = 2 * 3.0517578125e-05
        self.weight_decay = weight_decay
        self.optimizer = torch.optim.SGD(sgd_param_groups(self.net, weight_decay), lr=self.lr, momentum=self.m,
                                         weight_decay=weight_decay, nesterov=False)
        self.train_epoch = 0
        self.data_prepare(learnable_data, data_pool, seq_len)
        if self.pretrain is not None and os.path.isfile(self.pretrain):
            self.load_model_from_file(self.pretrain)
        self.sparsities = []
        self.compression_ratios = []
        self.communication_sizes = []
        self.avg_loss_per_epoch = 0.0
        self._epoch_loss_acc = None
        self.timer = 0.0
        self.forwardtime = 0.0
        self.backwardtime = 0.0
        self.iotime = 0.0
        self.epochs_info = []
        self.train_acc_top1 = []
        self._acc_acc = None
        self._acc_n = 0
        self.display = 40
        self._graph_body = False     # set while train/graph.py runs / captures its step body
        # per-step weight re-layouts of the convolutions, rebuilt in one batched
        # launch at the start of every step (ops/weight_prep.py)
        from ..ops.weight_prep import WeightPrep
        self.weight_prep = WeightPrep()
        logger.info("num_batches_per_epoch: %d" % self.num_batches_per_epoch)

    # ------------------------------------------------------------------
    def data_prepare(self, learnable: bool = False, pool: int = 4, seq_len: Optional[int] = None):
        ds = self.dataset
        if ds == "mnist" and self.dnn == "lenet":
            ds = "mnist32"
        if self.dnn.startswith("bert"):
            ds = "wikipedia"
        if ds not in DATASETS:
            raise ValueError("Unsupport dataset: %s" % ds)
        vocab = None
        if self.dnn == "bert_tiny":
            vocab = 1024
            seq_len = seq_len or 128
        self.test_data = None
        real = None
        if self.data_dir and os.path.isdir(self.data_dir) and not learnable:
            from ..data.real import open_dataset
            real = open_dataset(ds, self.data_dir, self.batch_size, self.device, self.rank, self.nworkers,
                                seed=self.seed, channels_last=self.channels_last and self.is_cuda,
                                num_steps=self.num_steps)
            if real is not None:
                self.test_data = open_dataset(ds, self.data_dir, self.batch_size, self.device, 0, 1, seed=self.seed,
                                              channels_last=self.channels_last and self.is_cuda,
                                              num_steps=self.num_steps, train=False)
                logger.info("real data: %s from %s, %d samples, rank %d of %d shards", ds, self.data_dir,
                            real.num_samples(), self.rank, self.nworkers)
            else:
                logger.info("no %s files under %s: synthetic data", ds, self.data_dir)
        if real is not None:
            self.data = real
        else:
            self.data = SyntheticData(ds, self.batch_size, self.device, seed=self.seed * 1000 + self.rank, pool=pool,
                                      learnable=learnable, seq_len=(self.num_steps if ds == "ptb" else seq_len),
                                      channels_last=self.channels_last and self.is_cuda, vocab_size=vocab,
                                      train_samples=self.train_samples)
        self.trainset_len = self.data.num_samples()
        self._input_shape = (self.batch_size,) + tuple(DATASETS[ds].shape)
        self._output_shape = (self.batch_size, self.num_classes)
        self.num_batches_per_epoch = (self.trainset_len + self.batch_size * self.nworkers - 1) // (
            self.batch_size * self.nworkers)

    def get_acc(self):
        return self.accuracy

    def get_loss(self):
        return self.loss

    def get_model_state(self):
        return self.net.state_dict()

    def get_data_shape(self):
        return self._input_shape, self._output_shape

    def get_train_epoch(self):
        return self.train_epoch

    def get_train_iter(self):
        return self.train_iter

    def set_train_epoch(self, epoch):
        self.train_epoch = epoch

    def set_train_iter(self, iteration):
        self.train_iter = iteration

    def seek_data(self, position: Optional[int] = None) -> None:
        """Point the (synthetic) batch stream at iteration ``position``
        (default: ``train_iter``) so a resumed run reads the batches the
        uninterrupted one would have; real loaders restart their epoch."""
        fn = getattr(self.data, "seek", None)
        if fn is not None:
            fn(self.train_iter if position is None else position)

    def get_num_of_training_samples(self):
        return self.trainset_len

    def update_optimizer(self, optimizer):
        self.optimizer = optimizer

    def update_nworker(self, nworkers, new_rank=-1):
        if new_rank >= 0:
            self.rank = new_rank
        self.nworkers = nworkers
        self.num_batches_per_epoch = (self.trainset_len + self.batch_size * self.nworkers - 1) // (
            self.batch_size * self.nworkers)

    def data_iter(self):
        return next(self.data)

    # ------------------------------------------------------------------
    def adjust_learning_rate(self, progress, optimizer):
        if self.dataset == "an4":
            lr = self.lstman4_sched(self.train_iter // max(1, self.num_batches_per_epoch))
        elif self.dnn == "lstm":
            lr = schedules.lstm_ptb_lr(self.base_lr, progress)
        else:
            lr = schedules.general_lr(self.base_lr, progress, self.train_iter, self.num_batches_per_epoch,
                                      self.dataset, warmup=settings.WARMUP)
        self.lr = lr
        for g in optimizer.param_groups:
            g["lr"] = lr
        return lr

    def cal_accuracy(self, output, target, topk=(1,)):
        """Top-k accuracy (%) as device tensors."""
        with torch.no_grad():
            maxk = max(topk)
            bs = target.size(0)
            if maxk == 1:
                # the per-step training top-1: one argmax reduction (torch's
                # sorted top-k path for k = 1 took 134 us per bs512 step on
                # MI355X, r5c55); the same prediction except on exactly tied logits
                pred = output.argmax(1).view(1, -1)
            else:
                _, pred = output.topk(maxk, 1, True, True)
                pred = pred.t()
            correct = pred.eq(target.view(1, -1).expand_as(pred))
            return [correct[:k].reshape(-1).float().sum(0, keepdim=True).mul_(100.0 / bs) for k in topk]

    def _autocast(self):
        if self.amp == "bf16":
            return torch.autocast(device_type=self.device.type, dtype=torch.bfloat16)
        if self.amp == "fp16":
            return torch.autocast(device_type=self.device.type, dtype=torch.float16)
        return contextlib.nullcontext()

    def forward_loss(self, inputs, labels, hidden=None):
        with self._autocast():
            if self.dnn == "lstm":
                hidden = repackage_hidden(hidden) if hidden is not None else self.net.init_hidden(inputs.shape[1])
                outputs, hidden = self.net(inputs, hidden)
                c = self.criterion
                if (isinstance(c, nn.CrossEntropyLoss) and c.reduction == "mean" and c.weight is None and
                        c.label_smoothing == 0.0):
                    # fused softmax cross-entropy on the bf16 logits on the GPU (ops/xent.py)
                    loss = xent.cross_entropy(outputs.reshape(-1, self.net.vocab_size), labels.reshape(-1),
                                              ignore_index=self.criterion.ignore_index)
                else:
                    loss = self.criterion(outputs.reshape(-1, self.net.vocab_size).float(), labels.reshape(-1))
            elif self.dnn.startswith("bert"):
                if isinstance(labels, (tuple, list)):     # (masked positions, labels)
                    outputs = self.net(inputs, masked_positions=labels[0])
                    loss = self.criterion(outputs, labels[1])
                else:                                     # dense [B, T] labels, -100 = unmasked
                    outputs = self.net(inputs)
                    loss = self.criterion(outputs, labels)
            elif self.dnn == "lstman4":
                targets, tgt_lens, in_lens = labels
                outputs, out_lens = self.net(inputs, in_lens)
                logp = outputs.float().log_softmax(-1).transpose(0, 1)  # T x N x C
                loss = self.criterion(logp, targets, out_lens, tgt_lens) / inputs.size(0)
            else:
                outputs = self.net(inputs)
                loss = self.criterion(outputs.float(), labels)
        return outputs, loss, hidden

    def _on_epoch_boundary(self):
        self.train_epoch += 1
        avg_loss = self._read_epoch_loss()
        acc = float(self._read_acc())
        logger.info("train iter: %d, num_batches_per_epoch: %d", self.train_iter, self.num_batches_per_epoch)
        logger.info("Epoch %d, avg train acc: %f, lr: %f, avg loss: %f" % (
            self.train_iter // self.num_batches_per_epoch, acc, self.lr, avg_loss))
        if self.rank == 0:
            self.test(self.train_epoch)
        self.epochs_info.append(avg_loss)
        if self.train_iter > 0 and self.train_epoch % self.checkpoint_every == 0:
            self.save_epoch_checkpoint()

    def _read_epoch_loss(self) -> float:
        if self._epoch_loss_acc is None:
            return 0.0
        v = float(self._epoch_loss_acc) / max(1, self.num_batches_per_epoch)
        self._epoch_loss_acc = None
        return v

    def _read_acc(self) -> float:
        if self._acc_acc is None or self._acc_n == 0:
            return 0.0
        v = float(self._acc_acc) / self._acc_n
        self._acc_acc = None
        self._acc_n = 0
        return v

    def train(self, num_of_iters=1, data=None, hidden=None):
        s = time.time()
        loss_sum = None
        for _ in range(num_of_iters):
            self.adjust_learning_rate(self.train_epoch, self.optimizer)
            # (a HIP-graph step, train/graph.py, runs the epoch-boundary logic --
            # eval, checkpoint, host syncs -- itself, outside its captured body)
            if self.train_iter % self.num_batches_per_epoch == 0 and self.train_iter > 0 and \
                    not self._graph_body:
                self._on_epoch_boundary()
            ss = time.time()
            d = data if data is not None else self.data_iter()
            inputs, labels = d[0], d[1]
            if inputs.device != self.device:
                inputs = inputs.to(self.device, non_blocking=True)
                labels = labels.to(self.device, non_blocking=True) if torch.is_tensor(labels) else labels
            self.iotime += time.time() - ss
            with self.weight_prep.step(self.device):
                sf = time.time()
                with trace.range("gk/forward"):
                    outputs, loss, hidden = self.forward_loss(inputs, labels, hidden)
                self.forwardtime += time.time() - sf
                sb = time.time()
                with trace.range("gk/backward"):
                    loss.backward()
                self.backwardtime += time.time() - sb
            ld = loss.detach()
            loss_sum = ld if loss_sum is None else loss_sum + ld
            self._epoch_loss_acc = ld.clone() if self._epoch_loss_acc is None else self._epoch_loss_acc + ld
            if self.dnn not in ("lstm", "lstman4") and not self.dnn.startswith("bert"):
                acc1, = self.cal_accuracy(outputs.detach(), labels, topk=(1,))
                self._acc_acc = acc1 if self._acc_acc is None else self._acc_acc + acc1
                self._acc_n += 1
            self.train_iter += 1
        self._loss_acc = loss_sum / num_of_iters
        self.timer += time.time() - s
        if self.train_iter % self.display == 0 and not self._graph_body:
            self.loss = float(self._loss_acc)
            logger.warning("[%3d][%5d/%5d][rank:%d] loss: %.3f, average forward (%f) and backward (%f) time: %f, "
                           "iotime: %f " % (self.train_epoch, self.train_iter, self.num_batches_per_epoch, self.rank,
                                            self.loss, self.forwardtime / self.display,
                                            self.backwardtime / self.display, self.timer / self.display,
                                            self.iotime / self.display))
            self.timer = self.iotime = self.forwardtime = self.backwardtime = 0.0
        if self.dnn == "lstm":
            # detached (the next call repackages it anyway): a caller holding the
            # state must not keep this step's autograd graph -- and its
            # AccumulateGrad nodes -- alive (a HIP-graph capture on another
            # stream refuses stale AccumulateGrad nodes)
            return num_of_iters, repackage_hidden(hidden)
        return num_of_iters

    def current_loss(self) -> float:
        """Loss of the last train() call (host sync)."""
        return float(self._loss_acc) if self._loss_acc is not None else float("nan")

    def _eval_batches(self, num_batches: Optional[int]):
        """Evaluation batches: the WHOLE test split, each sample once, when a
        real one is loaded (the reference's test() walks its testloader,
        dl_trainer.py:753); synthetic data has no split -> ``num_batches``
        sampled batches (default 2)."""
        src = self.test_data if getattr(self, "test_data", None) is not None else self.data
        if num_batches is None and hasattr(src, "full_pass"):
            return src.full_pass()
        return src.test_batches(num_batches if num_batches is not None else 2)

    @torch.no_grad()
    def test(self, epoch, num_batches: Optional[int] = None):
        """Reference dl_trainer.py:742-824: mean over batches of the batch loss
        and top-1 / top-5 accuracy; LSTM perplexity exp(sum cost / steps);
        lstman4 word error rate of the greedy CTC decode (sum over utterances
        of edit distance / reference words, over the number of utterances)."""
        self.net.eval()
        top1, top5, losses = [], [], []
        costs, steps = 0.0, 0
        wer_sum, utterances = 0.0, 0
        with self.weight_prep.step(self.device):
            for inputs, labels in self._eval_batches(num_batches):
                if self.dnn == "lstman4":
                    targets, tgt_lens, in_lens = labels
                    with self._autocast():
                        outputs, out_lens = self.net(inputs, in_lens)
                    hyps = ctc_greedy_decode(outputs.float(), out_lens)
                    refs = split_targets(targets, tgt_lens)
                    for h, r in zip(hyps, refs):
                        ref_s = AN4_LABELS_STR(r)
                        wer_sum += word_errors(AN4_LABELS_STR(h), ref_s) / float(max(1, len(ref_s.split())))
                    utterances += len(refs)
                    logp = outputs.float().log_softmax(-1).transpose(0, 1)
                    losses.append(float(self.criterion(logp, targets, out_lens, tgt_lens) / inputs.size(0)))
                    continue
                outputs, loss, _ = self.forward_loss(inputs, labels, None)
                losses.append(float(loss))
                if self.dnn == "lstm":
                    costs += float(loss) * self.num_steps
                    steps += self.num_steps
                elif not self.dnn.startswith("bert"):
                    k5 = min(5, outputs.shape[1])
                    a1, a5 = self.cal_accuracy(outputs.float(), labels, topk=(1, k5))
                    top1.append(float(a1))
                    top5.append(float(a5))
        test_loss = float(np.mean(losses)) if losses else 0.0
        if self.dnn == "lstm":
            acc, acc5 = float(np.exp(costs / max(1, steps))), 0.0
        elif self.dnn == "lstman4":
            acc, acc5 = wer_sum / max(1, utterances), 0.0
        elif self.dnn.startswith("bert"):
            acc, acc5 = float(np.exp(test_loss)), 0.0
        else:
            acc, acc5 = float(np.mean(top1)), float(np.mean(top5))
        logger.info("Epoch %d, lr: %f, val loss: %f, val top-1 acc: %f, top-5 acc: %f" % (
            epoch, self.lr, test_loss, acc, acc5))
        self.accuracy = acc
        self.net.train()
        return acc

    def update_model(self):
        self.optimizer.step()

    def zero_grad(self):
        self.optimizer.zero_grad()

    # ------------------------------------------------------------------
    # checkpoints
    # ------------------------------------------------------------------
    def checkpoint_dir(self) -> str:
        if self.prefix:
            return os.path.join(self.weights_dir, self.prefix, "%s-n%d-bs%d-lr%.4f" % (
                self.dnn, self.nworkers, self.batch_size, self.base_lr))
        return os.path.join(self.weights_dir, "%s-n%d-bs%d-lr%.4f" % (self.dnn, self.nworkers, self.batch_size,
                                                                       self.base_lr))

    def checkpoint_state(self) -> dict:
        state = {"iter": self.train_iter, "epoch": self.train_epoch, "state": self.get_model_state()}
        try:
            state["optimizer"] = self.optimizer.state_dict()
        except Exception:  # pragma: no cover
            pass
        if hasattr(self.optimizer, "compression_state"):
            state["compression"] = self.optimizer.compression_state()
        state["rng"] = {"torch": torch.get_rng_state()}
        return state

    def save_epoch_checkpoint(self):
        from ..utils.checkpoint import save_checkpoint
        # residuals / velocities are per rank: every rank saves when it has them
        has_residuals = hasattr(self.optimizer, "compression_state") and self.size > 1
        if self.rank != 0 and not has_residuals:
            return None
        fn = os.path.join(self.checkpoint_dir(), "%s-rank%d-epoch%d.pth" % (self.dnn, self.rank, self.train_epoch))
        save_checkpoint(self.checkpoint_state(), fn)   # one D2H of the state
        return fn

    def save_checkpoint(self, state, filename):
        from ..utils.checkpoint import save_checkpoint
        save_checkpoint(state, filename)

    def load_model_from_file(self, filename):
        from ..utils.checkpoint import load_checkpoint
        ck = load_checkpoint(filename, map_location=self.device)
        self.net.load_state_dict(ck["state"])
        self.train_epoch = ck.get("epoch", 0)
        self.train_iter = ck.get("iter", 0)
        if "optimizer" in ck:
            try:
                self.optimizer.load_state_dict(ck["optimizer"])
            except Exception as e:  # pragma: no cover
                logger.warning("optimizer state not restored: %s", e)
        if "compression" in ck and hasattr(self.optimizer, "load_compression_state"):
            self.optimizer.load_compression_state(ck["compression"])
        self._pending_compression = ck.get("compression")
        logger.info("Load pretrain model: %s, start from epoch %d and iter: %d", filename, self.train_epoch,
                    self.train_iter)

    def finish(self):
        if self.writer is not None:
            self.writer.close()


if __name__ == "__main__":
    # the reference's single-GPU entry is `python dl_trainer.py ...` (dl_trainer.py:907-927)
    from gaussiank_sgd_amd.train.single import main
    main()
