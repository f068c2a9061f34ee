"""On-device synthetic datasets with the reference's shapes.

| dataset   | sample            | classes / vocab | train samples |
|-----------|-------------------|-----------------|---------------|
| imagenet  | 3x224x224 fp32    | 1000            | 1,281,167     |
| cifar10   | 3x32x32           | 10              | 50,000        |
| mnist     | 1x28x28 (32x32 for lenet) | 10      | 60,000        |
| ptb       | 35 tokens         | 10,000          | 929,589 tokens|
| wikipedia | 512 tokens (MLM)  | 30,522          | 1,000,000     |

``learnable=True`` makes labels a fixed function of the inputs (argmax of a
random projection / next-token shift) so convergence tests see the loss fall.
A small pool of batches is generated once on the device and cycled.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np
import torch


@dataclass(frozen=True)
class DatasetSpec:
    name: str
    shape: Tuple[int, ...]
    num_classes: int
    train_samples: int
    test_samples: int
    kind: str  # image | tokens | mlm


DATASETS = {
    "imagenet": DatasetSpec("imagenet", (3, 224, 224), 1000, 1281167, 50000, "image"),
    "cifar10": DatasetSpec("cifar10", (3, 32, 32), 10, 50000, 10000, "image"),
    "mnist": DatasetSpec("mnist", (1, 28, 28), 10, 60000, 10000, "image"),
    "mnist32": DatasetSpec("mnist32", (1, 32, 32), 10, 60000, 10000, "image"),
    "ptb": DatasetSpec("ptb", (35,), 10000, 929589, 82430, "tokens"),
    "wikipedia": DatasetSpec("wikipedia", (512,), 30522, 1000000, 10000, "mlm"),
    # AN4 spectrograms: 161 frequency bins x ~2 s of 10 ms frames, 29 characters (CTC blank = 0)
    "an4": DatasetSpec("an4", (1, 161, 200), 29, 948, 130, "speech"),
}


class SyntheticData:
    def __init__(self, dataset: str, batch_size: int, device="cpu", seed: int = 0, pool: int = 4,
                 learnable: bool = False, seq_len: Optional[int] = None, channels_last: bool = False,
                 dtype: torch.dtype = torch.float32, vocab_size: Optional[int] = None,
                 train_samples: Optional[int] = None):
        if dataset not in DATASETS:
            raise ValueError("Unsupport dataset: %s" % dataset)
        self.spec = DATASETS[dataset]
        self.batch_size = int(batch_size)
        self.device = torch.device(device)
        self.learnable = learnable
        self.seq_len = seq_len or (self.spec.shape[0] if self.spec.kind != "image" else None)
        self.vocab = vocab_size or self.spec.num_classes
        # epoch length override (short synthetic epochs: resume / schedule tests)
        self.train_samples = train_samples
        g = torch.Generator(device="cpu")
        g.manual_seed(1234 + seed)
        self._batches = []
        proj = None
        if learnable and self.spec.kind == "image":
            feat = int(np.prod(self.spec.shape))
            proj = torch.randn(feat, self.spec.num_classes, generator=g) / feat ** 0.5
        for _ in range(max(1, pool)):
            self._batches.append(self._make(g, proj, channels_last, dtype))
        self._i = 0

    def _make(self, g, proj, channels_last, dtype):
        B = self.batch_size
        s = self.spec
        if s.kind == "image":
            x = torch.randn((B,) + s.shape, generator=g)
            if proj is not None:
                y = (x.reshape(B, -1) @ proj).argmax(1)
            else:
                y = torch.randint(0, s.num_classes, (B,), generator=g)
            x = x.to(self.device, dtype)
            if channels_last and x.dim() == 4:
                x = x.contiguous(memory_format=torch.channels_last)
            return x, y.to(self.device)
        if s.kind == "speech":
            x = torch.randn((B,) + s.shape, generator=g)
            T = s.shape[-1]
            in_lens = torch.randint(T // 2, T + 1, (B,), generator=g)
            in_lens[0] = T
            tgt_lens = torch.randint(5, 25, (B,), generator=g)
            targets = torch.randint(1, s.num_classes, (int(tgt_lens.sum()),), generator=g)
            return x.to(self.device, dtype), (targets.to(self.device), tgt_lens.to(self.device),
                                              in_lens.to(self.device))
        if s.kind == "tokens":
            T = self.seq_len
            if self.learnable:
                start = torch.randint(0, self.vocab, (1, B), generator=g)
                steps = torch.arange(T + 1).unsqueeze(1)
                seq = (start + steps) % self.vocab
            else:
                seq = torch.randint(0, self.vocab, (T + 1, B), generator=g)
            return seq[:-1].to(self.device), seq[1:].to(self.device)
        # masked LM, Google-BERT pre-training format: a fixed number of masked
        # positions per sequence (max_predictions_per_seq = 15% of T rounded up
        # to 8: 80 at T = 512, 20 at T = 128) with their labels, so the MLM
        # head and loss run on those rows only
        T = self.seq_len
        P = max(8, ((int(round(0.15 * T)) + 7) // 8) * 8)
        ids = torch.randint(5, self.vocab, (B, T), generator=g)
        pos = torch.argsort(torch.rand((B, T), generator=g), dim=1)[:, :P].sort(dim=1).values
        labels = ids.gather(1, pos)
        ids = ids.scatter(1, pos, 4)  # [MASK]
        return ids.to(self.device), (pos.to(self.device), labels.to(self.device))

    def __iter__(self):
        return self

    def __next__(self):
        b = self._batches[self._i % len(self._batches)]
        self._i += 1
        return b

    def get_batch(self):
        return next(self)

    def seek(self, position: int) -> None:
        """Continue from batch ``position`` (a resumed run reads the batch the
        uninterrupted run would have read at that iteration)."""
        self._i = int(position)

    def num_samples(self) -> int:
        if self.train_samples is not None:
            return int(self.train_samples)
        if self.spec.kind == "tokens":
            return self.spec.train_samples // self.seq_len
        return self.spec.train_samples

    def test_batches(self, n: int = 2):
        return [self._batches[i % len(self._batches)] for i in range(n)]


def make_data(dataset: str, batch_size: int, device="cpu", **kw) -> SyntheticData:
    return SyntheticData(dataset, batch_size, device, **kw)
