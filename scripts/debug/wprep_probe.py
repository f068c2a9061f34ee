#!/usr/bin/env python3
"""Which per-step weight re-layouts a ResNet-50 step registers (ops/weight_prep.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    from gaussiank_sgd_amd.ops import conv1x1
    from gaussiank_sgd_amd.ops import weight_prep as wpm
    from gaussiank_sgd_amd.train import DLTrainer
    bs = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    calls = {"fwd": 0, "wp": 0}
    orig = conv1x1._fwd

    def spy(x, w, s, stats_box=None, bias=None, wp=False):
        calls["fwd"] += 1
        calls["wp"] += int(bool(wp))
        return orig(x, w, s, stats_box, bias, wp=wp)
    conv1x1._fwd = spy
    t = DLTrainer(0, 1, dnn="resnet50", dataset="imagenet", batch_size=bs, lr=0.1, device="cuda",
                  channels_last=True, seed=0, data_pool=1)
    p0 = next(t.net.parameters())
    print("enabled", wpm.ENABLED, "param CL", p0.is_contiguous(memory_format=torch.channels_last), flush=True)
    for i in range(3):
        t.optimizer.zero_grad()
        t.train(1)
        t.optimizer.step()
        torch.cuda.synchronize()
        kinds = {}
        for k in t.weight_prep.entries:
            kinds[k[0]] = kinds.get(k[0], 0) + 1
        print("step", i, "fwd calls", calls, "entries", kinds, "launches", t.weight_prep.launches, flush=True)
    ch = {}
    for k, v in conv1x1.tuned_choices().items():
        ch[(k[0], v[0])] = ch.get((k[0], v[0]), 0) + 1
    print("choices", ch, flush=True)


if __name__ == "__main__":
    main()
