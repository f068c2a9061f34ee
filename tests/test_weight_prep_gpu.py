"""Batched per-step weight re-layouts (prep.hip / ops/weight_prep.py) against
the per-call builders they replace: Winograd filter transforms (forward and
flipped grad-input), 1x1 grad-input transposes and per-tap 3x3 flip-
transposes, fp32 and bf16; rebuilt from the CURRENT weights at every step
scope; and a ResNet-50 training step identical with and without batching."""
import pytest
import torch

from gaussiank_sgd_amd import ops
from gaussiank_sgd_amd.ops import weight_prep as wpm

pytestmark = pytest.mark.gpu
CL = torch.channels_last


def _refs(w3, w1, w3b, w1b):
    g = torch.ops.gksgd
    u0 = torch.empty(16 * w3.shape[0] * w3.shape[1], device=w3.device)
    u1 = torch.empty_like(u0)
    g.wino_weights(w3, u0, False)
    g.wino_weights(w3, u1, True)
    t1 = w1.reshape(w1.shape[0], -1).t().contiguous()
    t1b = w1b.reshape(w1b.shape[0], -1).t().contiguous()
    f3 = w3.flip(2, 3).transpose(0, 1).contiguous(memory_format=CL)
    f3b = w3b.flip(2, 3).transpose(0, 1).contiguous(memory_format=CL)
    return u0, u1, t1, t1b, f3, f3b


def _acquire_all(w3, w1, w3b, w1b):
    return (wpm.wino_filter(w3, False, True), wpm.wino_filter(w3, True, True), wpm.transposed_1x1(w1, True),
            wpm.transposed_1x1(w1b, True), wpm.flipped_3x3(w3, True), wpm.flipped_3x3(w3b, True))


@pytest.mark.parametrize("K,C", [(64, 64), (128, 256), (192, 128)])
def test_batched_relayouts_match_per_call_builders(K, C):
    assert ops.load()
    torch.manual_seed(0)
    dev = torch.device("cuda")
    w3 = torch.randn(K, C, 3, 3, device=dev).contiguous(memory_format=CL)
    w1 = torch.randn(K, C, 1, 1, device=dev)
    w3b = torch.randn(K, C, 3, 3, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
    w1b = torch.randn(K, C, 1, 1, device=dev).to(torch.bfloat16)
    prep = wpm.WeightPrep()
    with prep.step(dev):                        # first step: built per call, registered
        first = [t.clone() for t in _acquire_all(w3, w1, w3b, w1b)]
    assert prep.launches == 0 and len(prep.entries) == 6
    for t, r in zip(first, _refs(w3, w1, w3b, w1b)):
        assert torch.equal(t, r)
    for it in range(2):                         # later steps: ONE batched launch from the current weights
        with torch.no_grad():
            for t in (w3, w1, w3b, w1b):
                t.mul_(-0.5).add_(0.25)
        with prep.step(dev):
            got = _acquire_all(w3, w1, w3b, w1b)
            torch.cuda.synchronize()
            for t, r in zip(got, _refs(w3, w1, w3b, w1b)):
                assert torch.allclose(t.float(), r.float(), rtol=1e-6, atol=1e-6)
        assert prep.launches == it + 1
    # outside a scope nothing is cached
    assert wpm.current() is None


def test_transposes_ragged_tiles():
    """Transposes of shapes that are not multiples of the 64 x 64 tile."""
    torch.manual_seed(1)
    dev = torch.device("cuda")
    K, C = 100, 72
    ws = [torch.randn(K, C, 1, 1, device=dev), torch.randn(K, C, 1, 1, device=dev).to(torch.bfloat16)]
    w3 = [torch.randn(K, C, 3, 3, device=dev).contiguous(memory_format=CL),
          torch.randn(K, C, 3, 3, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)]
    prep = wpm.WeightPrep()
    for _ in range(2):
        with prep.step(dev):
            got = [wpm.transposed_1x1(w, True) for w in ws] + [wpm.flipped_3x3(w, True) for w in w3]
            torch.cuda.synchronize()
            ref = [w.reshape(K, C).t().contiguous() for w in ws] + \
                [w.flip(2, 3).transpose(0, 1).contiguous(memory_format=CL) for w in w3]
            for a, b in zip(got, ref):
                assert torch.equal(a, b)
    assert prep.launches == 1


@pytest.mark.parametrize("force", ["hip", "wino"])
def test_resnet50_step_same_with_and_without_batching(monkeypatch, force):
    """Three ResNet-50 training steps with every re-layout built per call and
    with the batched per-step launch give the same weights.  The kernel
    families are forced (fresh autotuner table) so the re-layouts the test
    needs are the ones registered: "hip" -> 1x1 transposes + 3x3 flips,
    "wino" -> Winograd filter transforms."""
    from gaussiank_sgd_amd.ops import conv1x1
    from gaussiank_sgd_amd.train import DLTrainer
    monkeypatch.setattr(conv1x1, "_choices", {})
    monkeypatch.setattr(conv1x1, "_FORCE", force)

    def run(enabled):
        monkeypatch.setattr(wpm, "ENABLED", enabled)
        t = DLTrainer(0, 1, dnn="resnet50", dataset="imagenet", batch_size=4, lr=0.1, device="cuda",
                      channels_last=True, seed=0, data_pool=1)
        for _ in range(3):
            t.optimizer.zero_grad()
            t.train(1)
            t.optimizer.step()
        torch.cuda.synchronize()
        return t, torch.cat([p.detach().flatten() for p in t.net.parameters()])
    t0, ref = run(False)
    t1, got = run(True)
    kinds = {k[0] for k in t1.weight_prep.entries}
    assert t0.weight_prep.launches == 0 and t1.weight_prep.launches == 2, t1.weight_prep.launches
    assert kinds >= ({"t1", "f3"} if force == "hip" else {"wino0", "wino1"}), kinds
    assert torch.allclose(got, ref, rtol=1e-5, atol=1e-6)
