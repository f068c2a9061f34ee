"""bf16 shadow weights + direct arena gradients vs plain autocast.

Both paths round the fp32 master weights to bf16 with round-to-nearest-even,
run the same bf16 convolutions and add the same bf16 gradients into fp32, so
the trajectories must agree to within MIOpen's run-to-run noise.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _make(cuda, shadow, compressor):
    from gaussiank_sgd_amd.compression import compressors
    from gaussiank_sgd_amd.models import resnet50
    from gaussiank_sgd_amd.parallel import DistributedOptimizer, install_bf16_shadow
    torch.manual_seed(0)
    net = resnet50(num_classes=10).to(cuda).to(memory_format=torch.channels_last)
    base = torch.optim.SGD(net.parameters(), lr=0.002, momentum=0.9, weight_decay=1e-4)
    opt = DistributedOptimizer(base, named_parameters=net.named_parameters(), compression=compressors[compressor],
                               is_sparse=compressor != "none", density=0.01, compress_single_rank=True,
                               density_warmup=False)
    n = install_bf16_shadow(net, opt) if shadow else 0
    return net, opt, n


def _grads(net, opt, cuda):
    g = torch.Generator(device=cuda).manual_seed(1)
    x = torch.randn(16, 3, 64, 64, device=cuda, generator=g).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (16,), device=cuda, generator=g)
    opt.zero_grad()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = torch.nn.functional.cross_entropy(net(x), y)
    loss.backward()
    opt.synchronize()
    grads = opt.arena.grads.clone()
    opt.step()
    return float(loss), grads


def _rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.parametrize("compressor", ["none", "gaussian"])
def test_shadow_matches_autocast(cuda, compressor):
    """MIOpen's split-K weight-gradient kernels accumulate with atomics, so two
    identical plain-autocast runs already differ slightly; the shadow path must
    stay within a small multiple of that run-to-run noise."""
    runs = []
    for shadow in (False, False, True):
        net, opt, n = _make(cuda, shadow, compressor)
        loss, grads = _grads(net, opt, cuda)
        runs.append((loss, grads, opt))
    (la, ga, oa), (la2, ga2, _), (lb, gb, ob) = runs
    assert n == sum(1 for _ in net.parameters())
    assert la == pytest.approx(lb, rel=1e-3)
    noise = _rel(ga2, ga)
    err = _rel(gb, ga)
    assert err <= 3 * noise + 2e-3, (err, noise)
    # the shadow tracks the master weights exactly (RNE cast in the SGD kernel)
    assert torch.equal(ob.arena.shadow, ob.arena.weights.to(torch.bfloat16))


def test_shadow_refresh_on_load_state_dict(cuda):
    net, opt, _ = _make(cuda, True, "none")
    sd = {k: v.clone() for k, v in net.state_dict().items()}
    for v in sd.values():
        if v.is_floating_point():
            v.add_(0.5)
    net.load_state_dict(sd)
    assert torch.equal(opt.arena.shadow, opt.arena.weights.to(torch.bfloat16))
