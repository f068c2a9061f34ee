"""Probe: plain autocast vs bf16-shadow forward/backward on the GPU."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from gaussiank_sgd_amd.compression import compressors
from gaussiank_sgd_amd.models import resnet50
from gaussiank_sgd_amd.parallel import DistributedOptimizer, install_bf16_shadow

cuda = torch.device("cuda", 0)


def make(shadow, fused_bn=True):
    torch.manual_seed(0)
    net = resnet50(num_classes=10).to(cuda).to(memory_format=torch.channels_last)
    if not fused_bn:
        for m in net.modules():
            if hasattr(m, "fused"):
                m.fused = False
    opt = DistributedOptimizer(torch.optim.SGD(net.parameters(), lr=0.002, momentum=0.9),
                               named_parameters=net.named_parameters(), compression=compressors["none"])
    if shadow:
        install_bf16_shadow(net, opt)
    return net, opt


def run(net, opt):
    g = torch.Generator(device=cuda).manual_seed(1)
    x = torch.randn(16, 3, 64, 64, device=cuda, generator=g).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (16,), device=cuda, generator=g)
    opt.zero_grad()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = net(x)
        loss = torch.nn.functional.cross_entropy(out, y)
    loss.backward()
    opt.synchronize()
    return float(loss), out.float().detach(), opt.arena.grads.clone()


for fused in (True, False):
    res = {}
    for name, sh in (("A", False), ("A2", False), ("B", True), ("B2", True)):
        net, opt = make(sh, fused)
        res[name] = run(net, opt)
        if sh:
            print("shadow==cast", torch.equal(opt.arena.shadow, opt.arena.weights.to(torch.bfloat16)))
    for k in ("A2", "B", "B2"):
        la, oa, ga = res["A"]
        lb, ob, gb = res[k]
        print("fused_bn=%s A vs %s: loss %.6f %.6f  out rel %.3e  grad rel %.3e" % (
            fused, k, la, lb, float((oa - ob).norm() / oa.norm()), float((ga - gb).norm() / ga.norm())))
