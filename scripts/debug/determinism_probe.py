"""Probe: is a ResNet-50 forward/backward bitwise repeatable on this GPU?
Runs the same model twice on the same input and reports the first module
whose output differs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from gaussiank_sgd_amd.models import resnet50  # noqa: E402

cuda = torch.device("cuda", 0)


def capture(net, x, amp):
    outs = {}
    hooks = []
    for name, m in net.named_modules():
        if len(list(m.children())) == 0:
            def h(mod, inp, out, name=name):
                o = out[0] if isinstance(out, tuple) else out
                outs[name] = o.detach().float().clone()
            hooks.append(m.register_forward_hook(h))
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
        y = net(x)
    y.float().sum().backward()
    for hk in hooks:
        hk.remove()
    grads = torch.cat([p.grad.reshape(-1).float() for p in net.parameters()])
    for p in net.parameters():
        p.grad = None
    return outs, y.detach().float(), grads


for fused in (True, False):
    for amp in (True, False):
        torch.manual_seed(0)
        net = resnet50(num_classes=10).to(cuda).to(memory_format=torch.channels_last)
        for m in net.modules():
            if hasattr(m, "fused"):
                m.fused = fused
        g = torch.Generator(device=cuda).manual_seed(1)
        x = torch.randn(16, 3, 64, 64, device=cuda, generator=g).contiguous(memory_format=torch.channels_last)
        o1, y1, g1 = capture(net, x, amp)
        o2, y2, g2 = capture(net, x, amp)
        first = None
        for name in o1:
            if not torch.equal(o1[name], o2[name]):
                first = (name, float((o1[name] - o2[name]).abs().max()), float(o1[name].abs().max()))
                break
        print("fused=%s amp=%s out_equal=%s grad_rel=%.3e first_diff=%s" % (
            fused, amp, torch.equal(y1, y2), float((g1 - g2).norm() / g1.norm()), first), flush=True)
