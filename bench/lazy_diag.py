#!/usr/bin/env python3
"""Diagnostic: per-parameter error of fp32 ResNet-50 gradients against an fp64
run for several paths (fused plain / fused lazy BN backward, repeated with a
warm autotune cache, and plain torch fp32); prints the lazy autotune choices."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from gaussiank_sgd_amd.models.resnet_imagenet import resnet50  # noqa: E402
from gaussiank_sgd_amd.ops import conv1x1  # noqa: E402
from gaussiank_sgd_amd.ops.bn import BNAct  # noqa: E402

CL = torch.channels_last
torch.manual_seed(0)
m0 = resnet50(num_classes=10)
B, R = int(os.environ.get("DIAG_B", "8")), int(os.environ.get("DIAG_R", "96"))
x = torch.randn(B, 3, R, R)
t = torch.randint(0, 10, (B,))


def run(lazy, dtype=torch.float32, torch_only=False):
    os.environ["GKSGD_BN_LAZY"] = "1" if lazy else "0"
    os.environ["GKSGD_FASTCONV_F32"] = "0" if torch_only else "1"
    m = resnet50(num_classes=10)
    m.load_state_dict(m0.state_dict())
    if torch_only:
        for mod in m.modules():
            if isinstance(mod, BNAct):
                mod.fused = False
    m = m.to(device="cuda", dtype=dtype).to(memory_format=CL)
    xi = x.to(device="cuda", dtype=dtype).contiguous(memory_format=CL)
    F.cross_entropy(m(xi), t.cuda()).backward()
    torch.cuda.synchronize()
    return {n: p.grad.detach().double() for n, p in m.named_parameters()}


ref = run(False, torch.float64)
runs = {}
for name, kw in [("torch32", dict(lazy=False, torch_only=True)), ("plainA", dict(lazy=False)),
                 ("lazyA", dict(lazy=True)), ("plainB", dict(lazy=False)), ("lazyB", dict(lazy=True))]:
    runs[name] = run(**kw)
print("%-30s " % "param" + " ".join("%9s" % k for k in runs))
for n in ref:
    sc = ref[n].abs().max().item() + 1e-12
    errs = [(runs[k][n] - ref[n]).abs().max().item() / sc for k in runs]
    flag = " <<<" if max(errs[1:]) > 5 * errs[0] + 1e-4 else ""
    print("%-30s " % n + " ".join("%9.2e" % e for e in errs) + flag)
for k, v in conv1x1.tuned_choices().items():
    if k[-1] == "lz":
        print("choice", json.dumps(list(k)), v)
