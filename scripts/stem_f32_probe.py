#!/usr/bin/env python3
"""Runs the fp32 stem kernels (forward with statistics, grad-weight) a few
times at ResNet-50 bs512 shapes -- a short program for rocprofv3 --pmc passes
(scripts/gpurun/stem_counters.sh).  usage: python scripts/stem_f32_probe.py [N] [iters] [fwd|wgrad|both]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gaussiank_sgd_amd import ops  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 512
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
which = sys.argv[3] if len(sys.argv) > 3 else "both"
assert torch.cuda.is_available() and ops.load()
g = torch.ops.gksgd
CL = torch.channels_last
x = torch.randn(N, 3, 224, 224, device="cuda").contiguous(memory_format=CL)
w = torch.randn(64, 3, 7, 7, device="cuda") * 0.1
y = torch.empty(N, 64, 112, 112, device="cuda").contiguous(memory_format=CL)
st = torch.empty(2, 512, 64, device="cuda")
dw = torch.zeros(64, 3, 7, 7, device="cuda")
part = torch.empty(int(g.stem_f32_wgrad_ws(N)), device="cuda")
for _ in range(iters):
    if which in ("fwd", "both"):
        g.stem_f32_fwd(x, w, y, st)
    if which in ("wgrad", "both"):
        g.stem_f32_wgrad(x, y, dw, part)
torch.cuda.synchronize()
print("ok", float(dw.abs().sum()))
