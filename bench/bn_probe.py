"""Streaming BatchNorm passes (ops/csrc/kernels/bn_act.hip) at ResNet-50
bs512 activation shapes: microseconds and achieved HBM bandwidth of

  fwd      stats + finalize + apply(+residual)(+ReLU mask)   (bn_act_forward)
  fwd_pre  finalize + apply from producer partials            (epilogue statistics)
  fwd_res_pre  the same + residual add (block output BN)
  bwd_pre  finalize + apply from the grad-input epilogue's partials
  bwd      reduce + finalize + apply (twin + residual: block output)

for each workgroup count in --blocks (bn_set_blocks), so the streaming grid can
be picked from measurements.  Bytes: the tensors each pass must move (--dtype bf16 | f32),
the mask / partials ignored.

    python bench/bn_probe.py [--batch 512] [--blocks 1024,2048,4096]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gaussiank_sgd_amd import ops  # noqa: E402

# (H, C): bottleneck BN shapes of ResNet-50 (bn1/bn2 width C, bn3 / block output 4C)
SHAPES = [(56, 64), (56, 256), (28, 128), (28, 512), (14, 256), (14, 1024), (7, 512), (7, 2048)]


def timeit(fn, iters=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--blocks", default="1024,2048,4096")
    ap.add_argument("--json-out", default="")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    a = ap.parse_args()
    dt = torch.float32 if a.dtype == "f32" else torch.bfloat16
    eb = 4 if a.dtype == "f32" else 2
    assert ops.load(), ops._load_error
    g = torch.ops.gksgd
    dev = torch.device("cuda", 0)
    out = {"batch": a.batch, "dtype": a.dtype, "rows": []}
    for H, C in SHAPES:
        M = a.batch * H * H
        x = torch.randn(M, C, device=dev).to(dt)
        res = torch.randn(M, C, device=dev).to(dt)
        y = torch.empty_like(x)
        dz = torch.randn(M, C, device=dev).to(dt)
        dx = torch.empty_like(x)
        dres = torch.empty_like(x)
        mask = torch.empty(g.bn_mask_bytes(M, C, eb), dtype=torch.uint8, device=dev)
        ws = torch.empty(g.bn_workspace_floats(M, C, eb), dtype=torch.float32, device=dev)
        w = torch.ones(C, device=dev)
        b = torch.zeros(C, device=dev)
        st = [torch.zeros(C, device=dev) for _ in range(4)]
        gg = [torch.zeros(C, device=dev) for _ in range(2)]
        part = torch.randn(2, 256, C, device=dev)
        mb = M * C * eb / 1e6
        for nb in [int(v) for v in a.blocks.split(",")]:
            g.bn_set_blocks(nb)

            def fwd():
                g.bn_act_forward(x, res, y, mask, w, b, None, None, st[0], st[1], st[2], st[3], ws, 1e-5, 0.1, True)

            def fwd_pre():
                g.bn_act_forward(x, None, y, mask, w, b, None, None, st[0], st[1], st[2], st[3], ws, 1e-5, 0.1, True,
                                 None, part, 256)

            def fwd_res_pre():
                g.bn_act_forward(x, res, y, mask, w, b, None, None, st[0], st[1], st[2], st[3], ws, 1e-5, 0.1, True,
                                 None, part, 256)

            def fwd_pre_norelu():
                g.bn_act_forward(x, None, y, mask, w, b, None, None, st[0], st[1], st[2], st[3], ws, 1e-5, 0.1, False,
                                 None, part, 256)

            def copy():
                y.copy_(x)

            def bwd_pre():
                g.bn_act_backward_pre(dz, x, dx, w, st[0], st[1], gg[0], gg[1], part, 256, None, None)

            def bwd():
                g.bn_act_backward(dz, mask, x, dx, dres, w, st[0], st[1], gg[0], gg[1], ws, True, None, None, res)

            fwd()   # valid statistics for the backward passes
            row = {"H": H, "C": C, "blocks": nb}
            # tensor passes: fwd reads x twice (stats, apply) + res, writes y: 4;
            # fwd_pre 2; bwd_pre reads dz, x, writes dx: 3; bwd reduce reads dy, dy2, x,
            # writes dz; apply reads dz, x, writes dx: 7
            for name, fn, passes in (("fwd", fwd, 4), ("fwd_pre", fwd_pre, 2), ("fwd_pre_norelu", fwd_pre_norelu, 2), ("copy", copy, 2), ("fwd_res_pre", fwd_res_pre, 3), ("bwd_pre", bwd_pre, 3), ("bwd", bwd, 7)):
                us = timeit(fn)
                row[name + "_us"] = round(us, 1)
                row[name + "_TBs"] = round(passes * mb / us, 3)
            out["rows"].append(row)
            print(json.dumps(row), flush=True)
    g.bn_set_blocks(1024)
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
