"""Fused residual-add + dropout + LayerNorm (ops/ln.py) at BERT-base's shape
(32 x 512 rows of 768, p = 0.1): forward / backward microseconds per call and
the achieved bandwidth (forward moves 4 row tensors, backward 4 + the
column partials), against the unfused PyTorch composition.

    python bench/ln_probe.py [--rows 16384] [--hidden 768] [--p 0.1]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gaussiank_sgd_amd import ops  # noqa: E402
from gaussiank_sgd_amd.ops.ln import add_layernorm  # noqa: E402


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
    ap.add_argument("--rows", type=int, default=16384)
    ap.add_argument("--hidden", type=int, default=768)
    ap.add_argument("--p", type=float, default=0.1)
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    assert ops.load(), ops._load_error
    R, H, p = a.rows, a.hidden, a.p
    ln = torch.nn.LayerNorm(H).cuda()
    x = torch.randn(R, H, device="cuda").to(torch.bfloat16).requires_grad_(True)
    y = torch.randn(R, H, device="cuda").to(torch.bfloat16).requires_grad_(True)
    dy = torch.randn(R, H, device="cuda").to(torch.bfloat16)
    mb = R * H * 2 / 1e6
    res = {"rows": R, "hidden": H, "p": p}

    def fused_f():
        with torch.no_grad():
            add_layernorm(y, x, ln, p, True)

    def fused_fb():
        add_layernorm(y, x, ln, p, True).backward(dy)

    def eager_f():
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            ln(x + torch.nn.functional.dropout(y, p))

    def eager_fb():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = ln(x + torch.nn.functional.dropout(y, p))
        out.backward(dy.float())

    for name, f, fb in [("fused", fused_f, fused_fb), ("torch", eager_f, eager_fb)]:
        tf, tfb = timeit(f), timeit(fb)
        res[name] = {"fwd_us": round(tf, 1), "bwd_us": round(tfb - tf, 1),
                     "fwd_TBps": round(4 * mb / tf, 2), "bwd_TBps": round(4 * mb / max(tfb - tf, 1e-3), 2)}
    print(json.dumps(res))
    if a.json_out:
        with open(a.json_out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
