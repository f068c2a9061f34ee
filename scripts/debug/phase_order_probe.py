#!/usr/bin/env python3
"""Does a small-batch fp32 phase slow a later bf16 bs512 phase in the same
process?  (round 4: bench.py's bf16 phase ran 57.8 ms/step after the bs32
phases, 41.0 ms right after the headline.)  Times bf16 bs512, then fp32 bs32,
then bf16 bs512 again, each in a fresh trainer, and prints the three
ms/step.  usage: python scripts/debug/phase_order_probe.py [--order b,s,b]"""
import argparse
import importlib.util
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--order", default="b,s,b", help="b: bf16 bs512, s: fp32 bs32 sparse, d: fp32 bs32 dense, f: fp32 bs512")
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    spec = importlib.util.spec_from_file_location("gk_bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    args.batch_size = 512
    args.threshold = 524288000
    import torch
    from gaussiank_sgd_amd import ops
    from gaussiank_sgd_amd.parallel import comm
    torch.cuda.set_device(0)
    comm.init()
    assert ops.load()
    res = []
    for tag in a.order.split(","):
        amp, bs, dense, thr = {"b": ("bf16", 512, False, 524288000), "s": ("fp32", 32, False, 524288000),
                               "d": ("fp32", 32, True, 6250000), "f": ("fp32", 512, False, 524288000)}[tag]
        ph = bench.build(args, amp, dense, thr, 1, 0, bs)
        el, _ = bench.run_phase(args, ph, a.steps, 3, 1)
        res.append((tag, round(el / a.steps * 1e3, 3)))
        print("phase", tag, res[-1][1], "ms/step", flush=True)
        bench.release(ph)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
