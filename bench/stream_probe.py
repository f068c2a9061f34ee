#!/usr/bin/env python3
"""Per-step time + caching-allocator counters of bench.py's fp32 ResNet-50
step with the grad-weight side stream on/off (GKSGD_WGRAD_STREAM)."""
import importlib.util
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
spec = importlib.util.spec_from_file_location("gk_bench", os.path.join(ROOT, "bench.py"))
gb = importlib.util.module_from_spec(spec)
spec.loader.exec_module(gb)
import torch  # noqa: E402

sys.argv = [sys.argv[0]] + sys.argv[1:]
args = gb.parse()
if args.batch_size is None:
    args.batch_size = 512
from gaussiank_sgd_amd.parallel import comm  # noqa: E402

comm.init()
amp = "bf16" if args.amp == "bf16" else "fp32"
from gaussiank_sgd_amd import ops  # noqa: E402
assert ops.load()
torch.cuda.set_device(0)
if args.threshold is None:
    args.threshold = gb.DEFAULT_THRESHOLD.get(args.model, 524288000)
from gaussiank_sgd_amd.ops import conv1x1  # noqa: E402
conv1x1.set_f32_matmul(args.f32_matmul)
ph = gb.build(args, amp, False, args.threshold, 1, 0, args.batch_size)
trainer, opt = ph.trainer, ph.opt


def step():
    opt.zero_grad()
    trainer.train(1)
    trainer.update_model()


for _ in range(args.warmup):
    step()
torch.cuda.synchronize()
torch.cuda.reset_peak_memory_stats()
for i in range(args.steps):
    s0 = torch.cuda.memory_stats()
    t0 = time.perf_counter()
    step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    s1 = torch.cuda.memory_stats()
    print("step %d %.1f ms retries %d device_allocs %d reserved %.1f GB peak %.1f GB" % (
        i, dt * 1e3, s1.get("num_alloc_retries", 0) - s0.get("num_alloc_retries", 0),
        s1.get("num_device_alloc", 0) - s0.get("num_device_alloc", 0), s1["reserved_bytes.all.current"] / 2**30,
        s1["allocated_bytes.all.peak"] / 2**30), flush=True)
