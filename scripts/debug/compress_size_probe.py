#!/usr/bin/env python3
"""Fixed vs per-element cost of the compression kernels: run the Gaussian-k
pipeline (EC, k_cap = 4k/3, training-like inputs) on buckets of several sizes
so a kernel trace (rocprofv3 --kernel-trace) separates each kernel's
launch + single-workgroup tail from its streaming part.
usage: rocprofv3 --kernel-trace -d out -- python3 scripts/debug/compress_size_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    from gaussiank_sgd_amd import ops
    from gaussiank_sgd_amd.utils.stats import gaussian_z
    assert ops.load(), ops._load_error
    dev = torch.device("cuda", 0)
    for n in (1 << 20, 1 << 22, 1 << 24, 25_557_032):
        k = max(n // 1000, 1)
        kc = (4 * k + 2) // 3
        bufs = ops.CompressBuffers(kc, dev)
        g = torch.empty(n, device=dev)
        r = torch.zeros(n, device=dev)
        pool = [torch.randn(n, device=dev) * 1e-3 * (1 + 0.1 * i) for i in range(4)]
        for it in range(40):
            g.copy_(pool[it % 4])
            ops.compress_(g, r, bufs, ops.MODE_GAUSSIAN, ec=True, zero_g=True, loops=3, z=gaussian_z(0.001), k=k,
                          k_cap=kc, seed=7, n_stats=n)
        torch.cuda.synchronize()
        print("n=%d done" % n, flush=True)


if __name__ == "__main__":
    main()
