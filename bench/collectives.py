#!/usr/bin/env python3
"""Collective latency / bandwidth curves for the sparse exchange.

Sweeps the packed-record all-gather (what every Gaussian-k bucket sends:
4 + 2*k_cap int32 words per rank) and the dense all-reduce (comparator) over
payload sizes, for the native RCCL engine (own ncclComm_t on the caller's
stream) and torch.distributed.  One process per GPU:

  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench/collectives.py
  (CPU plumbing check: --cpu, gloo backend)

Rank 0 prints one line per (op, engine, size): latency (us), algorithm
bandwidth (payload / time) and bus bandwidth (ring-equivalent bytes / time).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from gaussiank_sgd_amd.parallel import comm  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--json-out", default=None)
    args = ap.parse_args()
    dev = torch.device("cpu")
    if not args.cpu:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dev = torch.device("cuda", torch.cuda.current_device())
    comm.init(device="cpu" if args.cpu else None)
    P, rank = comm.size(), comm.rank()
    engines = [("torch", comm.Exchanger(dev, prefer_native=False))]
    if dev.type == "cuda" and P > 1:
        ex = comm.Exchanger(dev, prefer_native=True)
        if ex.kind == "rccl-native":
            engines.insert(0, ("rccl-native", ex))

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    rows = []
    ks = [256, 2_556, 25_557, 255_570, 2_555_703]   # ResNet-50 k at densities 1e-5 .. 0.1
    dense = [1 << 16, 1 << 20, 1 << 22, 25_557_032]
    for name, ex in engines:
        for k in ks:
            words = 4 + 2 * 2 * k   # k_cap = 2k
            inp = torch.zeros(words, dtype=torch.int32, device=dev)
            out = torch.zeros(P * words, dtype=torch.int32, device=dev)
            for _ in range(5):
                ex.allgather_(out, inp)
            sync()
            comm.barrier()
            t0 = time.perf_counter()
            for _ in range(args.iters):
                ex.allgather_(out, inp)
            sync()
            dt = (time.perf_counter() - t0) / args.iters
            nbytes = words * 4
            rows.append(dict(op="allgather_record", engine=name, P=P, k=k, bytes_per_rank=nbytes,
                             us=round(dt * 1e6, 1), algbw_GBs=round(P * nbytes / dt / 1e9, 2),
                             busbw_GBs=round((P - 1) * nbytes / dt / 1e9, 2)))
        for n in dense:
            t = torch.zeros(n, dtype=torch.float32, device=dev)
            for _ in range(3):
                ex.allreduce_(t, average=True)
            sync()
            comm.barrier()
            t0 = time.perf_counter()
            it = max(5, args.iters // 5)
            for _ in range(it):
                ex.allreduce_(t, average=True)
            sync()
            dt = (time.perf_counter() - t0) / it
            nbytes = n * 4
            rows.append(dict(op="allreduce_dense", engine=name, P=P, n=n, bytes=nbytes, us=round(dt * 1e6, 1),
                             algbw_GBs=round(nbytes / dt / 1e9, 2),
                             busbw_GBs=round(2 * (P - 1) / max(P, 1) * nbytes / dt / 1e9, 2)))
    if rank == 0:
        for r in rows:
            print(json.dumps(r), flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                json.dump(rows, f, indent=1)
    for _, ex in engines:
        ex.close()
    comm.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
