"""Diagnose reduce_records mismatches vs the CPU mirror (prints the first few)."""
import sys
import torch
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from test_kernels2_gpu import _records  # noqa: E402
from gaussiank_sgd_amd import ops  # noqa: E402

for P in (2, 3, 4):
    n, k_cap = 300_000, 6000
    counts = [1000 + (997 * p) % 5000 for p in range(P)]
    recs, per_rank = _records(P, k_cap, counts, 40_000, seed=P)
    dst = torch.randn(n) * 0.01
    want = dst.clone()
    ops.scatter_add_records_(want, recs, P, k_cap, 1.0 / P, True)
    got = dst.cuda()
    ops.scatter_add_records_(got, recs.cuda(), P, k_cap, 1.0 / P, True)
    got = got.cpu()
    bad = (got != want).nonzero().view(-1)
    print("P", P, "mismatches", bad.numel())
    maps = [dict(zip(i.tolist(), v.tolist())) for i, v in per_rank]
    for key in bad[:6].tolist():
        mem = [(q, maps[q].get(key)) for q in range(P) if key in maps[q]]
        print("  key", key, "dst0 %.9g want %.9g got %.9g" % (dst[key], want[key], got[key]), "members", mem,
              "got-dst %.9g" % (got[key] - dst[key]))
