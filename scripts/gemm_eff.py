#!/usr/bin/env python3
"""Per-shape efficiency table from an autotuner dump (bench.py with
GKSGD_GEMM_RETUNE=1 GKSGD_GEMM_DUMP=path): for every conv / linear GEMM key,
the chosen candidate, its measured time and the achieved TFLOP/s (direct
convolution FLOPs, so Winograd rows may exceed the MFMA peak).

usage: python scripts/gemm_eff.py DUMP.json [--batch N] [--dtype f32|bf16]"""
import argparse
import json


def flops(key):
    kind = key[0]
    if kind in ("fwd", "dgrad", "dgrad_bn", "wgrad"):
        N, C, H, W, K, k, s = key[1:8]
        OH, OW = (H + s - 1) // s, (W + s - 1) // s
        return 2.0 * N * OH * OW * C * K * k * k
    if kind in ("lin_fwd", "lin_dgrad", "lin_wgrad"):
        M, K, N = key[1:4]
        return 2.0 * M * K * N
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dump")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--dtype", default=None, help="f32 or bf16")
    a = ap.parse_args()
    rows = []
    for key, choice, log in json.load(open(a.dump)):
        f = flops(key)
        if f is None or not log:
            continue
        if a.batch is not None and key[0] != "lin_fwd" and key[1] != a.batch:
            continue
        is32 = "f32" in key
        if a.dtype == "f32" and not is32 or a.dtype == "bf16" and is32:
            continue
        times = [t for tag, t in log if isinstance(t, (int, float)) and list(tag) == list(choice)]
        if not times:
            times = [t for _, t in log if isinstance(t, (int, float))]
        if not times:
            continue
        ms = min(times)
        rows.append((ms, key, choice, f / (ms * 1e-3) / 1e12))
    rows.sort(key=lambda r: -r[0])
    tot = sum(r[0] for r in rows)
    print("total %.3f ms over %d keys (one call each)" % (tot, len(rows)))
    print("%9s %7s  %-48s %s" % ("ms", "TF/s", "key", "choice"))
    for ms, key, choice, tf in rows:
        print("%9.4f %7.1f  %-48s %s" % (ms, tf, ",".join(str(x) for x in key), choice))


if __name__ == "__main__":
    main()
