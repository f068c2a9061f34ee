"""Instruction mix of the kernels in a hipcc ``-S`` (gfx950) assembly file:
MFMA / VALU / transcendental / SALU / LDS / VMEM counts per kernel and for
its innermost loop (the largest basic-block range closed by a backward
``s_cbranch``), to price a kernel's VALU work against its MFMA work.

    hipcc --offload-arch=gfx950 -O3 --cuda-device-only -S k.hip -o k.s
    python scripts/isa_mix.py k.s [name-filter]
"""
import re
import sys
from collections import Counter


def classify(op: str) -> str:
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("v_exp", "v_log", "v_rcp", "v_sqrt", "v_rsq")):
        return "trans"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt") or op.startswith("s_barrier"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    return "other"


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    lines = open(path).read().split("\n")
    kernels = []
    for i, l in enumerate(lines):
        m = re.match(r"^([A-Za-z_][\w.$]*):\s*(;.*)?$", l)
        if m and not m.group(1).startswith(".") and "@" in (m.group(2) or ""):
            kernels.append((m.group(1), i))
    for kname, start in kernels:
        if filt not in kname:
            continue
        end = next((j for j in range(start, len(lines)) if lines[j].startswith(".Lfunc_end")), len(lines))
        body = lines[start + 1:end]
        labels = {}
        ins = []
        for l in body:
            s = l.split(";")[0].strip()
            if not s or s.startswith("//"):
                continue
            if s.endswith(":"):
                labels[s[:-1]] = len(ins)
                continue
            if s.startswith("."):
                continue
            ins.append(s.split()[0] + (" " + s.split()[1] if len(s.split()) > 1 else ""))
        tot = Counter(classify(i.split()[0]) for i in ins)
        # innermost hot loop: the longest backward-branch range
        best = None
        for k, i in enumerate(ins):
            op = i.split()
            if op[0].startswith("s_cbranch") or op[0] == "s_branch":
                tgt = op[1] if len(op) > 1 else ""
                if tgt in labels and labels[tgt] <= k:
                    rng = (labels[tgt], k)
                    if best is None or rng[1] - rng[0] > best[1] - best[0]:
                        best = rng
        print(kname)
        print("  kernel:", dict(tot), "total", len(ins))
        if best:
            loop = Counter(classify(i.split()[0]) for i in ins[best[0]:best[1] + 1])
            print("  loop  :", dict(loop), "total", best[1] - best[0] + 1)


if __name__ == "__main__":
    main()
