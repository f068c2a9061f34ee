#!/usr/bin/env python3
"""Host-side AddressSanitizer / UBSan pass over the native extension.

GPU ASan is not available on this pool, so the sanitizers cover the HOST code
only: ``python -m gaussiank_sgd_amd.ops.build --asan`` builds build/asan/_C.so
with -fsanitize=address,undefined on the C++ bindings, the RCCL engine and
the host side of every .hip file.  This script loads that library into a
CPU-only python (run it with the ASan runtime preloaded, see below) and drives
every host path reachable without a GPU: schema registration, workspace-size
helpers, support predicates, argument validation, the RCCL engine's unique-id
bootstrap, watchdog start/stop and statistics.  Any sanitizer report aborts
the process with a non-zero exit.

  LD_PRELOAD="$(g++ -print-file-name=libasan.so) $(g++ -print-file-name=libstdc++.so)" \\
      ASAN_OPTIONS=detect_leaks=0 \\
      python scripts/asan_check.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "build", "asan", "_C.so")


def main() -> int:
    torch.ops.load_library(LIB)
    o = torch.ops.gksgd
    checks = 0
    assert o.ctrl_bytes() > 0 and o.workspace_bytes() > 0 and o.sign_bucket_workspace_bytes() > 0
    for M, C, eb in ((512 * 56 * 56, 256, 2), (7, 64, 4), (1, 2048, 2)):
        assert o.bn_workspace_floats(M, C, eb) > 0
        o.bn_supported(C, eb)
        assert o.bn_mask_bytes(M, C, eb) >= 0
        checks += 3
    for N, K in ((64, 64), (256, 2304), (1000, 2048), (65, 7)):
        o.gemm_supported(N, K)
        checks += 1
    for H in (768, 1024, 100):
        o.add_ln_supported(H)
        if o.add_ln_supported(H):
            assert o.add_ln_ws_floats(4096, H) > 0
        checks += 1
    # argument validation paths: CPU tensors are rejected before any device work
    t = torch.zeros(16)
    for fn, args in ((o.fill_zero, (t,)), (o.cast_bf16, (t.bfloat16(), t)), (o.accum_grad, (t, t))):
        try:
            fn(*args)
        except RuntimeError:
            checks += 1
    # RCCL engine host paths (no communicator: no GPU here)
    E = torch.classes.gksgd.RcclEngine
    uid = E.unique_id()
    assert uid.numel() == 128 and uid.dtype == torch.uint8
    e = E()
    assert e.poll() == 0 and not e.failed() and e.in_flight() == 0
    e.reset_stats()
    assert e.stats(0) == [0.0, 0.0, 0.0, 0.0]
    e.start_watchdog(1.0, 1.0)
    e.stop_watchdog()
    e.check()
    try:
        e.allgather(torch.zeros(4, dtype=torch.int32), torch.zeros(4, dtype=torch.int32))
    except RuntimeError:
        checks += 1
    e.destroy()
    checks += 8
    print("asan host check: %d checks passed, no sanitizer reports (%s)" % (checks, LIB))
    return 0


if __name__ == "__main__":
    sys.exit(main())
