"""Two-level arrival counters of the compression hand-offs (compress.hip
arrive(): kSyncSub sub-counters, block b counts in at sub b % nsub, the last
arrival at a sub counts in at the top counter): a Python mirror of the
expected-count arithmetic, replayed over random arrival orders.  Exactly one
block -- the last to arrive -- is told it is last, and every counter is back
at zero afterwards (the counters are reused by the next kernel, and by the
fused fallback's grid barriers within one kernel)."""
import random

import pytest

K_SYNC_SUB = 32


def arrive(counters, G, bid):
    nsub = G if G < K_SYNC_SUB else K_SYNC_SUB
    j = bid % nsub
    expect = (G - j + nsub - 1) // nsub
    prev = counters["sub"][j]
    counters["sub"][j] += 1
    if prev == expect - 1:
        counters["sub"][j] = 0
        p2 = counters["top"]
        counters["top"] += 1
        if p2 == nsub - 1:
            counters["top"] = 0
            return True
    return False


@pytest.mark.parametrize("G", [1, 2, 7, 31, 32, 33, 63, 64, 65, 512, 893, 1024, 2048])
def test_exactly_the_last_arrival_is_last(G):
    rng = random.Random(G)
    counters = {"sub": [0] * K_SYNC_SUB, "top": 0}
    for rep in range(5):   # counters reused call after call
        order = list(range(G))
        rng.shuffle(order)
        lasts = [i for i, b in enumerate(order) if arrive(counters, G, b)]
        assert lasts == [G - 1], (G, rep, lasts)
        assert counters["top"] == 0 and not any(counters["sub"])


def test_ctrl_sync_timeouts_offset_matches_header():
    """ops.CTRL_SYNC_TIMEOUTS_U32 is the word the kernels count expired
    bounded spins into (GkCtrl::sync_timeouts, static_assert in gk_kernels.h);
    a fresh control block reports none."""
    import os
    import re
    from gaussiank_sgd_amd import ops
    hdr = os.path.join(os.path.dirname(ops.__file__), "csrc", "kernels", "gk_kernels.h")
    m = re.search(r"offsetof\(GkCtrl, sync_timeouts\) == (\d+)", open(hdr).read())
    assert m and int(m.group(1)) == ops.CTRL_SYNC_TIMEOUTS_U32 * 4
    b = ops.CompressBuffers(8, "cpu")
    assert ops.sync_timeouts(b) == 0 and ops.ctrl_fields(b)["sync_timeouts"] == 0
