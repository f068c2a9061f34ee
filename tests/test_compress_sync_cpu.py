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
