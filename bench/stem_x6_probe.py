"""Times the fp32 stem forward kernels at the headline shape (bs128 x 224^2):
stem_f32_fwd (fp32 MFMA) vs stem_f32x6_fwd (bf16x6 products; occupancy variant
from GKSGD_STEM_X6_OCC) and the grad-weight stem_f32_wgrad fp32 MFMA vs
bf16x6. Prints one JSON line."""
import json
import os

import torch

from gaussiank_sgd_amd import ops


def _time(fn, iters=50):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    assert ops.load(), ops._load_error
    g = torch.ops.gksgd
    N = int(os.environ.get("N", "128"))
    x = torch.randn(N, 3, 224, 224, device="cuda").contiguous(memory_format=torch.channels_last)
    w = torch.randn(64, 3, 7, 7, device="cuda") * 0.1
    y = torch.empty(N, 64, 112, 112, device="cuda").contiguous(memory_format=torch.channels_last)
    st = torch.empty(2, 4096, 64, device="cuda")
    wp3 = torch.empty(int(g.stem_f32x6_wplanes()), dtype=torch.bfloat16, device="cuda")
    t32 = _time(lambda: g.stem_f32_fwd(x, w, y, st))
    t6 = _time(lambda: g.stem_f32x6_fwd(x, w, y, st, wp3))
    dy = torch.randn_like(y)
    out = torch.zeros(64, 3, 7, 7, device="cuda")
    part = torch.empty(int(g.stem_f32_wgrad_ws(N)), device="cuda")
    tw32 = _time(lambda: g.stem_f32_wgrad(x, dy, out, part, False))
    tw6 = _time(lambda: g.stem_f32_wgrad(x, dy, out, part, True))
    print(json.dumps({"N": N, "occ": os.environ.get("GKSGD_STEM_X6_OCC", "2"), "f32_ms": round(t32, 4),
                      "x6_ms": round(t6, 4),
                      "wgrad_f32_ms": round(tw32, 4), "wgrad_x6_ms": round(tw6, 4)}))


if __name__ == "__main__":
    main()
