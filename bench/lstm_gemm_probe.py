"""PTB LSTM step GEMMs (B = 128, H = 1500 -> Hp = 1536): hipBLASLt on the
unpadded operands vs the split-K rec_gemm kernel (lstm.hip) on the 64-padded
ones, for every K-slice count S; plus the cell kernels that sum the slices.
Prints one JSON dict of microseconds per call."""
import json

import torch

from gaussiank_sgd_amd import ops

assert ops.load()
g = torch.ops.gksgd


def t_us(fn, reps=100):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return round(a.elapsed_time(b) / reps * 1e3, 2)


res = {}
for B, H in ((128, 1500), (20, 1500)):
    Hp = (H + 63) // 64 * 64
    bf = dict(device="cuda", dtype=torch.bfloat16)
    h = torch.randn(B, H, **bf)
    w = torch.randn(4 * H, H, **bf)
    dG = torch.randn(B, 4 * H, **bf)
    res["blas_fwd_%d" % B] = t_us(lambda: torch.mm(h, w.t()))
    res["blas_bwd_%d" % B] = t_us(lambda: torch.mm(dG, w))
    hp = torch.randn(B, Hp, **bf)
    wf = torch.randn(4 * Hp, Hp, **bf)
    dGp = torch.randn(B, 4 * Hp, **bf)
    wb = torch.randn(Hp, 4 * Hp, **bf)
    for S in (1, 2, 3, 4, 6, 8, 12):
        if Hp % (64 * S) == 0:
            P = torch.empty(S, B, 4 * Hp, device="cuda")
            res["rec_fwd_%d_S%d" % (B, S)] = t_us(lambda: g.lstm_rec_gemm(hp, wf, P, S))
    for S in (2, 4, 8, 12, 16, 24, 32, 48):
        if 4 * Hp % (64 * S) == 0:
            P = torch.empty(S, B, Hp, device="cuda")
            res["rec_bwd_%d_S%d" % (B, S)] = t_us(lambda: g.lstm_rec_gemm(dGp, wb, P, S))
print(json.dumps(res, indent=1))
