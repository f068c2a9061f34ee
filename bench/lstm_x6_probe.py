"""fp32 PTB LSTM step GEMMs (H = 1500 -> Hp = 1536; B = 128 and the
reference's B = 20): hipBLASLt fp32 on the unpadded operands, the fp32-MFMA
split-K rec_gemm (lstm.hip rec_gemm_f32_kernel) and the bf16x6 split-K
rec_gemm_x6 (fp32-accurate on the bf16 matrix cores) on the 64-padded ones,
per K-slice count S; plus each kernel's relative RMS error against fp64.
Prints one JSON dict (microseconds per call, errors)."""
import json

import torch

from gaussiank_sgd_amd import ops

assert ops.load()
g = torch.ops.gksgd


def t_us(fn, reps=200):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return round(a.elapsed_time(b) / reps * 1e3, 2)


def split3(w):
    hi = w.to(torch.bfloat16)
    r = w - hi.float()
    mid = r.to(torch.bfloat16)
    return torch.stack([hi, mid, (r - mid.float()).to(torch.bfloat16)]).contiguous()


def rel(x, ref):
    return float((x.double() - ref).norm() / ref.norm())


res = {}
for B in (128, 20):
    H, Hp = 1500, 1536
    f = dict(device="cuda", dtype=torch.float32)
    for direction, (M, N, K) in (("fwd", (B, 4 * Hp, Hp)), ("bwd", (B, Hp, 4 * Hp))):
        a = torch.zeros(M, K, **f)
        w = torch.zeros(N, K, **f)
        if direction == "fwd":
            a[:, :H] = torch.randn(B, H, **f)
            w.view(4, Hp, Hp)[:, :H, :H] = torch.randn(4, H, H, **f) / H ** 0.5
        else:
            a.view(B, 4, Hp)[:, :, :H] = torch.randn(B, 4, H, **f)
            w.view(Hp, 4, Hp)[:H, :, :H] = torch.randn(H, 4, H, **f) / H ** 0.5
        ref = a.double() @ w.double().t()
        w3 = split3(w)
        res["blas_%s_%d" % (direction, B)] = t_us(lambda: torch.mm(a, w.t()))
        res["blas_%s_%d_err" % (direction, B)] = rel(torch.mm(a, w.t()), ref)
        for S in (1, 2, 3, 4, 6, 8, 12, 16, 24):
            if K % (64 * S):
                continue
            P = torch.empty(S, M, N, **f)
            res["f32_%s_%d_S%d" % (direction, B, S)] = t_us(lambda: g.lstm_rec_gemm(a, w, P, S))
            if S == 4:
                res["f32_%s_%d_err" % (direction, B)] = rel(P.sum(0), ref)
            res["x6_%s_%d_S%d" % (direction, B, S)] = t_us(lambda: g.lstm_rec_gemm_x6(a, w3, P, S))
            if S == 4:
                res["x6_%s_%d_err" % (direction, B)] = rel(P.sum(0), ref)
print(json.dumps(res, indent=1))
