"""Convolutions on channels-last activations through the MFMA GEMMs of
``csrc/kernels/gemm.hip``, autotuned per shape against MIOpen.

Two compute precisions share the kernels: bf16 (under bf16 autocast,
v_mfma_f32_16x16x32_bf16) and fp32 (fp32 inputs without autocast -- the
reference's precision, settings.py:28 USE_FP16=False -- on
v_mfma_f32_16x16x4_f32: exact fp32 products, fp32 accumulation).

* 1x1, stride 1: a plain GEMM over the ``M = N*H*W`` pixel rows (forward
  ``Y = X W^T``, grad-input ``dX = dY W``, grad-weight ``dW += dY^T X``).
* KxK (and strided 1x1): implicit GEMM -- the A-operand rows are gathered
  straight from the NHWC input per filter tap by the LDS-DMA loads (padding
  reads a zero row), K = KH*KW*C tap-major like a channels-last weight.
  Stride-1 grad-input is the forward convolution of dY with the flipped,
  transposed weight; grad-weight is the transposed GEMM over gathered rows.

For every distinct (direction, geometry) the first call times a small set of
kernel configurations *and* the MIOpen convolution with HIP events and keeps
the fastest (``GKSGD_GEMM_TUNE=0`` skips the search and uses the HIP
kernel's heuristic default; ``GKSGD_FASTCONV=0`` disables the path).  The
grad-weight kernels add their fp32 result straight into the optimizer's
gradient arena (float atomics) when the module is on the bf16-shadow path
(``parallel/shadow.py``), so no bf16 weight gradient is materialised.

Reference parity: the reference's ResNets use ``nn.Conv2d``
(models/resnet.py / torchvision Bottleneck); ``FastConv2d`` is a drop-in
``nn.Conv2d`` subclass with identical parameters and state_dict keys.
"""
from __future__ import annotations

import os
from typing import Callable, Dict, List, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import load
from . import streams
from . import weight_prep

_CL = torch.channels_last
_TUNE = os.environ.get("GKSGD_GEMM_TUNE", "1") != "0"
_ENABLED = os.environ.get("GKSGD_FASTCONV", "1") != "0"
_choices: Dict[tuple, tuple] = {}
# candidates that are this package's own kernels; a vendor-library choice
# (MIOpen / hipBLASLt) has to beat the best of them by more than this fraction
# of its time (GKSGD_GK_MARGIN, default 5%: the fp32 implicit-GEMM kernels
# trail MIOpen's by 1-5% on some 3x3 shapes -- kept, so the fp32 step runs on
# code this package owns; 0 = fastest wins)
_OWN = ("hip", "w3", "mat", "wino", "wx6")
_GK_MARGIN = float(os.environ.get("GKSGD_GK_MARGIN", "0.05"))
# convolution bias gradients through the fused column pass (GKSGD_CONV_BIAS_COLSUM=0: torch's reduction)
_BIAS_COLSUM = os.environ.get("GKSGD_CONV_BIAS_COLSUM", "1") != "0"
_timings: Dict[tuple, list] = {}      # key -> [(tag, ms or error)] of the search
# fp32 3x3 stride-1 forward / grad-input: Winograd F(2x2, 3x3) candidates
# (winograd.hip, 2.25x fewer MFMA FLOPs); GKSGD_WINO=0 leaves them out.  Their
# autotune keys carry a "wino" tag so choices cached before they existed are
# searched again.  _FORCE (GKSGD_CONV_FORCE=wino, tests) keeps only them.
_WINO = os.environ.get("GKSGD_WINO", "1") != "0"
_FORCE = os.environ.get("GKSGD_CONV_FORCE", "")
_WINO_GRIDS = (0, 1 << 20)
# candidate kernel configurations (gemm.hip: cfg digits = tile + 10*panel + 100*stages)
_NT_CFGS = [1, 2, 3, 4, 11, 13, 21, 22, 23, 24, 111, 113, 121, 122, 123, 124, 25, 26, 27, 125, 126, 127,
            211, 212, 213, 214, 221, 222, 223, 224]   # 2xx: four LDS stages (more bytes in flight)
# grid override: 0 = persistent (about two blocks per CU), else a fixed block count
_NT_GRIDS = (0, 512, 1 << 20)
_TN_CFGS = [(c, s) for c in (1, 2, 3, 4, 5, 6, 7, 8, 21, 22, 23, 24, 27, 9, 29, 101, 121, 102, 122) for s in (0, 128)]
# fp32: 64x64 wave tiles (gemm.hip maps NT tiles 5-7 onto them) and, cfg + 1000, 32x64 wave tiles
# (twice the waves: the small-M layers of small batches, e.g. the reference's bs32); TN cfg = tile +
# 10 * (1: two stages)
_NT_CFGS_F32 = [1, 2, 3, 4, 7, 11, 12, 13, 14, 21, 22, 23, 24, 101, 102, 103, 104, 201, 202, 203, 204,
                1001, 1002, 1003, 1004, 1005, 1006, 1007, 1021, 1022, 1101, 1102, 1103]
_TN_CFGS_F32 = [(c, s) for c in (1, 2, 3, 4, 5, 6, 7, 8, 9, 11, 12, 13, 14, 15, 16) for s in (0, 64)]
# grad-weight of small-batch layers (pixel rows <= _TN_SMALL_M, e.g. ResNet-50 bs32): the default split
# count (two rounds of block slots) trades partial-sum atomics against idle CUs; these let the tuner pick
_TN_SMALL_M = 1 << 17
_TN_SMALL_F32 = [(c, s) for c in (4, 5, 11, 14, 15) for s in (16, 32, 128)]


# fp32 matmul algorithm (GKSGD_F32_MATMUL / set_f32_matmul):
#   "native" -- fp32 operands on v_mfma_f32_16x16x4_f32 only;
#   "bf16x6" -- the fp32 GEMM / implicit-GEMM candidates also include the bf16x6
#   kernels (gemm_kern.h X6, cfg digit 100000): every fp32 operand split exactly
#   into three bf16 parts, the six part products of order <= 2 accumulated in
#   fp32 on v_mfma_f32_16x16x32_bf16 -- measured MORE accurate than the fp32
#   MFMA against an fp64 reference on every ResNet-50 / BERT shape
#   (bench/x6_probe.py, profiles/r05_x6_probe.json), so it is an fp32 algorithm,
#   not a reduced precision; the tuner picks the faster kernel per shape.
X6 = 100000
_NT_CFGS_X6 = [c + X6 for c in (1, 2, 3, 4, 5, 6, 7, 12, 13, 101, 102, 103, 104, 105, 106, 107, 202, 203, 1001, 1002, 1003)]
# register-staged bf16x6 row GEMMs (gemm_kern.h gemm_nt_x62_kernel, cfg digit 200000; tiles 1-7):
# plain row GEMMs only -- an implicit-GEMM / lazy / split-K call refuses them and the tuner moves on.
# Digit 300000: the same kernels with B split into bf16 planes once per call by the binding
# (split3_rows), no B split in the kernel: within +-3% of 200000, up to 8% faster on a few shapes (r5c33)
_NT_CFGS_X62 = [2 * X6 + t for t in range(1, 8)] + [3 * X6 + t for t in range(1, 8)]
# default bf16x6: the library, the trainers (dist_trainer --f32-matmul) and
# bench.py all run the same fp32 GEMM family unless told otherwise
_F32MM = os.environ.get("GKSGD_F32_MATMUL", "bf16x6")


def set_f32_matmul(mode: str) -> str:
    """Select the fp32 matmul algorithm ("native" or "bf16x6"); returns the
    previous one.  Autotune keys carry the mode, so each mode is tuned once."""
    global _F32MM
    if mode not in ("native", "bf16x6"):
        raise ValueError("f32 matmul mode must be 'native' or 'bf16x6', got %r" % (mode,))
    prev, _F32MM = _F32MM, mode
    return prev


def f32_matmul() -> str:
    return _F32MM


def _x6() -> bool:
    return _F32MM == "bf16x6"


# register-staged bf16x6 grad-weight (gemm_kern.h gemm_tn_x62_kernel, cfg digit 200000; tiles 1-8):
# plain row form only -- an implicit-GEMM / lazy call refuses them and the tuner moves on
_TN_CFGS_X62 = [(2 * X6 + t, sp) for t in (1, 2, 3, 4, 5, 6, 7, 8) for sp in (0, 64)]


def _tn_cfgs(dt: torch.dtype) -> List[Tuple[int, int]]:
    if dt == torch.float32:
        # (_TN_CFGS_X62 measured no faster than the LDS-DMA bf16x6 grad-weight on any ResNet-50 /
        # BERT shape, r5c27: not offered by default, GKSGD_TN_X62=1 adds them)
        extra = _TN_CFGS_X62 if os.environ.get("GKSGD_TN_X62", "0") == "1" else []
        return _TN_CFGS_F32 + ([(c + X6, sp) for c, sp in _TN_CFGS_F32] + extra if _x6() else [])
    return _TN_CFGS


def _nt_cfgs(dt: torch.dtype) -> List[int]:
    if dt == torch.float32:
        return _NT_CFGS_F32 + (_NT_CFGS_X6 + _NT_CFGS_X62 if _x6() else [])
    return _NT_CFGS


# fp32 split-K (cfg + 10000 S: S fp32 partial planes over K slices, then one
# reduce pass with the fused epilogue -- gemm.hip nt_splitk_reduce_kernel) for
# row GEMMs whose output tiles cannot fill 256 CUs over a deep K: the 1x1
# convolutions of stages 3-4 at the reference's batch 32 (M = 1568, N = 512,
# K = 2048 is 52 tiles of 128x128).
_SPLITK_BASE = (4, 1, 1001, 1002, 1003)
_SPLITK_MAX_OUT = 1 << 22
_SPLITK_GRIDS = (0, 1 << 20)


def _splitk_cfgs(dt: torch.dtype, M: int, N: int, K: int) -> List[int]:
    """Split-K candidate configs of an [M, K] x [N, K]^T fp32 GEMM (empty when
    its output alone fills the chip)."""
    if dt != torch.float32 or M * N > _SPLITK_MAX_OUT:
        return []
    base = list(_SPLITK_BASE) + ([c + X6 for c in _SPLITK_BASE] if _x6() else [])
    return [c + 10000 * S for S in (2, 4, 8) if K % (64 * S) == 0 and K // S >= 128 for c in base]


# (the implicit-GEMM convolutions split the same way over their (tap, channel)
# K slices: conv_nt with cfg + 10000 S)


def _dkey(dt: torch.dtype) -> tuple:
    """Autotune key suffix: fp32 keys are tagged, bf16 keys keep their
    round-2 form so the shipped tuning cache stays valid."""
    if dt == torch.float32:
        return ("f32", "x6") if _x6() else ("f32",)
    return ()
_zeros: Dict[torch.device, torch.Tensor] = {}


def _g():
    return torch.ops.gksgd


def _zero(dev: torch.device) -> torch.Tensor:
    z = _zeros.get(dev)
    if z is None:
        z = _zeros[dev] = torch.zeros(256, dtype=torch.bfloat16, device=dev)
    return z


def _time(fn: Callable[[], None], reps: int = 5) -> float:
    fn()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


def _pick(key: tuple, cands: List[Tuple[tuple, Callable[[], None]]]) -> tuple:
    """Fastest candidate for ``key`` (timed once per process, then cached):
    a 3-repetition screen of every candidate, then the best four re-timed
    with 12 repetitions (one noisy sample must not decide)."""
    got = _choices.get(key)
    if got is not None:
        return got
    if len(cands) == 1:
        _choices[key] = cands[0][0]
        return cands[0][0]
    if not _TUNE:
        # untuned: the first candidate that runs (a lazy-operand tile may refuse its LDS budget)
        for tag, fn in cands:
            try:
                fn()
            except RuntimeError:
                continue
            _choices[key] = tag
            return tag
        raise RuntimeError("no candidate ran for %s" % (key,))
    log = _timings.setdefault(key, [])
    screened = []
    for tag, fn in cands:
        try:
            t = _time(fn, reps=3)
        except RuntimeError as e:
            log.append((tag, "error: %s" % str(e).splitlines()[0][:200]))
            continue
        screened.append((t, tag, fn))
    screened.sort(key=lambda e: e[0])
    best, best_t = cands[-1][0], float("inf")
    timed = []
    for _, tag, fn in screened[:4]:
        t = _time(fn, reps=12)
        log.append((tag, round(t, 4)))
        timed.append((t, tag))
        if t < best_t:
            best, best_t = tag, t
    if best[0] not in _OWN and _GK_MARGIN > 0:
        # keep the hand-written kernel unless the vendor library is clearly faster
        own = [(t, tag) for t, tag in timed if tag[0] in _OWN]
        if own and min(own)[0] <= best_t * (1.0 + _GK_MARGIN):
            best = min(own)[1]
            log.append((best, "kept: within GKSGD_GK_MARGIN of %s" % (best_t,)))
    _choices[key] = best
    return best


def tuning_log() -> Dict[tuple, list]:
    """Per key, every candidate's measured ms (or its error) from the search."""
    return dict(_timings)


def load_choices(path: str) -> int:
    """Seed the autotune cache from a JSON file written by save_choices()."""
    import json
    try:
        with open(path) as f:
            rows = json.load(f)
    except (OSError, ValueError):
        return 0
    for k, v in rows:
        _choices.setdefault(tuple(k), tuple(v))
    return len(rows)


def save_choices(path: str) -> None:
    import json
    with open(path, "w") as f:
        json.dump([[list(k), list(v)] for k, v in sorted(_choices.items(), key=str)], f, indent=0)


_CACHE = os.environ.get("GKSGD_GEMM_CACHE", os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))), "tuning", "gemm_choices.json"))
if _TUNE and _CACHE and os.path.exists(_CACHE) and os.environ.get("GKSGD_GEMM_RETUNE", "0") == "0":
    load_choices(_CACHE)
    # GKSGD_GEMM_RETUNE_ONLY=dgrad_bn,...: retune only the keys of these directions
    _only = {d for d in os.environ.get("GKSGD_GEMM_RETUNE_ONLY", "").split(",") if d}
    if _only:
        for _k in [k for k in _choices if k and k[0] in _only]:
            del _choices[_k]


def tuned_choices() -> Dict[tuple, tuple]:
    """(direction, geometry...) -> chosen (impl, cfg, grid/splits)."""
    return dict(_choices)


def supported(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    """Shapes the HIP kernels take (either precision)."""
    k = conv.kernel_size
    return (_ENABLED and x.is_cuda and x.dim() == 4 and k[0] == k[1] and k[0] in (1, 3) and
            conv.stride[0] == conv.stride[1] and conv.stride[0] in (1, 2) and
            conv.padding == (k[0] // 2, k[0] // 2) and conv.dilation == (1, 1) and conv.groups == 1 and
            conv.padding_mode == "zeros" and x.is_contiguous(memory_format=_CL) and
            conv.in_channels % 64 == 0 and conv.out_channels % 64 == 0 and x.numel() > 0)


def _rows(t: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] channels-last -> [N*H*W, C] view."""
    N, C, H, W = t.shape
    return t.permute(0, 2, 3, 1).reshape(N * H * W, C)


def _geom(x_shape, w: torch.Tensor, s: int):
    N, C, H, W = x_shape
    K, k = w.shape[0], w.shape[2]
    p = k // 2
    OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    return N, C, H, W, K, k, p, OH, OW


def _wino_ok(dt: torch.dtype, k: int, s: int, C: int, K: int) -> bool:
    return _WINO and dt == torch.float32 and k == 3 and s == 1 and C % 8 == 0 and K % 64 == 0


# bf16x6 Winograd (wino_x6.hip: the 16 element-wise GEMMs on v_mfma_f32_16x16x32_bf16
# with split operands, fp32-accurate), offered beside the fp32-MFMA Winograd in the
# bf16x6 fp32 matmul mode with GKSGD_WINO_X6=1.  Opt-in: measured 1.5-1.7x SLOWER
# than the fp32-MFMA Winograd on every ResNet-50 bs512 shape (profiles/r06_wino_x6.txt:
# 7.7 VALU per MFMA for the per-wave transform + split, and the per-wave patch loads
# not hidden at one wave per SIMD)
_WX6 = os.environ.get("GKSGD_WINO_X6", "0") == "1"


def _wx6_ok(Ci: int, Co: int) -> bool:
    return _WX6 and _x6() and Ci % 32 == 0 and Co % 32 == 0


def _wino_tag(Ci: int, Co: int) -> tuple:
    """Autotune-key suffix of a Winograd-eligible convolution (Ci -> Co as run):
    the x6 candidates get their own tag so choices tuned without them are not reused."""
    return ("wino", "wx6") if _wx6_ok(Ci, Co) else ("wino",)


def _wino_shape_fits(N: int, H: int, W: int, C: int, K: int) -> bool:
    """Every operand a Winograd stride-1 3x3 kernel addresses through a 32-bit
    buffer descriptor is < 2^31 bytes: forward x [N, C, H, W] and y
    [N, K, H, W]; grad-input dy [N, K, H, W] and dx / the BN-backward
    epilogue's h, dy2, mask (dx-shaped) [N, C, H, W]; grad-weight x and dy.
    The hardware range check would silently zero loads past the limit, so
    the candidate is refused (the bindings also refuse it loudly)."""
    return N * H * W * max(C, K) * 4 < (1 << 31) and N * ((H + 1) // 2) * ((W + 1) // 2) < (1 << 31)


def _wino_cands(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor, flip: bool, st=None, bn=(),
                wp: bool = False) -> list:
    """Winograd candidates: filter transform (the weights change every step:
    rebuilt once per step for the whole model by ops/weight_prep.py when ``wp``,
    the weight being persistent storage) + wino_conv; ``bn`` = (h, dy2, mask)
    of the BN-backward epilogue."""
    g = _g()

    def run(mb, sp=1):
        u = weight_prep.wino_filter(w, flip, wp)
        return g.wino_conv(x, u, out, mb, st, *bn, splits=sp)
    cands = [(("wino", 0, mb), (lambda mb=mb: run(mb))) for mb in _WINO_GRIDS]
    # small batches: fewer (64-tile x 64-channel) blocks than CUs -> also offer
    # input-channel splits (fp32 partial planes + one reduce pass with the epilogue)
    N, Ci, H, W = x.shape
    blocks = -(-(N * ((H + 1) // 2) * ((W + 1) // 2)) // 64) * (out.shape[1] // 64)
    if blocks < 256:
        cands += [(("wino", sp, 0), (lambda sp=sp: run(0, sp))) for sp in (2, 4) if Ci % (8 * sp) == 0]
    if _wx6_ok(Ci, out.shape[1]):
        def run6(mb):
            u3 = weight_prep.wino_x6_filter(w, flip, wp)
            return g.wino_x6_conv(x, u3, out, mb, st, *bn)
        cands += [(("wx6", 0, mb), (lambda mb=mb: run6(mb))) for mb in _WINO_GRIDS]
    return cands


def _forced(cands: list) -> list:
    if _FORCE:
        sel = [c for c in cands if c[0][0] == _FORCE]
        if sel:
            return sel
    return cands


def _fwd(x: torch.Tensor, w: torch.Tensor, s: int, stats_box=None, bias=None, wp: bool = False) -> torch.Tensor:
    """y = conv(x, w).  With ``stats_box`` (a list) and the HIP kernel chosen,
    the kernel's epilogue also reduces the BatchNorm batch statistics of y
    and ``(partials [2, rows_max, K], rows)`` is appended to the box
    (ops/bn.py BNAct(stats=...) consumes it and skips its statistics pass)."""
    N, C, H, W, K, k, p, OH, OW = _geom(x.shape, w, s)
    M = N * OH * OW
    dt = x.dtype
    y = torch.empty((N, K, OH, OW), dtype=dt, device=x.device, memory_format=_CL)
    g = _g()
    st = None
    if stats_box is not None:
        st = torch.empty(2, min(1280, (M + 63) // 64), K, dtype=torch.float32, device=x.device)
    split = []
    if k == 1 and s == 1:
        X, Y, Wm = _rows(x), _rows(y), w.reshape(K, C)
        run = lambda c, mb: g.gemm_nt(X, Wm, Y, c, mb, st, bias)  # noqa: E731
        split = _splitk_cfgs(dt, M, K, C)
    else:
        z = _zero(x.device)
        run = lambda c, mb: g.conv_nt(x, w, y, z, s, p, c, mb, st, bias)  # noqa: E731
        split = _splitk_cfgs(dt, M, K, k * k * C)
    b16 = bias.to(dt) if bias is not None else None
    cands = [(("hip", c, mb), (lambda c=c, mb=mb: run(c, mb))) for c in _nt_cfgs(dt) for mb in _NT_GRIDS]
    cands += [(("hip", c, mb), (lambda c=c, mb=mb: run(c, mb))) for c in split for mb in _SPLITK_GRIDS]
    wino = bias is None and _wino_ok(dt, k, s, C, K) and _wino_shape_fits(N, H, W, C, K)
    if wino:
        cands += _wino_cands(x, w, y, False, st, wp=wp)

    def miopen():
        out = F.conv2d(x, w, b16, stride=s, padding=p)
        if st is not None and ws is not None:
            # a MIOpen output leaves the consuming BN its statistics pass: time it too
            g.bn_stats_partials(out.contiguous(memory_format=_CL), ws)
        return out
    ws = None
    if st is not None and (("fwd", N, C, H, W, K, k, s, True) + _dkey(dt)) not in _choices and \
            g.bn_supported(K, x.element_size()):
        ws = torch.empty(int(g.bn_workspace_floats(M, K, x.element_size())), dtype=torch.float32, device=x.device)
    cands.append((("miopen", 0, 0), miopen))
    ch = _pick(("fwd", N, C, H, W, K, k, s, st is not None) + _dkey(dt) + (_wino_tag(C, K) if wino else ()),
               _forced(cands))
    if ch[0] == "miopen":
        return F.conv2d(x, w, b16, stride=s, padding=p).contiguous(memory_format=_CL)
    if ch[0] in ("wino", "wx6"):
        rows = dict(cands)[ch]()
    else:
        rows = run(ch[1], ch[2])
    if st is not None:
        stats_box.append((st, int(rows)))
    return y


def _lz_kw(lz, rows: bool = False) -> dict:
    """Kernel keywords of a lazy BN-backward operand (ops/bn.py ProducerLink):
    the dz operand is the tensor passed in place of dy; x (the BN input) has
    its layout (``rows``: as an [M, C] row view)."""
    _, x, coef, padz, padx = lz
    return dict(lz_x=_rows(x) if rows else x, lz_coef=coef, lz_padz=padz, lz_padx=padx)


def _dgrad(dy: torch.Tensor, w: torch.Tensor, x_shape, s: int, lz=None, plink=None, wp: bool = False) -> torch.Tensor:
    """Grad-input.  ``lz``: dy is the dz of a lazy BN backward (the kernels
    compute dx from dz and the BN input themselves); the "mat" candidate
    materialises dx (``plink.materialize()``) and runs the plain path."""
    N, C, H, W, K, k, p, OH, OW = _geom(x_shape, w, s)
    g = _g()
    dt = dy.dtype
    xs = torch.empty(x_shape, dtype=dt, device=dy.device, memory_format=_CL)   # shape only
    kw = _lz_kw(lz, rows=(s == 1 and k == 1)) if lz is not None else {}

    def miopen():
        return torch.ops.aten.convolution_backward(dy, xs, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
                                                   [True, False, False])[0]
    cands = []
    split = []
    dx = None
    if s == 2:
        # stride 2: the four parity classes of dX as stride-1 implicit GEMMs over dY
        dx = xs
        z = _zero(dy.device)
        run = lambda c, mb: g.conv_dgrad_s2(dy, w, dx, z, c, mb, **kw)  # noqa: E731
        cands = [(("hip", c, mb), (lambda c=c, mb=mb: run(c, mb))) for c in _nt_cfgs(dt) for mb in _NT_GRIDS]
    if s == 1:
        dx = xs
        if k == 1:
            DY, DX = _rows(dy), _rows(dx)
            Wt = _lazy(lambda: weight_prep.transposed_1x1(w, wp))
            run = lambda c, mb: g.gemm_nt(DY, Wt(), DX, c, mb, **kw)  # noqa: E731
            if lz is None:
                split = _splitk_cfgs(dt, N * H * W, C, K)
        else:
            # dX = conv(dY, W') with W'[c][kh][kw][k] = W[k][KH-1-kh][KW-1-kw][c]
            wf = _lazy(lambda: weight_prep.flipped_3x3(w, wp))
            z = _zero(dy.device)
            run = lambda c, mb: g.conv_nt(dy, wf(), dx, z, 1, p, c, mb, **kw)  # noqa: E731
        cands = [(("hip", c, mb), (lambda c=c, mb=mb: run(c, mb))) for c in _nt_cfgs(dt) for mb in _NT_GRIDS]
        cands += [(("hip", c, mb), (lambda c=c, mb=mb: run(c, mb))) for c in split for mb in _SPLITK_GRIDS]
    if lz is not None:
        cands.append((("mat", 0, 0), lambda: _dgrad(plink.materialize(), w, x_shape, s, wp=wp)))
        ch = _pick(("dgrad", N, C, H, W, K, k, s) + _dkey(dt) + ("lz",), cands)
        if ch[0] == "mat":
            return _dgrad(plink.materialize(), w, x_shape, s, wp=wp)
        run(ch[1], ch[2])
        return dx
    wino = _wino_ok(dt, k, s, K, C) and _wino_shape_fits(N, H, W, C, K)
    if wino:
        cands += _wino_cands(dy, w, dx, True, wp=wp)
    cands.append((("miopen", 0, 0), miopen))
    ch = _pick(_dgrad_key(N, C, H, W, K, k, s, dt), _forced(cands))
    if ch[0] == "miopen":
        return miopen().contiguous(memory_format=_CL)
    if ch[0] in ("wino", "wx6"):
        dict(cands)[ch]()
        return dx
    run(ch[1], ch[2])
    return dx


# Grad-weight choices issued on the side stream (ops/streams.py; HIP kernels only: MIOpen's
# handle and workspace follow the stream it was set up on).  GKSGD_WGRAD_STREAM_WINO=0 keeps
# the Winograd grad-weight inline, GKSGD_WGRAD_STREAM_KINDS restricts the forked choice kinds
# (only "wino": -3%, r6c43).  The fork is issued BEFORE the grad-input GEMM;
# GKSGD_WGRAD_AFTER_DGRAD=1 issues it after (measured -1.4% fp32 / -1.5% bf16, r6c46).
_WGRAD_AFTER = os.environ.get("GKSGD_WGRAD_AFTER_DGRAD", "0") == "1"
# GKSGD_WGRAD_SIDE_QROUNDS=q: a forked TN grad-weight whose tuned split is auto (two rounds
# of the chip's block slots) launches q quarter rounds instead (0: unchanged)
_SIDE_QROUNDS = int(os.environ.get("GKSGD_WGRAD_SIDE_QROUNDS", "0"))
# GKSGD_WGRAD_STREAM_BIAS=1: a forked convolution's bias gradient goes to the side stream with
# its grad-weight (measured slower: VGG-16 bs512 76.4-77.1k vs 78.5k img/s on the main stream, r6c53)
_FORK_BIAS = os.environ.get("GKSGD_WGRAD_STREAM_BIAS", "0") == "1"
_FORKABLE = tuple(k for k in os.environ.get("GKSGD_WGRAD_STREAM_KINDS", "hip,w3,wino").split(",")
                  if k and (k != "wino" or os.environ.get("GKSGD_WGRAD_STREAM_WINO", "1") == "1"))


def _lazy(make):
    """Memoised weight re-layout: built on first use only, so a Winograd /
    MIOpen choice does not pay the transpose / flip copy it never reads."""
    box = []

    def get():
        if not box:
            box.append(make())
        return box[0]
    return get


def _dgrad_key(N, C, H, W, K, k, s, dt) -> tuple:
    wino = _wino_ok(dt, k, s, K, C) and _wino_shape_fits(N, H, W, C, K)
    return ("dgrad", N, C, H, W, K, k, s) + _dkey(dt) + (_wino_tag(K, C) if wino else ())


def _dgrad_bn(dy: torch.Tensor, w: torch.Tensor, x_shape, s: int, link, lz=None, plink=None,
              wp: bool = False) -> torch.Tensor:
    """Grad-input with the producing BatchNorm's backward reduction fused into
    the epilogue (gemm.hip BnBwd; ops/bn.py BnLink): returns dz = ReLU-masked
    (dX + dy2) and leaves the partials in ``link.part``.  Stride 1 only; the
    caller checks ``link.ready()``.  ``lz``: dy is a lazy BN-backward dz (see
    _dgrad)."""
    N, C, H, W, K, k, p, OH, OW = _geom(x_shape, w, s)
    kw = _lz_kw(lz, rows=(k == 1)) if lz is not None else {}
    g = _g()
    M = N * H * W
    dt = dy.dtype
    dz = torch.empty(x_shape, dtype=dt, device=dy.device, memory_format=_CL)
    st = torch.empty(2, min(1280, (M + 63) // 64), C, dtype=torch.float32, device=dy.device)
    h, mask, dy2 = link.h, link.mask, link.dy2
    if k == 1:
        DY, DZ = _rows(dy), _rows(dz)
        Wt = _lazy(lambda: weight_prep.transposed_1x1(w, wp))
        H2 = _rows(h)
        D2 = _rows(dy2) if dy2 is not None else None
        run = lambda c, mb: g.gemm_nt(DY, Wt(), DZ, c, mb, st, None, H2, D2, mask, **kw)  # noqa: E731
        split = _splitk_cfgs(dt, M, C, K) if lz is None else []
    else:
        split = []
        wf = _lazy(lambda: weight_prep.flipped_3x3(w, wp))
        z = _zero(dy.device)
        run = lambda c, mb: g.conv_nt(dy, wf(), dz, z, 1, p, c, mb, st, None, h, dy2, mask, **kw)  # noqa: E731
    # 64x64-per-wave tiles (cfg digit 1-4) and the fp32 32x64 family (cfg >= 1000) carry the
    # BN-backward epilogue
    cands = [(("hip", c, mb), (lambda c=c, mb=mb: run(c, mb))) for c in _nt_cfgs(dt) if c % 10 <= 4 or c >= 1000
             for mb in _NT_GRIDS]
    cands += [(("hip", c, mb), (lambda c=c, mb=mb: run(c, mb))) for c in split for mb in _SPLITK_GRIDS]
    key = ("dgrad_bn", N, C, H, W, K, k, s, dy2 is not None) + _dkey(dt)
    if lz is not None:
        cands.append((("mat", 0, 0), lambda: _dgrad_bn(plink.materialize(), w, x_shape, s, link, wp=wp)))
        ch = _pick(key + ("lz",), cands)
        if ch[0] == "mat":
            return _dgrad_bn(plink.materialize(), w, x_shape, s, link, wp=wp)
    else:
        if _wino_ok(dt, k, s, K, C) and _wino_shape_fits(N, H, W, C, K):
            cands += _wino_cands(dy, w, dz, True, st, (h, dy2, mask), wp=wp)
            key = key + _wino_tag(K, C)
        ch = _pick(key, _forced(cands))
    if ch[0] in ("wino", "wx6"):
        rows = dict(cands)[ch]()
    else:
        rows = run(ch[1], ch[2])
    link.part = (st, int(rows))
    link.dz = dz
    return dz


def _bn_fusable(link, s: int, dgrad_key: tuple) -> bool:
    """Fuse the producing BN's backward reduction into this grad-input?  Only
    when its inputs are ready and the tuned plain grad-input is the HIP kernel
    (a MIOpen choice means the HIP GEMM is the slower one for this shape)."""
    if link is None or s != 1 or os.environ.get("GKSGD_BN_LINK", "1") == "0" or not link.ready():
        return False
    if link.h.dtype != dgrad_key_dtype(dgrad_key):
        return False
    ch = _choices.get(dgrad_key)
    return ch is None or ch[0] in ("hip", "wino", "wx6")


def dgrad_key_dtype(key: tuple) -> torch.dtype:
    return torch.float32 if "f32" in key[8:] else torch.bfloat16


def _wgrad_key(x: torch.Tensor, w: torch.Tensor, s: int, lz=None) -> tuple:
    N, C, H, W, K, k, p, OH, OW = _geom(x.shape, w, s)
    wino = lz is None and _wino_ok(x.dtype, k, s, C, K) and C % 64 == 0 and _wino_shape_fits(N, H, W, C, K)
    return ("wgrad", N, C, H, W, K, k, s) + _dkey(x.dtype) + (("lz",) if lz is not None else ()) + \
        (("wino",) if wino else ())


def _wgrad_into(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor, s: int, out_f32: torch.Tensor, lz=None,
                plink=None, side: bool = False) -> None:
    """out_f32 ([K, C, k, k] channels-last fp32) += dW.  ``lz``: dy is a lazy
    BN-backward dz (see _dgrad)."""
    N, C, H, W, K, k, p, OH, OW = _geom(x.shape, w, s)
    g = _g()
    dt = x.dtype
    key = _wgrad_key(x, w, s, lz)
    scratch = torch.zeros_like(out_f32) if key not in _choices else None
    kw = _lz_kw(lz, rows=(k == 1 and s == 1)) if lz is not None else {}

    def miopen():
        return torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
                                                   [False, True, False])[1]
    if k == 1 and s == 1:
        DY, X = _rows(dy), _rows(x)
        run = lambda o, c, sp: g.gemm_tn_acc(DY, X, o.view(K, C), c, sp, **kw)  # noqa: E731
    else:
        z = _zero(x.device)
        run = lambda o, c, sp: g.conv_tn_acc(dy, x, o, z, s, p, c, sp, **kw)  # noqa: E731
    tn = list(_tn_cfgs(dt))
    if dt == torch.float32 and N * OH * OW <= _TN_SMALL_M:
        tn += _TN_SMALL_F32   # small batches: more / fewer pixel splits than the two-rounds default
        if _x6():
            tn += [(c + X6, sp) for c, sp in _TN_SMALL_F32]
    cands = [(("hip", c, sp), (lambda c=c, sp=sp: run(scratch, c, sp))) for c, sp in tn]
    if lz is not None:
        cands.append((("mat", 0, 0), lambda: _wgrad_into(plink.materialize(), x, w, s, scratch)))
        ch = _pick(key, cands)
        if ch[0] == "mat":
            _wgrad_into(plink.materialize(), x, w, s, out_f32)
        else:
            run(out_f32, ch[1], ch[2])
        return
    if key[-1] == "wino":
        # Winograd F(2x2, 3x3) grad-weight (winograd.hip): per-split dU partials + finalize
        def wino_w(o, sp):
            part = torch.empty(int(g.wino_wgrad_ws(N, H, W, C, K, sp)), dtype=torch.float32, device=x.device)
            g.wino_wgrad(x, dy, o, part, sp)
        for sp in (0, 512):
            cands.append((("wino", 0, sp), (lambda sp=sp: wino_w(scratch, sp))))
    w3 = None
    if k == 3 and s == 1 and dt == torch.bfloat16 and g.wgrad3_supported(H, W, C, K):
        # tap-parallel kernel (wgrad3.hip): dY and X staged once per band for all 9 taps
        def w3(o):
            part = torch.empty(int(g.wgrad3_ws(N, H, W, C, K)), dtype=torch.float32, device=x.device)
            g.conv3_wgrad(dy, x, o, part, _zero(x.device))
        cands.append((("w3", 0, 0), lambda: w3(scratch)))

    def miopen_acc(o):
        # MIOpen writes a fresh (zero-filled) gradient that is then added into the
        # arena: the candidate is timed with that accumulation
        from . import accum_grad_
        accum_grad_(o, miopen().contiguous(memory_format=_CL))
    cands.append((("miopen", 0, 0), lambda: miopen_acc(scratch)))
    ch = _pick(key, _forced(cands))
    if ch[0] == "miopen":
        miopen_acc(out_f32)
        return
    if ch[0] == "wino":
        wino_w(out_f32, ch[2])
        return
    if ch[0] == "w3" and w3 is not None:
        w3(out_f32)
        return
    sp = ch[2]
    if side and sp == 0 and _SIDE_QROUNDS > 0:
        sp = -_SIDE_QROUNDS     # a smaller auto grid beside the critical path (gemm_kern.h launch_tn*)
    run(out_f32, ch[1], sp)


class _FastConvFn(torch.autograd.Function):
    """y = conv(x, w) in the compute dtype ``dt`` (bf16 or fp32).  ``param``
    is the fp32 master weight; ``w_bf16`` its bf16-shadow view (bf16 path);
    with a ``sink`` (the optimizer's gradient arena: bf16-shadow or fp32
    direct-gradient path) the weight gradient is added into the arena in the
    backward and None is returned for it."""

    @staticmethod
    def forward(ctx, x, param, w_bf16, sink, stride, stats_box=None, bias=None, bias_sink=None, link=None,
                dt=torch.bfloat16, plink=None):
        if x.dtype != dt:
            x = x.to(dt)
        x = x.contiguous(memory_format=_CL)
        if dt == torch.bfloat16:
            w = w_bf16 if w_bf16 is not None else param.detach().to(torch.bfloat16)
        else:
            w = param.detach()
        w = w.contiguous(memory_format=_CL)
        # persistent weight storage (the parameter or its bf16 shadow view): its
        # per-step re-layouts are batched by ops/weight_prep.py
        wp = w.data_ptr() == param.data_ptr() or (w_bf16 is not None and w.data_ptr() == w_bf16.data_ptr())
        b = bias.detach().float().contiguous() if bias is not None else None
        y = _fwd(x, w, stride, stats_box, b, wp=wp)
        ctx.wp = wp
        ctx.prep = weight_prep.current() if wp else None
        ctx.sink = sink
        ctx.bias_sink = bias_sink
        ctx.has_bias = bias is not None
        ctx.stride = stride
        ctx.param_dtype = param.dtype
        ctx.link = link
        ctx.dt = dt
        ctx.plink = plink       # the consuming BN may hand back a lazy dz (ops/bn.py ProducerLink)
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        s = ctx.stride
        dy = dy.to(ctx.dt).contiguous(memory_format=_CL)
        link, ctx.link = ctx.link, None
        plink, ctx.plink = ctx.plink, None
        # lazy BN backward: dy is the consuming BN's dz; dx is formed inside the GEMMs
        lz = plink.lazy if plink is not None and plink.matches(dy) else None
        if plink is not None and plink.lazy is not None and lz is None:
            # autograd summed the BN's dz with another consumer's gradient: the sum is not dx
            raise RuntimeError("FastConv2d: lazy BN gradient mixed with another consumer of the conv output; "
                               "set GKSGD_BN_LAZY=0 for this model")
        # grad-weight into the optimizer's arena: off the critical path on the side
        # stream (ops/streams.py), issued first so it overlaps the grad-input GEMM and
        # the BatchNorm passes that follow it; tuned shapes whose choice is a HIP kernel
        # only (the search times candidates on the current stream; MIOpen calls stay
        # on the stream its handle and workspace were set up for)
        sink = ctx.sink if ctx.needs_input_grad[1] else None
        direct = sink is not None and getattr(sink, "grad_view", None) is not None and \
            sink.grad_view.is_contiguous(memory_format=_CL)
        fork = direct and lz is None and not getattr(sink, "shared", False) and \
            streams.worth(x.device, 2.0 * dy.numel() * x.shape[1] * w.shape[2] * w.shape[3]) and \
            _choices.get(_wgrad_key(x, w, s), ("",))[0] in _FORKABLE

        # the bias gradient (a column pass over dy into its arena view) rides along
        bs0 = ctx.bias_sink if ctx.has_bias and ctx.needs_input_grad[6] else None
        gvb = getattr(bs0, "grad_view", None) if bs0 is not None else None
        bias_fork = fork and _FORK_BIAS and _BIAS_COLSUM and gvb is not None and gvb.is_contiguous() and \
            not getattr(bs0, "shared", False) and dy.is_contiguous(memory_format=_CL)

        def fork_wgrad():
            sink.check()
            if bias_fork:
                bs0.check()
            side = streams.fork(x.device)
            with torch.cuda.stream(side):
                _wgrad_into(dy, x, w, s, sink.grad_view, side=True)
                if bias_fork:
                    from .linear import bias_grad_acc_
                    bias_grad_acc_(gvb, _rows(dy))
            streams.hold(x.device, dy, x, w)    # alive until the side work is done / joined
        if fork and not _WGRAD_AFTER:
            fork_wgrad()
        dx = None
        if ctx.needs_input_grad[0]:
            N, C, H, W = x.shape
            key = _dgrad_key(N, C, H, W, w.shape[0], w.shape[2], s, ctx.dt)
            prep, ctx.prep = ctx.prep, None
            with weight_prep.use(prep):      # the step scope of the forward (autograd thread)
                if _bn_fusable(link, s, key):
                    dx = _dgrad_bn(dy, w, x.shape, s, link, lz, plink, wp=ctx.wp)
                else:
                    dx = _dgrad(dy, w, x.shape, s, lz, plink, wp=ctx.wp)
        if fork and _WGRAD_AFTER:
            fork_wgrad()    # waits for the grad-input: overlaps the BN passes that follow it
        gparam = None
        if ctx.needs_input_grad[1] and not fork:
            if direct:
                sink.check()
                _wgrad_into(dy, x, w, s, sink.grad_view, lz, plink)
            else:
                out = torch.zeros(w.shape, dtype=torch.float32, device=x.device).contiguous(memory_format=_CL)
                _wgrad_into(dy, x, w, s, out, lz, plink)
                if sink is not None:
                    sink(out)
                else:
                    gparam = out.to(ctx.param_dtype)
        gbias = None
        if ctx.has_bias and ctx.needs_input_grad[6] and not bias_fork:
            src = plink.materialize() if lz is not None else dy
            bs = ctx.bias_sink
            gv = getattr(bs, "grad_view", None) if bs is not None else None
            if src.is_contiguous(memory_format=_CL) and _BIAS_COLSUM:
                # one HIP column pass over the [N*H*W, C] rows of the channels-last
                # gradient (linear.hip colsum_acc), added straight into the arena
                # view when there is one (torch's NHWC sum(0, 2, 3) reduction took
                # 22.6 us per VGG-16 bs512 layer, profiles/r06_vgg16_bs512_fp32_kernel_stats.csv)
                from .linear import bias_grad_acc_
                if gv is not None and gv.is_contiguous():
                    bs.check()
                    bias_grad_acc_(gv, _rows(src))
                    bs = None
                    db = None
                else:
                    db = torch.zeros(src.shape[1], dtype=torch.float32, device=src.device)
                    bias_grad_acc_(db, _rows(src))
            else:
                db = src.sum(dim=(0, 2, 3), dtype=torch.float32)
            if bs is not None:
                bs(db)          # into the optimizer's fp32 arena (shadow path)
            elif db is not None:
                gbias = db
        if plink is not None:
            plink.clear()
        return dx, gparam, None, None, None, None, gbias, None, None, None, None


class FastConv2d(nn.Conv2d):
    """``nn.Conv2d`` whose 1x1 / 3x3 (stride 1 or 2, 'same' padding)
    training path on a GPU runs the autotuned MFMA kernels: bf16 compute
    under bf16 autocast, fp32 compute for fp32 inputs without autocast;
    everything else is the stock convolution."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self._run(x, None)

    def forward_stats(self, x: torch.Tensor):
        """(y, stats): stats = (partials, rows) of y's BatchNorm statistics
        when the fused HIP kernel produced them, else None."""
        box = []
        y = self._run(x, box)
        return y, (box[0] if box else None)

    def _run(self, x: torch.Tensor, box):
        dev = x.device.type
        autocast = torch.is_autocast_enabled(dev)
        bf16 = x.dtype == torch.bfloat16 or (autocast and torch.get_autocast_dtype(dev) == torch.bfloat16)
        f32 = not autocast and x.dtype == torch.float32 and self.weight.dtype == torch.float32 and \
            os.environ.get("GKSGD_FASTCONV_F32", "1") != "0"
        if (bf16 or f32) and supported(x, self) and load():
            if bf16:
                table = getattr(self, "_gk_shadow", None)
                info = table.get("weight") if table else None
                binfo = table.get("bias") if table else None
                use_shadow = info is not None and autocast
                w_bf16, sink = (info[0], info[1]) if use_shadow else (None, None)
                bsink = binfo[1] if (use_shadow and binfo is not None) else None
            else:
                # fp32 direct-gradient path (parallel/shadow.py install_direct_grads)
                table = getattr(self, "_gk_direct_grads", None) or {}
                w_bf16, sink, bsink = None, table.get("weight"), table.get("bias")
            if not torch.is_grad_enabled() or not self.weight.requires_grad:
                sink = None
            if not torch.is_grad_enabled() or self.bias is None or not self.bias.requires_grad:
                bsink = None
            link = getattr(x, "_gk_bn_link", None)
            plink = None
            if f32 and not bf16 and torch.is_grad_enabled():
                from .bn import ProducerLink
                plink = ProducerLink()
            y = _FastConvFn.apply(x, self.weight, w_bf16, sink, self.stride[0], box, self.bias, bsink, link,
                                  torch.bfloat16 if bf16 else torch.float32, plink)
            if plink is not None:
                y._gk_plink = plink
            return y
        slow = getattr(self, "_gk_slow", None)
        return slow(x) if slow is not None else super().forward(x)


def conv_stats(conv: nn.Module, x: torch.Tensor):
    """(conv(x), BatchNorm partials of the output or None) -- FastConv2d and
    the stem conv (ops/stem.py) reduce them in their GEMM epilogue."""
    fs = getattr(conv, "forward_stats", None)
    if fs is not None:
        return fs(x)
    return conv(x), None


class Conv1x1(FastConv2d):
    """``nn.Conv2d(in, out, 1, stride, bias=False)``."""

    def __init__(self, inp: int, out: int, stride: int = 1):
        super().__init__(inp, out, 1, stride=stride, bias=False)


class Conv3x3(FastConv2d):
    """``nn.Conv2d(in, out, 3, stride, padding=1, bias=False)``."""

    def __init__(self, inp: int, out: int, stride: int = 1, groups: int = 1, dilation: int = 1):
        super().__init__(inp, out, 3, stride=stride, padding=dilation, groups=groups, bias=False,
                         dilation=dilation)
