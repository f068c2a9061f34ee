"""Python front-end of the gfx950 kernel library (``gaussiank_sgd_amd/_C.so``).

Dispatch rule: GPU tensors ALWAYS go to the HIP kernels; if the extension is
missing on a GPU box the call raises (no silent eager fallback).  CPU tensors
run a pure-torch mirror of the same pipeline with identical semantics -- this
is what the gloo/CPU tests exercise and what the GPU numerics tests compare
against.

Packed record layout (one per rank and bucket, int32 words)::

    [0] sent  [1] total  [2] chosen candidate  [3] threshold (fp32 bits)
    [4 : 4+k_cap]            int32 indices (ascending)
    [4+k_cap : 4+2*k_cap]    fp32 values (bit-cast)
"""
from __future__ import annotations

import os
import threading
from pathlib import Path
from typing import List, Optional, Sequence, Tuple

import torch

# GKSGD_EXT overrides the library (e.g. build/asan/_C.so, the host-sanitizer build)
_LIB = Path(os.environ.get("GKSGD_EXT") or (Path(__file__).resolve().parents[1] / "_C.so"))
_lock = threading.Lock()
_loaded = False
_load_error: Optional[BaseException] = None

MODE_GAUSSIAN = 0
MODE_REDSYNC = 1
MODE_REDSYNCTRIM = 2
MODE_TOPK = 3
MODE_RANDOMK = 4
MODE_THRESHOLD = 5
MODE_DGC = 6
MODE_GAUSSIAN_CAL = 7

CAL_FALLBACK = 16   # record header `chosen` when the calibrated mode used the exact radix key
OVERFLOW_EXACT = 17  # ... when a threshold mode overflowed k_cap with every candidate (exact top-k_cap)
CAL_CAND = 8        # calibrated ladder size (gk::kCalCand)

MAX_CAND = 16
CTRL_SYNC_TIMEOUTS_U32 = 364 // 4   # GkCtrl::sync_timeouts (static_assert in gk_kernels.h)
CHUNK_ELEMS = 16384
REC_HDR = 4


def load(build_if_missing: bool = False) -> bool:
    """Load the native extension once.  Returns True when available."""
    global _loaded, _load_error
    if _loaded:
        return True
    with _lock:
        if _loaded:
            return True
        try:
            if not _LIB.exists() and build_if_missing:
                from . import build as _b
                _b.build()
            torch.ops.load_library(str(_LIB))
            _loaded = True
            if os.environ.get("GKSGD_BN_BLOCKS"):
                # workgroups per BatchNorm streaming pass (bn_act.hip, default 1024)
                torch.ops.gksgd.bn_set_blocks(int(os.environ["GKSGD_BN_BLOCKS"]))
        except BaseException as e:  # noqa: BLE001
            _load_error = e
    return _loaded


def native_available() -> bool:
    return load()


def library_path() -> str:
    return str(_LIB)


def require_native(t: torch.Tensor) -> None:
    if t.is_cuda and not load():
        raise RuntimeError(
            "gaussiank_sgd_amd native extension (%s) is not loadable on a GPU device: %r. "
            "Build it with `python -m gaussiank_sgd_amd.ops.build`." % (_LIB, _load_error))


def _ops():
    return torch.ops.gksgd


# ---------------------------------------------------------------------------
# per-bucket device buffers
# ---------------------------------------------------------------------------
class CompressBuffers:
    """ctrl block + workspace + packed send record for one bucket."""

    def __init__(self, k_cap: int, device: torch.device):
        device = torch.device(device)
        self.k_cap = int(k_cap)
        self.device = device
        if device.type == "cuda":
            require_native(torch.empty(0, device=device))
            ctrl_b = int(_ops().ctrl_bytes())
            ws_b = int(_ops().workspace_bytes())
        else:
            ctrl_b, ws_b = 512, 256
        # 256-byte alignment: the caching allocator returns >=512-byte aligned blocks
        self.ctrl = torch.zeros((ctrl_b + 7) // 8, dtype=torch.float64, device=device)
        self.ws = torch.zeros((ws_b + 255) // 256 * 64, dtype=torch.float32, device=device)
        self.record = torch.zeros(REC_HDR + 2 * self.k_cap, dtype=torch.int32, device=device)
        self.stats = torch.zeros(4, dtype=torch.float32, device=device)
        # calibrated Gaussian-k state of the CPU mirror (on GPU it lives in ctrl)
        self.cal = {"c": 0.0, "step": 0.0, "k": 0}

    def header(self) -> torch.Tensor:
        return self.record[:REC_HDR]

    def indices(self) -> torch.Tensor:
        return self.record[REC_HDR:REC_HDR + self.k_cap]

    def values(self) -> torch.Tensor:
        return self.record[REC_HDR + self.k_cap:].view(torch.float32)


def record_views(rec: torch.Tensor, k_cap: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    return rec[..., :REC_HDR], rec[..., REC_HDR:REC_HDR + k_cap], rec[..., REC_HDR + k_cap:].view(torch.float32)


# ---------------------------------------------------------------------------
# CPU mirror helpers
# ---------------------------------------------------------------------------
_M32 = 0xFFFFFFFF


# ---------------------------------------------------------------------------
# dropout / sampling seeds
# ---------------------------------------------------------------------------
_graph_words: dict = {}


def graph_seed_word(device) -> torch.Tensor:
    """The per-device int32 word that captured dropout kernels mix into their
    seed at run time (train/graph.py writes a new value before every replay)."""
    device = torch.device(device)
    w = _graph_words.get(device)
    if w is None:
        w = _graph_words[device] = torch.zeros(1, dtype=torch.int32, device=device)
    return w


def set_graph_seed(device, value: int) -> None:
    """Stream-ordered write of the replay word (before a graph replay)."""
    v = int(value) & 0xFFFFFFFF
    graph_seed_word(device).fill_(v - (1 << 32) if v >= (1 << 31) else v)


def capture_seed_word(device) -> Optional[torch.Tensor]:
    """The replay word when the current stream is being captured, else None."""
    if torch.device(device).type == "cuda" and torch.cuda.is_current_stream_capturing():
        return graph_seed_word(device)
    return None


def seed_generator() -> torch.Generator:
    """Host generator of the dropout seeds: derived from the process's torch
    seed (DLTrainer seeds it) and the rank, so ranks draw different masks and
    ``--seed`` changes them."""
    g = getattr(seed_generator, "_g", None)
    if g is None:
        import os
        base = (int(torch.initial_seed()) * 0x9E3779B97F4A7C15 + int(os.environ.get("RANK", "0")) * 7919) & (2 ** 63 - 1)
        g = seed_generator._g = torch.Generator().manual_seed(base)
    return g


def hash_u32(idx: torch.Tensor, seed: int) -> torch.Tensor:
    """Bit-exact mirror of gk::hash_u32 (murmur3 fmix32 of a Weyl sequence)."""
    i = idx.to(torch.int64) & _M32
    h = (i * 0x9E3779B1 + ((seed & _M32) * 0x85EBCA77 & _M32) + 0x27D4EB2F) & _M32
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & _M32
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & _M32
    h = h ^ (h >> 16)
    return h


def hash_key(idx: torch.Tensor, seed: int, valid: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Random-k key of gk::key_of<kKeyHash>: hash in [1, 2^32-2], 0 for invalid (padding) slots."""
    keys = hash_u32(idx, seed)
    keys = torch.where(keys == 0xFFFFFFFF, torch.full_like(keys, 0xFFFFFFFE), keys)
    keys = torch.where(keys == 0, torch.ones_like(keys), keys)
    if valid is not None:
        i = idx.to(torch.int64)
        words = valid.to(torch.int64) & 0xFFFFFFFF
        bit = (words[i >> 5] >> (i & 31)) & 1
        keys = torch.where(bit == 1, keys, torch.zeros_like(keys))
    return keys


def valid_bitmask(layout: Sequence[Tuple[int, int]], n: int, device) -> torch.Tensor:
    """int32 bitmask over n slots with bit i set for the real elements:
    ``layout`` = (offset, numel) per tensor (the rest is arena padding)."""
    bits = torch.zeros(((n + 31) // 32) * 32, dtype=torch.bool)
    for off, ln in layout:
        bits[off:off + ln] = True
    w = bits.view(-1, 32).to(torch.int64)
    words = (w << torch.arange(32, dtype=torch.int64)).sum(1)
    words = torch.where(words >= 2 ** 31, words - 2 ** 32, words)
    return words.to(torch.int32).to(device)


def abs_key(x: torch.Tensor) -> torch.Tensor:
    return x.contiguous().view(torch.int32).to(torch.int64) & 0x7FFFFFFF


def _bound_from_threshold(t: float) -> int:
    import struct
    tf = struct.unpack("f", struct.pack("f", t))[0] if t == t and abs(t) < 3.5e38 else t
    if not (tf >= 0.0):
        if tf < 0.0:
            return 0
        return 0x7FC00001
    if tf == float("inf"):
        return 0x7F800001
    bits = struct.unpack("I", struct.pack("f", tf))[0] & 0x7FFFFFFF
    return bits + 1


def _f32(x: float) -> float:
    import struct
    if x != x or abs(x) == float("inf"):
        return x
    if abs(x) >= 3.4028235677973366e38:
        return float("inf") if x > 0 else float("-inf")
    return struct.unpack("f", struct.pack("f", x))[0]


GAUSS_WALK = 6   # compress.hip kGaussWalk


def _gauss_ext(loops: int) -> bool:
    L = max(loops, 1)
    return min(L * (L + 1) // 2, MAX_CAND) <= GAUSS_WALK


def _candidates(mode: int, loops: int, z: float, fixed_thr: float, stats: Tuple[float, float, float, float]):
    """Candidate thresholds (|x| units) and key bounds, mirroring finalize_kernel."""
    mean, std, meanabs, maxabs = stats
    thr: List[float] = []
    if mode == MODE_GAUSSIAN:
        t0 = mean + z * std
        for s in range(loops):
            for b in range(s + 1):
                a = s - b
                t = t0
                for _ in range(b):
                    t *= 1.5
                for _ in range(a):
                    t *= 0.5
                thr.append(_f32(t))
        if _gauss_ext(loops):
            # overflow extension (compress.hip ladder_cands): dead slots up to
            # GAUSS_WALK, then t_top * 1.25^j above the walk's top node
            thr.extend([None] * (GAUSS_WALK - len(thr)))
            t = t0
            for _ in range(max(loops, 1) - 1):
                t *= 1.5
            for _ in range(MAX_CAND - GAUSS_WALK):
                t *= 1.25
                thr.append(_f32(t))
    elif mode in (MODE_REDSYNC, MODE_REDSYNCTRIM):
        mv = torch.tensor(meanabs, dtype=torch.float32)
        Mv = torch.tensor(maxabs, dtype=torch.float32)
        diff = Mv - mv
        if mode == MODE_REDSYNC:
            lo = [0.0] * 7
            hi = [0.0] * 7
            lo[0], hi[0] = 0.0, 1.0
            for i in range(7):
                mid = lo[i] + (hi[i] - lo[i]) / 2
                t = mv + torch.tensor(mid, dtype=torch.float32) * diff
                thr.append(float(t))
                if 2 * i + 2 < 7:
                    lo[2 * i + 1], hi[2 * i + 1] = lo[i], mid
                    lo[2 * i + 2], hi[2 * i + 2] = mid, hi[i]
        else:
            ratio = 1.0 - 0.2
            for _ in range(MAX_CAND):
                t = mv + torch.tensor(ratio, dtype=torch.float32) * diff
                thr.append(float(t))
                ratio = ratio - 0.2
    elif mode == MODE_THRESHOLD:
        thr.append(_f32(fixed_thr))
    return thr


def _decide(mode: int, loops: int, k: int, counts: Sequence[int]) -> int:
    if mode == MODE_GAUSSIAN:
        a = b = 0
        for loop in range(loops):
            c = counts[(a + b) * (a + b + 1) // 2 + b]
            if loop == loops - 1:
                break
            if c < 2 * k / 3:
                a += 1
            elif c > 4 * k / 3:
                b += 1
            else:
                break
        return (a + b) * (a + b + 1) // 2 + b
    if mode == MODE_REDSYNC:
        node = 0
        for depth in range(3):
            c = counts[node]
            if c > k and 2 * k > c:
                break
            if depth == 2:
                break
            node = 2 * node + 1 if c < k / 2 else 2 * node + 2
        return node
    if mode == MODE_REDSYNCTRIM:
        for j, c in enumerate(counts):
            if c >= k:
                return j
        return len(counts) - 1
    return 0


def _radix_topk_mask(keys: torch.Tensor, eligible: torch.Tensor, k: int) -> Tuple[torch.Tensor, int, int]:
    """Exact top-k by key with ties broken by lowest index (mirror of radix path).

    Returns (mask, K, quota): mask selects key > K plus the first `quota`
    elements with key == K in index order.
    """
    ek = keys[eligible]
    keff = min(int(k), int(ek.numel()))
    if keff <= 0:
        return torch.zeros_like(keys, dtype=torch.bool), 0, 0
    K = int(torch.topk(ek, keff).values[-1])
    gt = eligible & (keys > K)
    eq = eligible & (keys == K)
    quota = keff - int(gt.sum())
    eq_idx = torch.nonzero(eq).view(-1)[:quota]
    mask = gt.clone()
    mask[eq_idx] = True
    return mask, K, quota


def _cal_decide(bufs: CompressBuffers, k: int, thr: List[float], counts: Sequence[int], std: float) -> Tuple[int, bool]:
    """Mirror of decide_kernel's calibrated branch: (chosen, fallback); updates bufs.cal."""
    import math
    kd = float(k)
    best, closest, bestd, closed = -1, 0, 1e300, 1e300
    for j, c in enumerate(counts):
        d = abs(math.log((c if c > 0 else 0.5) / kd))
        if d < closed:
            closed, closest = d, j
        if 2.0 * kd / 3.0 <= c <= 4.0 * kd / 3.0 and d < bestd:
            bestd, best = d, j
    jc = best if best >= 0 else closest
    nc = len(counts)
    step = bufs.cal["step"]
    if best < 0 and (jc == 0 or jc == nc - 1):
        step *= 2.0
    elif 0 < jc < nc - 1 and counts[jc + 1] > 0:
        R = counts[jc - 1] / counts[jc + 1]
        if R > 1.0001:
            step *= min(max(math.log(1.7) / math.log(R), 0.5), 2.0)
        else:
            step *= 2.0
    bufs.cal["step"] = min(max(step, 0.002), 1.0)
    if std > 0.0 and thr[jc] > 0.0:
        bufs.cal["c"] = thr[jc] / std
    return jc, best < 0


def _overflow_alt(counts: Sequence[int], k: int, k_cap: int) -> int:
    """decide_kernel's magnitude-correct overflow rule: the candidate with the
    largest count in [2k/3, k_cap] (first on ties), -1 when none lands there."""
    alt, bc = -1, -1
    for j, c in enumerate(counts):
        if c <= k_cap and 3 * c >= 2 * k and c > bc:
            alt, bc = j, c
    return alt


def _key_thr(K: int) -> float:
    return float(torch.tensor([K & 0x7FFFFFFF], dtype=torch.int32).view(torch.float32))


def _cal_ladder(bufs: CompressBuffers, k: int, z: float, mean: float, std: float) -> List[float]:
    import math
    st = bufs.cal
    if st["k"] != k or not st["c"] > 0.0 or not st["step"] > 0.0:
        t0 = mean + z * std
        st["c"] = t0 / std if std > 0.0 and t0 > 0.0 else (z if z > 0.0 else 1.0)
        st["step"] = 0.105
        st["k"] = k
    tc = st["c"] * std
    return [tc * math.exp(st["step"] * (j - 0.5 * (CAL_CAND - 1))) for j in range(CAL_CAND)]


def compress_cpu_(g: torch.Tensor, r: torch.Tensor, bufs: CompressBuffers, mode: int, ec: bool, zero_g: bool,
                  loops: int, z: float, k: int, k_cap: int, seed: int = 0, fixed_thr: float = 0.0,
                  sample_p: float = 0.01, n_stats: int = 0, valid: Optional[torch.Tensor] = None,
                  u: Optional[torch.Tensor] = None) -> None:
    """Pure-torch mirror of gk::compress (same record layout and semantics).

    ``u``: DGC velocity (momentum correction already applied to g by the
    caller); sent indices are zeroed in it (momentum factor masking)."""
    with torch.no_grad():
        acc = g + r if ec else g.clone()
        r.copy_(acc)
        if zero_g:
            g.zero_()
        n = acc.numel()
        nst = int(n_stats) if n_stats and n_stats > 0 else n
        a64 = acc.double()
        s = float(a64.sum())
        ss = float((a64 * a64).sum())
        mean = s / nst
        var = (ss - s * s / nst) / (nst - 1) if nst > 1 else float("nan")
        std = max(var, 0.0) ** 0.5 if var == var else float("nan")
        absacc = acc.abs()
        meanabs = float(absacc.double().sum()) / nst
        maxabs = float(absacc.max()) if n else 0.0
        stats = (mean, std, meanabs, maxabs)
        bufs.stats.copy_(torch.tensor(stats, dtype=torch.float32))
        k = max(int(k), 1)
        ref_total = None   # the reference rule's count when it overflowed k_cap
        allm = torch.ones(n, dtype=torch.bool)

        def reselect(keys, bounds, thr, counts, chosen):
            # magnitude-correct overflow (decide_kernel): tighter candidate or exact top-k_cap
            alt = _overflow_alt(counts, k, k_cap)
            if alt >= 0:
                return keys >= bounds[alt], alt, thr[alt]
            m, K, _ = _radix_topk_mask(keys, allm, min(k_cap, n))
            return m, OVERFLOW_EXACT, _key_thr(K)

        if mode == MODE_GAUSSIAN_CAL:
            thr = _cal_ladder(bufs, k, z, mean, std)
            keys = abs_key(acc)
            bounds = [_bound_from_threshold(t) for t in thr]
            counts = [int((keys >= b).sum()) for b in bounds]
            chosen, fallback = _cal_decide(bufs, k, thr, counts, std)
            if fallback:
                mask, K, _ = _radix_topk_mask(keys, allm, k)
                chosen = CAL_FALLBACK
                thr_chosen = _key_thr(K)
            elif counts[chosen] > k_cap:
                ref_total = counts[chosen]
                mask, chosen, thr_chosen = reselect(keys, bounds, thr, counts, chosen)
            else:
                mask = keys >= bounds[chosen]
                thr_chosen = thr[chosen]
        elif mode in (MODE_GAUSSIAN, MODE_REDSYNC, MODE_REDSYNCTRIM, MODE_THRESHOLD):
            thr = _candidates(mode, loops, z, fixed_thr, stats)
            keys = abs_key(acc)
            bounds = [0xFFFFFFFF if t is None else _bound_from_threshold(t) for t in thr]
            thr = [0.0 if t is None else t for t in thr]
            counts = [int((keys >= b).sum()) for b in bounds]
            chosen = _decide(mode, loops, k, counts)
            if counts[chosen] > k_cap:
                ref_total = counts[chosen]
                mask, chosen, thr_chosen = reselect(keys, bounds, thr, counts, chosen)
            else:
                mask = keys >= bounds[chosen]
                thr_chosen = thr[chosen]
        elif mode in (MODE_TOPK, MODE_RANDOMK):
            idx = torch.arange(n, dtype=torch.int64)
            if mode == MODE_RANDOMK:
                keys = hash_key(idx, seed, valid)
            else:
                keys = abs_key(acc)
            mask, K, _ = _radix_topk_mask(keys, torch.ones(n, dtype=torch.bool), k)
            chosen = 0
            thr_chosen = float(torch.tensor([K & 0x7FFFFFFF], dtype=torch.int32).view(torch.float32))
        elif mode == MODE_DGC:
            idx = torch.arange(n, dtype=torch.int64)
            p = sample_p * 4294967296.0
            sthr = 0xFFFFFFFF if p >= 4294967295.0 else int(p)
            sampled = hash_u32(idx, seed) < sthr
            keys = abs_key(acc)
            skeys = torch.where(sampled, keys + 1, torch.zeros_like(keys))
            smask, Ks, _ = _radix_topk_mask(skeys, sampled, k)
            cand0 = keys >= Ks
            c0 = int(cand0.sum())
            if c0 > 4 * k / 3:
                mask, K, _ = _radix_topk_mask(keys, allm, k)
                chosen = 1
                thr_chosen = float(torch.tensor([K], dtype=torch.int32).view(torch.float32))
            elif c0 > k_cap:
                # only when k_cap < 4k/3: the three evaluated candidates of the GPU ladder
                _, K, _ = _radix_topk_mask(keys, allm, k)
                bounds = [Ks, K + 1, K]
                thr = [float(torch.tensor([max(Ks - 1, 0)], dtype=torch.int32).view(torch.float32)),
                       _key_thr(K), _key_thr(K)]
                counts = [int((keys >= b).sum()) for b in bounds]
                ref_total = c0
                mask, chosen, thr_chosen = reselect(keys, bounds, thr, counts, 0)
            else:
                mask = cand0
                chosen = 0
                thr_chosen = float(torch.tensor([max(Ks - 1, 0)], dtype=torch.int32).view(torch.float32))
        else:
            raise ValueError("bad mode %d" % mode)
        sel = torch.nonzero(mask).view(-1)
        total = int(sel.numel())
        sent = min(total, k_cap)
        sel = sel[:sent]
        rec = bufs.record
        rec.zero_()
        rec[0] = sent
        rec[1] = min(total if ref_total is None else ref_total, 0x7FFFFFFF)
        rec[2] = chosen
        rec[3] = torch.tensor([thr_chosen], dtype=torch.float32).view(torch.int32)[0]
        rec[REC_HDR:REC_HDR + sent] = sel.to(torch.int32)
        rec[REC_HDR + k_cap:REC_HDR + k_cap + sent] = acc[sel].view(torch.int32)
        r[sel] = 0.0
        if u is not None:
            u[sel] = 0.0


def compress_(g: torch.Tensor, r: torch.Tensor, bufs: CompressBuffers, mode: int, ec: bool = True,
              zero_g: bool = True, loops: int = 3, z: float = 0.0, k: int = 1, k_cap: Optional[int] = None,
              seed: int = 0, fixed_thr: float = 0.0, sample_p: float = 0.01, n_stats: int = 0,
              valid: Optional[torch.Tensor] = None, mc: Optional[dict] = None,
              seed_dev: Optional[torch.Tensor] = None, handoff: int = -1) -> None:
    """Sparsify ``g`` (+ residual ``r``) into ``bufs.record``.  Async on GPU.

    ``seed_dev``: optional int32 device word holding the seed (read by the
    kernels at run time instead of ``seed``): a captured hipGraph replays with
    whatever the host wrote there before the replay.

    ``n_stats``: element count used for mean/std (the real, unpadded bucket
    size; padding elements are zeros and do not change the sums).
    ``valid``: int32 bitmask of the real elements (``valid_bitmask``); random-k
    never picks padding slots.
    ``mc``: DGC momentum correction fused into the statistics pass -- dict with
    ``u`` and ``w`` (bucket slices of the velocity / weight arenas), ``chunks``
    (chunk table), ``begin``/``count`` (this bucket's rows), ``base`` (bucket
    arena offset), ``groups`` (param-group dicts with momentum/weight_decay),
    and optionally ``chunk_list`` (decoded rows, CPU path).  The sent indices
    are zeroed in ``u`` (momentum factor masking).
    """
    k_cap = bufs.k_cap if k_cap is None else int(k_cap)
    if g.is_cuda:
        require_native(g)
        kw = {}
        if valid is not None:
            kw["valid"] = valid
        if seed_dev is not None:
            kw["seed_dev"] = seed_dev
        if mc is not None:
            if not zero_g:
                raise ValueError("momentum-corrected compress zeroes g")
            kw.update(u=mc["u"], w=mc["w"], chunks=mc["chunks"], chunk_begin=int(mc["begin"]),
                      chunk_count=int(mc["count"]), chunk_base=int(mc["base"]),
                      mc_mu=[float(p["momentum"]) for p in mc["groups"]],
                      mc_wd=[float(p.get("weight_decay", 0.0)) for p in mc["groups"]])
        _ops().compress(g, r, bufs.ctrl, bufs.ws, bufs.record, int(mode), bool(ec), bool(zero_g), int(loops),
                        float(z), float(fixed_thr), float(sample_p), int(k), int(k_cap), int(seed) & 0xFFFFFFFF,
                        int(n_stats), bufs.stats, handoff=int(handoff), **kw)
    else:
        if seed_dev is not None:
            seed = int(seed_dev.view(-1)[0]) & 0xFFFFFFFF
        u = None
        if mc is not None:
            base = int(mc["base"])
            cl = mc.get("chunk_list")
            cl = cl if cl is not None else _decode_chunks(mc["chunks"])
            rows = [(st - base, ln, gi, sg) for st, ln, gi, sg in cl[int(mc["begin"]):int(mc["begin"]) + int(mc["count"])]]
            momentum_correct_(mc["u"], g, mc["w"], None, 0, len(rows), mc["groups"], rows)
            u = mc["u"]
        compress_cpu_(g, r, bufs, mode, ec, zero_g, loops, z, k, k_cap, seed, fixed_thr, sample_p, n_stats,
                      valid, u)


def ctrl_fields(bufs: CompressBuffers) -> dict:
    """Decode the GkCtrl block (host sync; tests/diagnostics only)."""
    raw = bufs.ctrl.detach().cpu()
    d = raw.numpy().view("float64")
    out = {"sum": d[0], "sumsq": d[1], "sumabs": d[2], "maxabs_raw": d[3], "mean": d[4], "std": d[5],
           "meanabs": d[6], "maxabs": d[7]}
    u32 = raw.numpy().view("uint32")
    out["bounds"] = [int(x) for x in u32[16:16 + MAX_CAND]]
    out["ncand"] = int(raw.numpy().view("int32")[16 + MAX_CAND])
    out["chosen"] = int(raw.numpy().view("int32")[17 + MAX_CAND])
    out["sync_timeouts"] = int(u32[CTRL_SYNC_TIMEOUTS_U32])
    return out


def sync_timeouts(bufs: CompressBuffers) -> int:
    """Sticky count of expired bounded spins in the fused decide / fallback
    grid of this bucket's calls (compress.hip sync_timeout; host sync)."""
    return int(bufs.ctrl.detach().cpu().numpy().view("uint32")[CTRL_SYNC_TIMEOUTS_U32])


# ---------------------------------------------------------------------------
# aggregation
# ---------------------------------------------------------------------------
def scatter_add_records_(dst: torch.Tensor, records: torch.Tensor, P: int, k_cap: int, scale: float,
                         deterministic: bool = False) -> None:
    """dst[idx_r] += val_r * scale for every rank r (records [P, 4+2k_cap])."""
    if dst.is_cuda:
        require_native(dst)
        _ops().scatter_add_records(dst, records.contiguous(), int(P), int(k_cap), float(scale), bool(deterministic))
        return
    rec = records.view(P, REC_HDR + 2 * k_cap)
    if P == 1:
        cnt = min(int(rec[0, 0]), k_cap)
        idx = rec[0, REC_HDR:REC_HDR + cnt].long()
        val = rec[0, REC_HDR + k_cap:REC_HDR + k_cap + cnt].view(torch.float32)
        dst.index_add_(0, idx, val * scale)
        return
    idx, s = _rank_ordered_sum(rec, P, k_cap, dst.numel())
    dst[idx] += s * torch.tensor(scale, dtype=torch.float32)   # fp32 scale, as the kernel


def _rank_ordered_sum(rec: torch.Tensor, P: int, k_cap: int, n: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """(unique indices, fp32 sums in rank order) of P packed records -- the
    arithmetic of reduce_records_kernel: s = ((0 + v_0) + v_1) + ..."""
    acc = torch.zeros(n, dtype=torch.float32)
    seen = torch.zeros(n, dtype=torch.bool)
    for r in range(P):
        cnt = min(int(rec[r, 0]), k_cap)
        idx = rec[r, REC_HDR:REC_HDR + cnt].long()
        val = rec[r, REC_HDR + k_cap:REC_HDR + k_cap + cnt].view(torch.float32)
        acc.index_add_(0, idx, val)   # unique within one record: one fp32 add per index
        seen[idx] = True
    idx = torch.nonzero(seen).view(-1)
    return idx, acc[idx]


def apply_records_sgd_(w: torch.Tensor, w_bf16: Optional[torch.Tensor], records: torch.Tensor, P: int, k_cap: int,
                       scale: float, lr: float, lr_mult: Optional[torch.Tensor] = None) -> None:
    """Sparse SGD from the packed records: w[i] -= lr * scale * sum_r val_r[i]."""
    if w.is_cuda:
        require_native(w)
        _ops().apply_records_sgd(w, w_bf16, records.contiguous(), int(P), int(k_cap), float(scale), float(lr), lr_mult)
        return
    rec = records.view(P, REC_HDR + 2 * k_cap)
    idx, s = _rank_ordered_sum(rec, P, k_cap, w.numel())
    lr_eff = torch.tensor(lr, dtype=torch.float32)
    if lr_mult is not None:
        lr_eff = lr_eff * lr_mult.float().cpu().view(())
    w[idx] = w[idx] - lr_eff * (s * torch.tensor(scale, dtype=torch.float32))
    if w_bf16 is not None:
        w_bf16[idx] = w[idx].to(torch.bfloat16)


def arena_digest(x: torch.Tensor) -> Tuple[int, int]:
    """(fp64 sum bits, 64-bit content hash) of a flat fp32 arena -- equal digests on
    two replicas mean bit-identical weights (up to a 2^-64 hash collision)."""
    if x.is_cuda:
        require_native(x)
        out = torch.zeros(2, dtype=torch.int64, device=x.device)
        ws = torch.zeros(2048, dtype=torch.int64, device=x.device)
        _ops().arena_digest(x, out, ws)
        a, b = out.cpu().tolist()
        return int(a) & 0xFFFFFFFFFFFFFFFF, int(b) & 0xFFFFFFFFFFFFFFFF
    import struct

    import numpy as np
    xs = x.detach().contiguous().view(-1)
    s = float(xs.double().sum())
    b = xs.view(torch.int32).numpy().view(np.uint32).astype(np.uint64)
    i = np.arange(xs.numel(), dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (b << np.uint64(32)) ^ (i * np.uint64(0x9E3779B97F4A7C15))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
        tot = int(z.sum(dtype=np.uint64))
    return struct.unpack("<Q", struct.pack("<d", s))[0], tot


def fill_zero_(dst: torch.Tensor) -> None:
    if dst.is_cuda:
        require_native(dst)
        _ops().fill_zero(dst)
    else:
        dst.zero_()


# ---------------------------------------------------------------------------
# sign-bucket compressor
# ---------------------------------------------------------------------------
def sign_bucket_compress_(x: torch.Tensor, mask: torch.Tensor, means: torch.Tensor, ws: Optional[torch.Tensor]) -> None:
    if x.is_cuda:
        require_native(x)
        _ops().sign_bucket_compress(x, mask, means, ws)
        return
    pos = x >= 0
    mask.copy_(pos.to(torch.uint8))
    mp = x[pos].mean() if bool(pos.any()) else torch.zeros((), dtype=x.dtype)
    mn = x[~pos].mean() if bool((~pos).any()) else torch.zeros((), dtype=x.dtype)
    means[0] = mp
    means[1] = mn
    x.sub_(torch.where(pos, means[0], means[1]))


def sign_bucket_decompress_(x: torch.Tensor, mask: torch.Tensor, means: torch.Tensor) -> None:
    if x.is_cuda:
        require_native(x)
        _ops().sign_bucket_decompress(x, mask, means)
        return
    x.add_(torch.where(mask.bool(), means[0], means[1]))


def sign_bucket_ws(device) -> Optional[torch.Tensor]:
    device = torch.device(device)
    if device.type != "cuda":
        return None
    require_native(torch.empty(0, device=device))
    nb = int(_ops().sign_bucket_workspace_bytes())
    return torch.zeros((nb + 7) // 8, dtype=torch.float64, device=device)


# ---------------------------------------------------------------------------
# fused optimizers
# ---------------------------------------------------------------------------
def make_chunk_table(segments: Sequence[Tuple[int, int, int, int]], device) -> torch.Tensor:
    """segments: (start, numel, group, seg_id) -> int64[nchunks*2] chunk table."""
    words: List[int] = []
    for start, numel, group, seg in segments:
        off = 0
        while off < numel:
            ln = min(CHUNK_ELEMS, numel - off)
            words.append(start + off)
            words.append((ln & 0xFFFFFFFF) | ((group & 0xFFFF) << 32) | ((seg & 0x7FFF) << 48))
            off += ln
    return torch.tensor(words, dtype=torch.int64, device=device)


def _decode_chunks(chunks: torch.Tensor):
    c = chunks.view(-1, 2).cpu()
    out = []
    for start, w in c.tolist():
        out.append((start, w & 0xFFFFFFFF, (w >> 32) & 0xFFFF, (w >> 48) & 0x7FFF))
    return out


def momentum_correct_(u: torch.Tensor, g: torch.Tensor, w: torch.Tensor, chunks: torch.Tensor, begin: int,
                      count: int, groups: Sequence[dict], chunk_list=None) -> None:
    """DGC momentum correction over chunks [begin, begin+count): u = mu*u + g + wd*w; g = u.

    ``groups``: dicts with ``momentum`` and ``weight_decay`` per param group.
    ``chunk_list``: decoded chunks (CPU path; avoids a device->host copy).
    """
    if u.is_cuda:
        require_native(u)
        _ops().momentum_correct(u, g, w, chunks, int(begin), int(count), [float(p["momentum"]) for p in groups],
                                [float(p.get("weight_decay", 0.0)) for p in groups])
        return
    cl = chunk_list if chunk_list is not None else _decode_chunks(chunks)
    for start, ln, gi, _ in cl[begin:begin + count]:
        p = groups[gi]
        us, gs, ws = u[start:start + ln], g[start:start + ln], w[start:start + ln]
        us.mul_(float(p["momentum"])).add_(gs).add_(ws, alpha=float(p.get("weight_decay", 0.0)))
        gs.copy_(us)


def mask_records_(u: torch.Tensor, record: torch.Tensor, k_cap: int) -> None:
    """Momentum factor masking: u[idx] = 0 for the indices one rank sent."""
    if u.is_cuda:
        require_native(u)
        _ops().mask_records(u, record, int(k_cap))
        return
    cnt = int(record[0])
    u[record[REC_HDR:REC_HDR + cnt].long()] = 0.0


def _same_order(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Same shape and the same element order in memory (size-1 dims ignored)."""
    if a.shape != b.shape:
        return False
    return all(n == 1 or sa == sb for n, sa, sb in zip(a.shape, a.stride(), b.stride()))


def _dense(t: torch.Tensor) -> bool:
    """Non-overlapping and dense: some permutation of the dims is contiguous."""
    dims = sorted((st, n) for n, st in zip(t.shape, t.stride()) if n != 1)
    expect = 1
    for st, n in dims:
        if st != expect:
            return False
        expect *= n
    return True


def accum_grad_(dst: torch.Tensor, src: torch.Tensor) -> None:
    """dst (fp32 arena view) += src (bf16/fp32 gradient with the same element order)."""
    native_ok = src.dtype in (torch.bfloat16, torch.float32) and _same_order(dst, src) and _dense(src) and \
        _dense(dst)
    if dst.is_cuda and native_ok:
        require_native(dst)
        _ops().accum_grad(dst, src)
    else:
        dst.add_(src.to(dst.dtype))


def cast_bf16_(dst: torch.Tensor, src: torch.Tensor) -> None:
    if dst.is_cuda:
        require_native(dst)
        _ops().cast_bf16(dst, src)
    else:
        dst.copy_(src)


def fused_sgd_(w: torch.Tensor, m: Optional[torch.Tensor], g: torch.Tensor, chunks: torch.Tensor,
               groups: Sequence[dict], zero_grad: bool = True, grad_scale: Optional[torch.Tensor] = None,
               w_bf16: Optional[torch.Tensor] = None, lr_mult: Optional[torch.Tensor] = None) -> None:
    """groups: dicts with lr, momentum, dampening, weight_decay, nesterov, first_step.

    ``w_bf16``: optional bf16 shadow arena rewritten from the new weights in
    the same pass (the compute copy used by bf16 convolutions / GEMMs).
    ``lr_mult``: optional fp32 device scalar multiplying every lr, read by the
    kernel (a captured HIP graph follows the host lr schedule through it).
    """
    if w.is_cuda:
        require_native(w)
        _ops().fused_sgd(w, m, g, chunks, [float(p["lr"]) for p in groups], [float(p["momentum"]) for p in groups],
                         [float(p.get("dampening", 0.0)) for p in groups],
                         [float(p.get("weight_decay", 0.0)) for p in groups],
                         [int(bool(p.get("nesterov", False))) for p in groups],
                         [int(bool(p.get("first_step", False))) for p in groups], bool(zero_grad), grad_scale,
                         w_bf16, lr_mult)
        return
    gs = float(grad_scale) if grad_scale is not None else 1.0
    lm = float(lr_mult) if lr_mult is not None else 1.0
    for start, ln, gi, _ in _decode_chunks(chunks):
        p = groups[gi]
        ws = w[start:start + ln]
        d = g[start:start + ln] * gs
        wd = float(p.get("weight_decay", 0.0))
        if wd != 0:
            d = d + wd * ws
        mom = float(p["momentum"])
        if mom != 0:
            ms = m[start:start + ln]
            if p.get("first_step", False):
                ms.copy_(d)
            else:
                ms.mul_(mom).add_(d, alpha=1 - float(p.get("dampening", 0.0)))
            d = d + mom * ms if p.get("nesterov", False) else ms
        ws.add_(d, alpha=-float(p["lr"]) * lm)
        if w_bf16 is not None:
            w_bf16[start:start + ln].copy_(ws)
        if zero_grad:
            g[start:start + ln].zero_()


def segmented_sumsq_(w: torch.Tensor, g: torch.Tensor, chunks: torch.Tensor, out: torch.Tensor) -> None:
    if w.is_cuda:
        require_native(w)
        _ops().segmented_sumsq(w, g, chunks, out)
        return
    for start, ln, _, seg in _decode_chunks(chunks):
        out[2 * seg] += float((w[start:start + ln].double() ** 2).sum())
        out[2 * seg + 1] += float((g[start:start + ln].double() ** 2).sum())


def fused_lars_(w: torch.Tensor, m: torch.Tensor, g: torch.Tensor, chunks: torch.Tensor, seg_sumsq: torch.Tensor,
                groups: Sequence[dict]) -> None:
    if w.is_cuda:
        require_native(w)
        _ops().fused_lars(w, m, g, chunks, seg_sumsq, [float(p["lr"]) for p in groups],
                          [float(p["momentum"]) for p in groups], [float(p["weight_decay"]) for p in groups],
                          [float(p["eeta"]) for p in groups], [float(p["epsilon"]) for p in groups])
        return
    for start, ln, gi, seg in _decode_chunks(chunks):
        p = groups[gi]
        wn = float(seg_sumsq[2 * seg]) ** 0.5
        gn = float(seg_sumsq[2 * seg + 1]) ** 0.5
        trust = 1.0
        if wn > 0 and gn > 0:
            trust = p["eeta"] * wn / (gn + p["weight_decay"] * wn + p["epsilon"])
        trust = min(max(trust, 0.0), 50.0)
        ws = w[start:start + ln]
        d = (g[start:start + ln] + p["weight_decay"] * ws).clamp_(-10.0, 10.0)
        ms = m[start:start + ln]
        ms.mul_(p["momentum"]).add_(d, alpha=p["lr"] * trust)
        ws.sub_(ms)


def clip_grad_norm_(g: torch.Tensor, max_norm: float, ws: Optional[torch.Tensor] = None,
                    coef: Optional[torch.Tensor] = None, norm: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Global-norm clip of a flat gradient arena, no host sync on GPU.  Returns the norm tensor."""
    if norm is None:
        norm = torch.zeros(1, dtype=torch.float32, device=g.device)
    if coef is None:
        coef = torch.zeros(1, dtype=torch.float32, device=g.device)
    if g.is_cuda:
        require_native(g)
        if ws is None:
            ws = torch.zeros(1024, dtype=torch.float64, device=g.device)
        _ops().clip_grad_norm(g, float(max_norm), ws, coef, norm)
        return norm
    nrm = float(g.double().norm())
    c = min(1.0, max_norm / (nrm + 1e-6))
    norm.fill_(nrm)
    coef.fill_(c)
    if c < 1.0:
        g.mul_(c)
    return norm


# ---------------------------------------------------------------------------
# RCCL engine
# ---------------------------------------------------------------------------
def rccl_engine_class():
    if not load():
        raise RuntimeError("native extension unavailable: %r" % (_load_error,))
    return torch.classes.gksgd.RcclEngine
