"""Fused multi-head self-attention (``csrc/kernels/attn.hip``), head dim 64.

``self_attention(qkv, heads, p)`` takes the packed QKV projection
``[B, T, 3 * heads * 64]`` (the ``[B, T, 3, heads, 64]`` layout of BERT's fused
QKV linear) and returns ``softmax(q k^T / 8) -> dropout_p -> @ v`` merged back
to ``[B, T, heads * 64]`` -- the input layout of the attention-output linear.
On a GPU with bf16 activations (or fp32, the reference's precision:
``csrc/kernels/attn_f32.hip`` on fp32 MFMA) this is one flash-style HIP kernel forward and
two backward (dQ with ``delta = rowsum(dO * O)``, then dK / dV); nothing of
size T x T is stored and there are no head split / merge copies: the kernels
read q, k, v with the packed row stride and write ``dqkv`` in the projection's
own layout.  The dropout mask is a hash of (seed, b*heads + h, query, key),
regenerated in the backward.  Elsewhere (CPU, masks, other head dims)
it is ``F.scaled_dot_product_attention`` with identical semantics.

Not in the reference (its model zoo has no transformer); BASELINE config 5
(BERT-base MLM) runs it.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import capture_seed_word, hash_u32, load, seed_generator

HEAD_DIM = 64


def _ops():
    return torch.ops.gksgd


def drop_threshold(p: float) -> int:
    """16-bit drop threshold of the kernels (keep iff hash >> 16 >= thr)."""
    if p <= 0.0:
        return 0
    return min(int(round(p * 65536.0)), 65535)


def drop_scale(p: float) -> float:
    thr = drop_threshold(p)
    return 65536.0 / (65536 - thr) if thr else 1.0


def dropout_mask(B: int, heads: int, T: int, p: float, seed: int, device, seed_dev=None) -> torch.Tensor:
    """The kernels' keep mask as bool [B, heads, T, T] (tests / CPU mirror);
    ``seed_dev``: the replay word the captured kernels mixed in."""
    device = torch.device(device)
    if device.type == "cuda":
        load()
        m = torch.empty(B, heads, T, T, dtype=torch.uint8, device=device)
        _ops().attn_dropout_mask(m, B, heads, T, float(p), int(seed), seed_dev)
        return m.bool()
    # one 32-bit hash per pair of keys: low half -> even key, high half -> odd key
    h = hash_u32(torch.arange(B * heads * T * T // 2, dtype=torch.int64), int(seed) & 0xFFFFFFFF)
    u = torch.stack([h & 0xFFFF, h >> 16], dim=1)
    return (u >= drop_threshold(p)).view(B, heads, T, T)


def reference_attention(qkv: torch.Tensor, heads: int, p: float = 0.0, seed: int = 0) -> torch.Tensor:
    """fp32 composition with the kernels' exact dropout mask (autograd-able)."""
    B, T, H3 = qkv.shape
    d = H3 // (3 * heads)
    x = qkv.float().view(B, T, 3, heads, d)
    q, k, v = (x[:, :, i].transpose(1, 2) for i in range(3))
    s = torch.matmul(q, k.transpose(-1, -2)) / d ** 0.5
    a = torch.softmax(s, dim=-1)
    if p > 0:
        keep = dropout_mask(B, heads, T, p, seed, qkv.device)
        a = a * keep.to(a.dtype) * drop_scale(p)
    o = torch.matmul(a, v)
    return o.transpose(1, 2).reshape(B, T, heads * d)


class _FlashAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, heads, p, seed, seed_dev=None):
        # seed_dev: the graph replay word (ops.graph_seed_word) under capture --
        # forward and backward of one replay read the same word
        B, T, _ = qkv.shape
        out = torch.empty(B, T, heads * HEAD_DIM, dtype=torch.bfloat16, device=qkv.device)
        lse = torch.empty(B * heads * T, dtype=torch.float32, device=qkv.device)
        _ops().attn_fwd(qkv, out, lse, int(heads), float(p), int(seed), seed_dev)
        ctx.save_for_backward(qkv, out, lse)
        ctx.heads, ctx.p, ctx.seed, ctx.seed_dev = int(heads), float(p), int(seed), seed_dev
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        dout = dout.to(torch.bfloat16).contiguous()
        delta = torch.empty_like(lse)
        dqkv = torch.empty_like(qkv)
        _ops().attn_bwd(qkv, out, dout, lse, delta, dqkv, ctx.heads, ctx.p, ctx.seed, ctx.seed_dev)
        return dqkv, None, None, None, None


class _FlashAttnF32Fn(torch.autograd.Function):
    """fp32 twin of _FlashAttnFn (csrc/kernels/attn_f32.hip): fp32 operands on
    v_mfma_f32_16x16x4_f32, the same dropout hashes."""

    @staticmethod
    def forward(ctx, qkv, heads, p, seed, seed_dev=None):
        B, T, _ = qkv.shape
        out = torch.empty(B, T, heads * HEAD_DIM, dtype=torch.float32, device=qkv.device)
        lse = torch.empty(B * heads * T, dtype=torch.float32, device=qkv.device)
        _ops().attn_f32_fwd(qkv, out, lse, int(heads), float(p), int(seed), seed_dev)
        ctx.save_for_backward(qkv, out, lse)
        ctx.heads, ctx.p, ctx.seed, ctx.seed_dev = int(heads), float(p), int(seed), seed_dev
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        dout = dout.to(torch.float32).contiguous()
        delta = torch.empty_like(lse)
        dqkv = torch.empty_like(qkv)
        _ops().attn_f32_bwd(qkv, out, dout, lse, delta, dqkv, ctx.heads, ctx.p, ctx.seed, ctx.seed_dev)
        return dqkv, None, None, None, None


def _compute_dtype(qkv: torch.Tensor):
    """bf16 under bf16 autocast; otherwise the storage dtype -- but an
    autocast to any OTHER dtype (fp16) takes the SDPA composition, which
    follows autocast (as ops/ln.py and ops/linear.py do)."""
    if torch.is_autocast_enabled("cuda"):
        return torch.bfloat16 if torch.get_autocast_dtype("cuda") == torch.bfloat16 else None
    return qkv.dtype if qkv.dtype in (torch.bfloat16, torch.float32) else None


def fused_available(qkv: torch.Tensor, heads: int) -> bool:
    """The HIP kernels take this call: bf16 (autocast or bf16 activations) or
    fp32 (no autocast: the reference's precision), head dim 64, T % 128 == 0."""
    if not qkv.is_cuda or qkv.dim() != 3 or qkv.shape[-1] != 3 * heads * HEAD_DIM:
        return False
    dt = _compute_dtype(qkv)
    if dt is None or not load():
        return False
    if dt == torch.float32:
        return bool(_ops().attn_f32_supported(qkv.shape[1], HEAD_DIM))
    return bool(_ops().attn_supported(qkv.shape[1], HEAD_DIM))


def _sdpa(qkv: torch.Tensor, heads: int, p: float, attn_mask=None) -> torch.Tensor:
    B, T, H3 = qkv.shape
    d = H3 // (3 * heads)
    x = qkv.view(B, T, 3, heads, d)
    q, k, v = (x[:, :, i].transpose(1, 2) for i in range(3))
    o = F.scaled_dot_product_attention(q, k, v, attn_mask=attn_mask, dropout_p=p)
    return o.transpose(1, 2).reshape(B, T, heads * d)


def self_attention(qkv: torch.Tensor, heads: int, p: float = 0.0, training: bool = True,
                   attn_mask=None, seed: int = None) -> torch.Tensor:
    """``[B, T, 3*heads*d]`` packed projection -> ``[B, T, heads*d]`` attention output."""
    p = float(p) if training else 0.0
    if attn_mask is None and fused_available(qkv, heads):
        if seed is None:
            seed = int(torch.randint(0, 2 ** 31 - 1, (1,), generator=seed_generator())) if p > 0 else 0
        seed_dev = capture_seed_word(qkv.device) if p > 0 else None
        if _compute_dtype(qkv) == torch.float32:
            return _FlashAttnF32Fn.apply(qkv.contiguous(), heads, p, seed, seed_dev)
        return _FlashAttnFn.apply(qkv.to(torch.bfloat16).contiguous(), heads, p, seed, seed_dev)
    return _sdpa(qkv, heads, p, attn_mask)
