"""fp32 matmul algorithm selection (ops/conv1x1.py set_f32_matmul) on the CPU:
the bf16x6 candidates are offered only in "bf16x6" mode and only for fp32
operands, their cfgs carry the 100000 digit (gemm.hip nt_unit_f32 /
tn_unit_f32x), split-K keeps both digits, autotune keys are tagged so the two
modes never share a cached choice, and bench.py defaults to bf16x6.

The split itself (exact hi + mid + lo decomposition, six products of order
<= 2) is mirrored here in numpy/torch to pin its error bound; the kernels are
checked against fp64 on the GPU (tests/test_gemm_x6_gpu.py)."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gaussiank_sgd_amd.ops import conv1x1 as cv  # noqa: E402


@pytest.fixture
def mode():
    prev = cv.f32_matmul()
    yield
    cv.set_f32_matmul(prev)


def test_modes_and_candidates(mode):
    cv.set_f32_matmul("native")
    nat = cv._nt_cfgs(torch.float32)
    assert all(c < cv.X6 for c in nat)
    assert cv._dkey(torch.float32) == ("f32",)
    assert all(c < cv.X6 for c, _ in cv._tn_cfgs(torch.float32))
    prev = cv.set_f32_matmul("bf16x6")
    assert prev == "native" and cv.f32_matmul() == "bf16x6"
    x6 = cv._nt_cfgs(torch.float32)
    assert set(nat) < set(x6)
    extra = [c for c in x6 if c >= cv.X6]
    assert extra and all(c // cv.X6 in (1, 2, 3) and (c % cv.X6) // 10000 == 0 for c in extra)
    assert cv._dkey(torch.float32) == ("f32", "x6")
    assert any(c >= cv.X6 for c, _ in cv._tn_cfgs(torch.float32))
    # bf16 operands are untouched by the fp32 algorithm choice
    assert cv._nt_cfgs(torch.bfloat16) == cv._NT_CFGS and cv._dkey(torch.bfloat16) == ()
    assert cv._tn_cfgs(torch.bfloat16) == cv._TN_CFGS
    # split-K: S in the 10000 digit, the bf16x6 flag in the 100000 digit
    sk = cv._splitk_cfgs(torch.float32, 1568, 512, 2048)
    assert any(c >= cv.X6 for c in sk)
    for c in sk:
        assert (c // 10000) % 10 in (2, 4, 8)
    with pytest.raises(ValueError):
        cv.set_f32_matmul("tf32")


def test_keys_do_not_collide(mode):
    cv.set_f32_matmul("native")
    k1 = cv._dgrad_key(512, 256, 14, 14, 1024, 1, 1, torch.float32)
    cv.set_f32_matmul("bf16x6")
    k2 = cv._dgrad_key(512, 256, 14, 14, 1024, 1, 1, torch.float32)
    assert k1 != k2 and k2[:len(k1)] == k1
    assert cv.dgrad_key_dtype(k2) == torch.float32


def _split3(x: np.ndarray):
    """numpy mirror of mfma_util.h split3x8: round-to-nearest-even bf16 parts."""
    def rne_bf16(v):
        u = v.astype(np.float32).view(np.uint32).astype(np.uint64)
        u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
        return u.astype(np.uint32).view(np.float32)
    hi = rne_bf16(x)
    r = (x - hi).astype(np.float32)
    mid = rne_bf16(r)
    lo = rne_bf16((r - mid).astype(np.float32))
    return hi, mid, lo


def test_split_is_exact_and_products_bound():
    rng = np.random.default_rng(0)
    x = (rng.standard_normal(100000) * np.exp(rng.uniform(-20, 20, 100000))).astype(np.float32)
    hi, mid, lo = _split3(x)
    # exact: the three parts sum back to x in fp64
    assert np.array_equal(hi.astype(np.float64) + mid + lo, x.astype(np.float64))
    assert np.all(np.abs(mid) <= 2.0 ** -8 * np.abs(x))
    assert np.all(np.abs(lo) <= 2.0 ** -16 * np.abs(x))
    # the dropped products (mid*lo, lo*mid, lo*lo) stay below ~2^-23 |a b|
    y = (rng.standard_normal(100000)).astype(np.float32)
    h2, m2, l2 = _split3(y)
    a = [v.astype(np.float64) for v in (hi, mid, lo)]
    b = [v.astype(np.float64) for v in (h2, m2, l2)]
    kept = sum(a[i] * b[j] for i in range(3) for j in range(3) if i + j <= 2)
    exact = x.astype(np.float64) * y
    rel = np.abs(kept - exact) / np.maximum(np.abs(exact), 1e-300)
    assert rel.max() <= 1.01 * 2.0 ** -23


def test_bench_defaults_to_bf16x6(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    monkeypatch.delenv("GKSGD_F32_MATMUL", raising=False)
    import importlib
    import bench
    importlib.reload(bench)
    assert bench.parse().f32_matmul == "bf16x6"
    monkeypatch.setattr(sys, "argv", ["bench.py", "--f32-matmul", "native"])
    assert bench.parse().f32_matmul == "native"


def _xcd_remap2(L_x, L_y, gx, gy):
    """Python mirror of gemm_kern.h xcd_remap2 (GK_XCD_REMAP = 1)."""
    G = gx * gy
    if G % 8 or G < 16:
        return L_x, L_y
    L = L_x + L_y * gx
    q = (L & 7) * (G >> 3) + (L >> 3)
    return (q % gx, q // gx) if gy >= 8 else (q // gy, q % gy)


def _xcd_remap3(x, y, z, gx, gy, gz):
    G = gx * gy * gz
    if G % 8 or G < 16:
        return x, y, z
    L = x + (y + z * gy) * gx
    q = (L & 7) * (G >> 3) + (L >> 3)
    return q % gx, (q // gx) % gy, q // (gx * gy)


@pytest.mark.parametrize("gx,gy", [(21, 24), (512, 2), (256, 1), (7, 3), (64, 12), (128, 8), (5, 16), (3, 1)])
def test_xcd_block_order_is_a_bijection(gx, gy):
    """Every logical (M start, N tile) of the grid is run by exactly one block,
    and (grids of >= 8 N tiles) an XCD's blocks cover a contiguous run of N
    tiles: the XCD-aware order changes only which CU runs a tile."""
    seen = {}
    for by in range(gy):
        for bx in range(gx):
            seen.setdefault(_xcd_remap2(bx, by, gx, gy), []).append((bx, by))
    assert len(seen) == gx * gy and all(len(v) == 1 for v in seen.values())
    assert all(0 <= x < gx and 0 <= y < gy for x, y in seen)
    G = gx * gy
    if G % 8 == 0 and G >= 16 and gy >= 8 and gy % 8 == 0:
        for xcd in range(8):
            ys = {_xcd_remap2(L % gx, L // gx, gx, gy)[1] for L in range(G) if L % 8 == xcd}
            assert len(ys) == gy // 8


@pytest.mark.parametrize("g", [(1, 4, 256), (2, 1, 1024), (4, 8, 32), (3, 5, 7), (1, 1, 16)])
def test_xcd_block_order_3d_is_a_bijection(g):
    gx, gy, gz = g
    out = {_xcd_remap3(x, y, z, gx, gy, gz) for z in range(gz) for y in range(gy) for x in range(gx)}
    assert len(out) == gx * gy * gz
    assert all(0 <= a < gx and 0 <= b < gy and 0 <= c < gz for a, b, c in out)


def test_library_trainer_and_bench_share_one_default(monkeypatch):
    """The fp32 GEMM family a user trains with is the one bench.py times:
    library default, ``dist_trainer --f32-matmul`` default and bench.py agree."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k != "GKSGD_F32_MATMUL"}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env["PYTHONPATH"] = root
    lib = subprocess.run([sys.executable, "-c", "from gaussiank_sgd_amd.ops import conv1x1; print(conv1x1.f32_matmul())"],
                         capture_output=True, text=True, env=env, timeout=300)
    assert lib.returncode == 0, lib.stderr[-1500:]
    assert lib.stdout.strip() == "bf16x6"
    monkeypatch.delenv("GKSGD_F32_MATMUL", raising=False)
    from gaussiank_sgd_amd.train.dist_trainer import build_parser
    assert build_parser().parse_args([]).f32_matmul == "bf16x6"
    helptext = " ".join(build_parser().format_help().split())
    assert "--f32-matmul" in helptext and "default: bf16x6" in helptext
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    import importlib
    import bench
    importlib.reload(bench)
    assert bench.parse().f32_matmul == build_parser().parse_args([]).f32_matmul
