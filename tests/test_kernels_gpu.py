"""Numerics of every HIP kernel against plain PyTorch fp32/fp64 references.

Run on the MI355X box: ``pytest -m gpu``.
"""
import math
import os

import pytest
import torch

from gaussiank_sgd_amd import ops
from gaussiank_sgd_amd.compression import reference
from gaussiank_sgd_amd.utils.stats import gaussian_z

pytestmark = pytest.mark.gpu


def _pair(n, seed=0, dist="normal", scale=1e-3):
    g = torch.Generator().manual_seed(seed)
    if dist == "normal":
        x = torch.randn(n, generator=g) * scale
        r = torch.randn(n, generator=g) * scale * 0.3
    else:
        # Student-t(2) from the seeded generator (t = z / sqrt(chi2_2 / 2),
        # chi2_2 = -2 log U): the data must not depend on the global RNG,
        # i.e. on which tests ran before
        z = torch.randn(n, generator=g, dtype=torch.float64)
        v = -2.0 * torch.log(torch.rand(n, generator=g, dtype=torch.float64).clamp_min(1e-300))
        x = (z / torch.sqrt(v / 2.0)).float() * scale
        r = torch.zeros(n)
    return x, r


def _run_both(x, r, mode, k, k_cap, ec=True, loops=3, z=0.0, seed=0, device=None):
    gb, rb = ops.CompressBuffers(k_cap, device), ops.CompressBuffers(k_cap, "cpu")
    xg, rg = x.clone().to(device), r.clone().to(device)
    xc, rc = x.clone(), r.clone()
    ops.compress_(xg, rg, gb, mode, ec=ec, zero_g=True, loops=loops, z=z, k=k, k_cap=k_cap, seed=seed)
    ops.compress_(xc, rc, rb, mode, ec=ec, zero_g=True, loops=loops, z=z, k=k, k_cap=k_cap, seed=seed)
    torch.cuda.synchronize()
    return (xg.cpu(), rg.cpu(), gb.record.cpu(), gb.stats.cpu()), (xc, rc, rb.record, rb.stats)


def _sel(rec, k_cap):
    sent = int(rec[0])
    idx = rec[4:4 + sent].long()
    val = rec[4 + k_cap:4 + k_cap + sent].view(torch.float32)
    return sent, int(rec[1]), idx, val


@pytest.mark.parametrize("n", [1 << 20, 1_000_003, 4096 * 7 + 5, 100])
@pytest.mark.parametrize("loops,ec", [(3, True), (5, False)])
def test_gaussian_pipeline(cuda, n, loops, ec):
    x, r = _pair(n, seed=n % 97)
    ratio = 0.001 if n > 10000 else 0.05
    k = max(int(n * ratio), 1)
    k_cap = 2 * k
    (xg, rg, recg, stg), (xc, rc, recc, stc) = _run_both(x, r, ops.MODE_GAUSSIAN, k, k_cap, ec, loops,
                                                         gaussian_z(ratio), device=cuda)
    acc = (x + r) if ec else x.clone()
    # statistics vs torch
    assert abs(float(stg[0]) - float(acc.double().mean())) < 1e-6 * max(1e-3, float(acc.abs().max()))
    assert math.isclose(float(stg[1]), float(acc.double().std()), rel_tol=1e-5)
    # gradient zeroed, selection consistent with the chosen threshold
    assert float(xg.abs().sum()) == 0.0
    sent, total, idx, val = _sel(recg, k_cap)
    thr = float(recg[3:4].view(torch.float32))
    if int(recg[2]) == ops.OVERFLOW_EXACT:
        # the reference threshold passed > k_cap: exact top-k_cap by magnitude
        assert sent == k_cap and total > k_cap
        unsent = torch.ones(n, dtype=torch.bool)
        unsent[idx] = False
        assert float(val.abs().min()) >= float(acc.abs()[unsent].max())
    else:
        mask = acc.abs() > thr
        expect = mask.nonzero().view(-1)
        assert total == int(mask.sum()) and sent == total
        assert torch.equal(idx, expect)
    assert torch.equal(val, acc[idx])
    res_expect = acc.clone()
    res_expect[idx] = 0
    assert torch.equal(rg, res_expect)
    # CPU mirror agrees on the decision (same candidate)
    assert int(recg[2]) == int(recc[2])
    assert abs(int(recg[1]) - int(recc[1])) <= max(2, total // 1000)


def test_gaussian_matches_reference_oracle(cuda):
    n = 1 << 18
    x, r = _pair(n, seed=3)
    ratio = 0.001
    k = int(n * ratio)
    bufs = ops.CompressBuffers(4 * k, cuda)
    xg, rg = x.clone().to(cuda), r.clone().to(cuda)
    ops.compress_(xg, rg, bufs, ops.MODE_GAUSSIAN, ec=True, zero_g=True, loops=3, z=gaussian_z(ratio), k=k,
                  k_cap=4 * k)
    torch.cuda.synchronize()
    st = bufs.stats.cpu()
    acc, idx, vals, res = reference.gaussian(x, r, ratio, loops=3, ec=True,
                                             stats=(float(st[0]), float(st[1])))
    sent, total, gidx, gval = _sel(bufs.record.cpu(), 4 * k)
    assert total == idx.numel()
    assert torch.equal(gidx, idx[:sent])
    assert torch.equal(rg.cpu(), res) if sent == total else True


@pytest.mark.parametrize("n", [1 << 20, 333_333])
def test_topk_exact(cuda, n):
    x, r = _pair(n, seed=5, dist="t")
    k = max(int(n * 0.001), 1)
    (xg, rg, recg, _), (xc, rc, recc, _) = _run_both(x, r, ops.MODE_TOPK, k, k, device=cuda)
    acc = x + r
    _, idx, vals, res = reference.topk_exact(x, r, 0.001)
    sent, total, gidx, gval = _sel(recg, k)
    assert sent == total == k
    assert torch.equal(gidx, idx)
    assert torch.equal(gval, acc[idx])
    assert torch.equal(rg, res)
    assert torch.equal(recg, recc)


def test_topk_ties_lowest_index(cuda):
    n = 50_000
    x = torch.zeros(n)
    x[::7] = 1.0  # many exact ties
    r = torch.zeros(n)
    k = 100
    (xg, rg, recg, _), (xc, rc, recc, _) = _run_both(x, r, ops.MODE_TOPK, k, k, device=cuda)
    sent, total, gidx, _ = _sel(recg, k)
    assert sent == k
    assert torch.equal(gidx, torch.arange(0, 7 * k, 7))
    assert torch.equal(recg, recc)


def test_randomk_hash_parity(cuda):
    n = 500_000
    x, r = _pair(n, seed=9)
    k = 500
    (xg, rg, recg, _), (xc, rc, recc, _) = _run_both(x, r, ops.MODE_RANDOMK, k, k, ec=False, seed=12345,
                                                     device=cuda)
    assert torch.equal(recg, recc)
    sent, total, idx, _ = _sel(recg, k)
    assert sent == k and idx.unique().numel() == k


@pytest.mark.parametrize("mode", [ops.MODE_REDSYNC, ops.MODE_REDSYNCTRIM, ops.MODE_DGC])
def test_threshold_modes_vs_mirror(cuda, mode):
    n = 400_000
    x, r = _pair(n, seed=11, dist="t")
    k = 400
    k_cap = 4 * k if mode != ops.MODE_REDSYNCTRIM else n
    (xg, rg, recg, _), (xc, rc, recc, _) = _run_both(x, r, mode, k, k_cap, seed=77, device=cuda)
    assert int(recg[2]) == int(recc[2])
    assert abs(int(recg[1]) - int(recc[1])) <= 2
    sent, total, idx, val = _sel(recg, k_cap)
    acc = x + r
    assert torch.equal(val, acc[idx])
    assert bool((idx[1:] > idx[:-1]).all())


def test_kcap_overflow_stays_in_residual(cuda):
    """Overflow past k_cap: the record holds the k_cap LARGEST entries (exact
    radix key at k_cap), the header the reference count, the rest stays in
    the residual (conservation)."""
    n = 1 << 16
    x, r = _pair(n, seed=13)
    k_cap = 10
    bufs = ops.CompressBuffers(k_cap, cuda)
    xg, rg = x.clone().to(cuda), r.clone().to(cuda)
    ops.compress_(xg, rg, bufs, ops.MODE_THRESHOLD, ec=True, zero_g=True, k=5, k_cap=k_cap, fixed_thr=0.0)
    torch.cuda.synchronize()
    rec = bufs.record.cpu()
    sent, total, idx, val = _sel(rec, k_cap)
    acc = x + r
    nz = (acc.abs() > 0).nonzero().view(-1)
    assert sent == k_cap and total == nz.numel()
    assert int(rec[2]) == ops.OVERFLOW_EXACT
    assert set(idx.tolist()) == set(torch.topk(acc.abs(), k_cap).indices.tolist())
    assert bool((idx[1:] > idx[:-1]).all())
    # conservation: acc == scatter(sent) + residual
    rebuilt = rg.cpu().clone()
    rebuilt[idx] += val
    assert torch.equal(rebuilt, acc)


@pytest.mark.parametrize("k_cap_mult", [4.0 / 3.0, 1.0, 3.0])
def test_gaussian_overflow_gpu_matches_mirror(cuda, k_cap_mult):
    """Heavy-tailed bucket whose reference threshold passes >> k_cap: the GPU
    record equals the CPU mirror's (exact top-k_cap) and holds the largest
    |x| -- every sent magnitude >= every unsent one."""
    n = 200_000
    g = torch.Generator().manual_seed(11)
    x = torch.randn(n, generator=g) * 1e-4
    hot = torch.randperm(n, generator=g)[: n // 50]
    x[hot] = (1.0 + torch.rand(hot.numel(), generator=g)) * torch.sign(torch.randn(hot.numel(), generator=g))
    r = torch.zeros(n)
    k = 200
    k_cap = max(1, math.ceil(k * k_cap_mult))
    (xg, rg, recg, _), (xc, rc, recc, _) = _run_both(x, r, ops.MODE_GAUSSIAN, k, k_cap, True, 3,
                                                     gaussian_z(0.001), device=cuda)
    assert int(recg[1]) > k_cap and int(recg[2]) == ops.OVERFLOW_EXACT
    assert torch.equal(recg, recc)
    assert torch.equal(rg, rc)
    sent, total, idx, val = _sel(recg, k_cap)
    unsent = torch.ones(n, dtype=torch.bool)
    unsent[idx] = False
    assert sent == k_cap and float(val.abs().min()) >= float((x + r).abs()[unsent].max())


@pytest.mark.parametrize("deterministic", [False, True])
def test_scatter_add_unequal_counts_and_duplicates(cuda, deterministic):
    n, P, k_cap = 100_000, 4, 3000
    g = torch.Generator().manual_seed(1)
    recs = torch.zeros(P, 4 + 2 * k_cap, dtype=torch.int32)
    per_rank = []
    for p in range(P):
        cnt = 1000 + 500 * p
        idx = torch.randperm(20_000, generator=g)[:cnt].sort().values  # overlapping index ranges
        val = torch.randn(cnt, generator=g)
        recs[p, 0] = cnt
        recs[p, 4:4 + cnt] = idx.int()
        recs[p, 4 + k_cap:4 + k_cap + cnt] = val.view(torch.int32)
        per_rank.append((idx, val))
    expect = reference.sparse_aggregate(n, per_rank, P)
    dst = torch.zeros(n, device=cuda)
    ops.scatter_add_records_(dst, recs.to(cuda), P, k_cap, 1.0 / P, deterministic)
    torch.cuda.synchronize()
    assert torch.allclose(dst.cpu(), expect, atol=1e-6, rtol=1e-5)
    if deterministic:
        dst2 = torch.zeros(n, device=cuda)
        ops.scatter_add_records_(dst2, recs.to(cuda), P, k_cap, 1.0 / P, True)
        assert torch.equal(dst, dst2)


def test_fused_sgd_vs_torch(cuda):
    torch.manual_seed(0)
    shapes = [(64, 3, 3, 3), (64,), (1000, 64), (1000,), (7,)]
    groups_cfg = [dict(lr=0.1, momentum=0.9, dampening=0.0, weight_decay=1e-4, nesterov=False),
                  dict(lr=0.05, momentum=0.875, dampening=0.1, weight_decay=0.0, nesterov=False),
                  dict(lr=0.02, momentum=0.9, dampening=0.0, weight_decay=5e-4, nesterov=True)]
    assign = [0, 1, 0, 1, 2]
    params = [torch.randn(s) for s in shapes]
    ref_params = [p.clone().requires_grad_(True) for p in params]
    opt = torch.optim.SGD([{"params": [ref_params[i] for i in range(5) if assign[i] == gi], **cfg}
                           for gi, cfg in enumerate(groups_cfg)], lr=0.1)
    pad = lambda n: (n + 63) // 64 * 64
    offs, o = [], 0
    for s in shapes:
        offs.append(o)
        o += pad(math.prod(s))
    w = torch.zeros(o, device=cuda)
    m = torch.zeros(o, device=cuda)
    gr = torch.zeros(o, device=cuda)
    for i, p in enumerate(params):
        w[offs[i]:offs[i] + p.numel()] = p.view(-1).to(cuda)
    chunks = ops.make_chunk_table([(offs[i], pad(params[i].numel()), assign[i], i) for i in range(5)], cuda)
    for step in range(3):
        grads = [torch.randn(s) for s in shapes]
        for i, gg in enumerate(grads):
            ref_params[i].grad = gg.clone()
            gr[offs[i]:offs[i] + gg.numel()] = gg.view(-1).to(cuda)
        opt.step()
        hp = [dict(cfg, first_step=(step == 0)) for cfg in groups_cfg]
        shadow = torch.zeros(o, dtype=torch.bfloat16, device=cuda)
        ops.fused_sgd_(w, m, gr, chunks, hp, zero_grad=True, w_bf16=shadow)
        torch.cuda.synchronize()
        assert float(gr.abs().sum()) == 0.0
        assert torch.equal(shadow, w.to(torch.bfloat16))  # RNE cast written in the same pass
        for i, p in enumerate(ref_params):
            got = w[offs[i]:offs[i] + p.numel()].cpu().view(p.shape)
            assert torch.allclose(got, p.detach(), atol=1e-6, rtol=1e-5), (step, i)


@pytest.mark.parametrize("n,off", [(1 << 20, 0), (12345, 0), (4097, 3), (7, 1)])
def test_accum_grad_and_cast_bf16(cuda, n, off):
    torch.manual_seed(0)
    base = torch.randn(n + off, device=cuda)
    dst = base[off:]                     # possibly unaligned fp32 view
    src = torch.randn(n + off, device=cuda).to(torch.bfloat16)[off:]
    want = dst.clone() + src.float()
    ops.accum_grad_(dst, src)
    assert torch.equal(dst, want)
    src32 = torch.randn(n, device=cuda)
    want = dst.clone() + src32
    ops.accum_grad_(dst, src32)
    assert torch.equal(dst, want)
    sh = torch.empty(n, dtype=torch.bfloat16, device=cuda)
    ops.cast_bf16_(sh, dst)
    assert torch.equal(sh, dst.to(torch.bfloat16))


def test_accum_grad_channels_last(cuda):
    w = torch.zeros(64, 32, 3, 3, device=cuda).to(memory_format=torch.channels_last)
    g = torch.randn(64, 32, 3, 3, device=cuda).to(torch.bfloat16).to(memory_format=torch.channels_last)
    ops.accum_grad_(w, g)
    assert torch.equal(w, g.float())
    g2 = torch.randn(64, 32, 3, 3, device=cuda).to(torch.bfloat16)  # contiguous: different strides
    ops.accum_grad_(w, g2)
    assert torch.allclose(w, g.float() + g2.float())


def test_fused_lars_vs_reference(cuda):
    from gaussiank_sgd_amd.optim.lars import LARS
    torch.manual_seed(1)
    shapes = [(128, 64), (64,), (10, 128)]
    params = [torch.randn(s).requires_grad_(True) for s in shapes]
    opt = LARS(params, lr=0.1, momentum=0.9, weight_decay=5e-4, eeta=1e-3, epsilon=1e-5)
    pad = lambda n: (n + 63) // 64 * 64
    offs, o = [], 0
    for s in shapes:
        offs.append(o)
        o += pad(math.prod(s))
    w = torch.zeros(o, device=cuda)
    m = torch.ones(o, device=cuda)
    gr = torch.zeros(o, device=cuda)
    for i, p in enumerate(params):
        w[offs[i]:offs[i] + p.numel()] = p.detach().view(-1).to(cuda)
    chunks = ops.make_chunk_table([(offs[i], pad(params[i].numel()), 0, i) for i in range(3)], cuda)
    ss = torch.zeros(6, dtype=torch.float64, device=cuda)
    hp = [dict(lr=0.1, momentum=0.9, weight_decay=5e-4, eeta=1e-3, epsilon=1e-5)]
    for step in range(3):
        for i, p in enumerate(params):
            gg = torch.randn(p.shape)
            p.grad = gg.clone()
            gr[offs[i]:offs[i] + gg.numel()] = gg.view(-1).to(cuda)
        opt.step()
        ss.zero_()
        ops.segmented_sumsq_(w, gr, chunks, ss)
        ops.fused_lars_(w, m, gr, chunks, ss, hp)
        torch.cuda.synchronize()
        for i, p in enumerate(params):
            got = w[offs[i]:offs[i] + p.numel()].cpu().view(p.shape)
            assert torch.allclose(got, p.detach(), atol=1e-5, rtol=1e-5), (step, i)


def test_clip_grad_norm(cuda):
    x = torch.randn(300_001) * 3
    g = x.clone().to(cuda)
    norm = ops.clip_grad_norm_(g, 5.0)
    torch.cuda.synchronize()
    ref = x.clone()
    rn = torch.nn.utils.clip_grad_norm_([torch.nn.Parameter(torch.zeros(1))], 1.0)  # API smoke
    n = float(x.double().norm())
    assert math.isclose(float(norm), n, rel_tol=1e-5)
    assert torch.allclose(g.cpu(), ref * (5.0 / (n + 1e-6)), rtol=1e-5, atol=1e-7)


def test_sign_bucket(cuda):
    x = torch.randn(123_457)
    res, means, pos = reference.sign_bucket_mean(x)
    g = x.clone().to(cuda)
    mask = torch.zeros(x.numel(), dtype=torch.uint8, device=cuda)
    mm = torch.zeros(2, device=cuda)
    ops.sign_bucket_compress_(g, mask, mm, ops.sign_bucket_ws(cuda))
    torch.cuda.synchronize()
    assert torch.allclose(mm.cpu(), means, rtol=1e-5, atol=1e-7)
    assert torch.equal(mask.cpu().bool(), pos)
    assert torch.allclose(g.cpu(), res, atol=1e-6)
    ops.sign_bucket_decompress_(g, mask, mm)
    torch.cuda.synchronize()
    assert torch.allclose(g.cpu(), x, atol=1e-6)


def test_rccl_engine_world1(cuda):
    cls = ops.rccl_engine_class()
    e = cls()
    e.init(cls.unique_id(), 0, 1, 0)
    t = torch.arange(10, dtype=torch.float32, device=cuda)
    out = torch.zeros(10, device=cuda)
    e.allgather(t, out)
    e.allreduce(t, 1)
    torch.cuda.synchronize()
    assert torch.equal(out, t)
    e.destroy()


def test_momentum_correct_and_mask(cuda):
    """DGC momentum correction over a chunk range + momentum factor masking."""
    torch.manual_seed(0)
    pad = lambda n: (n + 63) // 64 * 64
    sizes = [40000, 100, 7]
    offs, o = [], 0
    for n in sizes:
        offs.append(o)
        o += pad(n)
    chunks = ops.make_chunk_table([(offs[i], pad(sizes[i]), i % 2, i) for i in range(3)], cuda)
    nchunks = chunks.numel() // 2
    groups = [dict(momentum=0.9, weight_decay=1e-4), dict(momentum=0.5, weight_decay=0.0)]
    u = torch.randn(o, device=cuda)
    g = torch.randn(o, device=cuda)
    w = torch.randn(o, device=cuda)
    uc, gc, wc = u.cpu(), g.cpu(), w.cpu()
    cl = ops._decode_chunks(chunks)
    begin, count = 1, nchunks - 1          # skip the first chunk: it must stay untouched
    ops.momentum_correct_(u, g, w, chunks, begin, count, groups)
    ops.momentum_correct_(uc, gc, wc, chunks, begin, count, groups, cl)
    torch.cuda.synchronize()
    assert torch.allclose(u.cpu(), uc, atol=1e-6, rtol=1e-6)
    assert torch.allclose(g.cpu(), gc, atol=1e-6, rtol=1e-6)
    uc = u.cpu()          # masking is checked bit-exactly against the GPU state
    k_cap = 64
    rec = torch.zeros(ops.REC_HDR + 2 * k_cap, dtype=torch.int32)
    idx = torch.randperm(o)[:50].sort().values.int()
    rec[0] = 50
    rec[ops.REC_HDR:ops.REC_HDR + 50] = idx
    ops.mask_records_(u, rec.to(cuda), k_cap)
    uc[idx.long()] = 0
    assert torch.equal(u.cpu(), uc)


def test_rccl_communicator_self_test_world1(cuda):
    """The non-blocking bootstrap (init_async / init_poll with a deadline) +
    its start-up all-gather self-test, through the process-wide cache."""
    from gaussiank_sgd_amd.parallel import comm
    comm.init()
    c = comm.native_communicator(cuda)
    assert c is not None
    c.self_test(30.0)
    assert comm.native_communicator(cuda) is c
    torch.cuda.synchronize()
    comm.release_native()


def test_two_optimizers_share_one_communicator(cuda):
    """Every DistributedOptimizer of the process reuses ONE native
    communicator (bench.py's phases, a re-created trainer): one init per
    process, like hvd.init() (reference dist_trainer.py:125-126)."""
    from gaussiank_sgd_amd.compression import compressors
    from gaussiank_sgd_amd.parallel import comm
    from gaussiank_sgd_amd.parallel.distributed_optimizer import DistributedOptimizer
    comm.init()
    opts = []
    for _ in range(2):
        net = torch.nn.Sequential(torch.nn.Linear(64, 32), torch.nn.ReLU(), torch.nn.Linear(32, 8)).to(cuda)
        opts.append(DistributedOptimizer(torch.optim.SGD(net.parameters(), lr=0.1, momentum=0.9),
                                         named_parameters=net.named_parameters(),
                                         compression=compressors["gaussian"], is_sparse=True, density=0.05,
                                         compress_single_rank=True, density_warmup=False, native_rccl="force"))
        x = torch.randn(16, 64, device=cuda)
        opts[-1].zero_grad()
        net(x).square().mean().backward()
        opts[-1].step()
    torch.cuda.synchronize()
    e0, e1 = opts[0]._exchanger, opts[1]._exchanger
    assert e0.kind == e1.kind == "rccl-native"
    assert e0.native is e1.native and e0.native.users == 2
    inp = torch.arange(8, dtype=torch.int32, device=cuda)
    out = torch.zeros_like(inp)
    e0.reset_stats()
    e0.allgather_(out, inp)
    e1.allgather_(out, inp)
    torch.cuda.synchronize()
    assert torch.equal(out, inp)
    assert e1.stats()["allgather"]["calls"] == 2      # one communicator counts both Exchangers' calls
    e0.close()
    assert e1.native is not None and e1.native.users == 1
    comm.release_native()


_INIT_TIMEOUT_PROBE = """
import sys, time, torch
from gaussiank_sgd_amd import ops
torch.cuda.set_device(0)
cls = ops.rccl_engine_class()
e = cls()
t0 = time.time()
e.init_async(cls.unique_id(), 0, 2, 0)      # world 2, the peer never arrives
try:
    e.init_wait(3.0)
except RuntimeError as err:
    print("raised after %.1f s: %s" % (time.time() - t0, err), flush=True)
    sys.exit(0)
print("init completed without a peer", flush=True)
sys.exit(1)
"""


def test_rccl_init_deadline_aborts_without_peer(cuda):
    """The hang the bootstrap guards against, on the real engine: rank 0 of a
    world of 2 whose peer never joins.  The non-blocking init must end in
    ncclCommAbort + an exception at the deadline (run in a child process with
    its own time limit so a regression cannot hang the test session)."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, "-c", _INIT_TIMEOUT_PROBE], capture_output=True, text=True, timeout=90,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, (r.stdout, r.stderr[-2000:])
    assert "raised after" in r.stdout and "not complete" in r.stdout, r.stdout


def test_rccl_engine_failure_races_enqueue(cuda):
    """The watchdog's failure path (inject_failure = fail + abort, what the
    timeout / async-error poll runs) fired from another thread while the
    owning thread keeps enqueuing collectives: every enqueue either completes
    or raises the failure -- none touches the aborted communicator -- and the
    engine tears down cleanly afterwards (rccl_engine.cpp failure protocol)."""
    import threading
    import time
    cls = ops.rccl_engine_class()
    e = cls()
    e.init(cls.unique_id(), 0, 1, 0)
    e.start_watchdog(600.0, 1.0)
    t = torch.arange(1 << 16, dtype=torch.float32, device=cuda)
    out = torch.zeros_like(t)
    fire = threading.Event()

    def killer():
        fire.wait()
        time.sleep(0.002)
        e.inject_failure("test: injected failure")

    th = threading.Thread(target=killer)
    th.start()
    raised = None
    ok = 0
    for i in range(20000):
        if i == 50:
            fire.set()
        try:
            e.allgather(t, out)
            e.allreduce(t, 1)
            ok += 1
        except RuntimeError as err:
            raised = str(err)
            break
    th.join()
    torch.cuda.synchronize()
    assert ok >= 50
    assert raised is not None and "injected failure" in raised, raised
    assert e.failed() and "injected failure" in e.error()
    with pytest.raises(RuntimeError):
        e.allgather(t, out)
    e.stop_watchdog()
    e.destroy()


@pytest.mark.parametrize("mode", [ops.MODE_GAUSSIAN, ops.MODE_GAUSSIAN_CAL, ops.MODE_TOPK])
def test_compress_reused_buffers_varying_sizes(cuda, mode):
    """One CompressBuffers pair reused across buckets of different sizes (grid
    sizes): the last-block hand-off counters (stats -> finalize, count ->
    decide, radix -> fallback key) must be back at zero after every call, so
    each record equals the CPU mirror's."""
    k_cap = 3000
    gb, rb = ops.CompressBuffers(k_cap, cuda), ops.CompressBuffers(k_cap, "cpu")
    for i, n in enumerate([1_200_000, 5_000, 300_007 * 4, 64, 1_200_000]):
        x, r = _pair(n, seed=31 + i)
        k = max(int(n * 0.001), 1)
        xg, rg = x.clone().to(cuda), r.clone().to(cuda)
        xc, rc = x.clone(), r.clone()
        for g_, r_, b_ in ((xg, rg, gb), (xc, rc, rb)):
            ops.compress_(g_, r_, b_, mode, ec=True, zero_g=True, loops=3, z=gaussian_z(0.001), k=k, k_cap=k_cap,
                          seed=5)
        torch.cuda.synchronize()
        recg = gb.record.cpu()
        sg, tg, ig, vg = _sel(recg, k_cap)
        sc, tc, ic, vc = _sel(rb.record, k_cap)
        assert (sg, tg) == (sc, tc), (n, mode, sg, tg, sc, tc)
        assert torch.equal(ig, ic) and torch.equal(vg, vc)
        assert torch.equal(rg.cpu(), rc)


def _set_handoff(monkeypatch, handoff):
    """launch: launch hand-offs (finalize / decide as their own launches, the
    default); launch_ingrid: the same with the finalize / decide in the stats /
    count passes' last blocks (GKSGD_STEP_INGRID=1); lastblock: the in-grid
    hand-off of the buckets compressed during the backward."""
    monkeypatch.setenv("GKSGD_HANDOFF", "lastblock" if handoff == "lastblock" else "launch")
    monkeypatch.setenv("GKSGD_STEP_INGRID", "1" if handoff == "launch_ingrid" else "0")


@pytest.mark.parametrize("handoff", ["launch", "launch_ingrid", "lastblock"])
@pytest.mark.parametrize("mode", [ops.MODE_GAUSSIAN, ops.MODE_GAUSSIAN_CAL, ops.MODE_TOPK, ops.MODE_DGC])
def test_last_block_handoff_stress(cuda, mode, handoff, monkeypatch):
    """The last-block hand-offs (stats -> finalize, count -> decide, radix ->
    fallback key; compress.hip last_block) at the LARGEST grids
    (kMaxStatsBlocks / kMaxCountBlocks), back to back on one set of buffers,
    with an unrelated GEMM loading the chip from a second stream (uneven
    load, L1/L2 warm).  Every call is checked word by word: the statistics
    against fp64 torch (stale partials would move them), the header's total
    against the count above its own threshold (count -> decide), the record's
    indices / values / residual against that selection (decide's offsets),
    and for exact top-k the whole record against the CPU mirror."""
    _set_handoff(monkeypatch, handoff)   # compress.hip handoff_by_launch() / step_ingrid_env()
    n = 2048 * 4096 * 2 + 4093          # > kMaxStatsBlocks full tiles: every grid at its cap
    k = n // 1000
    k_cap = (4 * k + 2) // 3 if mode != ops.MODE_TOPK else k
    gb = ops.CompressBuffers(k_cap, cuda)
    cb = ops.CompressBuffers(k_cap, "cpu")
    side = torch.cuda.Stream()
    a = torch.randn(4096, 4096, device=cuda)
    z = gaussian_z(0.001)
    for it in range(5):
        x, r = _pair(n, seed=100 + it, dist="t" if it % 2 else "normal")
        xg, rg = x.to(cuda), r.to(cuda)
        with torch.cuda.stream(side):
            for _ in range(4):
                a = torch.tanh(a @ a * 1e-3)
        ops.compress_(xg, rg, gb, mode, ec=True, zero_g=True, loops=3, z=z, k=k, k_cap=k_cap, seed=it)
        torch.cuda.synchronize()
        acc = x + r
        recg = gb.record.cpu()
        st = gb.stats.cpu()
        assert abs(float(st[0]) - float(acc.double().mean())) < 1e-5 * float(acc.abs().max()), it
        assert math.isclose(float(st[1]), float(acc.double().std()), rel_tol=1e-5), it
        sent, total, idx, val = _sel(recg, k_cap)
        # total = the reference rule's count; past k_cap the selection is the
        # tighter candidate with the largest count in [2k/3, k_cap] (sent <
        # k_cap) or the exact top-k_cap key (sent == k_cap)
        overflow_alt = total > k_cap and sent < k_cap
        assert 0 < sent <= k_cap, it
        assert sent == min(total, k_cap) or (overflow_alt and 3 * sent >= 2 * k), (it, sent, total)
        assert bool((idx[1:] > idx[:-1]).all()), it
        assert torch.equal(val, acc[idx]), it
        res = acc.clone()
        res[idx] = 0
        assert torch.equal(rg.cpu(), res), it
        chosen = int(recg[2])
        if mode == ops.MODE_TOPK:
            ops.compress_(x.clone(), r.clone(), cb, mode, ec=True, zero_g=True, loops=3, z=z, k=k, k_cap=k_cap,
                          seed=it)
            assert torch.equal(recg, cb.record), it
        elif chosen not in (ops.OVERFLOW_EXACT, ops.CAL_FALLBACK) and mode != ops.MODE_DGC:
            thr = float(recg[3:4].view(torch.float32))
            expect = (acc.abs() > thr).nonzero().view(-1)
            assert (sent if overflow_alt else total) == expect.numel() and torch.equal(idx, expect[:sent]), it
        else:
            # exact-key selections: every sent magnitude >= every unsent one
            unsent = torch.ones(n, dtype=torch.bool)
            unsent[idx] = False
            assert float(val.abs().min()) >= float(acc.abs()[unsent].max()), it


def test_gaussian_overflow_extension_gpu_matches_mirror(cuda):
    """Power-law tail: an overflow-extension threshold (ladder slots 6..15,
    counted for the rare elements above the lowest of them) resolves the k_cap
    overflow; GPU record and residual equal the CPU mirror's."""
    n = 400_000 + 37
    g = torch.Generator().manual_seed(21)
    u = torch.rand(n, generator=g).clamp_min(1e-12)
    x = (u ** (-1.0 / 2.5) - 1.0) * 1e-3 * torch.sign(torch.randn(n, generator=g))
    r = torch.zeros(n)
    k = n // 1000
    k_cap = math.ceil(4 * k / 3)
    (xg, rg, recg, _), (xc, rc, recc, _) = _run_both(x, r, ops.MODE_GAUSSIAN, k, k_cap, True, 3,
                                                     gaussian_z(0.001), device=cuda)
    assert 6 <= int(recg[2]) < ops.MAX_CAND and int(recg[1]) > k_cap
    assert torch.equal(recg, recc)
    assert torch.equal(rg, rc)


@pytest.mark.parametrize("fused", ["1", "0"])
@pytest.mark.parametrize("handoff", ["launch", "launch_ingrid", "lastblock"])
def test_fused_fallback_fires_under_load(cuda, fused, handoff, monkeypatch):
    """The conditional exact fallback FIRING in decide_fb_kernel (one launch:
    decide, three radix passes, key resolve, conditional count, second decide,
    separated by grid barriers) on a bucket large enough for every grid at its
    cap, with GEMMs loading the chip from a second stream: the record, header
    and residual equal the CPU mirror's word for word, call after call on one
    set of buffers (the flag / barrier words are reused).  fused=0, or the
    in-grid hand-off (handoff=lastblock: the buckets compressed while the
    backward runs), take the chain of separate launches instead."""
    monkeypatch.setenv("GKSGD_FB_FUSED", fused)
    _set_handoff(monkeypatch, handoff)
    n = 6_000_000
    k = 300
    k_cap = 400
    gb = ops.CompressBuffers(k_cap, cuda)
    cb = ops.CompressBuffers(k_cap, "cpu")
    side = torch.cuda.Stream()
    a = torch.randn(4096, 4096, device=cuda)
    for it in range(3):
        g = torch.Generator().manual_seed(50 + it)
        x = torch.randn(n, generator=g) * 1e-4
        hot = torch.randperm(n, generator=g)[: n // 100]
        x[hot] = (1.0 + torch.rand(hot.numel(), generator=g)) * torch.sign(torch.randn(hot.numel(), generator=g))
        r = torch.zeros(n)
        xg, rg = x.to(cuda), r.to(cuda)
        with torch.cuda.stream(side):
            for _ in range(4):
                a = torch.tanh(a @ a * 1e-3)
        ops.compress_(xg, rg, gb, ops.MODE_GAUSSIAN, ec=True, zero_g=True, loops=3, z=gaussian_z(0.001), k=k,
                      k_cap=k_cap, seed=it)
        xc, rc = x.clone(), r.clone()
        ops.compress_(xc, rc, cb, ops.MODE_GAUSSIAN, ec=True, zero_g=True, loops=3, z=gaussian_z(0.001), k=k,
                      k_cap=k_cap, seed=it)
        torch.cuda.synchronize()
        recg = gb.record.cpu()
        assert int(recg[2]) == ops.OVERFLOW_EXACT, (it, recg[:4].tolist())
        assert torch.equal(recg, cb.record), it
        assert torch.equal(rg.cpu(), rc), it
        assert ops.sync_timeouts(gb) == 0, it   # every grid barrier / flag poll completed
