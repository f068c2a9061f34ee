"""bench.py's fail-soft phase runner and defaults, on CPU (no GPU needed)."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("gk_bench", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_optional_phase_records_error(bench, monkeypatch):
    out = {}

    def boom(holder):
        raise ValueError("bad shape\nsecond line")
    assert bench.optional_phase("dense", out, 1, boom) is True     # ranks can still agree: go on
    assert out["dense_error"] == "ValueError: bad shape"


def test_optional_phase_injection_and_success(bench, monkeypatch):
    out = {}
    ran = []
    monkeypatch.setenv("GKSGD_BENCH_FAIL_PHASE", "bf16")
    assert bench.optional_phase("bf16", out, 1, lambda h: ran.append(1)) is True
    assert "injected failure" in out["bf16_error"] and not ran
    assert bench.optional_phase("ref_bs32", out, 1, lambda h: ran.append(1)) is True
    assert ran == [1] and "ref_bs32_error" not in out


def test_reference_batches_and_bert_buckets(bench):
    # the reference's per-worker batches (/root/reference/exp_configs/*.conf:2)
    assert bench.REF_BATCH["resnet50"] == 32 and bench.REF_BATCH["vgg16"] == 128 and bench.REF_BATCH["lstm"] == 20
    # BERT: bucketed compression (~25 MB fp32 buckets) by default
    assert bench.DEFAULT_THRESHOLD["bert"] * 4 == pytest.approx(26e6, rel=0.1)


def test_bert_default_threshold_gives_buckets(bench):
    """The BERT default threshold splits the 110 M gradients into >= 4 buckets
    (reference grouping rule: reverse registration order until >= threshold)."""
    import torch
    from gaussiank_sgd_amd.models.bert import bert_base
    from gaussiank_sgd_amd.parallel.buckets import group_with_threshold
    with torch.device("meta"):
        net = bert_base()
    names = [n for n, p in net.named_parameters()]
    sizes = {n: p.numel() for n, p in net.named_parameters()}
    groups = group_with_threshold(names, sizes, bench.DEFAULT_THRESHOLD["bert"])
    assert len(groups) >= 4


def _asym_worker(rank, port, outdir):
    """Rank 1 fails the phase (GKSGD_BENCH_FAIL_PHASE_RANK) while rank 0 waits
    in the phase's own point-to-point exchange for it: the agreement
    collective cannot pair up, so only the phase deadline ends the run."""
    import time
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK=str(rank), GKSGD_BENCH_FAIL_PHASE="dense", GKSGD_BENCH_FAIL_PHASE_RANK="1",
                      GKSGD_BENCH_PHASE_TIMEOUT_S="3")
    spec = importlib.util.spec_from_file_location("gk_bench", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    from gaussiank_sgd_amd.parallel import comm
    comm.init(device="cpu")
    bench._EMIT["json_out"] = os.path.join(outdir, "line.json")
    out = {"metric": "m", "value": 1.0}

    def phase(holder):
        t = torch.zeros(1)
        torch.distributed.recv(t, src=1)     # rank 1 never sends: it failed before
    t0 = time.time()
    bench.optional_phase("dense", out, 2, phase)
    # not reached when the deadline fired (os._exit); reached only if the ranks agreed
    with open(os.path.join(outdir, "returned%d" % rank), "w") as f:
        f.write("%.1f" % (time.time() - t0))


def test_asymmetric_phase_failure_keeps_the_headline_line():
    import json
    import socket
    import tempfile
    import time
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    with tempfile.TemporaryDirectory() as d:
        t0 = time.time()
        mp.spawn(_asym_worker, args=(port, d), nprocs=2, join=True)
        assert time.time() - t0 < 60
        line = json.loads(open(os.path.join(d, "line.json")).read())
        assert line["value"] == 1.0 and "timeout" in line["dense_error"], line
        assert not os.path.exists(os.path.join(d, "returned0"))


def test_per_rank_injection(bench, monkeypatch):
    monkeypatch.setenv("GKSGD_BENCH_FAIL_PHASE", "bf16")
    monkeypatch.setenv("GKSGD_BENCH_FAIL_PHASE_RANK", "1")
    assert not bench._injected("bf16")          # this process is rank 0
    monkeypatch.setenv("GKSGD_BENCH_FAIL_PHASE_RANK", "0")
    assert bench._injected("bf16") and not bench._injected("dense")
