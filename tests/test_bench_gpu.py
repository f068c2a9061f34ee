"""bench.py's own multi-rank path, rehearsed on ONE GPU.

The driver's scaling run launches ``bench.py --gpus N`` under
torch.distributed.run with one rank per GPU over RCCL.  RCCL refuses two ranks
on one device, so here two ranks share cuda:0 over gloo
(``GKSGD_DIST_BACKEND=gloo``, ``--no-native-rccl``) and everything else is the
real thing: the self-launch of torch.distributed.run as a child, comm.init,
the coalesced parameter broadcast, barriers, the MAX-over-ranks elapsed time,
the packed all-gather + rank-ordered decompress, the selected-count
collection, the replica digest and Exchanger.close().
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench(*extra, gpus=2, timeout=480, probe=False, env_extra=None, native=False):
    env = dict(os.environ, GKSGD_DIST_BACKEND="gloo", MASTER_PORT=str(_free_port()), HSA_ENABLE_IPC_MODE_LEGACY="0",
               GKSGD_BENCH_PROBE="1" if probe else "0")
    env.update(env_extra or {})
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus)] + \
        ([] if native else ["--no-native-rccl"]) + list(extra)
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, "bench.py failed (%d):\n%s\n%s" % (p.returncode, p.stdout[-3000:], p.stderr[-3000:])
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-3000:]     # rank 0 prints exactly one JSON line
    return json.loads(lines[0])


def test_bench_resnet50_two_ranks_one_gpu(cuda):
    out = _bench("--steps", "3", "--warmup", "2", "--batch-size", "16", "--ref-batch", "8", "--ref-steps", "2")
    assert out["n_gpus"] == 2 and out["world"] == 2
    assert out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 32
    assert out["exchange"] == "torch"
    assert out["replicas_consistent"] is True
    assert out["value"] > 0 and out["ms_per_step"] > 0
    # headline precision is the reference's fp32; the bf16 phase is a second timed loop
    assert out["dtype"] == "fp32"
    assert out["bf16_value"] > 0 and out["bf16_ms_per_step"] > 0
    # sent <= k_cap per bucket; the header's total keeps the reference rule's count
    assert 0 < out["selected_over_k"] <= 1.0 + 1e-3
    assert out["candidates_per_step"] >= out["selected_per_step"]
    # wire ratio: dense fp32 bytes / fixed record bytes, Gaussian-k k_cap = k:
    # the reference's 500x at d = 0.001 (fp32 values + int32 indices)
    assert 490 <= out["effective_compression_ratio"] <= 501
    assert out["config"]["k_cap_factor"] == 1.0
    assert out["exposed_comm_ms"] is not None and out["exposed_comm_ms"] >= 0
    # dense comparator: bucketed (25 MB), backward-overlapped all-reduce after the sparse loop
    assert out["dense_ms_per_step"] > 0 and out["dense_buckets"] > 1
    assert out["speedup_vs_dense"] == pytest.approx(out["dense_ms_per_step"] / out["ms_per_step"], rel=1e-2)
    # reference-batch phases (the reference's per-worker batch; here shrunk to 8)
    assert out["ref_bs8_value"] > 0 and out["ref_bs8_dense_value"] > 0
    assert out["ref_bs8_speedup_vs_dense"] == pytest.approx(
        out["ref_bs8_dense_ms_per_step"] / out["ref_bs8_ms_per_step"], rel=1e-2)
    # per-phase exchanger kind (gloo: torch.distributed) and no recorded failure
    ph = out["phases"]
    assert set(ph) >= {"headline", "dense", "ref_bs8", "ref_bs8_dense", "bf16"}
    assert all(p["exchange"] == "torch" for p in ph.values())
    assert ph["ref_bs8"]["per_gpu_batch"] == 8 and ph["dense"]["buckets"] > 1
    assert not [k for k in out if k.endswith("_error")]


def test_bench_phase_failure_keeps_headline(cuda):
    """A failing secondary phase (injected into the dense comparator) is
    recorded as dense_error; the headline line still comes out, rc 0, and the
    phases after it still run."""
    out = _bench("--model", "resnet20", "--steps", "2", "--warmup", "1", "--batch-size", "32", "--ref-batch", "16",
                 "--ref-steps", "2", env_extra={"GKSGD_BENCH_FAIL_PHASE": "dense"})
    assert out["value"] > 0 and out["n_gpus"] == 2
    assert "injected failure" in out["dense_error"]
    assert "dense_ms_per_step" not in out and "speedup_vs_dense" not in out
    assert out["ref_bs16_value"] > 0 and out["bf16_value"] > 0


def test_bench_dense_two_ranks_one_gpu(cuda):
    out = _bench("--model", "resnet20", "--steps", "3", "--warmup", "1", "--batch-size", "64", "--dense",
                 "--no-bf16-phase", probe=True)
    assert out["replicas_consistent"] is True and out["config"]["compressor"] == "none"
    # the post-run fabric probe (alpha-beta of all-gather / all-reduce through the bench's exchanger)
    c = out["collectives"]
    assert c["allgather"]["points_bytes_us"] and c["allreduce"]["dense_grad_us"] > 0


def test_bench_native_bootstrap_failure_falls_back(cuda):
    """The native RCCL engine's bootstrap on real hardware where it CANNOT
    succeed: two ranks on one device (RCCL refuses duplicate GPUs, or its
    init never completes).  The non-blocking init must fail or hit its
    deadline on both ranks, the ranks agree, and every phase runs on the
    torch.distributed exchanger -- one bootstrap per process, no hang."""
    out = _bench("--model", "resnet20", "--steps", "2", "--warmup", "1", "--batch-size", "32", "--ref-batch", "0",
                 "--no-bf16-phase", "--no-dense-phase", native=True, timeout=400,
                 env_extra={"GKSGD_RCCL_INIT_TIMEOUT_S": "30"})
    assert out["value"] > 0 and out["n_gpus"] == 2
    assert out["exchange"] == "torch" and out["replicas_consistent"] is True
    assert out["native_inits"] == 1
    assert not [k for k in out if k.endswith("_error")]
