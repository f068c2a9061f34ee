#!/usr/bin/env python3
"""Headline benchmark: whole-node images/s of ResNet-50 data-parallel training
with Gaussian-k gradient sparsification at density 0.1% on MI355X.

Metric (BASELINE.json): "images/sec (whole node) ResNet-50 k=0.1% at 1/2/4/8
MI355X; effective grad compression ratio".  One process per GPU; launched
by ``torch.distributed.run`` for N > 1 (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*).

Each timed step is the FULL training step: zero_grad, forward
(channels_last), backward, per-bucket fused Gaussian-k compression with error
feedback, packed all-gather over RCCL, scatter-add average, fused
momentum-SGD update of every parameter.  The compressor also runs at N = 1
(world of one) so the per-GPU work is identical at every N (weak scaling).
Data: synthetic ImageNet-shaped batches generated on the device; weights:
random init.

Precision: the headline is fp32 compute (fp32 weights, activations and
gradients -- the reference trained in fp32, settings.py:28 USE_FP16=False),
on the hand-written fp32-MFMA convolutions (ops/conv1x1.py); a second timed
phase in the same process measures the bf16-autocast step and reports it as
``bf16_value`` / ``bf16_ms_per_step`` (``--no-bf16-phase`` skips it;
``--amp bf16`` makes bf16 the headline).  fp32 GEMMs: ``--f32-matmul bf16x6``
(default) also offers the fp32-accurate bf16x6 kernels to the per-shape tuner
(ops/conv1x1.py set_f32_matmul); a further phase then times the same step with
the fp32-MFMA GEMMs only (``fp32_native_value``; ``--no-native-phase`` skips).

N > 1 also times, after the sparse loop, a dense comparator: the same model
with a bucketed (``--dense-bucket-mb``, 25 MB), backward-overlapped RCCL
all-reduce of fp32 gradients and no compression -- ``dense_ms_per_step`` /
``speedup_vs_dense`` answer whether sparsification pays on xGMI.

At every N the same compressed step and the dense comparator are also timed
at the reference's own per-worker batch (``REF_BATCH``: ResNet-50 32,
/root/reference/exp_configs/resnet50.conf:2), where the exchange is a far
larger share of the step: ``ref_bs32_value`` / ``ref_bs32_dense_value`` /
``ref_bs32_speedup_vs_dense``.

After those, the other BASELINE configs are timed in the same process at the
headline's precision with the same compressor, density and momentum
correction (``--model-phases``, default ``vgg16,lstm,bert``): VGG-16 CIFAR
bs512 and the reference's bs128, the 2-layer LSTM on PTB bs128 x 35 and the
reference's bs20, BERT-base MLM seq 512 bs32 in ~25 MB buckets -- keys
``<model>_value`` (images/s or tokens/s), ``_ms_per_step``, ``_dtype``,
``_selected_over_k``, ``<model>_ref_bs<B>_value``.

Fail-soft: only the headline phase is fatal.  Every secondary phase (fabric
probe, dense comparator, reference-batch phases, bf16) runs under
``optional_phase``: an exception is recorded as ``<phase>_error`` in the one
JSON line (``GKSGD_BENCH_FAIL_PHASE=<phase>`` injects one, tests).  ``phases``
records per phase the exchanger kind and, on the native engine, the
event-timed collectives of its timed loop.
``exposed_comm_ms`` is the mean time, per timed step, from the end of the
backward pass on the compute stream to the end of the update (event pair):
the communication + decompression + update that the backward did not hide.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch-size B]
       [--compressor gaussian] [--density 0.001] [--model resnet50]

N > 1: after the timed loop every rank digests its fp32 weight arena (fp64
sum + 64-bit content hash, one HIP reduction) and the digests are all-gathered:
``replicas_consistent`` in the JSON line says whether all replicas are still
bit-identical.  ``GKSGD_DIST_BACKEND=gloo`` (with ``--no-native-rccl``) runs
the multi-rank path with several ranks on one GPU (tests/test_bench_gpu.py).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from typing import Optional

# MIOpen tuning state lives in the repo so a fresh box reuses the convolution
# solutions found once by `bench.py --cudnn-benchmark` (tuning/miopen/*.udb).
_HERE = os.path.dirname(os.path.abspath(__file__))
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(_HERE, "tuning", "miopen"))
os.makedirs(os.environ["MIOPEN_USER_DB_PATH"], exist_ok=True)

import torch  # noqa: E402

METRIC = "images/sec (whole node) ResNet-50 k=0.1% at 1/2/4/8 MI355X; effective grad compression ratio"

# Secondary BASELINE configs (--model): dataset, default per-GPU batch,
# throughput unit, tokens per sample (sequence models), data description.
MODELS = {
    "resnet50": ("imagenet", 512, "images/s", 1, "synthetic (ImageNet-shaped 3x224x224, on-device)"),
    "resnet18": ("imagenet", 512, "images/s", 1, "synthetic (ImageNet-shaped 3x224x224, on-device)"),
    "resnet101": ("imagenet", 256, "images/s", 1, "synthetic (ImageNet-shaped 3x224x224, on-device)"),
    "vgg16i": ("imagenet", 128, "images/s", 1, "synthetic (ImageNet-shaped 3x224x224, on-device)"),
    "vgg16": ("cifar10", 512, "images/s", 1, "synthetic (CIFAR-shaped 3x32x32, on-device)"),
    "resnet20": ("cifar10", 512, "images/s", 1, "synthetic (CIFAR-shaped 3x32x32, on-device)"),
    "lstm": ("ptb", 128, "tokens/s", 35, "synthetic (PTB-shaped: vocab 10k, 35-step BPTT, on-device)"),
    "bert": ("wikipedia", 32, "tokens/s", 512, "synthetic (BERT MLM, vocab 30522, seq 512, on-device)"),
    "fcn5net": ("mnist", 1024, "images/s", 1, "synthetic (MNIST-shaped 1x28x28, on-device)"),
}

# The reference's own per-worker batch (/root/reference/exp_configs/<dnn>.conf:2):
# the "ref_bs" phases time the same step at that batch, where the exchange is a
# larger share of the step than at the headline batch.
REF_BATCH = {"resnet50": 32, "vgg16i": 128, "vgg16": 128, "resnet20": 1024, "lstm": 20, "fcn5net": 128}

# BERT (BASELINE config 5, "bucketed compression"): default bucket threshold in
# elements (~25 MB of fp32 gradients per bucket, overlapped with the backward)
# instead of the reference's single 524,288,000-element group.
DEFAULT_THRESHOLD = {"bert": 6_500_000}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch-size", type=int, default=None,
                    help="per-GPU batch (default: per model; ResNet-50 512, env GKSGD_BENCH_BS)")
    ap.add_argument("--cudnn-benchmark", action="store_true", help="MIOpen find (exhaustive conv algorithm search)")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--compressor", default="gaussian")
    ap.add_argument("--density", type=float, default=0.001)
    ap.add_argument("--threshold", type=int, default=None,
                    help="bucket threshold (elements); default: the reference's 524288000 (one group), "
                         "BERT 6.5 M (~25 MB buckets, BASELINE config 5 'bucketed compression')")
    ap.add_argument("--planner", default="threshold", choices=["threshold", "mgs", "mgwfbp"],
                    help="bucket planner: reference threshold grouping, or MGS / MG-WFBP on measured layer-wise "
                         "backward times (utils/profiler.benchmark) and the perf models (utils/perf_model.py)")
    ap.add_argument("--plan-world", type=int, default=None,
                    help="world size the planner's cost models assume (default: this world)")
    ap.add_argument("--amp", default="none", choices=["bf16", "none"],
                    help="headline compute precision: none = fp32 (the reference's), bf16 = bf16 autocast")
    ap.add_argument("--f32-matmul", default=os.environ.get("GKSGD_F32_MATMUL", "bf16x6"),
                    choices=["native", "bf16x6"],
                    help="fp32 convolution / linear GEMM algorithm: native = fp32 MFMA only; bf16x6 = also the "
                         "fp32-accurate bf16x6 product kernels (ops/conv1x1.py set_f32_matmul)")
    ap.add_argument("--no-native-phase", action="store_true",
                    help="skip the secondary fp32-MFMA-only phase of a bf16x6 headline run")
    ap.add_argument("--no-bf16-phase", action="store_true",
                    help="skip the secondary bf16 phase of an fp32 headline run")
    ap.add_argument("--no-dense-phase", action="store_true", help="skip the dense comparator at N > 1")
    ap.add_argument("--ref-batch", type=int, default=None,
                    help="per-GPU batch of the reference-batch phases (default: the reference's exp_configs "
                         "batch of the model, ResNet-50 32; 0 skips them)")
    ap.add_argument("--ref-steps", type=int, default=10, help="timed steps of each reference-batch phase")
    ap.add_argument("--ref-graph", default="auto", choices=["auto", "on", "off"],
                    help="replay the reference-batch steps as one HIP graph (auto: on one GPU)")
    ap.add_argument("--dense-bucket-mb", type=float, default=25.0,
                    help="bucket size of the dense comparator's overlapped all-reduce (MB of fp32 gradients)")
    ap.add_argument("--no-channels-last", action="store_true")
    ap.add_argument("--dense", action="store_true", help="dense RCCL all-reduce comparator (compressor none)")
    ap.add_argument("--no-native-rccl", action="store_true")
    ap.add_argument("--no-momentum-correction", action="store_true",
                    help="plain momentum SGD on the aggregate instead of DGC momentum correction "
                         "(BASELINE config: GaussianK k=0.1%% + momentum correction)")
    ap.add_argument("--no-shadow", action="store_true",
                    help="disable bf16 shadow weights / direct arena gradients (plain autocast)")
    ap.add_argument("--graph", action="store_true",
                    help="capture the whole training step in a HIP graph and replay it (train/graph.py)")
    ap.add_argument("--k-cap-factor", type=float, default=None,
                    help="record capacity k_cap = factor * k of the sparse compressor (default: the compressor's: "
                         "Gaussian-k 1.0 -- at most k entries, what the reference's 500x assumes, the overflow "
                         "staying in the residual; gaussian_cal 4/3)")
    ap.add_argument("--model-phases", default="vgg16,lstm,bert",
                    help="comma list of further BASELINE models timed after the headline in the same process "
                         "(same precision / compressor / density); 'none' skips them")
    ap.add_argument("--model-steps", type=int, default=10, help="timed steps of each further model phase")
    ap.add_argument("--json-out", default=None)
    return ap.parse_args()


def probe_collectives(ex, P: int, dev, rec_bytes: int, dense_bytes: int, iters: int = 10):
    """Short alpha-beta probe of this node's fabric through the bench's own
    exchanger (after the timed loop): the packed-record all-gather at several
    per-rank sizes around the real record, and the dense all-reduce the
    sparse exchange replaces (up to the full fp32 gradient).  Times are the MAX
    over ranks; fits t = alpha + beta * bytes_per_rank (utils/perf_model.py)."""
    from gaussiank_sgd_amd.parallel import comm
    from gaussiank_sgd_amd.utils import perf_model

    def timed(fn):
        for _ in range(3):
            fn()
        comm.barrier()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        torch.cuda.synchronize()
        t = torch.tensor([a.elapsed_time(b) / iters * 1e-3], dtype=torch.float64, device="cuda")
        if comm.backend() == "nccl":
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        return float(t)

    out = {}
    pts = []
    for nb in sorted({4096, 65536, rec_bytes, 4 * rec_bytes, 1 << 22}):
        words = max(nb // 4, 1)
        inp = torch.zeros(words, dtype=torch.int32, device=dev)
        o = torch.zeros(P * words, dtype=torch.int32, device=dev)
        pts.append((words * 4, timed(lambda: ex.allgather_(o, inp))))
    a, b = perf_model.fit_alpha_beta([x for x, _ in pts], [t for _, t in pts])
    out["allgather"] = {"alpha_us": round(a * 1e6, 2), "beta_GBps": round(1e-9 / b, 1) if b > 0 else None,
                        "points_bytes_us": [[x, round(t * 1e6, 1)] for x, t in pts],
                        "record_us": round(dict(pts)[(rec_bytes // 4) * 4] * 1e6, 1) if rec_bytes else None}
    pts = []
    for nb in sorted({1 << 16, 1 << 20, 1 << 24, dense_bytes}):
        t = torch.zeros(max(nb // 4, 1), dtype=torch.float32, device=dev)
        pts.append((t.numel() * 4, timed(lambda t=t: ex.allreduce_(t, average=True))))
        del t
    a2, b2 = perf_model.fit_alpha_beta([x for x, _ in pts], [t for _, t in pts])
    out["allreduce"] = {"alpha_us": round(a2 * 1e6, 2), "beta_GBps": round(1e-9 / b2, 1) if b2 > 0 else None,
                        "points_bytes_us": [[x, round(t * 1e6, 1)] for x, t in pts],
                        "dense_grad_us": round(pts[-1][1] * 1e6, 1)}
    out["_fit"] = {"allgather": (a, b), "allreduce": (a2, b2)}
    return out


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class Phase:
    """One timed phase's objects.  ``release()`` clears every reference held
    here (trainer, optimizer, step closure / GraphedStep with its graph pool)
    so the next phase is timed without the previous one's memory resident."""

    def __init__(self, trainer, opt, comp_name: str, is_sparse: bool, batch: int, model: str):
        self.trainer, self.opt, self.comp_name, self.is_sparse, self.batch = trainer, opt, comp_name, is_sparse, batch
        self.model = model
        self.step = None


def build(args, amp: str, dense: bool, threshold: int, P: int, rank: int, batch: int,
          model: Optional[str] = None) -> Phase:
    """Trainer + DistributedOptimizer of one timed phase.  amp: "fp32" / "bf16";
    model: a MODELS key (default: --model)."""
    from gaussiank_sgd_amd.compression import compressors
    from gaussiank_sgd_amd.parallel import comm
    from gaussiank_sgd_amd.parallel.distributed_optimizer import DistributedOptimizer
    from gaussiank_sgd_amd.train import DLTrainer

    model = model or args.model
    dataset, _, _, _, _ = MODELS[model]
    trainer = DLTrainer(rank, P, dnn=model, dataset=dataset, batch_size=batch,
                        lr=0.1, nworkers=P, device="cuda", amp="bf16" if amp == "bf16" else None,
                        channels_last=not args.no_channels_last, seed=0)
    comp_name = "none" if dense else args.compressor
    is_sparse = not dense and comp_name not in ("none", "bucket")
    seq_names = layer_times = None
    if args.planner != "threshold" and not dense and model == args.model:
        # reference dist_trainer.py:38-47: layer-wise backward profile, shared from rank 0
        from gaussiank_sgd_amd.utils.profiler import benchmark
        seq_names, layer_times, _ = benchmark(trainer, warmup=3, iterations=10)
        layer_times = comm.broadcast_object(list(layer_times), 0)
    opt = DistributedOptimizer(trainer.optimizer, named_parameters=trainer.net.named_parameters(),
                               compression=compressors[comp_name], is_sparse=is_sparse, density=args.density,
                               threshold=threshold, compress_single_rank=True, density_warmup=False,
                               native_rccl=not args.no_native_rccl, seq_layernames=seq_names,
                               layerwise_times=layer_times,
                               planner=args.planner if not dense and model == args.model else "threshold",
                               planner_world=args.plan_world,
                               momentum_correction=is_sparse and not args.no_momentum_correction)
    comm.broadcast_parameters(trainer.net.state_dict(), root_rank=0)
    if not args.no_shadow:
        from gaussiank_sgd_amd.parallel import install_bf16_shadow, install_direct_grads
        if amp == "bf16":
            install_bf16_shadow(trainer.net, opt)
        else:
            install_direct_grads(trainer.net, opt)
    trainer.update_optimizer(opt)
    trainer.display = 10 ** 9  # no host-syncing log lines inside the timed loop
    return Phase(trainer, opt, comp_name, is_sparse, batch, model)


def run_phase(args, ph: Phase, steps: int, warmup: int, P: int, graph: Optional[bool] = None):
    """W untimed warm-up steps, then EXACTLY K steps bracketed by a barrier +
    synchronize on both sides; returns (elapsed seconds, max over ranks;
    exposed-comm ms per step, max over ranks).  The step callable is kept
    on ``ph``."""
    from gaussiank_sgd_amd.parallel import comm

    trainer, opt = ph.trainer, ph.opt
    state = {"hidden": None}
    lstm = ph.model == "lstm"
    clip = 0.25 if lstm else None  # reference dist_trainer.py:80-85
    marks = []   # (end of backward, end of update) event pairs of the timed steps

    def step():
        opt.zero_grad()
        if lstm:
            _, state["hidden"] = trainer.train(1, hidden=state["hidden"])
        else:
            trainer.train(1)
        ev = None
        if state.get("mark"):
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
        if clip is not None:
            opt.synchronize()
            opt.clip_grad_norm_(clip)
        trainer.update_model()
        if ev is not None:
            e2 = torch.cuda.Event(enable_timing=True)
            e2.record()
            marks.append((ev, e2))

    graph = args.graph if graph is None else graph
    run = step
    if graph:
        # whole-step HIP graph: capture after the eager warm-up, replay in the timed loop
        from gaussiank_sgd_amd.train.graph import GraphedStep
        for _ in range(warmup):
            step()
        run = GraphedStep(trainer, opt, clip)
    ph.step = run
    for _ in range(warmup):
        run()
    torch.cuda.synchronize()
    opt._collect_selected()  # drop warm-up counts
    if opt._exchanger is not None:
        opt._exchanger.reset_stats()   # shared communicator: count this phase's timed loop only
    state["mark"] = not graph and os.environ.get("GKSGD_BENCH_NO_MARKS", "0") != "1"
    comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    comm.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    state["mark"] = False
    exposed = sum(a.elapsed_time(b) for a, b in marks) / len(marks) if marks else float("nan")
    t = torch.tensor([elapsed, exposed], dtype=torch.float64, device="cuda")
    if P > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t[0]), float(t[1])


def sync_timeouts(opt) -> int:
    """Expired bounded spins of the fused compression decide / fallback grid
    over every compressed bucket (0 unless a grid was not co-resident)."""
    from gaussiank_sgd_amd import ops
    n = 0
    for b in opt.arena.buckets:
        bufs = getattr(b, "bufs", None)
        if bufs is not None and getattr(bufs, "ctrl", None) is not None and bufs.ctrl.is_cuda:
            n += ops.sync_timeouts(bufs)
    return n


def selection(ph: Phase, steps: int, density: float) -> dict:
    """Entries sent per step over k, and the per-rank wire compression ratio,
    of a phase's timed loop (its selected counts since the warm-up drain)."""
    opt = ph.opt
    if not ph.is_sparse:
        return {}
    from gaussiank_sgd_amd.compression import compressors
    comp = compressors[ph.comp_name]
    pairs = opt._collect_selected(with_totals=True)
    k_total = sum(comp.k_of(b.numel, density) for b in opt.arena.buckets)
    sent = sum(p[0] for p in pairs) / max(1, steps)
    nparams = sum(b.numel for b in opt.arena.buckets)
    wb = opt.wire_bytes_per_step(density)
    return {"selected_over_k": round(sent / k_total, 4) if k_total else None,
            "effective_compression_ratio": round(nparams * 4.0 / wb, 1) if wb else None}


def phase_info(ph: Phase) -> dict:
    """Exchanger kind and the event-timed collectives of the phase's timed
    loop (native engine; empty for torch.distributed / local)."""
    ex = ph.opt._exchanger if ph is not None and ph.opt is not None else None
    info = {"exchange": ex.kind if ex is not None else "none", "buckets": len(ph.opt.arena.buckets) if ph else None}
    wp = getattr(ph.trainer, "weight_prep", None) if ph is not None else None
    if wp is not None:
        info["weight_prep"] = {"relayouts": len(wp.entries), "batched_launches": wp.launches}
    if ph is not None and ph.opt is not None:
        info["compress_sync_timeouts"] = sync_timeouts(ph.opt)
    if ex is not None:
        try:
            info["timed_loop"] = ex.stats() or None
        except Exception as e:  # noqa: BLE001 - diagnostics only
            info["timed_loop"] = "error: %s" % e
    return info


def release(ph) -> None:
    import gc
    if ph is None:
        return
    opt = ph.opt
    if opt is not None and opt._exchanger is not None:
        try:
            opt._exchanger.close()
        finally:
            opt._exchanger = None
    ph.trainer = ph.opt = ph.step = None
    del opt
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def _agree(ok: bool, P: int):
    """(all ranks ok, communicator alive): the MIN of every rank's verdict on
    a phase; a failing agreement collective means the communicator is broken
    and ends the optional phases."""
    if P == 1:
        return ok, True
    from gaussiank_sgd_amd.parallel import comm
    try:
        dev = "cuda" if comm.backend() == "nccl" else "cpu"
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MIN)
        return int(t) == 1, True
    except Exception:  # noqa: BLE001
        return False, False


_EMIT = {"json_out": None}


def emit(out: dict) -> None:
    """Rank 0's one JSON line (stdout, and --json-out)."""
    line = json.dumps(out)
    print(line, flush=True)
    if _EMIT["json_out"]:
        with open(_EMIT["json_out"], "w") as f:
            f.write(line + "\n")


def _phase_deadline(name: str, out: dict, rank: int):
    """A secondary phase that does not finish in ``GKSGD_BENCH_PHASE_TIMEOUT_S``
    (default 240 s) ends the process: rank 0 first prints the JSON line with
    the headline and the phases finished so far plus ``<name>_error``.  This
    covers the ASYMMETRIC failure the agreement collective cannot: one rank
    raises while the others still wait inside the phase's collectives, which
    would otherwise hang until the 1800 s collective timeout and lose the
    line.  Every rank arms its own timer, so every rank exits."""
    import threading
    s = float(os.environ.get("GKSGD_BENCH_PHASE_TIMEOUT_S", "240"))
    if os.environ.get("GKSGD_GEMM_RETUNE"):
        s *= 4      # a first-time GEMM autotune is slow but healthy

    def fire():
        out[name + "_error"] = "timeout: phase not finished after %.0f s on rank %d" % (s, rank)
        # machine-readable: the line is cut short (the process still exits 0 so
        # the headline, measured and complete, is not discarded with the phase)
        out["bench_incomplete"] = True
        print("bench.py: phase %s timed out after %.0f s; exiting" % (name, s), file=sys.stderr, flush=True)
        if rank == 0:
            try:
                emit(out)
            finally:
                os._exit(0)
        os._exit(0)

    t = threading.Timer(s, fire)
    t.daemon = True
    t.start()
    return t


def _injected(name: str) -> bool:
    """GKSGD_BENCH_FAIL_PHASE=<phase> fails that phase on every rank;
    GKSGD_BENCH_FAIL_PHASE_RANK=<r> restricts it to rank r (asymmetric)."""
    if os.environ.get("GKSGD_BENCH_FAIL_PHASE") != name:
        return False
    only = os.environ.get("GKSGD_BENCH_FAIL_PHASE_RANK")
    if only is None or only == "":
        return True
    from gaussiank_sgd_amd.parallel import comm
    return int(only) == comm.rank()


def optional_phase(name: str, out: dict, P: int, fn) -> bool:
    """Run one secondary phase fail-soft: an exception (or the injected one,
    ``GKSGD_BENCH_FAIL_PHASE=<name>``) is recorded as ``<name>_error`` in the
    JSON line instead of losing the headline; a phase that hangs (one rank
    failed while the others wait in its collectives) hits ``_phase_deadline``.
    Returns whether the ranks could still agree afterwards (False: skip the
    remaining phases)."""
    from gaussiank_sgd_amd.parallel import comm
    holder = []
    err = None
    timer = _phase_deadline(name, out, comm.rank()) if P > 1 else None
    try:
        if _injected(name):
            raise RuntimeError("injected failure (GKSGD_BENCH_FAIL_PHASE=%s)" % name)
        fn(holder)
    except Exception as e:  # noqa: BLE001 - fail-soft by design
        msg = str(e).strip().splitlines()
        err = "%s: %s" % (type(e).__name__, msg[0][:300] if msg else "")
        print("bench.py: phase %s failed: %s" % (name, err), file=sys.stderr, flush=True)
    for ph in holder:
        try:
            release(ph)
        except Exception as e:  # noqa: BLE001
            err = err or "release: %s" % e
    ok, alive = _agree(err is None, P)
    if timer is not None:
        timer.cancel()
    if err is not None:
        out[name + "_error"] = err
    elif not ok:
        out[name + "_error"] = "failed on another rank"
    return alive


def main() -> int:
    args = parse()
    _EMIT["json_out"] = args.json_out
    from gaussiank_sgd_amd import ops
    from gaussiank_sgd_amd.compression import compressors
    from gaussiank_sgd_amd.parallel import comm

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and world_env == 1:
        # self-launch: start torch.distributed.run as a child (never exec after touching the GPU);
        # a free port unless MASTER_PORT pins one (a busy fixed port would fail the whole run)
        import subprocess
        port = os.environ.get("MASTER_PORT") or str(free_port())
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
               "--master-addr", "127.0.0.1", "--master-port", port,
               os.path.abspath(__file__)] + sys.argv[1:]
        return subprocess.call(cmd)

    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if not torch.cuda.is_available():
        print("bench.py needs a GPU", file=sys.stderr)
        return 2
    # several ranks may share a device (gloo rehearsal of the multi-rank path on one GPU)
    torch.cuda.set_device(local_rank % torch.cuda.device_count())
    comm.init(backend=os.environ.get("GKSGD_DIST_BACKEND") or None)
    P = comm.size()
    rank = comm.rank()
    if not ops.load():
        raise RuntimeError("native extension missing: run `python -m gaussiank_sgd_amd.ops.build`")
    torch.backends.cudnn.benchmark = args.cudnn_benchmark or os.environ.get("GKSGD_CUDNN_BENCHMARK", "0") == "1"

    if args.model not in MODELS:
        raise SystemExit("bench.py --model must be one of %s" % sorted(MODELS))
    dataset, default_bs, unit, tok_per_sample, data_desc = MODELS[args.model]
    if args.batch_size is None:
        args.batch_size = int(os.environ.get("GKSGD_BENCH_BS", default_bs)) if args.model == "resnet50" else default_bs
    if args.threshold is None:
        args.threshold = DEFAULT_THRESHOLD.get(args.model, 524288000)
    ref_bs = REF_BATCH.get(args.model) if args.ref_batch is None else args.ref_batch
    amp = "bf16" if args.amp == "bf16" else "fp32"
    if args.k_cap_factor is not None:
        compressors[args.compressor].kcap_factor = float(args.k_cap_factor)
    from gaussiank_sgd_amd.ops import conv1x1
    conv1x1.set_f32_matmul(args.f32_matmul)

    # ---- headline phase: any failure here is fatal (non-zero exit, no JSON line)
    ph = build(args, amp, args.dense, args.threshold, P, rank, args.batch_size)
    trainer, opt, comp_name, is_sparse = ph.trainer, ph.opt, ph.comp_name, ph.is_sparse
    nparams = sum(p.numel() for p in trainer.net.parameters() if p.requires_grad)
    elapsed, exposed = run_phase(args, ph, args.steps, args.warmup, P)
    loss = trainer.current_loss()
    pairs = opt._collect_selected(with_totals=True)
    sent = sum(p[0] for p in pairs) / max(1, args.steps)
    total = sum(p[1] for p in pairs) / max(1, args.steps)
    # What goes on the wire per rank and step: one fixed-size record per
    # bucket, (4 header + k_cap indices + k_cap values) int32 words.
    comp = compressors[comp_name]
    k_total = sum(comp.k_of(b.numel, args.density) for b in opt.arena.buckets) if is_sparse else 0
    wire_bytes = opt.wire_bytes_per_step(args.density if is_sparse else 1.0)
    ratio = (nparams * 4.0) / wire_bytes if wire_bytes else 1.0
    n_buckets = len(opt.arena.buckets)
    kind = opt._exchanger.kind if opt._exchanger is not None else "none"
    phases = {"headline": phase_info(ph)}
    replicas = None
    if P > 1:
        # bit-identical replicas: all-gather a digest of every rank's weight arena
        torch.cuda.synchronize()
        d = ops.arena_digest(opt.arena.weights)
        mine = torch.tensor([x - (1 << 64) if x >= (1 << 63) else x for x in d], dtype=torch.int64,
                            device="cuda" if comm.backend() == "nccl" else "cpu")
        allv = [torch.zeros_like(mine) for _ in range(P)]
        torch.distributed.all_gather(allv, mine)
        replicas = all(torch.equal(allv[0], v) for v in allv[1:])
    ms = elapsed / args.steps * 1e3
    imgs = P * args.batch_size * tok_per_sample * args.steps / elapsed
    metric = METRIC if args.model == "resnet50" else "%s (whole node) %s k=%g%% on MI355X" % (
        unit, args.model, 100.0 * (args.density if is_sparse else 1.0))
    out = {
        "metric": metric,
        "value": round(imgs, 2),
        "unit": unit,
        "n_gpus": P,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": amp,
        "data": data_desc + ", random-init weights",
        "config": {
            "model": args.model,
            "global_batch": P * args.batch_size,
            "per_gpu_batch": args.batch_size,
            "seq_len": tok_per_sample if tok_per_sample > 1 else None,
            "image_size": {"imagenet": 224, "cifar10": 32, "mnist": 28}.get(dataset),
            "parallelism": "dp%d" % P,
            "compressor": comp_name,
            "density": args.density if is_sparse else 1.0,
            "buckets": n_buckets,
            "threshold": args.threshold,
            "planner": args.planner if args.planner == "threshold" else "%s@P=%s" % (args.planner, args.plan_world or P),
            "exchange": kind,
            "momentum_correction": bool(opt._mc),
            "hip_graph": bool(args.graph),
            "f32_matmul": args.f32_matmul if amp == "fp32" else None,
            "k_cap_factor": round(float(getattr(compressors[comp_name], "kcap_factor", 0.0)), 4) if is_sparse else None,
        },
        "graph_captures": getattr(ph.step, "captures", None),
        "world": P,
        "exchange": kind,
        "replicas_consistent": replicas,
        "compress_sync_timeouts": sync_timeouts(opt),
        "exposed_comm_ms": round(exposed, 3) if exposed == exposed else None,
        "collectives": None,
        "effective_compression_ratio": round(ratio, 1),
        "wire_bytes_per_rank_step": wire_bytes,
        # sent: entries actually in the records (<= k_cap per bucket); total:
        # entries that passed the threshold before the k_cap overflow cut
        "selected_per_step": round(sent, 1),
        "candidates_per_step": round(total, 1),
        "k_per_step": k_total if is_sparse else None,
        "selected_over_k": round(sent / k_total, 4) if is_sparse and k_total else None,
        "params": nparams,
        "final_loss": round(loss, 4) if loss == loss else None,
        "phases": phases,
    }
    del trainer, opt   # the Phase holder keeps the only references; release() drops them

    def collectives_probe(holder):
        # alpha-beta probe of the fabric through the headline's exchanger (N > 1)
        ex = ph.opt._exchanger
        if ex is None:
            return
        timed_loop = ex.stats()     # event-timed collectives of the timed loop (native engine)
        col = probe_collectives(ex, P, torch.device("cuda", torch.cuda.current_device()),
                                wire_bytes // max(1, n_buckets) if is_sparse else 4096, nparams * 4)
        fit = col.pop("_fit")
        if timed_loop:
            col["timed_loop"] = timed_loop
        out["collectives"] = col
        out_path = os.environ.get("GKSGD_PERF_MODEL_OUT")
        if out_path and rank == 0:
            from gaussiank_sgd_amd.utils import perf_model
            for op in ("allgather", "allreduce"):
                perf_model.update(out_path, op, {
                    "alpha_s": fit[op][0], "beta_s_per_byte": fit[op][1], "measured": True,
                    "source": "bench.py probe, %d x %s, exchanger %s, points %s" % (
                        P, torch.cuda.get_device_name(), ex.kind, col[op]["points_bytes_us"])},
                    key=str(P))

    alive = True
    if P > 1 and os.environ.get("GKSGD_BENCH_PROBE", "1") == "1":
        alive = optional_phase("collectives", out, P, collectives_probe)
    release(ph)
    ph = None

    def timed(holder, name, amp_, dense, threshold, batch, steps, warmup, graph=None, model=None):
        p = build(args, amp_, dense, threshold, P, rank, batch, model)
        holder.append(p)
        el, exp_ = run_phase(args, p, steps, warmup, P, graph)
        info = phase_info(p)
        info["hip_graph"] = bool(args.graph if graph is None else graph)
        tps = MODELS[p.model][3]
        info.update(ms_per_step=round(el / steps * 1e3, 3),
                    value=round(P * batch * tps * steps / el, 2),
                    exposed_comm_ms=round(exp_, 3) if exp_ == exp_ else None, per_gpu_batch=batch, steps=steps)
        info.update(selection(p, steps, args.density))
        phases[name] = info
        return info

    # ---- secondary bf16 phase of an fp32 headline
    if alive and amp == "fp32" and not args.no_bf16_phase:
        def bf16_phase(holder):
            i = timed(holder, "bf16", "bf16", args.dense, args.threshold, args.batch_size, args.steps, args.warmup)
            out["bf16_ms_per_step"] = i["ms_per_step"]
            out["bf16_value"] = i["value"]
            out["bf16_exposed_comm_ms"] = i["exposed_comm_ms"]
        alive = optional_phase("bf16", out, P, bf16_phase)

    # ---- secondary fp32 phase with the fp32-MFMA GEMMs only (the bf16x6 kernels
    # off): the same step on the other fp32 GEMM algorithm, for comparison
    if alive and amp == "fp32" and args.f32_matmul == "bf16x6" and not args.no_native_phase:
        def native_phase(holder):
            prev = conv1x1.set_f32_matmul("native")
            try:
                i = timed(holder, "fp32_native", "fp32", args.dense, args.threshold, args.batch_size,
                          max(5, min(args.steps, 10)), max(3, min(args.warmup, 5)))
            finally:
                conv1x1.set_f32_matmul(prev)
            out["fp32_native_ms_per_step"] = i["ms_per_step"]
            out["fp32_native_value"] = i["value"]
        alive = optional_phase("fp32_native", out, P, native_phase)

    # ---- dense comparator (N > 1): bucketed, backward-overlapped RCCL all-reduce
    dense_elems = max(1, int(args.dense_bucket_mb * 1e6 / 4))
    if alive and P > 1 and not args.dense and not args.no_dense_phase:
        def dense_phase(holder):
            i = timed(holder, "dense", amp, True, dense_elems, args.batch_size, max(5, min(args.steps, 10)),
                      max(3, min(args.warmup, 5)))
            out["dense_ms_per_step"] = i["ms_per_step"]
            out["dense_value"] = i["value"]
            out["dense_buckets"] = i["buckets"]
            out["dense_exposed_comm_ms"] = i["exposed_comm_ms"]
            out["speedup_vs_dense"] = round(i["ms_per_step"] / ms, 4)
        alive = optional_phase("dense", out, P, dense_phase)

    # ---- reference-batch phases: the same compressed step, and the dense
    # comparator, at the reference's per-worker batch (exp_configs/<dnn>.conf)
    if alive and ref_bs and not args.dense:
        tag = "ref_bs%d" % ref_bs
        rsteps, rwarm = max(1, args.ref_steps), max(2, min(args.warmup, 5))
        # the reference batch is launch-bound: the whole step replays as one HIP
        # graph (train/graph.py) by default on one GPU; at N > 1 eager, with the
        # side-stream overlap (--ref-graph on|off overrides)
        ref_graph = (P == 1) if args.ref_graph == "auto" else args.ref_graph == "on"

        def ref_sparse(holder):
            i = timed(holder, tag, amp, False, args.threshold, ref_bs, rsteps, rwarm, graph=ref_graph)
            out[tag + "_value"] = i["value"]
            out[tag + "_ms_per_step"] = i["ms_per_step"]
            out[tag + "_exposed_comm_ms"] = i["exposed_comm_ms"]

        def ref_dense(holder):
            i = timed(holder, tag + "_dense", amp, True, dense_elems, ref_bs, rsteps, rwarm, graph=ref_graph)
            out[tag + "_dense_value"] = i["value"]
            out[tag + "_dense_ms_per_step"] = i["ms_per_step"]
            if (tag + "_ms_per_step") in out:
                out[tag + "_speedup_vs_dense"] = round(i["ms_per_step"] / out[tag + "_ms_per_step"], 4)
        alive = optional_phase(tag, out, P, ref_sparse)
        if alive:
            alive = optional_phase(tag + "_dense", out, P, ref_dense)

    # ---- the other BASELINE configs (3-5) in the same process, at the same
    # precision as the headline and the same compressor / density / momentum
    # correction: VGG-16 CIFAR bs512 (+ the reference's bs128), 2-layer LSTM
    # PTB bs128 x 35 (+ the reference's bs20), BERT-base MLM seq512 bs32 (14
    # buckets of ~25 MB).  Each is fail-soft and adds <model>_value /
    # _ms_per_step / _dtype / _unit / _selected_over_k (and _ref_bs<B>_value).
    if alive and not args.dense and args.model_phases != "none":
        for m in [x for x in args.model_phases.split(",") if x and x != args.model]:
            if not alive:
                break
            if m not in MODELS:
                out[m + "_error"] = "unknown model"
                continue
            mbatch = MODELS[m][1]
            mthr = DEFAULT_THRESHOLD.get(m, 524288000)
            msteps, mwarm = max(3, min(args.steps, args.model_steps)), max(2, min(args.warmup, 3))

            def model_phase(holder, m=m, mbatch=mbatch, mthr=mthr, msteps=msteps, mwarm=mwarm):
                i = timed(holder, m, amp, False, mthr, mbatch, msteps, mwarm, graph=False, model=m)
                out[m + "_value"] = i["value"]
                out[m + "_unit"] = MODELS[m][2]
                out[m + "_ms_per_step"] = i["ms_per_step"]
                out[m + "_dtype"] = amp
                out[m + "_per_gpu_batch"] = mbatch
                out[m + "_selected_over_k"] = i.get("selected_over_k")
                out[m + "_effective_compression_ratio"] = i.get("effective_compression_ratio")
            alive = optional_phase(m, out, P, model_phase)
            rb = REF_BATCH.get(m)
            if alive and rb and rb != mbatch and args.ref_batch != 0:
                tag = "%s_ref_bs%d" % (m, rb)

                # the reference batch replays as one HIP graph on one GPU, as the
                # headline model's reference-batch phase (--ref-graph)
                rgraph = (P == 1) if args.ref_graph == "auto" else args.ref_graph == "on"

                def model_ref_phase(holder, m=m, rb=rb, mthr=mthr, msteps=msteps, mwarm=mwarm, tag=tag, rgraph=rgraph):
                    i = timed(holder, tag, amp, False, mthr, rb, msteps, mwarm, graph=rgraph, model=m)
                    out[tag + "_value"] = i["value"]
                    out[tag + "_ms_per_step"] = i["ms_per_step"]
                alive = optional_phase(tag, out, P, model_ref_phase)

    # every phase's shapes (the reference-batch phases tune their own keys)
    if rank == 0 and os.environ.get("GKSGD_GEMM_DUMP"):
        from gaussiank_sgd_amd.ops.conv1x1 import tuned_choices, tuning_log
        log = tuning_log()
        with open(os.environ["GKSGD_GEMM_DUMP"], "w") as f:
            json.dump([[list(k), list(v), [[list(t), r] for t, r in log.get(k, [])]]
                       for k, v in tuned_choices().items()], f)
    if rank == 0 and os.environ.get("GKSGD_GEMM_SAVE"):
        from gaussiank_sgd_amd.ops.conv1x1 import save_choices
        save_choices(os.environ["GKSGD_GEMM_SAVE"])
    out["native_inits"] = comm.native_bootstraps()   # one per process: the communicator is shared by every phase
    if rank == 0:
        emit(out)
    try:
        comm.shutdown()
    except Exception as e:  # noqa: BLE001 - the result line is already out
        print("bench.py: shutdown: %s" % e, file=sys.stderr)
    if replicas is False:
        print("bench.py: replicas diverged", file=sys.stderr)
        return 3
    return 0


if __name__ == "__main__":
    sys.exit(main())
