"""Horovod-compatible communication facade over torch.distributed (RCCL / gloo).

Parity: reference ``distributed_optimizer.py:21-26`` re-exports Horovod's
``init, size, local_size, rank, local_rank, broadcast, allreduce_async_,
allgather_async, broadcast_async_, synchronize`` and defines
``broadcast_parameters`` / ``broadcast_optimizer_state`` (:588-736); the
trainer also uses ``mpi4py`` ``COMM_WORLD.bcast`` (dist_trainer.py:16-17,40)
-> ``broadcast_object`` here.

Design: one process per GPU.  ``init()`` reads the torchrun variables
(RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR) or, for mpirun launches, the
OpenMPI ones (OMPI_COMM_WORLD_*).  On GPUs the backend is ``nccl`` (= RCCL on
ROCm over xGMI), on CPU ``gloo``.  Async handles wrap torch Work objects; for
RCCL ``synchronize`` only makes the current HIP stream wait (no host block),
matching how the hot path is meant to run.  A world of one process needs no
process group at all.
"""
from __future__ import annotations

import contextlib
import datetime
import os
import threading
import time
from typing import Any, Callable, Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

_state: Dict[str, Any] = {"initialized": False, "rank": 0, "size": 1, "local_rank": 0, "local_size": 1,
                          "backend": None, "owns_pg": False}
# per-thread world state of a loopback (in-process fake) world; see loopback_world()
_tls = threading.local()


def _S() -> Dict[str, Any]:
    st = getattr(_tls, "state", None)
    return st if st is not None else _state


class _LoopbackWorld:
    """P virtual ranks = P threads of one process.  Every collective is an
    exchange: each rank deposits its payload, all meet at a barrier, every
    rank reads all P payloads in rank order (so reductions are deterministic
    and identical on every rank), and a second barrier frees the slots."""

    def __init__(self, P: int, timeout_s: float):
        self.P = P
        self.slots: List[Any] = [None] * P
        self.barrier = threading.Barrier(P, timeout=timeout_s)

    def exchange(self, rank: int, payload: Any) -> List[Any]:
        self.slots[rank] = payload
        self.barrier.wait()
        got = list(self.slots)
        self.barrier.wait()
        return got


def loopback_world(P: int, fn: Callable[[int], Any], timeout_s: float = 120.0) -> List[Any]:
    """Run ``fn(rank)`` on P virtual ranks (threads) whose comm calls --
    ``size/rank``, all-reduce, all-gather, broadcast, barrier, the hot-path
    ``Exchanger`` -- go through an in-process loopback world with the real
    collective semantics.  Unit-tests the whole hook -> bucket -> compress ->
    exchange -> decompress -> step path of ``DistributedOptimizer`` for any P
    without processes.  Returns fn's results in rank
    order; an exception on any rank breaks the barrier for the others and is
    re-raised here."""
    world = _LoopbackWorld(P, timeout_s)
    results: List[Any] = [None] * P
    errors: List[Optional[BaseException]] = [None] * P

    def run(r: int) -> None:
        _tls.state = {"initialized": True, "rank": r, "size": P, "local_rank": r, "local_size": P,
                      "backend": "loopback", "owns_pg": False, "world": world}
        try:
            results[r] = fn(r)
        except BaseException as e:  # noqa: BLE001 - re-raised on the caller's thread
            errors[r] = e
            world.barrier.abort()
        finally:
            _tls.state = None

    threads = [threading.Thread(target=run, args=(r,), name="loopback-rank%d" % r) for r in range(P)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    first = next((e for e in errors if e is not None and not isinstance(e, threading.BrokenBarrierError)), None)
    if first is None:
        first = next((e for e in errors if e is not None), None)
    if first is not None:
        raise first
    return results


def _loopback() -> Optional[_LoopbackWorld]:
    st = getattr(_tls, "state", None)
    return st["world"] if st is not None else None


def _lb_exchange(payload: Any) -> List[Any]:
    # GPU payloads: the producing stream finishes before another rank (thread,
    # own current / comm stream) may read the tensor
    if torch.is_tensor(payload) and payload.is_cuda:
        torch.cuda.current_stream(payload.device).synchronize()
    return _loopback().exchange(rank(), payload)


def _lb_settle(t: torch.Tensor) -> None:
    # the other ranks' payloads were allocated on THEIR streams: finish reading
    # them before they are released to (and reused by) those streams
    if t.is_cuda:
        torch.cuda.current_stream(t.device).synchronize()


def _env_int(*names: str, default: int) -> int:
    for n in names:
        v = os.environ.get(n)
        if v is not None and v != "":
            return int(v)
    return default


def init(backend: Optional[str] = None, timeout_s: Optional[float] = None, device: Optional[str] = None) -> None:
    """Initialise the world (idempotent).  Equivalent of ``hvd.init()``."""
    if _S()["initialized"]:  # (always true on a loopback rank)
        return
    rank = _env_int("RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK", default=0)
    size = _env_int("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", default=1)
    local_rank = _env_int("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", default=rank)
    local_size = _env_int("LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE", default=size)
    if dist.is_available() and dist.is_initialized():
        rank, size = dist.get_rank(), dist.get_world_size()
        _S()["backend"] = dist.get_backend()
    elif size > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        os.environ["RANK"] = str(rank)
        os.environ["WORLD_SIZE"] = str(size)
        if backend is None:
            want_gpu = device != "cpu" and torch.cuda.device_count() > 0
            backend = "nccl" if want_gpu else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))
        kw = {}
        t = timeout_s if timeout_s is not None else float(os.environ.get("GKSGD_COLLECTIVE_TIMEOUT_S", "1800"))
        kw["timeout"] = datetime.timedelta(seconds=t)
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
        dist.init_process_group(backend=backend, **kw)
        _S()["backend"] = backend
        _S()["owns_pg"] = True
    _S().update(initialized=True, rank=rank, size=size, local_rank=local_rank, local_size=local_size)


def shutdown() -> None:
    if _loopback() is not None:
        return
    release_native()
    if _S()["owns_pg"] and dist.is_initialized():
        dist.destroy_process_group()
    _S().update(initialized=False, rank=0, size=1, local_rank=0, local_size=1, backend=None, owns_pg=False)


def is_initialized() -> bool:
    return _S()["initialized"]


def size() -> int:
    return _S()["size"]


def rank() -> int:
    return _S()["rank"]


def local_rank() -> int:
    return _S()["local_rank"]


def local_size() -> int:
    return _S()["local_size"]


def backend() -> Optional[str]:
    return _S()["backend"]


def _distributed() -> bool:
    return _S()["size"] > 1 and dist.is_initialized() and _loopback() is None


class Handle:
    """Async handle: ``synchronize(handle)`` returns the output tensor."""

    __slots__ = ("work", "output", "post")

    def __init__(self, work, output, post=None):
        self.work = work
        self.output = output
        self.post = post


def synchronize(handle: Handle) -> torch.Tensor:
    if handle.work is not None:
        handle.work.wait()
        handle.work = None
    if handle.post is not None:
        handle.output = handle.post(handle.output)
        handle.post = None
    return handle.output


def barrier() -> None:
    if _loopback() is not None:
        _loopback().barrier.wait()
    elif _distributed():
        if backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


# ----------------------------------------------------------------------------
# collectives
# ----------------------------------------------------------------------------
def allreduce_async_(tensor: torch.Tensor, average: bool = True, name: Optional[str] = None) -> Handle:
    if _loopback() is not None:
        parts = _lb_exchange(tensor.detach().clone())
        acc = parts[0].clone()
        for p in parts[1:]:
            acc.add_(p)
        tensor.copy_(acc.div_(len(parts)) if average else acc)
        _lb_settle(tensor)
        return Handle(None, tensor)
    if not _distributed():
        return Handle(None, tensor)
    if average and backend() == "nccl":
        work = dist.all_reduce(tensor, op=dist.ReduceOp.AVG, async_op=True)
        return Handle(work, tensor)
    work = dist.all_reduce(tensor, op=dist.ReduceOp.SUM, async_op=True)
    if average:
        n = size()
        return Handle(work, tensor, post=lambda t: t.div_(n))
    return Handle(work, tensor)


def allreduce_(tensor: torch.Tensor, average: bool = True, name: Optional[str] = None) -> torch.Tensor:
    return synchronize(allreduce_async_(tensor, average, name))


def allreduce(tensor: torch.Tensor, average: bool = True, name: Optional[str] = None) -> torch.Tensor:
    return allreduce_(tensor.clone(), average, name)


def allgather_into_(out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
    """Fixed-size all-gather: out = concat over ranks of inp (out numel = P * inp numel)."""
    if _loopback() is not None:
        parts = _lb_exchange(inp.detach().reshape(-1).clone())
        out.view(-1).copy_(torch.cat(parts))
        _lb_settle(out)
        return None
    if not _distributed():
        out.view(-1)[: inp.numel()].copy_(inp.view(-1))
        return None
    if backend() == "gloo":
        chunks = list(out.view(size(), -1).unbind(0))
        return dist.all_gather(chunks, inp.view(-1).contiguous(), async_op=async_op)
    return dist.all_gather_into_tensor(out.view(-1), inp.view(-1).contiguous(), async_op=async_op)


def allgather_async(tensor: torch.Tensor, name: Optional[str] = None) -> Handle:
    """Horovod semantics: first dimension may differ per rank; result is the concat."""
    if _loopback() is not None:
        res = torch.cat(_lb_exchange(tensor.detach().clone()), 0)
        _lb_settle(res)
        return Handle(None, res)
    if not _distributed():
        return Handle(None, tensor.clone())
    t = tensor.contiguous()
    n0 = torch.tensor([t.shape[0] if t.dim() > 0 else 1], dtype=torch.int64, device=t.device)
    sizes = torch.zeros(size(), dtype=torch.int64, device=t.device)
    allgather_into_(sizes, n0)
    sizes_l = [int(x) for x in sizes.cpu().tolist()]
    mx = max(sizes_l)
    rest = tuple(t.shape[1:])
    padded = torch.zeros((mx,) + rest, dtype=t.dtype, device=t.device)
    if t.shape[0] > 0:
        padded[: t.shape[0]].copy_(t)
    out = torch.empty((size() * mx,) + rest, dtype=t.dtype, device=t.device)
    work = allgather_into_(out, padded, async_op=True)

    def post(o):
        parts = [o[i * mx: i * mx + s] for i, s in enumerate(sizes_l)]
        return torch.cat(parts, 0)

    return Handle(work, out, post)


def allgather(tensor: torch.Tensor, name: Optional[str] = None) -> torch.Tensor:
    return synchronize(allgather_async(tensor, name))


def broadcast_async_(tensor: torch.Tensor, root_rank: int, name: Optional[str] = None) -> Handle:
    if _loopback() is not None:
        src = _lb_exchange(tensor.detach().clone() if rank() == root_rank else None)[root_rank]
        if rank() != root_rank:
            tensor.copy_(src)
            _lb_settle(tensor)
        return Handle(None, tensor)
    if not _distributed():
        return Handle(None, tensor)
    work = dist.broadcast(tensor, src=root_rank, async_op=True)
    return Handle(work, tensor)


def broadcast_(tensor: torch.Tensor, root_rank: int, name: Optional[str] = None) -> torch.Tensor:
    return synchronize(broadcast_async_(tensor, root_rank, name))


def broadcast(tensor: torch.Tensor, root_rank: int, name: Optional[str] = None) -> torch.Tensor:
    return broadcast_(tensor.clone(), root_rank, name)


def broadcast_object(obj: Any, root: int = 0) -> Any:
    """Replacement for mpi4py ``COMM_WORLD.bcast`` (dist_trainer.py:40)."""
    if _loopback() is not None:
        import copy
        return copy.deepcopy(_lb_exchange(obj if rank() == root else None)[root])
    if not _distributed():
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=root)
    return lst[0]


# storage data_ptr -> callbacks run after a broadcast overwrote that storage
# (the bf16 shadow arena re-casts itself from the fp32 weight arena).  Bound
# methods are held weakly: a registered optimizer (and its arenas) can still be
# garbage-collected.
_storage_listeners: Dict[int, List] = {}


def on_storage_overwritten(ptr: int, fn) -> None:
    import weakref
    ref = weakref.WeakMethod(fn) if hasattr(fn, "__self__") else (lambda f=fn: f)
    lst = [r for r in _storage_listeners.get(int(ptr), []) if r() is not None]
    lst.append(ref)
    _storage_listeners[int(ptr)] = lst


def _notify_storage(ptr: int) -> None:
    live = []
    for ref in _storage_listeners.get(ptr, ()):
        fn = ref()
        if fn is not None:
            fn()
            live.append(ref)
    if ptr in _storage_listeners:
        if live:
            _storage_listeners[ptr] = live
        else:
            del _storage_listeners[ptr]


def broadcast_parameters(params, root_rank: int = 0) -> None:
    """Broadcast a state_dict / named_parameters from root (distributed_optimizer.py:588-617).

    Tensors sharing one storage (our flat arenas) are broadcast once per
    storage, so a whole model normally costs one or two collectives.
    """
    if isinstance(params, dict):
        items = sorted(params.items())
    elif isinstance(params, list):
        items = params
    else:
        raise ValueError("invalid params of type: %s" % type(params))
    if not _distributed() and _loopback() is None:
        return
    seen = set()
    handles: List[Handle] = []
    for name, p in items:
        t = p.data if hasattr(p, "data") else p
        if not torch.is_tensor(t) or t.numel() == 0:
            continue
        st = t.untyped_storage()
        key = (st.data_ptr(), st.nbytes())
        if key in seen:
            continue
        seen.add(key)
        # Tensors that are views of one storage (our flat arenas) are broadcast
        # as ONE flat tensor over the whole storage.
        n = st.nbytes() // t.element_size()
        if t.is_contiguous() and t.storage_offset() == 0 and t.numel() == n:
            flat = t
        else:
            flat = t.new_empty(0).set_(st, 0, (n,), (1,))
        handles.append(broadcast_async_(flat, root_rank, name))
    for h in handles:
        synchronize(h)
    for ptr, _ in seen:
        _notify_storage(ptr)


def broadcast_optimizer_state(optimizer: torch.optim.Optimizer, root_rank: int = 0) -> None:
    """Broadcast optimizer hyper-parameters and state from root (distributed_optimizer.py:620-736)."""
    if not _distributed() and _loopback() is None:
        return
    sd = optimizer.state_dict()
    scalars = {"param_groups": [{k: v for k, v in g.items() if k != "params"} for g in sd["param_groups"]]}
    scalars = broadcast_object(scalars, root_rank)
    for g, src in zip(optimizer.param_groups, scalars["param_groups"]):
        for k, v in src.items():
            g[k] = v
    for group in optimizer.param_groups:
        for p in group["params"]:
            st = optimizer.state.get(p, {})
            flags = broadcast_object(sorted(k for k, v in st.items() if torch.is_tensor(v)), root_rank)
            for k in flags:
                if k not in st:
                    st[k] = torch.zeros_like(p.data)
                    optimizer.state[p] = st
                broadcast_(st[k], root_rank)


# ----------------------------------------------------------------------------
# native RCCL engine
# ----------------------------------------------------------------------------
def _all_ok(ok: bool) -> bool:
    """MIN over the ranks of a per-rank verdict: every rank gets the same answer."""
    if _loopback() is not None:
        return all(bool(x) for x in _lb_exchange(bool(ok)))
    if not _distributed():
        return bool(ok)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t.item()) == 1


def agree_ints(vals: List[int]) -> Tuple[bool, List[int], List[int]]:
    """Do all ranks hold the same integer vector?  Returns ``(all equal, mins,
    maxs)`` -- the per-entry minimum and maximum over the ranks -- identically
    on every rank.  Two small all-reduces (MIN of ``[x, -x]`` gives both
    extremes at once): the vector LENGTH first, so ranks holding vectors of
    different lengths agree on "unequal" without ever entering a collective
    of mismatched size; then the entries."""
    v = [int(x) for x in vals]
    if _loopback() is not None:
        parts = _lb_exchange(list(v))
        if len({len(p) for p in parts}) != 1:
            return False, [], []
        mins = [min(col) for col in zip(*parts)]
        maxs = [max(col) for col in zip(*parts)]
        return mins == maxs, mins, maxs
    if not _distributed():
        return True, v, v
    dev = torch.device("cuda", torch.cuda.current_device()) if backend() == "nccl" else torch.device("cpu")

    def minmax(x: List[int]) -> Tuple[List[int], List[int]]:
        t = torch.tensor(x + [-y for y in x], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        h = t.cpu().tolist()
        return h[:len(x)], [-y for y in h[len(x):]]

    lmin, lmax = minmax([len(v)])
    if lmin != lmax:
        return False, [], []
    if not v:
        return True, [], []
    mins, maxs = minmax(v)
    return mins == maxs, mins, maxs


def _wait_event(ev, timeout_s: float, what: str) -> None:
    """Host wait for a recorded HIP event with a deadline (no blocking
    synchronize: a collective whose peer never arrives must not hang us)."""
    deadline = time.monotonic() + timeout_s
    while not ev.query():
        if time.monotonic() > deadline:
            raise TimeoutError("%s not complete after %.1f s" % (what, timeout_s))
        time.sleep(0.0005)


class RcclCommunicator:
    """Own RCCL communicator (C++ ``gk::RcclComm``), built ONCE per process and
    device by ``native_communicator`` (the bootstrap protocol below) and shared
    by every ``Exchanger`` / ``DistributedOptimizer`` of the process, as
    ``hvd.init()`` is called once per process in the reference
    (dist_trainer.py:125-126).  Collectives run on the CALLER's current stream."""

    def __init__(self, engine, device: torch.device, rank_: int, world: int):
        self.engine = engine
        self.device = torch.device(device)
        self.rank = rank_
        self.world = world
        self.users = 0          # Exchangers that attached to it (diagnostics)

    def self_test(self, timeout_s: float = 120.0) -> None:
        """One all-gather of the rank ids on the current stream, checked on the
        host with a deadline at start-up: a mis-bootstrapped communicator fails
        here (and every rank falls back to torch.distributed) instead of
        corrupting gradients later."""
        inp = torch.full((4,), self.rank, dtype=torch.int32, device=self.device)
        out = torch.full((4 * self.world,), -1, dtype=torch.int32, device=self.device)
        self.engine.allgather(inp, out)
        if self.device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
            _wait_event(ev, timeout_s, "native RCCL all-gather self-test")
        got = out.view(self.world, 4).cpu()
        want = torch.arange(self.world, dtype=torch.int32)[:, None].expand(self.world, 4)
        if not torch.equal(got, want):
            raise RuntimeError("native RCCL all-gather self-test failed: %s" % got[:, 0].tolist())

    def allgather_(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        self.engine.allgather(inp, out)

    def allgather_many_(self, outs: List[torch.Tensor], inps: List[torch.Tensor]) -> None:
        self.engine.allgather_many(inps, outs)

    def check(self) -> None:
        self.engine.check()

    def stats(self) -> Dict[str, Dict[str, float]]:
        """Event-timed per-op statistics of the completed collectives."""
        self.engine.poll()
        out = {}
        for i, name in enumerate(("allgather", "allreduce", "broadcast", "allgather_grouped")):
            calls, nbytes, ms, mx = self.engine.stats(i)
            if calls:
                out[name] = {"calls": int(calls), "bytes_per_call": nbytes / calls, "us_mean": 1e3 * ms / calls,
                             "us_max": 1e3 * mx}
        return out

    def reset_stats(self) -> None:
        self.engine.poll()
        self.engine.reset_stats()

    def allreduce_(self, t: torch.Tensor, average: bool = True) -> None:
        self.engine.allreduce(t, 1 if average else 0)

    def broadcast_(self, t: torch.Tensor, root: int = 0) -> None:
        self.engine.broadcast(t, root)

    def destroy(self) -> None:
        self.engine.stop_watchdog()
        self.engine.destroy()


def _bootstrap_native(device: torch.device, engine_cls=None,
                      timeout_s: Optional[float] = None) -> Optional[RcclCommunicator]:
    """Build the native communicator with every blocking step bounded and
    agreed over the process group before the next one starts:

    1. rank 0 makes the ncclUniqueId; it is broadcast (None if that failed)
       and the ranks agree that the engine class loaded everywhere;
    2. every rank starts a NON-BLOCKING ``ncclCommInitRankConfig`` and polls it
       against ``GKSGD_RCCL_INIT_TIMEOUT_S`` (default 120 s); on the deadline the
       communicator is aborted (ncclCommAbort);  agree;
    3. a start-up all-gather self-test, waited for with the same deadline;
       agree.

    A failure on ANY rank at ANY step aborts the communicator on every rank
    that built one and returns None everywhere, so all ranks take the
    torch.distributed path together; nothing waits without a deadline except
    the agreement collectives themselves, which every rank reaches in bounded
    time.  ``engine_cls`` substitutes the C++ engine (fault-injection tests)."""
    from ..settings import logger
    _BOOTSTRAPS[0] += 1
    r, P = rank(), size()
    tmo = float(timeout_s if timeout_s is not None else os.environ.get("GKSGD_RCCL_INIT_TIMEOUT_S", "120"))
    err: Optional[str] = None
    cls = engine_cls
    if cls is None:
        try:
            from .. import ops
            cls = ops.rccl_engine_class()
        except Exception as e:  # noqa: BLE001 - agreed below
            err = "engine class: %s" % e
    uid = None
    if r == 0 and err is None:
        try:
            uid = [int(x) for x in cls.unique_id().tolist()]
        except Exception as e:  # noqa: BLE001
            err = "unique id: %s" % e
    uid = broadcast_object(uid, 0)
    if not _all_ok(err is None and uid is not None):
        logger.warning("native RCCL engine not used (bootstrap step 1 on rank %d: %s)", r,
                       err or "another rank failed")
        return None

    # step 2: non-blocking init with a deadline
    eng = None
    aborted = False
    try:
        eng = cls()
        idx = device.index if device.index is not None else 0
        eng.init_async(torch.tensor(uid, dtype=torch.uint8), r, P, idx)
        deadline = time.monotonic() + tmo
        while int(eng.init_poll()) != 0:
            if time.monotonic() > deadline:
                eng.abort()
                aborted = True
                raise TimeoutError("RCCL communicator init not complete after %.1f s" % tmo)
            time.sleep(0.001)
    except Exception as e:  # noqa: BLE001 - agreed below
        err = "init: %s" % e
        aborted = True        # init_poll / init_async abort (or never built) the communicator on error
    if not _all_ok(err is None):
        if eng is not None and not aborted:
            eng.abort()
        logger.warning("native RCCL engine not used (bootstrap step 2 on rank %d: %s)", r,
                       err or "another rank failed")
        return None

    # step 3: start-up self-test with a deadline
    c = RcclCommunicator(eng, device, r, P)
    try:
        c.self_test(tmo)
    except Exception as e:  # noqa: BLE001
        err = "self-test: %s" % e
        eng.abort()           # releases RCCL kernels still spinning on a missing peer
        aborted = True
    if not _all_ok(err is None):
        if not aborted:
            eng.abort()
        logger.warning("native RCCL engine not used (bootstrap step 3 on rank %d: %s)", r,
                       err or "another rank failed")
        return None
    # hang / async-error watchdog: aborts the communicator instead of letting a
    # dead peer hang the GPU; the next hot-path call raises
    wd = float(os.environ.get("GKSGD_RCCL_WATCHDOG_S", "600"))
    if wd > 0:
        eng.start_watchdog(wd, 5.0)
    return c


_BOOTSTRAPS = [0]


def native_bootstraps() -> int:
    """How many times this process ran the native bootstrap (one per device
    is the design: bench.py reports it as ``native_inits``)."""
    return _BOOTSTRAPS[0]


def native_communicator(device, engine_cls=None) -> Optional[RcclCommunicator]:
    """The process's native communicator for ``device`` (one per device,
    built on first use by ``_bootstrap_native`` -- a COLLECTIVE call: every
    rank must ask for it at the same point -- and reused afterwards; None when
    the ranks agreed to use torch.distributed).  The verdict is cached too,
    identical on every rank, so later calls are local.  ``shutdown()`` /
    ``release_native()`` destroy it."""
    dev = torch.device(device)
    if dev.type == "cuda" and dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    cache = _S().setdefault("native", {})
    key = (str(dev), engine_cls)
    if key not in cache:
        cache[key] = _bootstrap_native(dev, engine_cls)
    return cache[key]


def release_native() -> None:
    """Destroy the cached native communicators (after their devices are idle)."""
    cache = _S().pop("native", None) or {}
    for c in cache.values():
        if c is None:
            continue
        if c.device.type == "cuda":
            torch.cuda.synchronize(c.device)
        c.destroy()


class Exchanger:
    """Stream-ordered fixed-size collectives used by the hot path.

    backend 'rccl-native' -> the process's shared RcclCommunicator,
    'torch' -> torch.distributed, 'loopback' -> in-process virtual ranks
    (loopback_world), 'local' -> world of one (copies).  All calls are issued
    on the current stream and return without blocking the host.

    ``force_native`` uses the native engine even in a world of one (GPU tests
    of the shared communicator); ``engine_cls`` substitutes the C++ engine.
    """

    def __init__(self, device: torch.device, prefer_native: bool = True, engine_cls=None,
                 force_native: bool = False):
        self.device = torch.device(device)
        self.P = size()
        self.native: Optional[RcclCommunicator] = None
        self._lb_state = getattr(_tls, "state", None)
        lb = _loopback() is not None
        if self.P > 1:
            self.kind = "loopback" if lb else "torch"
        else:
            self.kind = "local"
        want = prefer_native and (self.P > 1 or force_native) and os.environ.get("GKSGD_NATIVE_RCCL", "1") == "1"
        # a loopback world's ranks are threads of one process (one device):
        # only a substituted engine can stand in for RCCL there
        if want and (engine_cls is not None or (self.device.type == "cuda" and not lb)):
            self.native = native_communicator(self.device, engine_cls)
            if self.native is not None:
                self.native.users += 1
                self.kind = "rccl-native"

    @contextlib.contextmanager
    def _bound(self):
        # a loopback rank's collectives may be issued from another thread
        prev = getattr(_tls, "state", None)
        if self.kind == "loopback":
            _tls.state = self._lb_state
        try:
            yield
        finally:
            _tls.state = prev

    def allgather_(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        if self.native is not None:
            self.native.allgather_(out, inp)
        elif self.kind == "local":
            if out.data_ptr() != inp.data_ptr():
                out.view(-1)[: inp.numel()].copy_(inp.view(-1))
        else:
            with self._bound():
                allgather_into_(out, inp, async_op=False)

    def allgather_many_(self, outs: List[torch.Tensor], inps: List[torch.Tensor]) -> None:
        """Several fixed-size all-gathers; one grouped RCCL launch on the native engine."""
        if self.native is not None:
            self.native.allgather_many_(outs, inps)
        else:
            for o, i in zip(outs, inps):
                self.allgather_(o, i)

    def check(self) -> None:
        if self.native is not None:
            self.native.check()

    def stats(self) -> Dict[str, Dict[str, float]]:
        return self.native.stats() if self.native is not None else {}

    def reset_stats(self) -> None:
        """Start a fresh statistics window (the communicator is shared, so a
        phase's collectives are counted from here)."""
        if self.native is not None:
            self.native.reset_stats()

    def allreduce_(self, t: torch.Tensor, average: bool = True) -> None:
        if self.native is not None:
            self.native.allreduce_(t, average)
        elif self.kind == "local":
            return
        else:
            with self._bound():
                allreduce_(t, average)

    def broadcast_(self, t: torch.Tensor, root: int = 0) -> None:
        if self.native is not None:
            self.native.broadcast_(t, root)
        elif self.kind == "local":
            return
        else:
            with self._bound():
                broadcast_(t, root)

    def close(self) -> None:
        """Detach from the shared native communicator (it stays alive for the
        next optimizer of the process; ``comm.shutdown()`` destroys it)."""
        if self.native is not None:
            self.native.users -= 1
            self.native = None
            self.kind = ("loopback" if self._lb_state is not None else "torch") if self.P > 1 else "local"
