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
from typing import Any, Callable, Dict, List, Optional

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
class RcclCommunicator:
    """Own RCCL communicator (C++ ``gk::RcclComm``) bootstrapped through the
    torch.distributed store.  Collectives run on the CALLER's current stream."""

    def __init__(self, device: torch.device):
        from .. import ops
        cls = ops.rccl_engine_class()
        self.engine = cls()
        self.device = torch.device(device)
        self.world = size()
        self.rank = rank()
        if self.rank == 0:
            uid = cls.unique_id()
        else:
            uid = None
        uid_list = broadcast_object(uid.tolist() if uid is not None else None, 0)
        uid_t = torch.tensor(uid_list, dtype=torch.uint8)
        self.engine.init(uid_t, self.rank, self.world, self.device.index or 0)
        self.self_test()
        # hang / async-error watchdog: aborts the communicator instead of
        # letting a dead peer hang the GPU; the next hot-path call raises
        wd = float(os.environ.get("GKSGD_RCCL_WATCHDOG_S", "600"))
        if wd > 0:
            self.engine.start_watchdog(wd, 5.0)

    def self_test(self) -> None:
        """One all-gather of the rank ids on the current stream, checked on the
        host once at start-up: a mis-bootstrapped communicator fails here
        (and the Exchanger falls back to torch.distributed on every rank)
        instead of corrupting gradients later."""
        inp = torch.full((4,), self.rank, dtype=torch.int32, device=self.device)
        out = torch.full((4 * self.world,), -1, dtype=torch.int32, device=self.device)
        self.engine.allgather(inp, out)
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

    def allreduce_(self, t: torch.Tensor, average: bool = True) -> None:
        self.engine.allreduce(t, 1 if average else 0)

    def broadcast_(self, t: torch.Tensor, root: int = 0) -> None:
        self.engine.broadcast(t, root)

    def destroy(self) -> None:
        self.engine.stop_watchdog()
        self.engine.destroy()


class Exchanger:
    """Stream-ordered fixed-size collectives used by the hot path.

    backend 'rccl-native' -> RcclCommunicator, 'torch' -> torch.distributed,
    'loopback' -> in-process virtual ranks (loopback_world), 'local' -> world
    of one (copies).  All calls are issued on the current
    stream and return without blocking the host.
    """

    def __init__(self, device: torch.device, prefer_native: bool = True):
        self.device = torch.device(device)
        self.P = size()
        self.native: Optional[RcclCommunicator] = None
        self.kind = "local"
        self._lb_state = getattr(_tls, "state", None)
        if self.P > 1 and _loopback() is not None:
            self.kind = "loopback"          # module collectives take the loopback branch
        elif self.P > 1:
            self.kind = "torch"
            if prefer_native and self.device.type == "cuda" and os.environ.get("GKSGD_NATIVE_RCCL", "1") == "1":
                ok = 1
                try:
                    self.native = RcclCommunicator(self.device)
                except Exception as e:  # pragma: no cover - GPU only
                    from ..settings import logger
                    logger.warning("native RCCL engine unavailable (%s); using torch.distributed", e)
                    ok = 0
                # every rank takes the same path: one failed self-test sends all to torch.distributed
                flag = torch.tensor([ok], dtype=torch.int32,
                                    device=self.device if backend() == "nccl" else "cpu")
                dist.all_reduce(flag, op=dist.ReduceOp.MIN)
                if int(flag) == 1:
                    self.kind = "rccl-native"
                elif self.native is not None:
                    self.native.destroy()
                    self.native = None

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
        if self.kind == "local":
            if out.data_ptr() != inp.data_ptr():
                out.view(-1)[: inp.numel()].copy_(inp.view(-1))
        elif self.native is not None:
            self.native.allgather_(out, inp)
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

    def allreduce_(self, t: torch.Tensor, average: bool = True) -> None:
        if self.kind == "local":
            return
        if self.native is not None:
            self.native.allreduce_(t, average)
        else:
            with self._bound():
                allreduce_(t, average)

    def broadcast_(self, t: torch.Tensor, root: int = 0) -> None:
        if self.kind == "local":
            return
        if self.native is not None:
            self.native.broadcast_(t, root)
        else:
            with self._bound():
                broadcast_(t, root)

    def close(self) -> None:
        """Release the native communicator (after the device is idle)."""
        if self.native is not None:
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            self.native.destroy()
            self.native = None
            self.kind = "torch"
