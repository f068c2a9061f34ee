"""Reference-compatible module path: ``import gaussiank_sgd_amd.distributed_optimizer as hvd``
gives ``hvd.init/size/rank/local_rank/broadcast/broadcast_parameters/
broadcast_optimizer_state/DistributedOptimizer`` like the reference's
``distributed_optimizer`` module (distributed_optimizer.py:21-26,550-736)."""
from .parallel.distributed_optimizer import *  # noqa: F401,F403
from .parallel.distributed_optimizer import DistributedOptimizer, _DistributedOptimizer  # noqa: F401
