"""Global flags and the shared logger.

Parity: reference ``settings.py:5-43`` keeps module constants that users edit
by hand.  Here every constant keeps its name and default but can also be set
from the environment (``GKSGD_<NAME>``), so launch scripts do not need to
patch source files.  The logger uses the reference's line format
(``settings.py:41``) because ``tools/plot.py`` parses those lines.
"""
from __future__ import annotations

import logging
import os
import socket


def _env_bool(name: str, default: bool) -> bool:
    v = os.environ.get("GKSGD_" + name)
    if v is None:
        return default
    return v.strip().lower() in ("1", "true", "yes", "on")


def _env_int(name: str, default: int) -> int:
    v = os.environ.get("GKSGD_" + name)
    return default if v is None else int(v)


DEBUG = _env_int("DEBUG", 0)
SERVER_PORT = _env_int("SERVER_PORT", 5911)
PORT = _env_int("PORT", 5922)

WARMUP = _env_bool("WARMUP", True)

PREFIX = ""
if WARMUP:
    PREFIX = PREFIX + "gwarmup"

LOGGING_ASSUMPTION = _env_bool("LOGGING_ASSUMPTION", False)
# The reference dumps the full merged gradient EVERY iteration when this is on
# (distributed_optimizer.py:409-411).  We keep the flag but sample the dumps:
# see DUMP_GRAD_EVERY.
LOGGING_GRADIENTS = _env_bool("LOGGING_GRADIENTS", False)
DUMP_GRAD_EVERY = _env_int("DUMP_GRAD_EVERY", 100)

EXP = "-convergence"
PREFIX = PREFIX + EXP
ADAPTIVE_MERGE = _env_bool("ADAPTIVE_MERGE", False)
ADAPTIVE_SPARSE = _env_bool("ADAPTIVE_SPARSE", False)
if ADAPTIVE_MERGE:
    PREFIX = PREFIX + "-ada"

TENSORBOARD = _env_bool("TENSORBOARD", False)
# reference: apex amp O2 (dead code).  Here: bf16 autocast on MI355X.
USE_FP16 = _env_bool("USE_FP16", False)
USE_BF16 = _env_bool("USE_BF16", False)

MAX_EPOCHS = _env_int("MAX_EPOCHS", 10)

# Bitwise-reproducible aggregation (sorted/per-rank scatter instead of atomics).
DETERMINISTIC = _env_bool("DETERMINISTIC", False)

hostname = socket.gethostname()
logger = logging.getLogger("gksgd")

if DEBUG:
    logger.setLevel(logging.DEBUG)
else:
    logger.setLevel(logging.INFO)

formatter = logging.Formatter("%(asctime)s [%(filename)s:%(lineno)d] %(levelname)s %(message)s")
if not logger.handlers:
    strhdlr = logging.StreamHandler()
    strhdlr.setFormatter(formatter)
    logger.addHandler(strhdlr)
logger.propagate = False
