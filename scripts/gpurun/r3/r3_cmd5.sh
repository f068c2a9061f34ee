#!/bin/bash
set -u
mkdir -p gpurun_out/r3e
timeout -k 10 300 python -u bench/lazy_diag.py > gpurun_out/r3e/diag2.log 2>&1
rc=$?; echo rc=$rc; exit $rc
