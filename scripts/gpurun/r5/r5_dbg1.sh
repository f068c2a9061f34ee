#!/bin/bash
set -u
mkdir -p gpurun_out/r5d1
timeout -k 10 300 python3 -u scripts/debug/wprep_probe.py 4 > gpurun_out/r5d1/probe4.log 2>&1; echo rc=$?; grep -v INFO gpurun_out/r5d1/probe4.log | tail -8
timeout -k 10 300 python3 -u scripts/debug/wprep_probe.py 32 > gpurun_out/r5d1/probe32.log 2>&1; echo rc=$?; grep -v INFO gpurun_out/r5d1/probe32.log | tail -8
