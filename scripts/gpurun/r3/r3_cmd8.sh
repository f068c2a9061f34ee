#!/bin/bash
set -u
D=gpurun_out/r3h
mkdir -p $D
timeout -k 10 300 python -u bench/stream_probe.py --steps 4 --warmup 4 > $D/probe_on.log 2>&1
echo on_rc=$?; grep step $D/probe_on.log
GKSGD_WGRAD_STREAM=0 timeout -k 10 300 python -u bench/stream_probe.py --steps 4 --warmup 4 > $D/probe_off.log 2>&1
echo off_rc=$?; grep step $D/probe_off.log
