set -o pipefail
mkdir -p gpurun_out/bn
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_bn_gpu.py tests/test_bnlink_gpu.py tests/test_stem_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/bn/tests.log 2>&1 || { tail -n 30 gpurun_out/bn/tests.log; exit 1; }
tail -n 2 gpurun_out/bn/tests.log
timeout -k 10 200 python bench/bn_probe.py --blocks 1024,2048,4096 --json-out gpurun_out/bn/u4.json > gpurun_out/bn/u4.log 2>&1 || exit 1
GKSGD_EXT=variants/bnu1/_C.so timeout -k 10 200 python bench/bn_probe.py --blocks 1024,4096 --json-out gpurun_out/bn/u1.json > gpurun_out/bn/u1.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/bn/bench.json > gpurun_out/bn/bench.log 2>&1 || { tail -n 20 gpurun_out/bn/bench.log; exit 1; }
tail -n 1 gpurun_out/bn/bench.log
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bn/prof -o run -- python3 bench.py --steps 8 --warmup 6 > gpurun_out/bn/prof.log 2>&1 || exit 1
echo done
