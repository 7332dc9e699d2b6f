#!/bin/bash
# One GPU session: parity tests, bench, kernel-trace profile. Each GPU step has
# its own time limit and the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py --steps 30 --warmup 5 --cpu-seconds 5 > gpurun_out/bench_${TAG}.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_${TAG}.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run -- python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/prof_${TAG}.log 2>&1 || { echo "prof failed"; tail -30 gpurun_out/prof_${TAG}.log; exit 1; }
echo done
