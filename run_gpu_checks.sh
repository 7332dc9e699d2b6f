#!/bin/bash
# One GPU session: parity tests, smoke, bench, kernel-trace profile. Each GPU
# step has its own time limit and the chain stops at the first failure.
#   run_gpu_checks.sh TAG [PYTEST_SELECTION]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r02}
SEL=${2:-}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $SEL > gpurun_out/pytest_gpu_${TAG}.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_${TAG}.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_${TAG}.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke_${TAG}.log; exit 1; }
tail -1 gpurun_out/smoke_${TAG}.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 10 > gpurun_out/bench_${TAG}.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_${TAG}.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python bench.py --steps 20 --warmup 3 --no-cpu --long-updates 0 > gpurun_out/prof_${TAG}.log 2>&1 || { echo "prof failed"; tail -30 gpurun_out/prof_${TAG}.log; exit 1; }
echo done
