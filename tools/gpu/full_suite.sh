#!/bin/bash
# full GPU suite, phase clocks, bench (no CPU leg)
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03}
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_${TAG}.log; exit 1; }
tail -3 gpurun_out/pytest_${TAG}.log
timeout -k 10 300 python tools/phase_clocks.py 1024 10 150 > gpurun_out/clocks_${TAG}.json 2>&1 || { echo "clocks failed"; tail -20 gpurun_out/clocks_${TAG}.json; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_${TAG}.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_${TAG}.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; r=d["roofline"]; print("value %.4g ms/step %.3f c0 %.3f never %.1f over %.1f spills %.1f" % (d["value"], d["ms_per_step"], r["kernel_ms"], c["births_never_placed_per_update"], c["births_overwritten_per_update"], c["spills_per_update"]))'
