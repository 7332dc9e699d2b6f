#!/bin/bash
# GPU sweep of the interpreter's slow-op batch size (after the parity tests).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-sweep}
shift
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_${TAG}.log; exit 1; }
tail -1 gpurun_out/pytest_${TAG}.log
for B in "$@"; do
  AVGPU_SLOW_BATCH=$B timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu > gpurun_out/bench_${TAG}_$B.log 2>&1 || { echo "bench $B failed"; tail -20 gpurun_out/bench_${TAG}_$B.log; exit 1; }
  python -c "
import json; b=json.loads(open('gpurun_out/bench_${TAG}_$B.log').read().strip().splitlines()[-1])
print('batch $B value %.4g ms/step %.3f lane_eff %.3f c0_ms %.3f' % (b['value'], b['ms_per_step'], b['roofline']['lane_efficiency'], b['roofline']['kernel_ms']))"
done
