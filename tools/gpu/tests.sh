#!/bin/bash
# GPU tests (optionally a -k selection), smoke
#   tools/gpu/tests.sh TAG ["k-expression"]
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05}
SEL=${2:-}
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread ${SEL:+-k "$SEL"} > gpurun_out/pytest_${TAG}.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_${TAG}.log; exit 1; }
tail -3 gpurun_out/pytest_${TAG}.log
grep -E "PASSED|FAILED" gpurun_out/pytest_${TAG}.log | tail -80 | awk '{print $1, $2}' > gpurun_out/pytest_${TAG}.summary
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_${TAG}.log; exit 1; }
tail -1 gpurun_out/smoke_${TAG}.log
