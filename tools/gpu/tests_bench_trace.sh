#!/bin/bash
# selected GPU tests, bench, kernel-trace stats + per-update tail breakdown
#   tools/gpu/tests_bench_trace.sh TAG [pytest -k expression]
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03}
SEL=${2:-}
if [ -n "$SEL" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread -k "$SEL" > gpurun_out/pytest_${TAG}.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_${TAG}.log; exit 1; }
  tail -3 gpurun_out/pytest_${TAG}.log
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_${TAG}.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_${TAG}.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; r=d["roofline"]; print("value %.4g ms/step %.3f c0 %.3f never %.1f over %.1f spills %.1f" % (d["value"], d["ms_per_step"], r["kernel_ms"], c["births_never_placed_per_update"], c["births_overwritten_per_update"], c["spills_per_update"]))'
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_${TAG} -o run -- python bench.py --steps 40 --warmup 2 --no-cpu --long-updates 0 > gpurun_out/kt_${TAG}.log 2>&1 || { echo "kernel trace failed"; tail -20 gpurun_out/kt_${TAG}.log; exit 1; }
python tools/tail_summary.py $(ls gpurun_out/kt_${TAG}/*/*kernel_trace.csv gpurun_out/kt_${TAG}/*kernel_trace.csv 2>/dev/null | head -1) > gpurun_out/${TAG}_tail_per_update.txt
cat gpurun_out/${TAG}_tail_per_update.txt
cp $(ls gpurun_out/kt_${TAG}/*/*kernel_stats.csv gpurun_out/kt_${TAG}/*kernel_stats.csv 2>/dev/null | head -1) gpurun_out/${TAG}_kernel_stats_bench.csv || true
