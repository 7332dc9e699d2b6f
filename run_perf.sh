#!/bin/bash
# Quick GPU iteration: parity tests, per-block loop clocks, bench (no CPU leg).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-perf}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_${TAG}.log; exit 1; }
tail -1 gpurun_out/pytest_${TAG}.log
timeout -k 10 300 python tools/phase_clocks.py 1024 10 150 > gpurun_out/clocks_${TAG}.json 2>&1 || { echo "clocks failed"; tail -20 gpurun_out/clocks_${TAG}.json; exit 1; }
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu > gpurun_out/bench_${TAG}.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_${TAG}.log; exit 1; }
python - <<PY
import json
b = json.loads(open("gpurun_out/bench_${TAG}.log").read().strip().splitlines()[-1])
c = json.loads(open("gpurun_out/clocks_${TAG}.json").read()[open("gpurun_out/clocks_${TAG}.json").read().index("{"):])
print("value %.4g ms/step %.3f lane_eff %.3f c0_ms %.3f" % (b["value"], b["ms_per_step"], b["roofline"]["lane_efficiency"], b["roofline"]["kernel_ms"]))
print("cyc/iter %.0f" % c["loop_cycles_per_iter"], {k: round(v) for k, v in c["loop_cycles_per_iter_by_block"].items()})
PY
