#!/bin/bash
# GPU parity tests, then the bench (spill-row lanes per wave 1 and 64), then a kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_lpw.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_lpw.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_lpw.log
for v in 1 64; do
  AVGPU_SPILL_LPW=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu > gpurun_out/bench_lpw$v.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/bench_lpw$v.log; exit 1; }
  echo "lpw=$v $(tail -1 gpurun_out/bench_lpw$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["class_ms"])')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lpw -o run -- python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/prof_lpw.log 2>&1 || { echo "prof failed"; exit 1; }
echo done
