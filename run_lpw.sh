#!/bin/bash
# per-class timing events on / off (AVGPU_CLASS_TIMING), bench only
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1 0 1 0; do
  AVGPU_CLASS_TIMING=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu > gpurun_out/bench_ct$v.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/bench_ct$v.log; exit 1; }
  echo "timing_all=$v $(tail -1 gpurun_out/bench_ct$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["class_ms"])')"
done
