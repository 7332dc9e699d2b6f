#!/bin/bash
# bench the in-tree library under several values of one environment knob:
#   tools/sweep_env.sh TAG VAR v1 v2 ...
set -o pipefail
mkdir -p gpurun_out
TAG=$1; VAR=$2; shift 2
for V in "$@"; do
  env "$VAR=$V" timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --long-updates 100 > gpurun_out/sw_${TAG}_$V.log 2>&1 || { echo "bench $V failed"; tail -5 gpurun_out/sw_${TAG}_$V.log; exit 1; }
  python - "$VAR=$V" gpurun_out/sw_${TAG}_$V.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"]
print("%-14s value %.4g  long %.4g  ms/step %.3f  c0 %.3f ms  classes %s" % (sys.argv[1], d["value"],
      d["config"]["long_run"]["value"], d["ms_per_step"], r["kernel_ms"], [round(x, 3) for x in r["class_ms"]]))
PY
done
