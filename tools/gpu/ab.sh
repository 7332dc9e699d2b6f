#!/bin/bash
# A/B bench of variant libraries (avida_amd/libavida_gpu_<V>.so) on one box:
#   tools/gpu/ab.sh TAG V1 V2 ...   ("main" = the in-tree product library)
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=$1; shift
for V in "$@"; do
  if [ "$V" = main ]; then unset AVGPU_DIAG_LIB; else export AVGPU_DIAG_LIB=$PWD/avida_amd/libavida_gpu_$V.so; fi
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --long-updates 100 > gpurun_out/ab_${TAG}_$V.log 2>&1 || { echo "bench $V failed"; tail -5 gpurun_out/ab_${TAG}_$V.log; exit 1; }
  python - "$V" gpurun_out/ab_${TAG}_$V.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"]
print("%-6s value %.4g  long %.4g  ms/step %.3f  c0 %.3f ms  classes %s" % (sys.argv[1], d["value"],
      d["config"]["long_run"]["value"], d["ms_per_step"], r["kernel_ms"], [round(x, 3) for x in r["class_ms"]]))
PY
done
