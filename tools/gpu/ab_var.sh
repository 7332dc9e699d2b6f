#!/bin/bash
# A/B bench of variants on one box.  Each variant is LIB[,ENV=VAL...][:bench args]
# (LIB "main" = the in-tree product library, else avida_amd/libavida_gpu_<LIB>.so):
#   tools/gpu/ab_var.sh TAG main main:--time-every=4 lab,AVGPU_SLOW_BATCH=16
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=$1; shift
i=0
for V in "$@"; do
  i=$((i + 1))
  spec=${V%%:*}; args=""; [ "$spec" != "$V" ] && args=${V#*:}
  lib=${spec%%,*}; envs=""; [ "$lib" != "$spec" ] && envs=${spec#*,}
  (
    if [ "$lib" = main ]; then unset AVGPU_DIAG_LIB; else export AVGPU_DIAG_LIB=$PWD/avida_amd/libavida_gpu_$lib.so; fi
    for e in ${envs//,/ }; do export "$e"; done
    timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --long-updates 100 ${args//=/ } > gpurun_out/ab_${TAG}_$i.log 2>&1
  ) || { echo "bench $V failed"; tail -5 gpurun_out/ab_${TAG}_$i.log; exit 1; }
  python - "$V" gpurun_out/ab_${TAG}_$i.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"]
print("%-40s value %.4g  long %.4g  ms/step %.3f  c0 %.3f ms" % (sys.argv[1], d["value"],
      d["config"]["long_run"]["value"], d["ms_per_step"], r["kernel_ms"]))
PY
done
