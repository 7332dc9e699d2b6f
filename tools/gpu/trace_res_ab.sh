#!/bin/bash
# k_res_step time per variant library (rocprofv3 kernel trace of the configs[4] bench)
#   tools/gpu/trace_res_ab.sh TAG LIB...   (LIB "main" = the in-tree library)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=$1; shift
for L in "$@"; do
  if [ "$L" = main ]; then unset AVGPU_DIAG_LIB; else export AVGPU_DIAG_LIB=$PWD/avida_amd/libavida_gpu_$L.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tres_${TAG}_$L -o run -- \
    python bench.py --env resources --steps 20 --warmup 5 --no-cpu --long-updates 0 > gpurun_out/tres_${TAG}_$L.log 2>&1 || { echo "trace $L failed"; exit 1; }
  python - gpurun_out/tres_${TAG}_$L/run_kernel_stats.csv "$L" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_res_step" in r["Name"] or "k_interpret<320" in r["Name"]:
        print("%-6s %-40s %8.1f us" % (sys.argv[2], r["Name"][:40], float(r["AverageNs"]) / 1e3))
PY
done
