#!/bin/bash
# k_res_step band heights A/B (AVGPU_RES_ROWS) on configs[4]: a kernel trace
# of bench.py --env resources per height, then one PMC pass over the default.
# usage (GPU box): bash tools/gpu/res_step_ab.sh TAG "8 16 24 32"
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=${1:-res}
mkdir -p gpurun_out/$TAG
for R in ${2:-16}; do
  AVGPU_RES_ROWS=$R timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$TAG/kt_$R -o run -- \
    python bench.py --env resources --no-cpu --long-updates 0 > gpurun_out/$TAG/bench_$R.json 2> gpurun_out/$TAG/bench_$R.err || exit 1
done
if [ -n "$3" ]; then
  timeout -s KILL 120 rocprofv3 --pmc $3 --output-format csv -d gpurun_out/$TAG/pmc -o run -- \
    python bench.py --env resources --steps 5 --warmup 2 --no-cpu --long-updates 0 > gpurun_out/$TAG/pmc.log 2>&1 || exit 1
fi
