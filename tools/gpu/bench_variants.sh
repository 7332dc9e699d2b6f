#!/bin/bash
# bench lines of the default world and its variants (no CPU leg)
#   tools/gpu/bench_variants.sh TAG "ARGS1" "ARGS2" ...
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
K=0
for A in "$@"; do
  timeout -k 10 400 python bench.py --no-cpu $A > gpurun_out/bench_${TAG}_$K.log 2>&1 || { echo "bench $A failed"; tail -20 gpurun_out/bench_${TAG}_$K.log; exit 1; }
  grep '^{"metric"' gpurun_out/bench_${TAG}_$K.log > gpurun_out/${TAG}_bench_$K.json
  python -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_bench_$K.json')); r=d['roofline']; print(sys.argv[1], 'value %.4g ms/step %.3f c0 %.3f long %.4g' % (d['value'], d['ms_per_step'], r['kernel_ms'], (d['config']['long_run'] or {}).get('value', 0)))" "$A"
  K=$((K + 1))
done
