#!/bin/bash
# round-end check: the whole GPU suite (statistical included), smoke, the
# default bench line (with its CPU leg), class-0 PMC passes
#   tools/gpu/r04_final.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r04}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_${TAG}.log; exit 1; }
tail -3 gpurun_out/pytest_${TAG}.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_${TAG}.log; exit 1; }
tail -2 gpurun_out/smoke_${TAG}.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default_${TAG}.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_default_${TAG}.log; exit 1; }
grep '^{"metric"' gpurun_out/bench_default_${TAG}.log > gpurun_out/${TAG}_bench_default.json
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_default.json')); print('value %.4g ms/step %.3f roofline %s cpu %s' % (d['value'], d['ms_per_step'], d['roofline'].get('frac'), d['cpu_baseline'].get('value')))"
bash tools/pmc_passes.sh ${TAG} || { echo "pmc failed"; exit 1; }
cat gpurun_out/${TAG}_pmc_k_interpret320.txt
