#!/bin/bash
# round-5 measurement pass on one box: class-0 PMC passes (their JSON, stamped
# with the library's build hash, copied into this box's profiles/ so that the
# bench line pairs it with its own timing), the default bench line (with its
# CPU leg), a rocprofv3 kernel trace of the bench with the per-update tail
#   tools/gpu/r05_final.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r05}
bash tools/pmc_passes.sh ${TAG} || { echo "pmc failed"; exit 1; }
cp gpurun_out/pmc_k_interpret320.json profiles/pmc_k_interpret320.json
timeout -k 10 400 python bench.py > gpurun_out/bench_default_${TAG}.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_default_${TAG}.log; exit 1; }
grep '^{"metric"' gpurun_out/bench_default_${TAG}.log > gpurun_out/${TAG}_bench_default.json
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_default.json')); r=d['roofline']; print('value %.4g ms/step %.3f issue %s hbm %s traffic %s cpu %s' % (d['value'], d['ms_per_step'], r.get('frac'), r['hbm'].get('frac'), r['hbm'].get('traffic_over_algorithmic'), d['cpu_baseline'].get('value')))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_${TAG} -o run -- \
  python bench.py --steps 20 --warmup 5 --no-cpu --long-updates 0 > gpurun_out/trace_${TAG}.log 2>&1 || { echo "trace failed"; tail -20 gpurun_out/trace_${TAG}.log; exit 1; }
python tools/tail_summary.py gpurun_out/trace_${TAG}/run_kernel_trace.csv > gpurun_out/${TAG}_tail_per_update.txt
cp gpurun_out/trace_${TAG}/run_kernel_stats.csv gpurun_out/${TAG}_kernel_stats_bench.csv
tail -3 gpurun_out/${TAG}_tail_per_update.txt
