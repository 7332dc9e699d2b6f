#!/bin/bash
# split-memory round: parity/determinism/resource tests, bench + trace, A/B
# against the unsplit build, the resources bench (configs[4]) with its trace
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=$1; shift
bash tools/gpu/tests_bench_trace.sh "$TAG" "parity or determinism or resources" || exit 1
if [ $# -gt 0 ]; then bash tools/gpu/ab_var.sh "$TAG" main "$@" || exit 1; fi
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ktres_${TAG} -o run -- python bench.py --env resources --steps 20 --warmup 3 --no-cpu --long-updates 0 > gpurun_out/benchres_${TAG}.log 2>&1 || { echo "resources bench failed"; tail -20 gpurun_out/benchres_${TAG}.log; exit 1; }
grep "^{\"metric\"" gpurun_out/benchres_${TAG}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("resources value %.4g ms/step %.3f" % (d["value"], d["ms_per_step"]))'
python tools/res_roofline.py gpurun_out/ktres_${TAG}/run_kernel_stats.csv 1024 9 > gpurun_out/${TAG}_res_step_roofline.json && cat gpurun_out/${TAG}_res_step_roofline.json
