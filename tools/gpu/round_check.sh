#!/bin/bash
# GPU suite without the statistical tests, bench + kernel-trace tail, strip
# timing (2 and 8 strips on one GPU)
#   tools/gpu/round_check.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=${1:-r03}
bash tools/gpu/tests_bench_trace.sh "$TAG" "not statistical" || exit 1
timeout -k 10 400 python tools/strip_timing.py 1024 2048 2 150 20 > gpurun_out/strips2_${TAG}.json 2> gpurun_out/strips2_${TAG}.err || { echo "strip timing 2 failed"; tail -5 gpurun_out/strips2_${TAG}.err; exit 1; }
cat gpurun_out/strips2_${TAG}.json
timeout -k 10 600 python tools/strip_timing.py 4096 4096 8 150 10 > gpurun_out/strips8_${TAG}.json 2> gpurun_out/strips8_${TAG}.err || { echo "strip timing 8 failed"; tail -5 gpurun_out/strips8_${TAG}.err; exit 1; }
cat gpurun_out/strips8_${TAG}.json
