#!/bin/bash
# Profiling session: kernel-trace stats of the bench, PMC passes of the
# class-0 interpreter, phase clocks of the diagnostic build.
#   run_prof.sh TAG
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r02}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python bench.py --steps 20 --warmup 3 --no-cpu --long-updates 0 > gpurun_out/prof_${TAG}.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_${TAG}.log; exit 1; }
bash tools/pmc_passes.sh $TAG || exit 1
timeout -k 10 300 python tools/phase_clocks.py 1024 10 150 > gpurun_out/clocks_${TAG}.json 2>&1 || { echo "clocks failed"; tail -20 gpurun_out/clocks_${TAG}.json; exit 1; }
echo done
