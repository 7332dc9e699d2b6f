#!/bin/bash
# measurement call: bench, configs[4] bench + k_res_step roofline,
# PMC passes of the class-0 kernel, strip-tile timing (multi-GPU cost model)
#   tools/gpu/measure.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03}
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_${TAG}.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_${TAG}.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("logic9 value %.4g ms/step %.3f c0 %.3f" % (d["value"], d["ms_per_step"], r["kernel_ms"]))'
timeout -k 10 300 python bench.py --env resources --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_res_${TAG}.log 2>&1 || { echo "bench res failed"; tail -20 gpurun_out/bench_res_${TAG}.log; exit 1; }
tail -1 gpurun_out/bench_res_${TAG}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("resources value %.4g ms/step %.3f c0 %.3f" % (d["value"], d["ms_per_step"], r["kernel_ms"]))'
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ktres_${TAG} -o run -- python bench.py --env resources --steps 10 --warmup 2 --no-cpu --long-updates 0 > gpurun_out/ktres_${TAG}.log 2>&1 || { echo "res trace failed"; tail -20 gpurun_out/ktres_${TAG}.log; exit 1; }
python tools/res_roofline.py $(ls gpurun_out/ktres_${TAG}/*/*kernel_stats.csv gpurun_out/ktres_${TAG}/*kernel_stats.csv 2>/dev/null | head -1) 1024 > gpurun_out/${TAG}_res_step_roofline.json
cat gpurun_out/${TAG}_res_step_roofline.json
bash tools/pmc_passes.sh ${TAG} || { echo "pmc failed"; exit 1; }
head -30 gpurun_out/${TAG}_pmc_k_interpret320.txt
timeout -k 10 400 python tools/strip_timing.py 1024 2048 2 150 20 > gpurun_out/strips2_${TAG}.json 2> gpurun_out/strips2_${TAG}.err || { echo "strip timing 2 failed"; tail -5 gpurun_out/strips2_${TAG}.err; exit 1; }
cat gpurun_out/strips2_${TAG}.json
timeout -k 10 600 python tools/strip_timing.py 4096 4096 8 150 10 > gpurun_out/strips8_${TAG}.json 2> gpurun_out/strips8_${TAG}.err || { echo "strip timing 8 failed"; tail -5 gpurun_out/strips8_${TAG}.err; exit 1; }
cat gpurun_out/strips8_${TAG}.json
