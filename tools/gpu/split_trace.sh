#!/bin/bash
# kernel-trace tail of a diagnostic variant library (tools/build_variant.py)
#   tools/gpu/split_trace.sh TAG VARIANT
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; VAR=$2
export AVGPU_DIAG_LIB=$PWD/avida_amd/libavida_gpu_$VAR.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_${TAG} -o run -- python bench.py --steps 40 --warmup 2 --no-cpu --long-updates 0 > gpurun_out/kt_${TAG}.log 2>&1 || { echo "kernel trace failed"; tail -20 gpurun_out/kt_${TAG}.log; exit 1; }
python tools/tail_summary.py $(ls gpurun_out/kt_${TAG}/*/*kernel_trace.csv gpurun_out/kt_${TAG}/*kernel_trace.csv 2>/dev/null | head -1) > gpurun_out/${TAG}_tail_per_update.txt
cat gpurun_out/${TAG}_tail_per_update.txt
