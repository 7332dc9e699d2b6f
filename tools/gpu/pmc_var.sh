#!/bin/bash
# class-0 PMC passes (waves / cycles / waits, instruction mix, memory) for
# each named library: "main" = the product, else avida_amd/libavida_gpu_<V>.so
#   tools/gpu/pmc_var.sh TAG main nosplit ...
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out
for V in "$@"; do
  if [ "$V" = main ]; then unset AVGPU_DIAG_LIB; else export AVGPU_DIAG_LIB=$PWD/avida_amd/libavida_gpu_$V.so; fi
  P=1
  for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE GRBM_COUNT GRBM_GUI_ACTIVE"; do
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmcv_${TAG}_${V}_$P -o run -- \
      python bench.py --steps 5 --warmup 2 --no-cpu --long-updates 0 > gpurun_out/pmcv_${TAG}_${V}_$P.log 2>&1 || { echo "pass $P of $V failed"; exit 1; }
    P=$((P + 1))
  done
  echo "== $V"
  python tools/pmc_summary.py "gpurun_out/pmcv_${TAG}_${V}_*/**/*counter_collection.csv" | tee gpurun_out/${TAG}_pmc_${V}.txt
done
