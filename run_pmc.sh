#!/bin/bash
# PMC passes on the bench (each pass its own rocprofv3 run, --pmc with kernel trace only).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
ARGS="python bench.py --steps 5 --warmup 2 --no-cpu"
i=0
for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_BUSY_CYCLES" \
            "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/pmc_${TAG}_$i -o p -- $ARGS > gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "pass $i failed"; tail -20 gpurun_out/pmc_${TAG}_$i.log; exit 1; }
done
echo pmc done
