#!/bin/bash
# PMC passes over the bench's tail kernels (diagnostic): one pass per counter
# group, then per-kernel averages over the last dispatches.
# usage (GPU box): bash tools/gpu/pmc_tail.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=${1:-tail}
mkdir -p gpurun_out/$TAG
P=1
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/$TAG/p$P -o run -- \
    python bench.py --steps 5 --warmup 2 --no-cpu --long-updates 0 > gpurun_out/$TAG/p$P.log 2>&1 || { echo "pass $P failed"; exit 1; }
  P=$((P + 1))
done
