#!/bin/bash
# class-0 PMC passes on the configs[4] world (bench.py --env resources): the
# simple-reaction kernel with finite resources (k_interpret<320, ..., RES>)
#   tools/gpu/pmc_res.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=${1:-r04}
mkdir -p gpurun_out
P=1
for C in "FETCH_SIZE" "WRITE_SIZE GRBM_COUNT GRBM_GUI_ACTIVE" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmcres_${TAG}_$P -o run -- \
    python bench.py --env resources --steps 5 --warmup 2 --no-cpu --long-updates 0 > gpurun_out/pmcres_${TAG}_$P.log 2>&1 || { echo "pass $P failed"; exit 1; }
  P=$((P + 1))
done
python tools/pmc_summary.py "gpurun_out/pmcres_${TAG}_*/**/*counter_collection.csv" "k_interpret<320, false, true, true, true, true>|k_interpretILi320ELb0ELb1ELb1ELb1ELb1E" > gpurun_out/${TAG}_pmc_k_interpret320_res.txt
cat gpurun_out/${TAG}_pmc_k_interpret320_res.txt
