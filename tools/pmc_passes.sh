#!/bin/bash
# rocprofv3 PMC passes over a short bench run (one pass per counter group,
# within the per-pass limits of MI355X_MICROARCH.md: <= 8 SQ, <= 4 TCC with
# FETCH_SIZE = 3 and WRITE_SIZE = 2, <= 2 GRBM), each pass under its own
# time limit; then the per-dispatch averages of the class-0 interpreter.
# usage (on the GPU box): bash tools/pmc_passes.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-r01}
mkdir -p gpurun_out
P=1
for C in "FETCH_SIZE" "WRITE_SIZE GRBM_COUNT GRBM_GUI_ACTIVE" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_${TAG}_$P -o run -- \
    python bench.py --steps 5 --warmup 2 --no-cpu --long-updates 0 > gpurun_out/pmc_${TAG}_$P.log 2>&1 || { echo "pass $P failed"; exit 1; }
  P=$((P + 1))
done
python tools/pmc_summary.py "gpurun_out/pmc_${TAG}_*/**/*counter_collection.csv" --last 7 \
  --json gpurun_out/pmc_k_interpret320.json --world 1024x1024 \
  --source "profiles/${TAG}_pmc_k_interpret320.txt (rocprofv3 --pmc, 5 passes over bench.py --steps 5 --warmup 2 --no-cpu after 150 burn-in updates; average over each pass's last 7 class-0 main-pass dispatches: the warmup and timed updates)" \
  > gpurun_out/${TAG}_pmc_k_interpret320.txt
python tools/pmc_summary.py "gpurun_out/pmc_${TAG}_*/**/*counter_collection.csv" 'k_interpret<(316|320),[^(]*true>\(' --last 7 \
  > gpurun_out/${TAG}_pmc_k_interpret320_newborn.txt
