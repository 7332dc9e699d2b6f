set -o pipefail
cd /root/repo
export TMPDIR=/tmp
P=1
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU" \
         "FETCH_SIZE" "WRITE_SIZE GRBM_COUNT GRBM_GUI_ACTIVE" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD"; do
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmcres_$P -o run -- \
    python bench.py --env resources --steps 5 --warmup 2 --no-cpu --long-updates 0 > gpurun_out/pmcres_$P.log 2>&1 || { echo "pass $P failed"; tail -5 gpurun_out/pmcres_$P.log; exit 1; }
  P=$((P + 1))
done
python tools/pmc_summary.py "gpurun_out/pmcres_*/**/*counter_collection.csv" "k_res_step" > gpurun_out/pmc_res_step.txt
cat gpurun_out/pmc_res_step.txt
