#!/bin/bash
# GPU tests (no statistical), bench + kernel-trace tail, an A/B of variants,
# the class-0 PMC passes
#   tools/gpu/r04_check.sh TAG [variant ...]
set -o pipefail
cd "$(dirname "$0")/../.."
TAG=$1; shift
bash tools/gpu/tests_bench_trace.sh "$TAG" "not statistical" || exit 1
if [ $# -gt 0 ]; then bash tools/gpu/ab_var.sh "$TAG" main "$@" || exit 1; fi
bash tools/pmc_passes.sh "$TAG" || { echo "pmc failed"; exit 1; }
grep -E "SQ_LDS_BANK_CONFLICT|SQ_LDS_IDX_ACTIVE|SQ_WAIT_ANY|SQ_WAVE_CYCLES|SQ_INSTS_VALU|FETCH_SIZE|WRITE_SIZE" gpurun_out/${TAG}_pmc_k_interpret320.txt
