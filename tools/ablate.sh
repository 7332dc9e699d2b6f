#!/bin/bash
# Diagnostic ablations of the interpreter (timing only: these builds break the
# semantics they remove).  Builds avida_amd/libavida_gpu_abl_<X>.so here; run
# the bench against each on the GPU box with tools/ablate.sh run.
set -e
cd "$(dirname "$0")/.."
if [ "$1" != run ]; then
  for X in IO LABEL SEARCHRQ; do
    /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -ffp-contract=off -Wno-unused-result -Wno-unused-value \
      -DAVGPU_ABL_$X -o avida_amd/libavida_gpu_abl_$X.so avida_amd/csrc/interp.hip avida_amd/csrc/world.hip avida_amd/csrc/resources.hip avida_amd/csrc/capi.hip &
  done
  wait
  exit 0
fi
mkdir -p gpurun_out
for X in BASE IO LABEL SEARCHRQ; do
  L=avida_amd/libavida_gpu_abl_$X.so; [ $X = BASE ] && L=avida_amd/libavida_gpu.so
  AVGPU_DIAG_LIB=$PWD/$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/abl_$X.log 2>&1
  python -c "
import json; b=json.loads(open('gpurun_out/abl_$X.log').read().strip().splitlines()[-1])
print('$X value %.4g ms/step %.3f c0_ms %.3f insts/upd %.3g' % (b['value'], b['ms_per_step'], b['roofline']['kernel_ms'], b['config']['insts_per_update']))"
done
