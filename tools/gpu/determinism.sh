#!/bin/bash
# the host driver's untiled world, twice per library: are the digests stable?
#   tools/gpu/determinism.sh LIB...   ("main" = in-tree library)
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/detlib
for V in "$@"; do
  if [ "$V" = main ]; then unset LD_LIBRARY_PATH; else
    mkdir -p gpurun_out/detlib/$V && cp avida_amd/libavida_gpu_$V.so gpurun_out/detlib/$V/libavida_gpu.so
    export LD_LIBRARY_PATH=$PWD/gpurun_out/detlib/$V; fi
  for i in 1 2 3; do
    timeout -k 10 120 avida_amd/bin/avgpu_strips --config tests/golden --side 256 --updates 12 --burn-in 0 --seed 7 --strips 2 --untiled > gpurun_out/det_${V}_$i.json 2>&1 || { echo "run $V $i failed"; tail -3 gpurun_out/det_${V}_$i.json; exit 1; }
    echo "$V $i $(tail -1 gpurun_out/det_${V}_$i.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["digest_rank0"], d["organisms"])')"
  done
done
