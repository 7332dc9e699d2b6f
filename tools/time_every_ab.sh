set -o pipefail
for TE in 1 4 1 4; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu --long-updates 100 --time-every $TE > gpurun_out/te_$TE.log 2>&1 || exit 1
  python - $TE gpurun_out/te_$TE.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); r = d["roofline"]
print("time_every %s value %.4g long %.4g ms/step %.3f c0 %.3f timed %d" % (sys.argv[1], d["value"], d["config"]["long_run"]["value"], d["ms_per_step"], r["kernel_ms"], r["timed_launches"]))
PY
done
