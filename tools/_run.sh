set -o pipefail
for a in "--pipeline 1" "--pipeline 2" "--pipeline 4" "--pipeline 8" "--pipeline 4 --xcorr-m 8192 --xcorr-variant 0" "--pipeline 8 --xcorr-m 8192 --xcorr-variant 0"; do
  echo "== $a"
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 $a 2>gpurun_out/bench_err.log | python -c "import json,sys; d=json.load(sys.stdin); print(d['ms_per_step'], d['value'], d['stages_ms'], d['check']['ok'])" || { tail -20 gpurun_out/bench_err.log; exit 1; }
done
