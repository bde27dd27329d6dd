set -o pipefail
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for cfg in "" "VSIG_XCORR_M=8192" "VSIG_FIR_M=8192" "VSIG_FIR_M=8192 VSIG_XCORR_M=8192"; do
  echo "== $cfg"
  env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print(d['ms_per_step'], d['value'], d['stages_ms'], d['check']['ok'])" || exit 1
done
