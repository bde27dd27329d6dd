set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_analysis.py -x -q -k pfb --timeout 120 --timeout-method thread > gpurun_out/r02_v34_tests.txt 2>&1 || { tail -30 gpurun_out/r02_v34_tests.txt; exit 1; }
tail -1 gpurun_out/r02_v34_tests.txt
VSIG_LIB=$GRAFT_REPO_ROOT/vector_amd/libvsig_pfbv3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_analysis.py -x -q -k pfb --timeout 120 --timeout-method thread > gpurun_out/r02_v34_tests3.txt 2>&1 || { tail -30 gpurun_out/r02_v34_tests3.txt; exit 1; }
tail -1 gpurun_out/r02_v34_tests3.txt
for rep in 1 2; do
for lib in base libvsig_pfbv3; do
  if [ "$lib" = base ]; then unset VSIG_LIB; else export VSIG_LIB=$GRAFT_REPO_ROOT/vector_amd/$lib.so; fi
  timeout -k 10 240 python3 bench.py --workload pfb --no-cpu-baseline > gpurun_out/r02_v34_${rep}_$lib.json 2> gpurun_out/r02_v34_${rep}_$lib.err
  python3 -c "import json; d=json.load(open('gpurun_out/r02_v34_${rep}_$lib.json')); print('$lib', d['ms_per_step'], d['value'])"
done
done
echo done
