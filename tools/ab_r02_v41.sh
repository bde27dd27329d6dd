set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_refine.py tests/test_gpu_alignment.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_v41_tests.txt 2>&1 || { tail -30 gpurun_out/r02_v41_tests.txt; exit 1; }
tail -1 gpurun_out/r02_v41_tests.txt
for rep in 1 2; do
bash tools/ab_run.sh r02_v41_c5_$rep "" libvsig_nol1tw base
bash tools/ab_run.sh r02_v41_c2_$rep "--workload c2" libvsig_nol1tw base
done
for lib in libvsig_nol1tw base libvsig_nol1tw base; do
  if [ "$lib" = base ]; then unset VSIG_LIB; else export VSIG_LIB=$GRAFT_REPO_ROOT/vector_amd/$lib.so; fi
  timeout -k 10 240 python3 bench.py --workload sync --no-cpu-baseline > gpurun_out/r02_v41_sync_$lib.json 2> gpurun_out/r02_v41_sync_$lib.err
  python3 -c "import json; d=json.load(open('gpurun_out/r02_v41_sync_$lib.json')); print('sync $lib', d['ms_per_step'])"
done
echo done
