set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_alignment.py tests/test_gpu_parity.py tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_v39_tests.txt 2>&1 || { tail -30 gpurun_out/r02_v39_tests.txt; exit 1; }
tail -1 gpurun_out/r02_v39_tests.txt
for rep in 1 2 3; do
bash tools/ab_run.sh r02_v39_c5_$rep "" libvsig_nobufld base
bash tools/ab_run.sh r02_v39_c2_$rep "--workload c2" libvsig_nobufld base
done
echo done
