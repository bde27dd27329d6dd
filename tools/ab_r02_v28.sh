set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_alignment.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_v28_tests.txt 2>&1 || { tail -30 gpurun_out/r02_v28_tests.txt; exit 1; }
tail -1 gpurun_out/r02_v28_tests.txt
for rep in 1 2; do
bash tools/ab_run.sh r02_v28_c5_$rep "" base libvsig_ilv50 libvsig_ilv61
bash tools/ab_run.sh r02_v28_c2_$rep "--workload c2" base libvsig_ilv50 libvsig_ilv61
done
echo done
