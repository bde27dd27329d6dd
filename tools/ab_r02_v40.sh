set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_refine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_v40_tests.txt 2>&1 || { tail -30 gpurun_out/r02_v40_tests.txt; exit 1; }
tail -1 gpurun_out/r02_v40_tests.txt
for rep in 1 2 3; do
bash tools/ab_run.sh r02_v40_n8_$rep "--samples 268435456 --steps 50" libvsig_rg1024 base
done
echo done
