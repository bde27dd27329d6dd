set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
VSIG_LIB=$GRAFT_REPO_ROOT/vector_amd/libvsig_xilv.so timeout -k 10 300 python -u -m pytest tests/test_gpu_alignment.py tests/test_gpu_refine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_v29_tests.txt 2>&1 || { tail -30 gpurun_out/r02_v29_tests.txt; exit 1; }
tail -1 gpurun_out/r02_v29_tests.txt
for rep in 1 2; do
bash tools/ab_run.sh r02_v29_c5_$rep "" libvsig_xilv base
bash tools/ab_run.sh r02_v29_c2_$rep "--workload c2" libvsig_xilv base
done
echo done
