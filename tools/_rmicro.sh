cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_refine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_v8_t.txt 2>&1; tail -1 gpurun_out/r03_v8_t.txt; grep -E "^FAILED" gpurun_out/r03_v8_t.txt | head -3
for lib in base rko1 rko2 rko3; do
  if [ $lib = base ]; then unset VSIG_LIB; else export VSIG_LIB=$GRAFT_REPO_ROOT/vector_amd/libvsig_$lib.so; fi
  timeout -k 10 120 python tools/refine_micro.py 30
done
