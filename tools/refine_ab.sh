# round 4: refine launch composition (rocprofv3 per-kernel durations) and numpy-pass grid A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_rprof -o run -- python3 tools/refine_micro.py 50 > gpurun_out/r04_rprof.log 2>&1
for lib in base libvsig_np256 libvsig_np64 libvsig_relaxed base libvsig_np256 libvsig_np64 libvsig_relaxed; do
  if [ "$lib" = base ]; then unset VSIG_LIB; else export VSIG_LIB=$GRAFT_REPO_ROOT/vector_amd/$lib.so; fi
  timeout -k 10 120 python3 tools/refine_micro.py 50
done
VSIG_LIB=$GRAFT_REPO_ROOT/vector_amd/libvsig_relaxed.so timeout -k 10 300 python3 -m pytest tests/test_gpu_refine.py tests/test_gpu_chain.py -q --timeout 120 --timeout-method thread 2>&1 | tail -2
