# round 4: refine (one launch) -- refine/chain GPU tests, micro and c5 bench timing, then phase
# timestamps (VSIG_REFINE_TRACE build) in the micro and the c5 bench
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_refine.py tests/test_gpu_chain.py tests/test_gpu_shard_threads.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_fused_tests.txt 2>&1
timeout -k 10 120 python3 tools/refine_micro.py 50 > gpurun_out/r04_fused_micro.txt 2>&1
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-c2-leg > gpurun_out/r04_fused_c5.json 2>/dev/null
export VSIG_LIB=$GRAFT_REPO_ROOT/vector_amd/libvsig_rtrace.so
timeout -k 10 120 python3 tools/refine_micro.py 6 > gpurun_out/r04_rtrace_micro.txt 2>&1
timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-c2-leg > gpurun_out/r04_rtrace_c5.txt 2>&1
