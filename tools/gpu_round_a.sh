set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -3 gpurun_out/gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"
timeout -k 10 400 python3 bench.py > gpurun_out/r01_v4_bench.json 2> gpurun_out/r01_v4_bench.err
cat gpurun_out/r01_v4_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r01_v4_prof -o run -- python3 bench.py --steps 10 --no-cpu-baseline > gpurun_out/r01_v4_prof.log 2>&1
echo prof done
