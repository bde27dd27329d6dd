#!/bin/bash
# End-of-round pass: GPU suite + smoke, then the profiling round (headline
# chain, PFB), config 3 (sync) with its kernel trace, and the mixer chain.
set -e
cd "$GRAFT_REPO_ROOT"
TAG=$1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gputests.log 2>&1
tail -2 gpurun_out/${TAG}_gputests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
cat gpurun_out/${TAG}_smoke.log
bash tools/profile_round.sh "$TAG"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 bench.py --workload sync > gpurun_out/${TAG}_sync_bench.json 2> gpurun_out/${TAG}_sync_bench.err
cat gpurun_out/${TAG}_sync_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_syncprof -o run -- python3 bench.py --workload sync --steps 10 --no-cpu-baseline > gpurun_out/${TAG}_syncprof.log 2>&1
timeout -k 10 200 python3 bench.py --freq-shift 3e8 --no-cpu-baseline > gpurun_out/${TAG}_mix_bench.json 2> gpurun_out/${TAG}_mix_bench.err
cat gpurun_out/${TAG}_mix_bench.json
echo "round done"
