#!/bin/bash
# Round-2 GPU pass: suite, bench lines (c5 default, c2), kernel stats.  TAG = $1
set -e
TAG=${1:-r02}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputests.txt 2>&1 || { tail -30 gpurun_out/${TAG}_gputests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_gputests.txt
timeout -k 10 300 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 python3 bench.py --workload c2 --no-cpu-baseline > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err
cat gpurun_out/${TAG}_c2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 10 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
echo done
