#!/bin/bash
# One GPU pass: GPU suite, smoke, default bench (c5 + CPU baseline), c2 bench,
# rocprofv3 kernel stats of the default workload.  Usage: tools/round_pass.sh TAG
set -e
TAG=${1:?tag}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gputests.txt 2>&1 || { tail -30 gpurun_out/${TAG}_gputests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_gputests.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1
tail -1 gpurun_out/${TAG}_smoke.txt
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 python3 bench.py --workload c2 --no-cpu-baseline > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err
cat gpurun_out/${TAG}_c2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 10 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
echo done
