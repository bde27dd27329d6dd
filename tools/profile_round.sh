#!/bin/bash
# One profiling pass: bench lines (c5 default, c2), rocprofv3 kernel stats and
# PMC counters of the default workload.  Usage: tools/profile_round.sh TAG
set -e
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
echo "bench done"; cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 python3 bench.py --workload c2 --no-cpu-baseline > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err
cat gpurun_out/${TAG}_c2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 10 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
echo "prof done"
bash tools/pmc.sh gpurun_out/${TAG}_pmc
echo "all done"
