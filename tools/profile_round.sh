#!/bin/bash
# One profiling pass for a round: bench lines, rocprofv3 kernel stats and PMC
# counters for the headline chain and the PFB workload.  Usage:
#   tools/profile_round.sh TAG      (outputs under gpurun_out/TAG_*)
set -e
TAG=$1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
echo "bench done"; cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 10 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
echo "prof done"
bash tools/pmc.sh gpurun_out/${TAG}_pmc
echo "pmc done"
timeout -k 10 300 python3 bench.py --workload pfb > gpurun_out/${TAG}_pfb_bench.json 2> gpurun_out/${TAG}_pfb_bench.err
cat gpurun_out/${TAG}_pfb_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_pfbprof -o run -- python3 bench.py --workload pfb --steps 10 --no-cpu-baseline > gpurun_out/${TAG}_pfbprof.log 2>&1
bash tools/pmc.sh gpurun_out/${TAG}_pfbpmc --workload pfb
echo "all done"
