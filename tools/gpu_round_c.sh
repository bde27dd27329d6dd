#!/bin/bash
# Round profiling pass + the fused FIR->PSD kernel's counters (bench --fuse).
set -e
cd "$GRAFT_REPO_ROOT"
bash tools/profile_round.sh "$1"
timeout -k 10 200 python3 bench.py --fuse --no-cpu-baseline > gpurun_out/$1_fused_bench.json 2> gpurun_out/$1_fused_bench.err
cat gpurun_out/$1_fused_bench.json
bash tools/pmc.sh gpurun_out/$1_fusedpmc --fuse
echo "fused done"
