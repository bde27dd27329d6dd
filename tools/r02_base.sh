#!/bin/bash
# Round-2 first GPU pass: suite, default bench, config-5 shape (D=4, 2^31 samples), kernel stats.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02a_gputests.txt 2>&1
tail -2 gpurun_out/r02a_gputests.txt
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/r02a_bench.json 2> gpurun_out/r02a_bench.err
cat gpurun_out/r02a_bench.json
timeout -k 10 300 python3 bench.py --decim 4 --samples 2147483648 --no-cpu-baseline --steps 10 > gpurun_out/r02a_c5.json 2> gpurun_out/r02a_c5.err
cat gpurun_out/r02a_c5.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02a_prof -o run -- python3 bench.py --steps 10 --no-cpu-baseline > gpurun_out/r02a_prof.log 2>&1
echo done
