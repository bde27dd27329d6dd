#!/bin/bash
# The first half of tools/round_pass.sh (one GPU call stays under gpurun's
# 20-minute limit): GPU suite, smoke, default bench (c5 + CPU baselines + the
# c2 FIR+PSD leg), c2 / sync / pfb lines, rocprofv3 kernel stats of the
# default workload.  Usage: tools/round_pass_a.sh TAG
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
for w in c2 sync pfb; do
  timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline > gpurun_out/${TAG}_$w.json 2> gpurun_out/${TAG}_$w.err
  cat gpurun_out/${TAG}_$w.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-c2-leg > gpurun_out/${TAG}_prof.log 2>&1
python3 tools/db_stats.py gpurun_out/${TAG}_prof/run_results.db gpurun_out/${TAG}_kernel_stats.csv > /dev/null
rm -rf gpurun_out/${TAG}_prof          # raw traces exceed what gpurun copies back
echo prof done
