#!/bin/bash
# Round-2 evidence pass: bench lines for every config (c5 default with CPU
# baseline, c2, sync = config 3, pfb = config 4), rocprofv3 kernel stats of the
# default line, PMC passes (tools/pmc.sh) for c5 and c2.  Usage: tools/r02_profile.sh TAG
set -e
TAG=${1:-r02}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 python3 bench.py --workload c2 --no-cpu-baseline > gpurun_out/${TAG}_c2_bench.json 2> gpurun_out/${TAG}_c2_bench.err
timeout -k 10 300 python3 bench.py --workload sync > gpurun_out/${TAG}_sync_bench.json 2> gpurun_out/${TAG}_sync_bench.err
timeout -k 10 300 python3 bench.py --workload pfb > gpurun_out/${TAG}_pfb_bench.json 2> gpurun_out/${TAG}_pfb_bench.err
echo "benches done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 10 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
python3 tools/db_stats.py gpurun_out/${TAG}_prof/run_results.db gpurun_out/${TAG}_kernel_stats.csv
rm -rf gpurun_out/${TAG}_prof
echo "kernel trace done"
bash tools/pmc.sh gpurun_out/${TAG}_pmc
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc gpurun_out/pmc_c5_${TAG}.json n=2147483648:ntaps=255:decim=4:nfft=8192:L=4096
bash tools/pmc.sh gpurun_out/${TAG}_pmc_c2 --workload c2
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc_c2 gpurun_out/pmc_c2_${TAG}.json n=268435456:ntaps=255:decim=1:nfft=8192:L=4096
rm -rf gpurun_out/${TAG}_pmc gpurun_out/${TAG}_pmc_c2
echo "all done"
