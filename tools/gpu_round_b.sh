set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
TAG=${1:-r01_v5}
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 10 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
echo prof done
bash tools/pmc.sh gpurun_out/${TAG}_pmc
echo pmc done
