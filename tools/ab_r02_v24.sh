set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_v24_gputests.txt 2>&1 || { tail -30 gpurun_out/r02_v24_gputests.txt; exit 1; }
tail -2 gpurun_out/r02_v24_gputests.txt
bash tools/ab_run.sh ab24c5 "" base libvsig_nokeyed
bash tools/ab_run.sh ab24c2 "--workload c2" base libvsig_nokeyed
bash tools/ab_run.sh ab24c2b "--workload c2" base libvsig_nokeyed
echo done
