set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_v6_gputests.txt 2>&1 || { tail -40 gpurun_out/r02_v6_gputests.txt; exit 1; }
tail -2 gpurun_out/r02_v6_gputests.txt
bash tools/ab_run.sh r02_v6ab "--workload c2 --steps 20" base libvsig_x32 libvsig_x32k1024
