set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_v19_gputests.txt 2>&1 || { tail -30 gpurun_out/r02_v19_gputests.txt; exit 1; }
tail -2 gpurun_out/r02_v19_gputests.txt
bash tools/ab_run.sh ab19c5 "" base libvsig_xsigma
bash tools/ab_run.sh ab19c2 "--workload c2" base libvsig_xsigma
echo done
