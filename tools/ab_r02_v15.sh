set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_run.sh ab15 "" base libvsig_firko libvsig_firkox4
echo done
