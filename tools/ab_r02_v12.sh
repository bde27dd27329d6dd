set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_run.sh ab12b "" base libvsig_firw2 libvsig_firw4 libvsig_firko libvsig_firkow4
echo done
