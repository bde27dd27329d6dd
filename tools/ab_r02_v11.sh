set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_run.sh ab11bp1 "" libvsig_solo
bash tools/ab_run.sh ab11bp4 "--pipeline 4 --three-streams" libvsig_solo
bash tools/ab_run.sh ab11bp8 "--pipeline 8 --three-streams" libvsig_solo
echo done
