# round 4 A/B: FIR pair loads with the unshared rows non-temporal (libvsig_ntmid)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/ab_run.sh r04_ntc2 "--workload c2 --steps 40" base libvsig_ntmid base libvsig_ntmid
bash tools/ab_run.sh r04_ntc5 "--steps 30 --no-c2-leg" base libvsig_ntmid base libvsig_ntmid
