set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2; do
bash tools/ab_run.sh r02_v28b_c5_$rep "" libvsig_ilv61 libvsig_ilv50 base
bash tools/ab_run.sh r02_v28b_c2_$rep "--workload c2" libvsig_ilv61 libvsig_ilv50 base
done
echo done
