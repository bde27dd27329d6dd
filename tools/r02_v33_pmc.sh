set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/pmc.sh gpurun_out/r02_v33_pmc --workload pfb
python3 tools/pmc_summary.py gpurun_out/r02_v33_pmc gpurun_out/pmc_pfbrun_r02_v33.json n=536870912:nchan=64:P=16
rm -rf gpurun_out/r02_v33_pmc
echo done
