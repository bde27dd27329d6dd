set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_v10_gputests.txt 2>&1 || { tail -30 gpurun_out/r02_v10_gputests.txt; exit 1; }
tail -2 gpurun_out/r02_v10_gputests.txt
bash tools/ab_run.sh ab10c5 "" base libvsig_noswz
bash tools/ab_run.sh ab10c2 "--workload c2" base libvsig_noswz
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/ab10_pmc -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab10_pmc.log 2>&1
echo done
