set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_v22_gputests.txt 2>&1 || { tail -30 gpurun_out/r02_v22_gputests.txt; exit 1; }
tail -2 gpurun_out/r02_v22_gputests.txt
timeout -k 10 300 python3 bench.py --no-cpu-baseline --samples 268435456 --steps 50 > gpurun_out/r02_v22_c5n8.json 2> gpurun_out/r02_v22_c5n8.err
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/r02_v22_c5.json 2> gpurun_out/r02_v22_c5.err
for f in c5n8 c5; do python3 -c "import json; d=json.load(open('gpurun_out/r02_v22_$f.json')); print('$f', d['ms_per_step'], d['stages_ms'], d['check']['ok'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02_v22_prof -o run -- python3 bench.py --no-cpu-baseline --samples 268435456 --steps 20 > gpurun_out/r02_v22_prof.log 2>&1
python3 tools/db_stats.py gpurun_out/r02_v22_prof/run_results.db gpurun_out/r02_v22_c5n8_kernel_stats.csv
rm -rf gpurun_out/r02_v22_prof
echo done
