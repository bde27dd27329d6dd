set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_refine.py tests/test_gpu_alignment.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_v27_gputests.txt 2>&1 || { tail -30 gpurun_out/r02_v27_gputests.txt; exit 1; }
tail -1 gpurun_out/r02_v27_gputests.txt
timeout -k 10 300 python3 bench.py --no-cpu-baseline --samples 268435456 --steps 50 > gpurun_out/r02_v27_c5n8.json 2> gpurun_out/r02_v27_c5n8.err
python3 -c "import json; d=json.load(open('gpurun_out/r02_v27_c5n8.json')); print('c5n8', d['ms_per_step'], d['stages_ms'], d['check']['ok'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02_v27_prof -o run -- python3 bench.py --no-cpu-baseline --samples 268435456 --steps 20 > gpurun_out/r02_v27_prof.log 2>&1
python3 tools/db_stats.py gpurun_out/r02_v27_prof/run_results.db gpurun_out/r02_v27_c5n8_kernel_stats.csv > /dev/null
rm -rf gpurun_out/r02_v27_prof
echo done
