cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_refine.py tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_v7_t.txt 2>&1; tail -2 gpurun_out/r03_v7_t.txt; grep -E "^FAILED" gpurun_out/r03_v7_t.txt | head
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03_v7_bench.json 2>gpurun_out/r03_v7_bench.err
python -c "import json; d=json.load(open('gpurun_out/r03_v7_bench.json')); print(d['ms_per_step'], d['stages_ms'], d['check'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_v7_prof -o run -- python3 bench.py --steps 5 --no-cpu-baseline > gpurun_out/r03_v7_prof.log 2>&1 && python tools/db_seq.py gpurun_out/r03_v7_prof/run_results.db refine | tail -6
