set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_v27_gputests.txt 2>&1 || { tail -30 gpurun_out/r02_v27_gputests.txt; exit 1; }
tail -1 gpurun_out/r02_v27_gputests.txt
timeout -k 10 300 python3 bench.py --no-cpu-baseline --samples 268435456 --steps 50 > gpurun_out/r02_v27_c5n8.json 2> gpurun_out/r02_v27_c5n8.err
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/r02_v27_c5.json 2> gpurun_out/r02_v27_c5.err
timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload c2 > gpurun_out/r02_v27_c2.json 2> gpurun_out/r02_v27_c2.err
timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload sync > gpurun_out/r02_v27_sync.json 2> gpurun_out/r02_v27_sync.err
for f in c5n8 c5 c2 sync; do python3 -c "import json; d=json.load(open('gpurun_out/r02_v27_$f.json')); print('$f', d['ms_per_step'], d.get('stages_ms'), d.get('check'))"; done
echo done
