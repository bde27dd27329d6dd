set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_v42_gputests.txt 2>&1 || { tail -30 gpurun_out/r02_v42_gputests.txt; exit 1; }
tail -1 gpurun_out/r02_v42_gputests.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_v42_smoke.txt 2>&1
tail -1 gpurun_out/r02_v42_smoke.txt
timeout -k 10 400 python3 bench.py > gpurun_out/r02_v42_bench.json 2> gpurun_out/r02_v42_bench.err
timeout -k 10 300 python3 bench.py --workload c2 --no-cpu-baseline > gpurun_out/r02_v42_c2_bench.json 2> gpurun_out/r02_v42_c2_bench.err
for f in r02_v42_bench r02_v42_c2_bench; do python3 -c "
import json; d=json.load(open('gpurun_out/$f.json')); print('$f', d['value'], d['ms_per_step'], d.get('stages_ms'), d['roofline'].get('practical_frac'), (d.get('cpu_baseline') or {}).get('value'))"; done
