set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SECONDS=0
timeout -k 10 400 python3 bench.py > gpurun_out/r02_v31_bench.json 2> gpurun_out/r02_v31_bench.err
echo "default bench wall: $SECONDS s"
timeout -k 10 300 python3 bench.py --workload sync > gpurun_out/r02_v31_sync_bench.json 2> gpurun_out/r02_v31_sync_bench.err
timeout -k 10 300 python3 bench.py --workload pfb > gpurun_out/r02_v31_pfb_bench.json 2> gpurun_out/r02_v31_pfb_bench.err
for f in r02_v31_bench r02_v31_sync_bench r02_v31_pfb_bench; do python3 -c "
import json; d=json.load(open('gpurun_out/$f.json')); print('$f', d['value'], d['ms_per_step'], json.dumps(d['cpu_baseline'])[:400])"; done
