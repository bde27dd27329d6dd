set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for K in 1 8 16 32; do
  if [ $K = 1 ]; then A=""; else A="--serial --pipeline $K"; fi
  timeout -k 10 300 python3 bench.py --no-cpu-baseline $A > gpurun_out/r02_v21_s$K.json 2> gpurun_out/r02_v21_s$K.err
  python3 -c "import json; d=json.load(open('gpurun_out/r02_v21_s$K.json')); print('serial K=$K', d['ms_per_step'], d['stages_ms'], d['check']['ok'])"
done
echo done
