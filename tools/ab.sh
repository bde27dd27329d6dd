# A/B the default library against an alternative build: tools/ab.sh ALT.so [bench args]
set -e
ALT=$1; shift
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/ab_gpu.log 2>&1 || { tail -30 gpurun_out/ab_gpu.log; exit 1; }
tail -1 gpurun_out/ab_gpu.log
for rep in 1 2; do
for lib in vector_amd/libvsig.so $ALT; do
  echo "== $lib chain"; VSIG_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline "$@" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['stages_ms'], d['check']['ok'])"
  echo "== $lib pfb"; VSIG_LIB=$lib timeout -k 10 300 python bench.py --workload pfb --steps 20 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['avg_launch_ms'], d['check']['ok'])"
done; done
