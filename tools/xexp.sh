set -e
for lib in vector_amd/libvsig.so; do
  echo "== $lib"; VSIG_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['stages_ms'], d['check'])"
done
