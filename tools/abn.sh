# interleaved A/B/C of library builds: tools/abn.sh lib1 lib2 ... (3 rounds each)
set -e
for rep in 1 2 3; do
for lib in "$@"; do
  VSIG_LIB=$lib timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['ms_per_step'], d['stages_ms'], d['check']['ok'])"
done; done
