set -e
for cfg in "0 2" "0 34" "0 42" "8192 32" "8192 40" "16384 34"; do
  set -- $cfg
  echo "== M=$1 var=$2"; timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline --xcorr-m $1 --xcorr-variant $2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['stages_ms'], d['check']['ok'])"
done
