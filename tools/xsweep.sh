set -e
for cfg in "16384 10" "16384 8" "16384 26" "16384 0" "8192 8" "8192 24" "8192 0"; do
  set -- $cfg
  echo "== M=$1 var=$2"; timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --xcorr-m $1 --xcorr-variant $2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['stages_ms'], d['check']['ok'])"
done
