# Size scan of the chain stages (c2 at 2^27..2^29, c5 at 2^29..2^31 samples): one bench line
# per size into gpurun_out/r04_scan_<cfg>_<log2 n>.json (round 4, FIR / PSD / correlator scaling).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for s in 27 28 29; do
  timeout -k 10 200 python3 bench.py --workload c2 --samples $((1<<s)) --steps 20 --no-cpu-baseline > gpurun_out/r04_scan_c2_$s.json 2>/dev/null
  python3 -c "import json; d=json.load(open('gpurun_out/r04_scan_c2_$s.json')); print('c2 2^$s', d['ms_per_step'], d['stages_ms'])"
done
for s in 29 30 31; do
  timeout -k 10 200 python3 bench.py --samples $((1<<s)) --steps 20 --no-cpu-baseline --no-c2-leg > gpurun_out/r04_scan_c5_$s.json 2>/dev/null
  python3 -c "import json; d=json.load(open('gpurun_out/r04_scan_c5_$s.json')); print('c5 2^$s', d['ms_per_step'], d['stages_ms'])"
done
