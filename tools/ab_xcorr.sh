#!/bin/bash
# A/B of correlator variants on the headline chain (bench.py, no CPU leg).
# Usage: tools/ab_xcorr.sh "VARIANT_ARGS" ...   (each arg one bench configuration)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for a in "$@"; do
  echo "== $a"
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 $a 2>gpurun_out/ab_err.log \
    | python -c "import json,sys; d=json.load(sys.stdin); print(d['ms_per_step'], d['value'], d['stages_ms'], d['check']['ok'])" \
    || { tail -20 gpurun_out/ab_err.log; exit 1; }
done
