#!/bin/bash
# A/B of library builds on the headline chain: tools/ab_libs.sh "LIB1 LIB2 ..." [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
LIBS=$1; shift
for rep in 1 2; do
for lib in $LIBS; do
  echo "== $lib"
  VSIG_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 "$@" 2>gpurun_out/ab_err.log \
    | python -c "import json,sys; d=json.load(sys.stdin); print(d['ms_per_step'], d['value'], d['stages_ms'], d['check']['ok'])" \
    || { tail -20 gpurun_out/ab_err.log; exit 1; }
done; done
