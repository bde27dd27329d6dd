#!/bin/bash
# A/B: chain history 254 vs 256 (VSIG_CHAIN_HIST16) x D=1 FIR offset lo16 library
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {  # tag lib hist16 args
  local tag=$1 lib=$2 h=$3; shift 3
  if [ "$lib" = base ]; then unset VSIG_LIB; else export VSIG_LIB=$GRAFT_REPO_ROOT/vector_amd/$lib.so; fi
  VSIG_CHAIN_HIST16=$h timeout -k 10 240 python3 bench.py "$@" --no-cpu-baseline > gpurun_out/r05_h_${tag}.json 2> gpurun_out/r05_h_${tag}.err
  python3 -c "import json; d=json.load(open('gpurun_out/r05_h_${tag}.json')); print('$tag', d['ms_per_step'], d['stages_ms'], d['check']['ok'])"
}
for rep in 1 2; do
  run c5_base_h0_$rep base 0 --no-c2-leg
  run c5_base_h1_$rep base 1 --no-c2-leg
  run c2_base_h0_$rep base 0 --workload c2
  run c2_base_h1_$rep base 1 --workload c2
  run c2_lo16_h0_$rep libvsig_lo16 0 --workload c2
  run c2_lo16_h1_$rep libvsig_lo16 1 --workload c2
done
