#!/bin/bash
# A/B of library builds on one bench line: tools/ab_run.sh TAG "bench args" lib1 lib2 ...
# (each lib: vector_amd/<name>.so built by _build.build(defines=..., out=...); "base" = libvsig.so)
set -e
TAG=$1; ARGS=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in "$@"; do
  if [ "$lib" = base ]; then unset VSIG_LIB; else export VSIG_LIB=$GRAFT_REPO_ROOT/vector_amd/$lib.so; fi
  timeout -k 10 240 python3 bench.py $ARGS --no-cpu-baseline > gpurun_out/${TAG}_$lib.json 2> gpurun_out/${TAG}_$lib.err
  python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_$lib.json')); print('$lib', d['ms_per_step'], d.get('stages_ms'), d.get('stages_ghz'), d['check']['ok'])"
done
