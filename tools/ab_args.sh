#!/bin/bash
# A/B of bench.py argument sets on one library: tools/ab_args.sh TAG "common args" "label=args" ...
# (each label=args pair is one bench.py run, in the order given; repeat pairs to alternate)
set -e
TAG=$1; COMMON=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
i=0
for pair in "$@"; do
  label=${pair%%=*}; args=${pair#*=}; i=$((i+1))
  timeout -k 10 240 python3 bench.py $COMMON $args --no-cpu-baseline > gpurun_out/${TAG}_${i}_$label.json 2> gpurun_out/${TAG}_${i}_$label.err
  python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_${i}_$label.json')); print('$label', d['ms_per_step'], d.get('stages_ms'), d.get('stages_ghz'), d['check']['ok'])"
done
