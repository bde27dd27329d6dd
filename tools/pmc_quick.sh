#!/bin/bash
# One PMC pass (FETCH_SIZE, then WRITE_SIZE) over a short bench run: tools/pmc_quick.sh OUT [bench args]
set -e
OUT=$1; shift; mkdir -p "$GRAFT_REPO_ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/p1" -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > "$OUT/p1.log" 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/p2" -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > "$OUT/p2.log" 2>&1
