#!/bin/bash
# One pfb line and one default (c5) line without CPU baselines: tools/quick_lines.sh TAG
set -e
TAG=${1:?tag}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --workload pfb --no-cpu-baseline > gpurun_out/${TAG}_pfb.json 2> gpurun_out/${TAG}_pfb.err
timeout -k 10 400 python3 bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
python3 - "$TAG" <<'PY'
import json, sys
t = sys.argv[1]
d = json.load(open(f"gpurun_out/{t}_pfb.json"))
print("pfb", d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["traffic_source"])
d = json.load(open(f"gpurun_out/{t}_bench.json"))
print("c5", d["ms_per_step"], d["stages_ms"], d["stages_ghz"], d["stages_roofline_c2"]["fir+psd"]["hbm_frac"])
PY
