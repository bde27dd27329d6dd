#!/bin/bash
# The second half of tools/round_pass.sh: the PMC passes of c5, c2, sync and
# pfb (tools/pmc.sh), summarised per kernel into gpurun_out/TAG_pmcsum.
# Usage: tools/round_pass_b.sh TAG
set -e
TAG=${1:?tag}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/${TAG}_pmcsum
pmc() {   # name keyspec bench-args...
  local name=$1 key=$2; shift 2
  bash tools/pmc.sh gpurun_out/${TAG}_pmc_$name "$@"
  python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc_$name gpurun_out/${TAG}_pmcsum/pmc_${name}_${TAG}.json "$key" > /dev/null
  rm -rf gpurun_out/${TAG}_pmc_$name
  echo "pmc $name done"
}
pmc c5 n=2147483648:ntaps=255:decim=4:nfft=8192:L=4096 --no-c2-leg
pmc c2 n=268435456:ntaps=255:decim=1:nfft=8192:L=4096 --workload c2
pmc sync n=1073741824:L=4096 --workload sync
pmc pfb n=536870912:nchan=64:P=16 --workload pfb
echo pmc done
