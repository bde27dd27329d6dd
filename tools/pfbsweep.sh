set -e
mkdir -p gpurun_out
for v in ${VARS:-1 3}; do for f in ${FPGS:-32 64 128}; do
  timeout -k 10 120 python bench.py --workload pfb --steps 10 --warmup 2 --no-cpu-baseline --pfb-variant $v --pfb-fpg $f 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($v,$f,d['roofline']['avg_launch_ms'],d['roofline']['achieved'],d['check']['ok'])"
done; done
