set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in base libvsig_pfb128 libvsig_pfb256 libvsig_pfb512; do
  if [ "$lib" = base ]; then unset VSIG_LIB; else export VSIG_LIB=$GRAFT_REPO_ROOT/vector_amd/$lib.so; fi
  timeout -k 10 240 python3 bench.py --workload pfb --no-cpu-baseline > gpurun_out/ab13_$lib.json 2> gpurun_out/ab13_$lib.err
  python3 -c "import json; d=json.load(open('gpurun_out/ab13_$lib.json')); print('$lib', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['check'])"
done
for lib in base libvsig_pfb256; do
  if [ "$lib" = base ]; then unset VSIG_LIB; else export VSIG_LIB=$GRAFT_REPO_ROOT/vector_amd/$lib.so; fi
  for grp in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/ab13_pmc_${lib}_$grp -o pmc -- python3 bench.py --workload pfb --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab13_pmc_${lib}_$grp.log 2>&1
  done
done
echo done
