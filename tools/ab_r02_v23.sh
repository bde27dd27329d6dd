set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_v23_gputests.txt 2>&1 || { tail -30 gpurun_out/r02_v23_gputests.txt; exit 1; }
tail -2 gpurun_out/r02_v23_gputests.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()"
for rep in 1 2; do
for lib in base libvsig_nox4; do
  if [ "$lib" = base ]; then unset VSIG_LIB; else export VSIG_LIB=$GRAFT_REPO_ROOT/vector_amd/$lib.so; fi
  timeout -k 10 240 python3 bench.py --workload pfb --no-cpu-baseline > gpurun_out/ab23_$lib.json 2> gpurun_out/ab23_$lib.err
  python3 -c "import json; d=json.load(open('gpurun_out/ab23_$lib.json')); print('$lib', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['check'])"
done
done
echo done
