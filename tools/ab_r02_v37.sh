set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_v37_gputests.txt 2>&1 || { tail -30 gpurun_out/r02_v37_gputests.txt; exit 1; }
tail -1 gpurun_out/r02_v37_gputests.txt
for rep in 1 2; do
bash tools/ab_run.sh r02_v37_c5_$rep "" libvsig_unphased base
bash tools/ab_run.sh r02_v37_c2_$rep "--workload c2" libvsig_unphased base
done
for lib in libvsig_unphased base; do
  if [ "$lib" = base ]; then unset VSIG_LIB; else export VSIG_LIB=$GRAFT_REPO_ROOT/vector_amd/$lib.so; fi
  timeout -k 10 240 python3 bench.py --workload sync --no-cpu-baseline > gpurun_out/r02_v37_sync_$lib.json 2> gpurun_out/r02_v37_sync_$lib.err
  timeout -k 10 240 python3 bench.py --workload pfb --no-cpu-baseline > gpurun_out/r02_v37_pfb_$lib.json 2> gpurun_out/r02_v37_pfb_$lib.err
  python3 -c "import json; d=json.load(open('gpurun_out/r02_v37_sync_$lib.json')); e=json.load(open('gpurun_out/r02_v37_pfb_$lib.json')); print('sync/pfb $lib', d['ms_per_step'], e['ms_per_step'])"
done
echo done
