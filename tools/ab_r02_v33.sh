set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_analysis.py -x -q -k pfb --timeout 120 --timeout-method thread > gpurun_out/r02_v33_tests.txt 2>&1 || { tail -30 gpurun_out/r02_v33_tests.txt; exit 1; }
tail -1 gpurun_out/r02_v33_tests.txt
for rep in 1 2; do
for lib in base libvsig_pfbfwd; do
  if [ "$lib" = base ]; then unset VSIG_LIB; else export VSIG_LIB=$GRAFT_REPO_ROOT/vector_amd/$lib.so; fi
  timeout -k 10 240 python3 bench.py --workload pfb --no-cpu-baseline > gpurun_out/r02_v33_${rep}_$lib.json 2> gpurun_out/r02_v33_${rep}_$lib.err
  python3 -c "import json; d=json.load(open('gpurun_out/r02_v33_${rep}_$lib.json')); print('$lib', d['ms_per_step'], d['value'])"
done
done
unset VSIG_LIB
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/v33_f -o pmc -- python3 bench.py --workload pfb --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/v33_f.log 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/v33_w -o pmc -- python3 bench.py --workload pfb --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/v33_w.log 2>&1
python3 - <<'PY'
import csv, glob
for tag in ("v33_f", "v33_w"):
    for f in glob.glob(f"gpurun_out/{tag}/**/*counter_collection.csv", recursive=True):
        vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "pfb_kernel" in r["Kernel_Name"]]
        print(tag, len(vals), vals[-3:])
PY
rm -rf gpurun_out/v33_f gpurun_out/v33_w
echo done
