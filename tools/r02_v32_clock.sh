set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for w in c2 sync; do
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/v32_$w -o run -- python3 bench.py --workload $w --samples 268435456 --no-cpu-baseline --steps 12 --warmup 2 > gpurun_out/v32_$w.log 2>&1
python3 tools/db_seq.py gpurun_out/v32_$w/run_results.db xcorr_half fir_os psd_pair > gpurun_out/r02_v32_${w}_seq.txt
rm -rf gpurun_out/v32_$w
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/v32_s30 -o run -- python3 bench.py --workload sync --no-cpu-baseline --steps 6 --warmup 2 > gpurun_out/v32_s30.log 2>&1
python3 tools/db_seq.py gpurun_out/v32_s30/run_results.db xcorr_half > gpurun_out/r02_v32_sync30_seq.txt
rm -rf gpurun_out/v32_s30
echo done
