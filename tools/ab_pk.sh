# A/B: packed-fp32 FFT engine (libvsig.so) vs scalar (libvsig_scalar.so)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_pk.log 2>&1 || { tail -30 gpurun_out/gpu_pk.log; exit 1; }
tail -2 gpurun_out/gpu_pk.log
echo "== fftbench packed"; timeout -k 10 120 python tools/fftbench.py
echo "== fftbench scalar"; VSIG_LIB=vector_amd/libvsig_scalar.so timeout -k 10 120 python tools/fftbench.py
echo "== bench packed"; timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline 2>/dev/null
echo "== bench scalar"; VSIG_LIB=vector_amd/libvsig_scalar.so timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline 2>/dev/null
echo "== pfb packed"; timeout -k 10 300 python bench.py --workload pfb --steps 10 --no-cpu-baseline 2>/dev/null
