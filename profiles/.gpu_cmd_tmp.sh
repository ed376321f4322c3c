set -o pipefail
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_host_adapter.py -q -m gpu -x --durations=8 > gpurun_out/t4.log 2>&1; echo "tests rc=$?"; tail -15 gpurun_out/t4.log
for U in 1 2 4; do PMDFC_GET_UNROLL=$U timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b_u$U.json 2> gpurun_out/b_u$U.err || { echo "bench U=$U failed"; tail -5 gpurun_out/b_u$U.err; break; }; echo "U=$U done"; done
