set -o pipefail
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py tests/test_gpu_host_adapter.py -q -m gpu -x --durations=8 > gpurun_out/t5.log 2>&1; echo "tests rc=$?"; tail -15 gpurun_out/t5.log
PMDFC_BUCKET_STAMPS=1 timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/b5s.json 2> gpurun_out/b5s.err; echo "stamps rc=$?"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/prof_r01b/trace -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/b5.json 2> gpurun_out/b5.err; echo "prof rc=$?"
