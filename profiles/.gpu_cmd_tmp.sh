set -o pipefail
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py tests/test_gpu_host_adapter.py -q -m gpu -x --durations=5 > gpurun_out/t7.log 2>&1; echo "tests rc=$?"; tail -20 gpurun_out/t7.log
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b7.json 2> gpurun_out/b7.err; echo "bench rc=$?"; python3 -c "import json;d=json.load(open('gpurun_out/b7.json'));print(d['value'],d['ms_per_step'],d['correct'],d['kernel_ms_per_step'])"
