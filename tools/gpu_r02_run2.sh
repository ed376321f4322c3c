set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "upsert or split_loss" tests/test_gpu_dropin.py > gpurun_out/r02_t2.log 2>&1; rc=$?; tail -3 gpurun_out/r02_t2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --upsert --no-cpu-baseline > gpurun_out/r02_bench2_upsert.json 2> gpurun_out/r02_bench2_upsert.err && echo upsert ok &&
timeout -k 10 300 python -u bench.py --config 8 --no-cpu-baseline > gpurun_out/r02_bench8.json 2> gpurun_out/r02_bench8.err && echo bench8 ok &&
timeout -k 10 120 python -u tools/phase_stamps.py 12 > gpurun_out/r02_stamps12.txt 2>&1 && echo st12 ok &&
timeout -k 10 120 python -u tools/phase_stamps.py 46 > gpurun_out/r02_stamps46.txt 2>&1 && echo st46 ok &&
cat /sys/fs/cgroup/cpu.max > gpurun_out/r02_cpumax.txt 2>&1; nproc >> gpurun_out/r02_cpumax.txt;
bash tools/run_profile.sh r02 > gpurun_out/r02_prof.log 2>&1 && echo prof ok
