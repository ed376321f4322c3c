set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/r02_bench2.json 2> gpurun_out/r02_bench2.err && echo bench2 ok &&
timeout -k 10 300 python -u bench.py --upsert --no-cpu-baseline > gpurun_out/r02_bench2_upsert.json 2> gpurun_out/r02_bench2_upsert.err && echo upsert ok &&
timeout -k 10 300 python -u bench.py --config 8 > gpurun_out/r02_bench8.json 2> gpurun_out/r02_bench8.err && echo bench8 ok &&
timeout -k 10 300 python -u bench.py --config 4 > gpurun_out/r02_bench4.json 2> gpurun_out/r02_bench4.err && echo bench4 ok &&
timeout -k 10 300 python -u bench.py --config 4 --route > gpurun_out/r02_bench4_route.json 2> gpurun_out/r02_bench4_route.err && echo bench4r ok &&
bash profiles/run_profile.sh r02 > gpurun_out/r02_prof.log 2>&1 && echo prof ok
