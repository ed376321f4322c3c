# the round's committed evidence: kernel trace + PMC (FETCH_SIZE, WRITE_SIZE
# passes) of the bench's own non-pipelined config-2 run, then the bench lines
# (config 2 with its CPU baseline, config 2 upsert, 3, 4, 4 routed, 5, 6, 7, 8)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
R=${1:-r04}
bash tools/run_profile.sh $R > gpurun_out/prof_$R.log 2>&1 || { tail -5 gpurun_out/prof_$R.log; exit 1; }
mkdir -p gpurun_out/ev profiles/$R
cp gpurun_out/prof_$R/pmc_config2.json profiles/$R/pmc_config2.json
timeout -k 10 600 python -u bench.py > gpurun_out/ev/bench_config2.json 2> gpurun_out/ev/bench_config2.err || exit 1
echo config2 done
for c in "--config 2 --upsert --no-cpu-baseline" "--config 2 --route --no-cpu-baseline" "--config 3 --no-cpu-baseline" "--config 4 --no-cpu-baseline" "--config 4 --route --no-cpu-baseline" "--config 5 --no-cpu-baseline" "--config 6 --no-cpu-baseline" "--config 7 --no-cpu-baseline" "--config 8 --steps 2" "--config 2 --init-cap 2 --no-cpu-baseline"; do
  tag=$(echo "$c" | tr -dc 'a-z0-9')
  timeout -k 10 600 python -u bench.py $c > gpurun_out/ev/bench_$tag.json 2> gpurun_out/ev/bench_$tag.err || { echo "failed: $c"; exit 1; }
  echo "$c done"
done
