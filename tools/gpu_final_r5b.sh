# round 5 final tree, part 2: every bench line (config 2 with its CPU
# baseline first), with this round's PMC summary in place for the roofline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ev
timeout -k 10 600 python -u bench.py > gpurun_out/ev/bench_config2.json 2> gpurun_out/ev/bench_config2.err || exit 1
echo config2 done
for c in "--config 2 --upsert --no-cpu-baseline" "--config 2 --route --no-cpu-baseline" "--config 3 --no-cpu-baseline" "--config 4 --no-cpu-baseline" "--config 4 --route --no-cpu-baseline" "--config 5 --no-cpu-baseline" "--config 6 --no-cpu-baseline" "--config 7 --no-cpu-baseline" "--config 8 --steps 2" "--config 2 --init-cap 2 --no-cpu-baseline"; do
  tag=$(echo "$c" | tr -dc 'a-z0-9')
  timeout -k 10 600 python -u bench.py $c > gpurun_out/ev/bench_$tag.json 2> gpurun_out/ev/bench_$tag.err || { echo "failed: $c"; exit 1; }
  echo "$c done"
done
