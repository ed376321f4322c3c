# End-of-round evidence on the final tree (usage: gpu_final.sh rNN a|b):
#   a: the whole GPU suite + smoke, then the kernel trace and the PMC passes of
#      the bench's own config-2 run (tools/run_profile.sh -> profiles/rNN/);
#   b: every bench line (config 2 with its CPU baseline first), with the
#      round's PMC summary in place for the roofline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
R=${1:?round}
case "${2:-a}" in
a)
  mkdir -p gpurun_out
  bash tools/gpu_full_tests.sh || exit 1
  bash tools/run_profile.sh $R > gpurun_out/prof_$R.log 2>&1 || { tail -5 gpurun_out/prof_$R.log; exit 1; }
  echo "profile done"
  ;;
b)
  O=gpurun_out/ev_$R
  mkdir -p $O
  timeout -k 10 600 python -u bench.py > $O/bench_config2.json 2> $O/bench_config2.err || exit 1
  echo config2 done
  for c in "--config 2 --upsert --no-cpu-baseline" "--config 2 --route --no-cpu-baseline" "--config 3 --no-cpu-baseline" \
           "--config 4 --no-cpu-baseline" "--config 4 --route --no-cpu-baseline" "--config 5 --no-cpu-baseline" \
           "--config 6 --no-cpu-baseline" "--config 7 --no-cpu-baseline" "--config 8 --steps 2" \
           "--config 2 --init-cap 2 --no-cpu-baseline"; do
    tag=$(echo "$c" | tr -dc 'a-z0-9')
    timeout -k 10 600 python -u bench.py $c > $O/bench_$tag.json 2> $O/bench_$tag.err || { echo "failed: $c"; exit 1; }
    echo "$c done"
  done
  ;;
esac
