# front-end A/B: bench_frontend (32 callers, 8 waves) under env settings,
# one run per argument ("VAR=value ..." or "-"); FE_EXE picks another binary
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/fe
i=0
for cfg in "$@"; do
  i=$((i + 1))
  [ "$cfg" = "-" ] && cfg=""
  exe=pmdfc_amd/lib/bench_frontend; case "$cfg" in *OLD=1*) exe=pmdfc_amd/lib/ab/feold/bench_frontend;; esac
  env $cfg timeout -k 10 200 $exe 32 65536 256 65536 ${FE_SPINUS:-10} ${FE_WAVES:-8} > gpurun_out/fe/r$i.json 2> gpurun_out/fe/r$i.err || exit 1
  python3 -c "
import json,sys; f=json.loads(open('gpurun_out/fe/r$i.json').read().strip().splitlines()[-1])
print(sys.argv[1] or '(default)', {k: f[k] for k in f if 'mops' in k or 'avg_batch' in k}); ph=f['phases']
print('   ', {p: (ph[p]['queue_us_per_op'], ph[p]['gpu_us_per_op'], ph[p]['deliver_us_per_op']) for p in ph})" "$cfg"
done
