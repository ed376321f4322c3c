# the CCEH_hybrid(2) ramp: 16 record buffers vs 3 (A/B build rb3)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5u
mkdir -p $O
for i in 1 2; do
for v in base rb3; do
  L=""; [ $v != base ] && L=pmdfc_amd/lib/ab/$v/libpmdfc_cceh.so
  PMDFC_LIB=$L timeout -k 10 400 python3 bench.py --config 2 --init-cap 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/ic2_$v.$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/ic2_$v.$i.json').read().strip().splitlines()[-1]);print('ic2 $v',d['value'],d['ms_per_step'],d.get('kernel_ms_per_step'))"
done
done
