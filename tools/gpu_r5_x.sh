# grids by ops per segment: the ramp and config 2, against oldgrids
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r5x
mkdir -p $O
for v in base oldgrids; do
  L=""; [ $v != base ] && L=pmdfc_amd/lib/ab/$v/libpmdfc_cceh.so
  PMDFC_LIB=$L timeout -k 10 400 python3 bench.py --config 2 --init-cap 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/ic2_$v.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/ic2_$v.json').read().strip().splitlines()[-1]);print('ic2 $v',d['value'],d['ms_per_step'],d.get('kernel_ms_per_step'))"
  PMDFC_LIB=$L timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/c2_$v.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$O/c2_$v.json'));print('config2 $v',d['value'],d['ms_per_step'],d['kernel_ms_per_step'], d['roofline']['random_access_roofline']['step_frac'])"
done
