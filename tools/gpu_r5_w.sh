# the CCEH_hybrid(2) ramp regression: grids at p1max (oldgrids: 1024/4096/1024, fin1024: final 1024 only) vs the round's first commit
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r5w
mkdir -p $O
for v in base oldgrids fin1024; do
  L=""; [ $v != base ] && L=pmdfc_amd/lib/ab/$v/libpmdfc_cceh.so
  PMDFC_LIB=$L timeout -k 10 400 python3 bench.py --config 2 --init-cap 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/ic2_$v.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/ic2_$v.json').read().strip().splitlines()[-1]);print('ic2 $v',d['value'],d['ms_per_step'],d.get('kernel_ms_per_step'))"
done
(cd ab_tree && timeout -k 10 400 python3 bench.py --config 2 --init-cap 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/ic2_old.json 2>/dev/null) || exit 1
python3 -c "import json;d=json.loads(open('$O/ic2_old.json').read().strip().splitlines()[-1]);print('ic2 old',d['value'],d['ms_per_step'],d.get('kernel_ms_per_step'))"
