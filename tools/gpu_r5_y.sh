# config 2: small vs round-4 grids, interleaved x3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r5y
mkdir -p $O
for i in 1 2 3; do
for v in base oldgrids; do
  L=""; [ $v != base ] && L=pmdfc_amd/lib/ab/$v/libpmdfc_cceh.so
  PMDFC_LIB=$L timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/c2_$v.$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$O/c2_$v.$i.json'));print('config2 $v',d['value'],d['ms_per_step'],d['kernel_ms_per_step'], d['roofline']['random_access_roofline']['step_frac'])"
done
done
