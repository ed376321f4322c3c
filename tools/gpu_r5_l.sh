# k_split: reload of the parent pairs with plain loads (A/B build reload1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5l
mkdir -p $O
AB=pmdfc_amd/lib/ab/reload1/libpmdfc_cceh.so
for i in 1 2; do
timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_r0.$i.json 2>/dev/null || exit 1
PMDFC_LIB=$AB timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_r1.$i.json 2>/dev/null || exit 1
for m in 0 1; do python3 -c "import json;d=json.load(open('$O/bench_r$m.$i.json'));print('reload',$m,d['value'],d['ms_per_step'],d['kernel_ms_per_step'])"; done
done
timeout -k 10 300 python -u tools/phase_stamps.py 46 > $O/stamps0.txt 2>&1 || exit 1
PMDFC_LIB=$AB timeout -k 10 300 python -u tools/phase_stamps.py 46 > $O/stamps1.txt 2>&1 || exit 1
grep -A12 "^k_split" $O/stamps0.txt; grep -A12 "^k_split" $O/stamps1.txt
