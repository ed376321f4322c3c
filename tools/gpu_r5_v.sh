# the CCEH_hybrid(2) ramp: this tree vs the round's first commit (ab_tree, 857dc4e), same box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r5v
mkdir -p $O
for i in 1 2; do
  timeout -k 10 400 python3 bench.py --config 2 --init-cap 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/ic2_new.$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/ic2_new.$i.json').read().strip().splitlines()[-1]);print('ic2 new',d['value'],d['ms_per_step'],d.get('kernel_ms_per_step'))"
  (cd ab_tree && timeout -k 10 400 python3 bench.py --config 2 --init-cap 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/ic2_old.$i.json 2>/dev/null) || exit 1
  python3 -c "import json;d=json.loads(open('$O/ic2_old.$i.json').read().strip().splitlines()[-1]);print('ic2 old',d['value'],d['ms_per_step'],d.get('kernel_ms_per_step'))"
done
