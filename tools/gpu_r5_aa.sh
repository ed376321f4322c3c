# split round + last parked pass in one launch (k_split_park): parity first, then A/B and the timeline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r5aa
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
for f in 1 0; do
  PMDFC_SPLIT_PARK=$f timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/c2_sp$f.$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$O/c2_sp$f.$i.json'));print('split_park=$f',d['value'],d['ms_per_step'],d['kernel_ms_per_step'], d['roofline']['random_access_roofline']['step_frac'])"
done
done
for f in 1 0; do
  PMDFC_SPLIT_PARK=$f timeout -k 10 400 python3 bench.py --config 2 --init-cap 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/ic2_sp$f.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/ic2_sp$f.json').read().strip().splitlines()[-1]);print('ic2 split_park=$f',d['value'],d['ms_per_step'],d.get('kernel_ms_per_step'))"
done
timeout -k 10 300 python3 -u tools/timeline.py 40 8 > $O/timeline.txt 2>&1 || exit 1
tail -16 $O/timeline.txt
