# last parked pass + final pass in one launch (k_apply_parked_fin): full GPU suite, A/B, timeline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5r
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
for f in 1 0; do
  PMDFC_FUSE_FINAL=$f timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_f$f.$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_f$f.$i.json'));print('fuse=$f',d['value'],d['ms_per_step'],d['kernel_ms_per_step'], d['roofline']['random_access_roofline']['step_frac'])"
done
done
timeout -k 10 400 python3 bench.py --config 2 --init-cap 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/ic2.json 2>/dev/null || exit 1
python3 -c "import json;d=json.loads(open('$O/ic2.json').read().strip().splitlines()[-1]);print('ic2',d['value'],d['ms_per_step'],d.get('kernel_ms_per_step'))"
PMDFC_FUSE_FINAL=0 timeout -k 10 400 python3 bench.py --config 2 --init-cap 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/ic2_f0.json 2>/dev/null || exit 1
python3 -c "import json;d=json.loads(open('$O/ic2_f0.json').read().strip().splitlines()[-1]);print('ic2 fuse=0',d['value'],d['ms_per_step'],d.get('kernel_ms_per_step'))"
timeout -k 10 300 python3 -u tools/timeline.py 40 8 > $O/timeline.txt 2>&1 || exit 1
cat $O/timeline.txt
