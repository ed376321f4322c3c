# grouped insert pipeline (PMDFC_PIPE_GROUP batches behind one event pair): parity, A/B, timeline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5q
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_route.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
for g in 8 1 4; do
  PMDFC_PIPE_GROUP=$g timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_g$g.$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_g$g.$i.json'));print('G=$g',d['value'],d['ms_per_step'],d['kernel_ms_per_step'], d['roofline']['random_access_roofline']['step_frac'])"
done
done
timeout -k 10 300 python3 -u tools/timeline.py 40 8 > $O/timeline.txt 2>&1 || exit 1
cat $O/timeline.txt
