# per-bucket early answers of mixed batches (k_mixed_early): parity, then
# config 3 / 4 A/B against the device-wide set (PMDFC_MIXED_EARLY=0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5j
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for c in 4 3; do
  for e in 1 0; do
    PMDFC_MIXED_EARLY=$e timeout -k 10 400 python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/c$c.e$e.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.loads(open('$O/c$c.e$e.json').read().strip().splitlines()[-1]);print('c$c early=$e',d['value'],d['ms_per_step'],d.get('kernel_ms_per_step'))"
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d $O/t4 -o run -- python3 bench.py --config 4 --steps 1 --warmup 0 --no-cpu-baseline > /dev/null 2> $O/t4.err || exit 1
head -25 $O/t4/run_kernel_stats.csv | cut -c1-150
