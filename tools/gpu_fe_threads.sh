set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/fet
for T in 1 4 8 16 32; do
  timeout -k 10 200 pmdfc_amd/lib/bench_frontend $T 32768 256 65536 10 8 > gpurun_out/fet/t$T.json 2> gpurun_out/fet/t$T.err || exit 1
  python3 -c "
import json; f=json.loads(open('gpurun_out/fet/t$T.json').read().strip().splitlines()[-1]); ph=f['phases']
print($T, 'ins', f['insert_mops'], 'mixed', f['mixed_mops'], 'amixed', f['async_mixed_mops'], {p: (ph[p]['queue_us_per_op'], ph[p]['gpu_us_per_op'], ph[p]['deliver_us_per_op'], ph[p]['ops_per_batch'], ph[p]['chunk_apply_us'], ph[p]['chunk_answer_us']) for p in ('insert','mixed')})"
done
