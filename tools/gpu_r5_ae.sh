# with the grouped pipeline: coarse partition on/off, partition stream priority
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r5ae
mkdir -p $O
for i in 1 2; do
for v in "X=1" "PMDFC_CP=0" "PMDFC_PSTREAM_PRIO=0"; do
  tag=$(echo "$v" | tr -dc 'A-Za-z0-9')
  env $v timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/c2_$tag.$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$O/c2_$tag.$i.json'));print('$v',d['value'],d['ms_per_step'],d['kernel_ms_per_step'], d['roofline']['random_access_roofline']['step_frac'])"
done
done
