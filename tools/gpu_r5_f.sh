# multi-wave serving: parity (serve tests, C++ KV test), front-end bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r5f
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_serve.py -x -v --timeout 200 --timeout-method thread > $O/serve.log 2>&1 || { tail -40 $O/serve.log; exit 1; }
tail -3 $O/serve.log
timeout -k 10 300 pmdfc_amd/lib/test_gpu_kv 200000 8 > $O/kv.log 2>&1 || { tail -20 $O/kv.log; exit 1; }
tail -14 $O/kv.log
timeout -k 10 600 python3 bench.py --config 8 --steps 2 --no-cpu-baseline > $O/c8.json 2> $O/c8.err || { tail -20 $O/c8.err; exit 1; }
python3 - <<'PY'
import json
d=json.load(open("gpurun_out/r5f/c8.json"))
for k in ("frontend","frontend_16_callers","frontend_one_wave"):
    f=d[k]; print(k, f.get("serve_waves"), "ins", f["insert_mops"], "get", f["get_mops"], "mixed", f["mixed_mops"], "async mixed", f["async_mixed_mops"])
print("value", d["value"])
PY
for w in 2 4 16; do
timeout -k 10 300 pmdfc_amd/lib/bench_frontend 32 65536 256 65536 10 $w > $O/fe_w$w.json 2>/dev/null || exit 1
python3 -c "import json;f=json.load(open('$O/fe_w$w.json'));print('waves',f['serve_waves'],'ins',f['insert_mops'],'get',f['get_mops'],'mixed',f['mixed_mops'])"
done
