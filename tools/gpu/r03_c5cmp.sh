# C5 one-launch time: bench.py's aux leg vs tools/exp_c5_list_order.py in a fresh process.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-c5cmp}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u tools/exp_c5_list_order.py --config c5 --only swizzle,swizzle_info > gpurun_out/$TAG/exp.json 2> gpurun_out/$TAG/exp.err || { tail -20 gpurun_out/$TAG/exp.err; exit 1; }
cat gpurun_out/$TAG/exp.json
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --aux c5 --no-recur --no-shadow --no-cpu-baseline --steady-steps 0 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -20 gpurun_out/$TAG/bench.err; exit 1; }
python - <<PY
import json
d = json.loads([l for l in open("gpurun_out/$TAG/bench.json") if l.startswith("{")][-1])
c5 = d["config"]["aux_configs"]["c5_san_miguel_primary_4k"]
print(json.dumps({k: c5.get(k) for k in ("trace_ms", "mrays_s", "two_parts_two_streams")}))
PY
