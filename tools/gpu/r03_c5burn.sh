# C5 one-launch time under sustained load (clock / power drift). Usage: bash tools/gpu/r03_c5burn.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-c5burn}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u tools/exp_c5_list_order.py --config c5 --only swizzle,swizzle_info > gpurun_out/$TAG/c5.json 2> gpurun_out/$TAG/c5.err || { tail -20 gpurun_out/$TAG/c5.err; exit 1; }
cat gpurun_out/$TAG/c5.json
for extra in "--parts 1" "--no-single"; do
  n=b_${extra//[- ]/_}
  timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --aux c5 --no-recur --no-shadow --no-cpu-baseline --steady-steps 0 $extra > gpurun_out/$TAG/$n.json 2> gpurun_out/$TAG/$n.err || { tail -20 gpurun_out/$TAG/$n.err; exit 1; }
  python - <<PY
import json
d = json.loads([l for l in open("gpurun_out/$TAG/$n.json") if l.startswith("{")][-1])
c5 = d["config"]["aux_configs"]["c5_san_miguel_primary_4k"]
print("$extra", json.dumps({k: c5.get(k) for k in ("trace_ms", "mrays_s")}))
PY
done
