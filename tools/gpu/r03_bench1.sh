# The driver's N = 1 bench (W = 5 / K = 20) once; prints value, step and roofline fields.
# Usage: bash tools/gpu/r03_bench1.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-b1}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -20 gpurun_out/$TAG/bench.err; exit 1; }
python - <<PY
import json
d = json.loads([l for l in open("gpurun_out/$TAG/bench.json") if l.startswith("{")][-1])
r = d["roofline"]
print(d["value"], d["ms_per_step"], r["frac"], json.dumps(r.get("step")))
PY
