# 2-rank gloo rehearsal on one GPU with the C5 4K tile leg (aux_c5_tiles: one launch, two parts, two parts + adaptive order).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-c5t}
mkdir -p gpurun_out/$TAG
TT_BENCH_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 6 --warmup 2 --no-cpu-baseline --no-shadow --steady-steps 0 > gpurun_out/$TAG/c5t.json 2> gpurun_out/$TAG/c5t.err || { tail -5 gpurun_out/$TAG/c5t.err; exit 1; }
python -c "
import json; d=json.loads([l for l in open('gpurun_out/$TAG/c5t.json') if l.startswith('{')][-1]); print(json.dumps(d['config'].get('aux_c5_tiles')))"
