# Multi-rank rehearsals on one GPU: 2 and 4 ranks over gloo (ranks share the device; host-side
# collectives, so timings are not the RCCL path's), and the RCCL path with a size-1 communicator.
# Usage: bash tools/gpu/r03_rehearse.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-reh}
mkdir -p gpurun_out/$TAG
COMMON="--steps 5 --warmup 2 --no-cpu-baseline --no-shadow --steady-steps 0 --no-c5-tiles"
TT_BENCH_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 $COMMON > gpurun_out/$TAG/gloo2.json 2> gpurun_out/$TAG/gloo2.err || exit $?
echo gloo2 done
TT_BENCH_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 4 $COMMON > gpurun_out/$TAG/gloo4.json 2> gpurun_out/$TAG/gloo4.err || exit $?
echo gloo4 done
RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29531 TT_BENCH_RCCL_WORLD1=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-shadow --steady-steps 0 --aux '' --no-recur > gpurun_out/$TAG/rccl1.json 2> gpurun_out/$TAG/rccl1.err || exit $?
python - <<PY
import json
for f in ("gloo2", "gloo4", "rccl1"):
    d = json.loads([l for l in open(f"gpurun_out/$TAG/{f}.json") if l.startswith("{")][-1])
    c = d["config"]
    print(f, d["n_gpus"], d["scaling"], d["value"], d["ms_per_step"], c["samples_per_frame"], c["gather_identical_to_1gpu"],
          json.dumps(c.get("aux_strong_tiles")), json.dumps(c.get("aux_sample_sharded")))
PY
