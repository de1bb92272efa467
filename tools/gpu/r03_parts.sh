# Parts per rank with one-wave blocks: rank 0's shard of an N-GPU C2 frame (strong scaling) in 2 vs 3 parts.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-parts}
mkdir -p gpurun_out/$TAG
for cp in "2 8" "3 8" "2 4" "3 4" "2 8" "3 8"; do
  set -- $cp
  timeout -k 10 300 python -u tools/exp_order.py --config c2 --parts $1 --ranks $2 --rounds 2 > gpurun_out/$TAG/p$1_r$2.json 2> gpurun_out/$TAG/p$1_r$2.err || { tail -5 gpurun_out/$TAG/p$1_r$2.err; exit 1; }
  echo "== parts $1 ranks $2"; grep -v amdgpu.ids gpurun_out/$TAG/p$1_r$2.err
done
