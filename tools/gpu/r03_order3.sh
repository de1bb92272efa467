# Adaptive order on the primary launches only: C2 1/2 parts, C4 2 parts, C2 rank-0 shard of 8 in 3 parts.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-order3}
mkdir -p gpurun_out/$TAG
for cp in "c2 1 1" "c2 2 1" "c4 2 1" "c2 3 8" "c2 2 2"; do
  set -- $cp
  timeout -k 10 300 python -u tools/exp_order.py --config $1 --parts $2 --ranks $3 --rounds 2 --primary-only > gpurun_out/$TAG/exp_$1_p$2_r$3.json 2> gpurun_out/$TAG/exp_$1_p$2_r$3.err || { tail -5 gpurun_out/$TAG/exp_$1_p$2_r$3.err; exit 1; }
  echo "== $1 parts $2 ranks $3 primary-only"; grep -v amdgpu.ids gpurun_out/$TAG/exp_$1_p$2_r$3.err
done
