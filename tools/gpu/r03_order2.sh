# Adaptive order on strong-scaling shards (rank 0's tiles of an N-GPU C2 / C5 frame), then the default bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-order2}
mkdir -p gpurun_out/$TAG
for cp in "c2 1 8" "c2 2 8" "c2 1 4" "c5 1 8"; do
  set -- $cp
  timeout -k 10 300 python -u tools/exp_order.py --config $1 --parts $2 --ranks $3 --rounds 2 > gpurun_out/$TAG/exp_$1_p$2_r$3.json 2> gpurun_out/$TAG/exp_$1_p$2_r$3.err || { tail -5 gpurun_out/$TAG/exp_$1_p$2_r$3.err; exit 1; }
  echo "== $1 parts $2 ranks $3"; grep -v amdgpu.ids gpurun_out/$TAG/exp_$1_p$2_r$3.err
done
timeout -k 10 500 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
rc=$?
tail -c 300 gpurun_out/$TAG/bench.json
exit $rc
