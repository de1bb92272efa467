# Adaptive dequeue order: its GPU tests, then tools/exp_order.py on C4 / C2 (1 and 2 parts);
# TT_ORDER_RECORD_ONLY=1 runs measure the cost-recording overhead alone.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-order}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_order.py -x -v --timeout 120 --timeout-method thread > gpurun_out/$TAG/order_tests.log 2>&1
rc=$?
tail -6 gpurun_out/$TAG/order_tests.log
[ $rc -eq 0 ] || exit $rc
for cp in "c4 1" "c2 1" "c2 2" "c4 2" "c4 1 rec" "c2 1 rec"; do
  set -- $cp
  if [ "$3" = rec ]; then export TT_ORDER_RECORD_ONLY=1; else unset TT_ORDER_RECORD_ONLY; fi
  timeout -k 10 300 python -u tools/exp_order.py --config $1 --parts $2 --rounds 2 > gpurun_out/$TAG/exp_$1_p$2$3.json 2> gpurun_out/$TAG/exp_$1_p$2$3.err || { tail -5 gpurun_out/$TAG/exp_$1_p$2$3.err; exit 1; }
  echo "== $1 parts $2 $3"; grep -v amdgpu.ids gpurun_out/$TAG/exp_$1_p$2$3.err
done
