# Hit-record stream: its GPU tests, the rehearsals (gloo 2/4 ranks on one GPU, RCCL size-1 tile path) and the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-hits}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_order.py tests/test_gpu_parts.py tests/test_bench_launch.py -x -q --timeout 200 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1
rc=$?
tail -3 gpurun_out/$TAG/tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu/r03_rehearse.sh $TAG || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
rc=$?
python -c "
import json; d=json.load(open('gpurun_out/$TAG/bench.json')); print('VALUE', d['value'], d['ms_per_step'])"
exit $rc
