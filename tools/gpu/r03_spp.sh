# spp (weak-scaling) multi-GPU layout: the 2-rank gloo self-launch test on one GPU, then the default
# N = 1 bench. Usage: bash tools/gpu/r03_spp.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-spp}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_bench_launch.py -m gpu -x -v --timeout 200 --timeout-method thread --durations=5 > gpurun_out/$TAG/launch_test.log 2>&1
rc=$?
tail -8 gpurun_out/$TAG/launch_test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
rc=$?
python -c "
import json; d=json.load(open('gpurun_out/$TAG/bench.json')); print('VALUE', d['value'], d['ms_per_step'], d['scaling'], d['config']['gather_identical_to_1gpu'])"
exit $rc
