# parity suite, full bench (aux + CPU baseline), ray-count sweep. Usage: bash tools/gpu/r02_full.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-full}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gputests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_gputests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err && python -c "
import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); c=d['config']
print('VALUE', d['value'], 'prim', c['trace_ms_primary'], 'bnc', c['trace_ms_bounce'], 'recur', c['aux_recur_unjittered'])" &&
timeout -k 10 300 python -u tools/ray_count_sweep.py > gpurun_out/${TAG}_sweep.json 2> gpurun_out/${TAG}_sweep.err && grep "\[sweep\]" gpurun_out/${TAG}_sweep.err
