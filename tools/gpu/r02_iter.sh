# quick iteration on the GPU box: parity suite, long-ray latencies, short metric bench
# (no aux configs, no CPU baseline). Usage: bash tools/gpu/r02_iter.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-iter}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gputests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_gputests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/long_rays.py > gpurun_out/${TAG}_long.json 2> gpurun_out/${TAG}_long.err && grep long_rays gpurun_out/${TAG}_long.err &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --aux '' --no-cpu-baseline --no-shadow > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err && python -c "
import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); c=d['config']
print('VALUE', d['value'], 'prim', c['trace_ms_primary'], 'bnc', c['trace_ms_bounce'])"
