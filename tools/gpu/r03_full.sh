# GPU parity suite, default bench, PMC unit passes (VALU-issue model for bench's roofline).
# Usage: bash tools/gpu/r03_full.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-full}
mkdir -p gpurun_out/$TAG
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/gputests.log 2>&1
rc=$?
tail -3 gpurun_out/$TAG/gputests.log
[ $rc -eq 0 ] || exit $rc
bash tools/pmc_units.sh gpurun_out/$TAG/pmcu > gpurun_out/$TAG/pmcu.log 2>&1 || { echo PMC_FAILED; tail gpurun_out/$TAG/pmcu.log; exit 1; }
tail -2 gpurun_out/$TAG/pmcu.log
cp gpurun_out/$TAG/pmcu/units.json profiles/units_latest.json
timeout -k 10 500 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
rc=$?
python -c "
import json; d=json.load(open('gpurun_out/$TAG/bench.json')); print('VALUE', d['value'], json.dumps(d['roofline'])[:900]); print(d['cpu_baseline'])"
exit $rc
