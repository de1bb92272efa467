# GPU parity suite + default bench. Usage: bash tools/gpu/r03_check.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-chk}
mkdir -p gpurun_out/$TAG
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/gputests.log 2>&1
rc=$?
tail -3 gpurun_out/$TAG/gputests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
rc=$?
tail -c 600 gpurun_out/$TAG/bench.json
exit $rc
