# GPU suite (indirect tests first) + the C4 work-order experiment (tools/exp_lpt.py --config c4).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-lpt}
mkdir -p gpurun_out/$TAG
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/gputests.log 2>&1
rc=$?
tail -3 gpurun_out/$TAG/gputests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/exp_lpt.py --config c4 > gpurun_out/$TAG/lpt_c4.json 2> gpurun_out/$TAG/lpt_c4.err
rc=$?
tail -3 gpurun_out/$TAG/lpt_c4.err
exit $rc
