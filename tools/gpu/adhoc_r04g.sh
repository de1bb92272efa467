set -o pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}"
export TMPDIR=/tmp
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.out 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.out 2> $O/bench.err || exit $?
timeout -k 10 900 python -u tools/strong_replay.py --configs c2,c5 --ns 1,2,4,8 --layouts 1x3,2x1,3x1,2x2 --steps 30 > $O/replay.json 2> $O/replay.err || exit $?
timeout -k 10 600 bash tools/pmc_units.sh $O/pmcu > $O/pmcu.out 2> $O/pmcu.err || exit $?
