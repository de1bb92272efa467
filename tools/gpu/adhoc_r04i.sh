set -o pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}"
export TMPDIR=/tmp
O=gpurun_out/r04i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.out 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.out 2> $O/bench.err || exit $?
timeout -k 10 900 bash tools/profile_round.sh r04i > $O/prof.out 2> $O/prof.err || exit $?
timeout -k 10 400 python -u tools/strong_replay.py --configs c5 --ns 8 --ranks 2,3 --layouts 1x5,1x6,1x8 --steps 30 > $O/rep_c5.json 2> $O/rep_c5.err || exit $?
timeout -k 10 400 python -u tools/strong_replay.py --configs c2 --ns 8 --layouts 1x6 --steps 30 > $O/rep_c2.json 2> $O/rep_c2.err || exit $?
