set -o pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}"
export TMPDIR=/tmp
O=gpurun_out/r04j; mkdir -p $O
timeout -k 10 1000 python -u tools/strong_replay.py --configs c2,c5 --ns 1,2,4,8 --layouts 1x4,1x6 --steps 30 > $O/replay.json 2> $O/replay.err || exit $?
