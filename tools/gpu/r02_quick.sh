# a subset of the GPU parity suite: bash tools/gpu/r02_quick.sh "<pytest -k expression>"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "$1" --timeout 120 --timeout-method thread 2>&1 | tail -15
