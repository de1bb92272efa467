set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "refit" --timeout 120 --timeout-method thread 2>&1 | tail -3 &&
timeout -k 10 300 python -u bench.py --steps 20 --aux refit --no-cpu-baseline --no-shadow > gpurun_out/refit_bench.json 2> gpurun_out/refit_bench.err && grep "aux refit" gpurun_out/refit_bench.err
