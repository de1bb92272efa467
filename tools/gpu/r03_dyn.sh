# update-path tests + the C4 dynamic-frame bench leg
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/dyn
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "update or incremental or refit" --timeout 120 --timeout-method thread > gpurun_out/dyn/tests.log 2>&1
rc=$?; tail -3 gpurun_out/dyn/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --aux c4,dyn --no-cpu-baseline --no-recur --no-shadow --steady-steps 0 > gpurun_out/dyn/bench.json 2> gpurun_out/dyn/bench.err
rc=$?; grep "dynamic\|aux c4" gpurun_out/dyn/bench.err; exit $rc
