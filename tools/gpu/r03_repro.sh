# Repro: the shadow random-soup test alone, then after the adaptive-order tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-repro}
mkdir -p gpurun_out/$TAG
timeout -k 10 200 python -u -m pytest "tests/test_gpu_parity.py::test_shadow_random_soup" -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/alone.log 2>&1
echo "alone rc=$?"; tail -2 gpurun_out/$TAG/alone.log
timeout -k 10 200 python -u -m pytest tests/test_gpu_order.py "tests/test_gpu_parity.py::test_shadow_random_soup" -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/after_order.log 2>&1
echo "after_order rc=$?"; tail -2 gpurun_out/$TAG/after_order.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_builder.py tests/test_gpu_configs.py "tests/test_gpu_parity.py::test_shadow_random_soup" -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/after_cfg.log 2>&1
echo "after_cfg rc=$?"; tail -2 gpurun_out/$TAG/after_cfg.log
exit 0
