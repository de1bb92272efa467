set -o pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}"
export TMPDIR=/tmp
O=gpurun_out/r04f; mkdir -p $O
V=truetrace-unity-pathtracer_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.out 2>&1 || exit $?
timeout -k 10 300 env TT_HIP_LIB=$V/libtruetrace_hip_pk.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_pk.out 2>&1 || exit $?
for i in 1 2; do for v in product pk pk5; do
  lib=$V/libtruetrace_hip_$v.so; [ $v = product ] && lib=truetrace-unity-pathtracer_amd/lib/libtruetrace_hip.so
  timeout -k 10 300 env TT_HIP_LIB=$lib python -u bench.py --steps 20 --warmup 5 --aux "" --no-cpu-baseline --no-recur --no-shadow > $O/ab_${v}_$i.out 2> $O/ab_${v}_$i.err || exit $?
done; done
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.out 2> $O/bench.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python -u tools/strong_replay.py --configs c2 --ns 8 --layouts 1x3,2x1 --steps 20 > $O/rep_kt.json 2> $O/rep_kt.err || exit $?
