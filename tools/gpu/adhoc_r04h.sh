set -o pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}"
export TMPDIR=/tmp
O=gpurun_out/r04h; mkdir -p $O
V=truetrace-unity-pathtracer_amd/lib/variants
timeout -k 10 400 env TT_HIP_LIB=$V/libtruetrace_hip_lp128.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_parts.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_lp128.out 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_bench_launch.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_launch.out 2>&1 || exit $?
for i in 1 2; do for v in product rlsetup lp128 lp64p2; do
  lib=$V/libtruetrace_hip_$v.so; [ $v = product ] && lib=truetrace-unity-pathtracer_amd/lib/libtruetrace_hip.so
  timeout -k 10 300 env TT_HIP_LIB=$lib python -u bench.py --steps 20 --warmup 5 --aux "" --no-cpu-baseline --no-shadow > $O/ab_${v}_$i.out 2> $O/ab_${v}_$i.err || exit $?
done; done
for v in product lp128 lp64p2 prio2; do
  lib=$V/libtruetrace_hip_$v.so; [ $v = product ] && lib=truetrace-unity-pathtracer_amd/lib/libtruetrace_hip.so
  timeout -k 10 400 env TT_HIP_LIB=$lib python -u tools/strong_replay.py --configs c5 --ns 8 --ranks 2,3 --layouts 1x3,1x4 --steps 30 > $O/rep_c5_$v.json 2> $O/rep_c5_$v.err || exit $?
done
timeout -k 10 400 python -u tools/strong_replay.py --configs c2 --ns 8 --layouts 1x4 --steps 30 > $O/rep_c2_prod.json 2> $O/rep_c2_prod.err || exit $?
