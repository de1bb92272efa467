set -o pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}"
export TMPDIR=/tmp
O=gpurun_out/r04e; mkdir -p $O
V=truetrace-unity-pathtracer_amd/lib/variants
timeout -k 10 600 env TT_HIP_LIB=$V/libtruetrace_hip_idle.so python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_idle.out 2>&1 || exit $?
for i in 1 2; do for v in product idle; do
  lib=$V/libtruetrace_hip_$v.so; [ $v = product ] && lib=truetrace-unity-pathtracer_amd/lib/libtruetrace_hip.so
  timeout -k 10 300 env TT_HIP_LIB=$lib python -u bench.py --steps 20 --warmup 5 --aux "" --no-cpu-baseline --no-recur --no-shadow > $O/ab_${v}_$i.out 2> $O/ab_${v}_$i.err || exit $?
done; done
timeout -k 10 300 python -u tools/strong_replay.py --configs c2 --ns 8 --ranks 0,1,2,3 --layouts 1x3,2x1 --steps 30 > $O/rep_prod.json 2> $O/rep_prod.err || exit $?
timeout -k 10 300 env TT_HIP_LIB=$V/libtruetrace_hip_prio2.so python -u tools/strong_replay.py --configs c2 --ns 8 --ranks 0,1,2,3 --layouts 1x3,2x1 --steps 30 > $O/rep_prio2.json 2> $O/rep_prio2.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python -u tools/strong_replay.py --configs c2 --ns 8 --ranks 0,1 --layouts 1x3 --steps 30 > $O/rep_kt.json 2> $O/rep_kt.err || exit $?
