# Drain-phase hoisted node test (TT_WIDE_HOIST): A/B on C2 (+ the UseReCur launch), C4, the C5 4K
# one-launch frame (MaxBounce = 1: the degenerate-ray tail) and the C2 two-part step.
# Usage: bash tools/gpu/r03_hoist.sh TAG v1 v2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
mkdir -p gpurun_out/$TAG
V=truetrace-unity-pathtracer_amd/lib/variants
RV_RECUR=1 timeout -k 10 400 python -u tools/run_variants.py "$@" "$@" > gpurun_out/$TAG/rv_c2.txt 2>&1 || { tail -5 gpurun_out/$TAG/rv_c2.txt; exit 1; }
cat gpurun_out/$TAG/rv_c2.txt
RV_CFG=c4 timeout -k 10 400 python -u tools/run_variants.py "$@" > gpurun_out/$TAG/rv_c4.txt 2>&1 || { tail -5 gpurun_out/$TAG/rv_c4.txt; exit 1; }
cat gpurun_out/$TAG/rv_c4.txt
for v in "$@" "$@"; do
  TT_HIP_LIB=$PWD/$V/libtruetrace_hip_$v.so timeout -k 10 300 python -u tools/exp_c5_list_order.py --config c5 --max-bounce 1 --only swizzle,swizzle_info --rounds 2 > gpurun_out/$TAG/c5_$v.json 2> gpurun_out/$TAG/c5_$v.err || { tail -5 gpurun_out/$TAG/c5_$v.err; exit 1; }
  echo "== c5 $v $(python -c "import json; d=json.load(open('gpurun_out/$TAG/c5_$v.json')); print(d['identical_to_swizzle'], d['ms_median'])")"
done
for v in "$@" "$@"; do
  TT_HIP_LIB=$PWD/$V/libtruetrace_hip_$v.so timeout -k 10 300 python -u tools/exp_order.py --config c2 --parts 2 --rounds 1 --steps 60 > gpurun_out/$TAG/p2_$v.json 2> gpurun_out/$TAG/p2_$v.err || { tail -5 gpurun_out/$TAG/p2_$v.err; exit 1; }
  echo "== c2 parts 2 $v $(grep -v amdgpu.ids gpurun_out/$TAG/p2_$v.err)"
done
