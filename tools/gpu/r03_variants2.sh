# Variant A/B: run_variants (one launch per bounce + strided oracle check) on C2 and C4, then the C2
# two-part step (tools/exp_order.py "off" = the metric layout) per variant. Usage: r03_variants2.sh TAG v1 v2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
mkdir -p gpurun_out/$TAG
V=truetrace-unity-pathtracer_amd/lib/variants
timeout -k 10 400 python -u tools/run_variants.py "$@" "$@" > gpurun_out/$TAG/rv_c2.txt 2>&1 || { tail -5 gpurun_out/$TAG/rv_c2.txt; exit 1; }
cat gpurun_out/$TAG/rv_c2.txt
RV_CFG=c4 timeout -k 10 400 python -u tools/run_variants.py "$@" > gpurun_out/$TAG/rv_c4.txt 2>&1 || { tail -5 gpurun_out/$TAG/rv_c4.txt; exit 1; }
cat gpurun_out/$TAG/rv_c4.txt
for v in "$@" "$@"; do
  TT_HIP_LIB=$PWD/$V/libtruetrace_hip_$v.so timeout -k 10 300 python -u tools/exp_order.py --config c2 --parts 2 --rounds 1 --steps 60 > gpurun_out/$TAG/p2_$v.json 2> gpurun_out/$TAG/p2_$v.err || { tail -5 gpurun_out/$TAG/p2_$v.err; exit 1; }
  echo "== c2 parts 2 $v $(grep -v amdgpu.ids gpurun_out/$TAG/p2_$v.err)"
done
