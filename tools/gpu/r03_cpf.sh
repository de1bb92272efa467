# Child prefetch in the drain phase (TT_WIDE_CHILD_PREFETCH, LDS-destination loads): run_variants on C2 with the
# UseReCur launch (RV_RECUR=1), C4, then the C2 two-part step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-cpf}
mkdir -p gpurun_out/$TAG
V=truetrace-unity-pathtracer_amd/lib/variants
RV_RECUR=1 timeout -k 10 400 python -u tools/run_variants.py cur cpf cur cpf > gpurun_out/$TAG/rv_c2.txt 2>&1 || { tail -5 gpurun_out/$TAG/rv_c2.txt; exit 1; }
cat gpurun_out/$TAG/rv_c2.txt
RV_CFG=c4 timeout -k 10 400 python -u tools/run_variants.py cur cpf cur cpf > gpurun_out/$TAG/rv_c4.txt 2>&1 || { tail -5 gpurun_out/$TAG/rv_c4.txt; exit 1; }
cat gpurun_out/$TAG/rv_c4.txt
for v in cur cpf cur cpf; do
  TT_HIP_LIB=$PWD/$V/libtruetrace_hip_$v.so timeout -k 10 300 python -u tools/exp_order.py --config c2 --parts 2 --rounds 1 --steps 60 > gpurun_out/$TAG/p2_$v.json 2> gpurun_out/$TAG/p2_$v.err || { tail -5 gpurun_out/$TAG/p2_$v.err; exit 1; }
  echo "== c2 parts 2 $v $(grep -v amdgpu.ids gpurun_out/$TAG/p2_$v.err)"
done
