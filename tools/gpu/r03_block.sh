# Block-size experiment: 256 (cur) vs 128 vs 64-thread persistent blocks. run_variants (single stream +
# strided oracle check) on C2 / C4, then the two-part step (tools/exp_order.py "off" mode) per variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-block}
mkdir -p gpurun_out/$TAG
V=truetrace-unity-pathtracer_amd/lib/variants
timeout -k 10 400 python -u tools/run_variants.py cur b128 b64 cur b128 b64 > gpurun_out/$TAG/rv_c2.txt 2>&1 || { tail -5 gpurun_out/$TAG/rv_c2.txt; exit 1; }
cat gpurun_out/$TAG/rv_c2.txt
RV_CFG=c4 timeout -k 10 400 python -u tools/run_variants.py cur b128 b64 > gpurun_out/$TAG/rv_c4.txt 2>&1 || { tail -5 gpurun_out/$TAG/rv_c4.txt; exit 1; }
cat gpurun_out/$TAG/rv_c4.txt
for v in cur b128 b64; do
  TT_HIP_LIB=$PWD/$V/libtruetrace_hip_$v.so timeout -k 10 300 python -u tools/exp_order.py --config c2 --parts 2 --rounds 2 > gpurun_out/$TAG/p2_$v.json 2> gpurun_out/$TAG/p2_$v.err || { tail -5 gpurun_out/$TAG/p2_$v.err; exit 1; }
  echo "== c2 parts 2 $v"; grep -v amdgpu.ids gpurun_out/$TAG/p2_$v.err
done
