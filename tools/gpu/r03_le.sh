set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/var
for lib in cur oldupd; do TT_HIP_LIB=truetrace-unity-pathtracer_amd/lib/variants/libtruetrace_hip_$lib.so timeout -k 10 200 python -u tools/update_bench.py 2>&1 | tail -1 | tee -a gpurun_out/var/update_bench.txt || exit 1; done
RV_CFG=c4 RV_RECUR=0 timeout -k 10 600 python -u tools/run_variants.py cur le1 le2 cur le1 le2 2>&1 | tee gpurun_out/var/le_c4.txt || exit 1
RV_CFG=c2 RV_RECUR=0 timeout -k 10 300 python -u tools/run_variants.py cur le2 cur le2 2>&1 | tee gpurun_out/var/le_c2.txt
