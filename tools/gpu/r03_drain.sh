set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/var
V=truetrace-unity-pathtracer_amd/lib/variants
RV_CFG=c2 RV_RECUR=1 timeout -k 10 600 python -u tools/run_variants.py cur at8 coop s11 cur at8 coop s11 2>&1 | tee gpurun_out/var/drain_c2.txt || exit 1
RV_CFG=c4 RV_RECUR=0 timeout -k 10 400 python -u tools/run_variants.py cur coop cur coop 2>&1 | tee gpurun_out/var/coop_c4.txt || exit 1
for v in cur at8; do TT_HIP_LIB=$V/libtruetrace_hip_$v.so timeout -k 10 300 python -u tools/ray_count_sweep.py > gpurun_out/var/sweep_$v.json 2> gpurun_out/var/sweep_$v.err || exit 1; grep "\[sweep\]" gpurun_out/var/sweep_$v.err | tail -3; done
