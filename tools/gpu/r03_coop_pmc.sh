set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
V=truetrace-unity-pathtracer_amd/lib/variants
mkdir -p gpurun_out/pmc_cur gpurun_out/pmc_coop gpurun_out/var
for v in cur coop; do
  TT_HIP_LIB=$V/libtruetrace_hip_$v.so timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_$v -o p --output-format csv -- python bench.py --parts 1 --steps 2 --warmup 1 --steady-steps 0 --no-single --no-cpu-baseline --no-shadow --no-recur --aux '' > gpurun_out/pmc_$v/run.log 2>&1 || { mkdir -p gpurun_out/pmc_$v; echo FAIL $v; exit 1; }
done
python tools/pmc_compare.py cur=gpurun_out/pmc_cur coop=gpurun_out/pmc_coop | tee gpurun_out/var/coop_pmc.json
