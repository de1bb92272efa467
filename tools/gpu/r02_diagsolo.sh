set -o pipefail
cd "$GRAFT_REPO_ROOT"
TT_HIP_LIB=$PWD/truetrace-unity-pathtracer_amd/lib/variants/libtruetrace_hip_diagsolo.so timeout -k 10 120 python -u tools/solo_diag.py
