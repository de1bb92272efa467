set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/long_rays.py > gpurun_out/r02_long.json 2> gpurun_out/r02_long.err && echo LONG_OK
