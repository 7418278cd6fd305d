set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh prof pmc
