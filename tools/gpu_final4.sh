set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_run.sh tests smoke benchq
