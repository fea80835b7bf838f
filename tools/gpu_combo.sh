set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=prof_r05a CONFIGS="cfg2" bash tools/gpu_profile.sh || exit 1
A=prio ROUNDS=3 bash tools/ab_bench.sh || exit 1
