# round-3 tree after the persistent GEMM: full GPU tier, smoke, driver-default bench, b256 serving
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu.sh r3s9 smoke tests bench serve
