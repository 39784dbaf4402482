# One GPU call: GPU test tier, smoke, 1-GPU bench (the round-end driver sequence).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/check
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -8 $O/$name.log; echo "== $name rc=$rc"; return $rc; }
run tests 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread && \
run smoke 300 python __graft_entry__.py smoke && \
run bench 300 python bench.py
