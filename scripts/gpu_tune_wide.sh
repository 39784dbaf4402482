# One GPU call: decode numerics (incl. the deep-chunk variants 20-23), serving
# GPU tests, then the variant x split-K sweep at batch 128 and 256.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/tune_wide
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -4 $O/$name.log; echo "== $name rc=$rc"; return $rc; }
run tests 400 python -u -m pytest tests/test_decode_gpu.py tests/test_serve_gpu.py -x -v --timeout 120 --timeout-method thread && \
run tune 900 python -u bench/decode_bench.py --tune --iters 20 --ms 128,256
