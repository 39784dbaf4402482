# One GPU call: decode-kernel numerics, then the decode microbenchmarks.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/decode
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -12 $O/$name.log; echo "== $name rc=$rc"; return $rc; }
run tests 300 python -u -m pytest tests/test_decode_gpu.py -x -v --timeout 120 --timeout-method thread && \
run bench 600 python -u bench/decode_bench.py --iters 30 --sweep --gemm --ms 1,8,16,32,48,64
