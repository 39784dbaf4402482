# One GPU call: decode-kernel numerics, then the skinny-GEMM variant x split-K tuning sweep.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/tune
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -6 $O/$name.log; echo "== $name rc=$rc"; return $rc; }
run tests 300 python -u -m pytest tests/test_decode_gpu.py -x -v --timeout 120 --timeout-method thread && \
run tune 900 python -u bench/decode_bench.py --tune --iters 20 --ms 1,16,32,64,128,256 && run tune_fp8 600 python -u bench/decode_bench.py --tune --fp8 --iters 20 --ms 1,16,32,64
