# One GPU call: split-K GEMM numerics, then its timing at decode batch sizes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/splitk
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -4 $O/$name.log; echo "== $name rc=$rc"; return $rc; }
run tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "splitk or bounded" --timeout 120 --timeout-method thread && \
run wide 600 python -u bench/decode_bench.py --wide --ms 128,256,512 --iters 30
