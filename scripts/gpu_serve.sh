# One GPU call: serving-engine GPU tests, then a short offline serving benchmark.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/serve
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -15 $O/$name.log; echo "== $name rc=$rc"; return $rc; }
run tests 400 python -u -m pytest tests/test_serve_gpu.py tests/test_decode_gpu.py -x -v --timeout 200 --timeout-method thread && \
run bench_small 500 python -u -m kgs.serve bench --requests 64 --input-len 512 --output-len 128 --max-batch 64 --max-model-len 2048
