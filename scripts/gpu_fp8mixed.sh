# One GPU call: fp8 projections in mixed steps (numerics), online 32 req/s with them.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fp8mixed
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-600; echo "== $name rc=$rc"; return $rc; }
run tests 300 python -u -m pytest tests/test_serve_gpu.py -x -v -k "fp8_prefill" --timeout 200 --timeout-method thread && \
run online64 300 python -u -m kgs.serve bench --requests 256 --input-len 512 --output-len 256 --max-batch 256 --max-model-len 2048 --request-rate 64 --chunked-prefill 2048 --prefill-weights fp8
