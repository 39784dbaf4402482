# One GPU call: prefix-caching numerics, then offline/online serving with a
# 384-token shared system prompt (of 512), with and without prefix caching.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prefix
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-1200; echo "== $name rc=$rc"; return $rc; }
B="python -u -m kgs.serve bench --requests 256 --input-len 512 --output-len 256 --max-batch 256 --max-model-len 2048 --shared-prefix 384"
run tests 300 python -u -m pytest tests/test_serve_gpu.py -x -v --timeout 120 --timeout-method thread && \
run off_base 300 $B && \
run off_prefix 300 $B --prefix-caching --chunked-prefill 16384 && \
run on_base 300 $B --request-rate 32 --chunked-prefill 2048 && \
run on_prefix 300 $B --request-rate 32 --chunked-prefill 2048 --prefix-caching
