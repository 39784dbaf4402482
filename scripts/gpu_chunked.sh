# One GPU call: chunked-prefill numerics (chunk attention + engine), then online
# serving with and without chunked prefill at 32 req/s.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/chunked
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-900; echo "== $name rc=$rc"; return $rc; }
run tests 300 python -u -m pytest tests/test_serve_gpu.py tests/test_kernels_gpu.py -x -v -k "chunk or engine or attention or splitk" --timeout 120 --timeout-method thread && \
run online_chunk 300 python -u -m kgs.serve bench --requests 256 --input-len 512 --output-len 256 --max-batch 256 --max-model-len 2048 --request-rate 32 --chunked-prefill 2048 && \
run online_chunk64 300 python -u -m kgs.serve bench --requests 256 --input-len 512 --output-len 256 --max-batch 256 --max-model-len 2048 --request-rate 64 --chunked-prefill 2048 && \
run offline_chunk 300 python -u -m kgs.serve bench --requests 256 --input-len 512 --output-len 256 --max-batch 256 --max-model-len 2048 --chunked-prefill 4096
