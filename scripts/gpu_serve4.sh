# One GPU call: decode + serving tests, then serving throughput: bf16 (fused 32 vs 64), fp8 KV at b256, b512.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/serve4
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -2 $O/$name.log; echo "== $name rc=$rc"; return $rc; }
B="python -u -m kgs.serve bench --input-len 512 --output-len 256 --max-model-len 2048"
run tests 400 python -u -m pytest tests/test_decode_gpu.py tests/test_serve_gpu.py -x -q --timeout 200 --timeout-method thread && \
run b64_f32 300 $B --requests 64 --max-batch 64 && \
run b64_f64 300 $B --requests 64 --max-batch 64 --fused-max-batch 64 && \
run b256 400 $B --requests 256 --max-batch 256 && \
run b256_kv8 400 $B --requests 256 --max-batch 256 --kv-cache-dtype fp8 && \
run b512 500 $B --requests 512 --max-batch 512 && \
run b1 300 $B --requests 2 --max-batch 1 && \
run b16 300 $B --requests 16 --max-batch 16
