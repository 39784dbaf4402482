# One GPU call: decode + serving GPU tests, then bf16 vs fp8-weight decode throughput at batch 1/16/32.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fp8serve
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -3 $O/$name.log; echo "== $name rc=$rc"; return $rc; }
run tests 400 python -u -m pytest tests/test_decode_gpu.py tests/test_serve_gpu.py -x -v --timeout 200 --timeout-method thread && \
run b1_fp8 300 python -u -m kgs.serve bench --requests 2 --input-len 512 --output-len 256 --max-batch 1 --max-model-len 2048 --decode-weights fp8 && \
run b16_fp8 300 python -u -m kgs.serve bench --requests 16 --input-len 512 --output-len 256 --max-batch 16 --max-model-len 2048 --decode-weights fp8 && \
run b32_bf16 300 python -u -m kgs.serve bench --requests 32 --input-len 512 --output-len 256 --max-batch 32 --max-model-len 2048 && \
run b32_fp8 300 python -u -m kgs.serve bench --requests 32 --input-len 512 --output-len 256 --max-batch 32 --max-model-len 2048 --decode-weights fp8 && \
run b64_fp8 300 python -u -m kgs.serve bench --requests 64 --input-len 512 --output-len 256 --max-batch 64 --max-model-len 2048 --decode-weights fp8 --fused-max-batch 64
