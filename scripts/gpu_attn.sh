# One GPU call: decode + serving GPU tests, attention microbench, b32/b64/b256 serving.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/attn
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -3 $O/$name.log; echo "== $name rc=$rc"; return $rc; }
run tests 400 python -u -m pytest tests/test_decode_gpu.py tests/test_serve_gpu.py -x -v --timeout 200 --timeout-method thread && \
run attn 200 python -u bench/decode_bench.py --attn --iters 30 && \
run b32 300 python -u -m kgs.serve bench --requests 32 --input-len 512 --output-len 256 --max-batch 32 --max-model-len 2048 && \
run b64 300 python -u -m kgs.serve bench --requests 64 --input-len 512 --output-len 256 --max-batch 64 --max-model-len 2048 && \
run b256 400 python -u -m kgs.serve bench --requests 256 --input-len 512 --output-len 256 --max-batch 256 --max-model-len 2048
