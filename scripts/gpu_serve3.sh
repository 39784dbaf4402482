# One GPU call: decode + serving GPU tests, then fused vs unfused decode throughput.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/serve3
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -3 $O/$name.log; echo "== $name rc=$rc"; return $rc; }
run tests 400 python -u -m pytest tests/test_decode_gpu.py tests/test_serve_gpu.py -x -v --timeout 200 --timeout-method thread && \
run b64_fused 300 python -u -m kgs.serve bench --requests 64 --input-len 512 --output-len 256 --max-batch 64 --max-model-len 2048 && \
run b64_unfused 300 python -u -m kgs.serve bench --requests 64 --input-len 512 --output-len 256 --max-batch 64 --max-model-len 2048 --fused-max-batch 0 && \
run b16_fused 300 python -u -m kgs.serve bench --requests 16 --input-len 512 --output-len 256 --max-batch 16 --max-model-len 2048 && \
run b1_fused 300 python -u -m kgs.serve bench --requests 2 --input-len 512 --output-len 256 --max-batch 1 --max-model-len 2048
