# One GPU call: decode + serving GPU tests, then serving throughput at batch 1/16/64/256.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/serve2
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -3 $O/$name.log; echo "== $name rc=$rc"; return $rc; }
run tests 400 python -u -m pytest tests/test_decode_gpu.py tests/test_serve_gpu.py -x -v --timeout 200 --timeout-method thread && \
run kgs_b256 400 python -u -m kgs.serve bench --requests 256 --input-len 512 --output-len 256 --max-batch 256 --max-model-len 2048 && \
run kgs_b64 300 python -u -m kgs.serve bench --requests 64 --input-len 512 --output-len 256 --max-batch 64 --max-model-len 2048 && \
run kgs_b16 300 python -u -m kgs.serve bench --requests 16 --input-len 512 --output-len 256 --max-batch 16 --max-model-len 2048 && \
run kgs_b1 300 python -u -m kgs.serve bench --requests 2 --input-len 512 --output-len 256 --max-batch 1 --max-model-len 2048
