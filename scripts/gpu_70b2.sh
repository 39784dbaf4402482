# One GPU call: Llama-3-70B serving with the 70B split-K routing (batch 64 / 256).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/l70b2
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-300; echo "== $name rc=$rc"; return $rc; }
run tests 300 python -u -m pytest tests/test_serve_gpu.py tests/test_kernels_gpu.py -x -v -k "unpacked or splitk" --timeout 200 --timeout-method thread && \
run b64 500 python -u -m kgs.serve bench --model llama3-70b --requests 64 --input-len 512 --output-len 128 --max-batch 64 --max-model-len 2048 && \
run b256 600 python -u -m kgs.serve bench --model llama3-70b --requests 256 --input-len 512 --output-len 128 --max-batch 256 --max-model-len 2048
