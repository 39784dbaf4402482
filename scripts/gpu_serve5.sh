# One GPU call: serving GPU tests, then kgs.serve at batch 128 / 256 / 512
# with the split-K routing.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/serve5
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-900; echo "== $name rc=$rc"; return $rc; }
run tests 300 python -u -m pytest tests/test_serve_gpu.py tests/test_kernels_gpu.py -x -v -k "serve or engine or splitk" --timeout 120 --timeout-method thread && \
run b256 300 python -u -m kgs.serve bench --requests 256 --input-len 512 --output-len 256 --max-batch 256 --max-model-len 2048 && \
run b128 300 python -u -m kgs.serve bench --requests 128 --input-len 512 --output-len 256 --max-batch 128 --max-model-len 2048 && \
run b512 400 python -u -m kgs.serve bench --requests 512 --input-len 512 --output-len 256 --max-batch 512 --max-model-len 2048
