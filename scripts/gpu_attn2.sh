# One GPU call: attention numerics + microbench, b64 serving.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/attn2
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -7 $O/$name.log; echo "== $name rc=$rc"; return $rc; }
run dbg 200 python scripts/attn_dbg.py && \
run tests 300 python -u -m pytest tests/test_decode_gpu.py -x -q -k "paged or rope" --timeout 200 --timeout-method thread && \
run attn 200 python -u bench/decode_bench.py --attn --iters 30 && \
run b64 300 python -u -m kgs.serve bench --requests 64 --input-len 512 --output-len 256 --max-batch 64 --max-model-len 2048
