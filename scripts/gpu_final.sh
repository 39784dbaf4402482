# One GPU call at round end: full GPU tier, smoke, 1-GPU bench, serving b256
# (bf16 KV and fp8 KV).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/final
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -2 $O/$name.log | cut -c1-700; echo "== $name rc=$rc"; return $rc; }
run tests 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread && \
run smoke 300 python __graft_entry__.py smoke && \
run bench 300 python bench.py && \
run serve_b256 400 python -u -m kgs.serve bench --requests 256 --input-len 512 --output-len 256 --max-batch 256 --max-model-len 2048 && \
run serve_b256_fp8kv 400 python -u -m kgs.serve bench --requests 256 --input-len 512 --output-len 256 --max-batch 256 --max-model-len 2048 --kv-cache-dtype fp8
