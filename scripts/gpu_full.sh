# One GPU call: full GPU test tier, smoke, 1-GPU bench, serving bench at batch 256.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/full
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -4 $O/$name.log; echo "== $name rc=$rc"; return $rc; }
run tests 900 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread && \
run smoke 300 python __graft_entry__.py smoke && \
run bench 300 python bench.py && \
run serve_b256 400 python -u -m kgs.serve bench --requests 256 --input-len 512 --output-len 256 --max-batch 256 --max-model-len 2048 && \
run wide 300 python -u bench/decode_bench.py --wide --ms 64,128,256,512 --iters 30
