# One GPU call: fp8 numerics, fp8 skinny tuning sweep, and b32 decode-step profiles (fused vs unfused bf16).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof_b32
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -3 $O/$name.log; echo "== $name rc=$rc"; return $rc; }
run tests 300 python -u -m pytest tests/test_decode_gpu.py -x -q -k "fp8 or fused" --timeout 200 --timeout-method thread && \
run tune_fp8 600 python -u bench/decode_bench.py --tune --fp8 --iters 20 --ms 1,16,32,64 && \
run fused 300 rocprofv3 --kernel-trace --output-format csv -d $O/fused -o d -- python3 -m kgs.serve bench --requests 32 --input-len 512 --output-len 64 --max-batch 32 --max-model-len 2048 && \
run unfused 300 rocprofv3 --kernel-trace --output-format csv -d $O/unfused -o d -- python3 -m kgs.serve bench --requests 32 --input-len 512 --output-len 64 --max-batch 32 --max-model-len 2048 --fused-max-batch 0
