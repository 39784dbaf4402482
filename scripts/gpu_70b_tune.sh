# One GPU call: split-K vs hipBLASLt on the Llama-3-70B decode shapes, then
# 70B serving at batch 64 with fp8 (W8A16) packed decode weights.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/l70b_tune
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-900; echo "== $name rc=$rc"; return $rc; }
run wide 600 python -u bench/decode_bench.py --wide --model llama3-70b --ms 64,128,256 --iters 20 && \
run b64_fp8 600 python -u -m kgs.serve bench --model llama3-70b --requests 64 --input-len 512 --output-len 128 --max-batch 64 --max-model-len 2048 --decode-weights fp8
