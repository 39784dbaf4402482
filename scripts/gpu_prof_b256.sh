# One GPU call: kernel-trace profile of batch-256 decode (bf16 and fp8 KV).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof_b256
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -2 $O/$name.log; echo "== $name rc=$rc"; return $rc; }
run b256 300 rocprofv3 --kernel-trace --output-format csv -d $O/b256 -o d -- python3 -m kgs.serve bench --requests 256 --input-len 512 --output-len 32 --max-batch 256 --max-model-len 2048
