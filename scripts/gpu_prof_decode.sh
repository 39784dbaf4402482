# One GPU call: kernel-trace profiles of batch-1 and batch-16 decode (fused layer).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof_decode
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -3 $O/$name.log; echo "== $name rc=$rc"; return $rc; }
run b1 300 rocprofv3 --kernel-trace --output-format csv -d $O/b1 -o d -- python3 -m kgs.serve bench --requests 1 --input-len 512 --output-len 64 --max-batch 1 --max-model-len 2048 && \
run b16 300 rocprofv3 --kernel-trace --output-format csv -d $O/b16 -o d -- python3 -m kgs.serve bench --requests 16 --input-len 512 --output-len 64 --max-batch 16 --max-model-len 2048
