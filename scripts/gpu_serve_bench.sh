# One GPU call: full offline serving benchmark (kgs engine vs HF transformers) + a kernel-trace profile.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/serve_bench
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -4 $O/$name.log; echo "== $name rc=$rc"; return $rc; }
run kgs_b256 400 python -u -m kgs.serve bench --requests 256 --input-len 512 --output-len 256 --max-batch 256 --max-model-len 2048 && \
run kgs_b64 300 python -u -m kgs.serve bench --requests 64 --input-len 512 --output-len 256 --max-batch 64 --max-model-len 2048 && \
run hf_b64 400 python -u -m kgs.serve bench --requests 64 --input-len 512 --output-len 256 --max-batch 64 --max-model-len 2048 --hf-only && \
run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o serve -- python3 -m kgs.serve bench --requests 64 --input-len 512 --output-len 64 --max-batch 64 --max-model-len 2048
