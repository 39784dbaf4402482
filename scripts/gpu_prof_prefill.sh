# One GPU call: kernel trace of serving prefill (64 prompts x 512 tokens, 2 output tokens).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof_prefill
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o p -- python3 -m kgs.serve bench --requests 64 --input-len 512 --output-len 2 --max-batch 64 --max-model-len 2048 > $O/run.log 2>&1
rc=$?; tail -2 $O/run.log; find $O -name "*kernel_stats.csv" | head; exit $rc
