# One GPU call: online serving sweep (Poisson arrivals), chunked prefill 2048 (the server default).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/online_sweep
mkdir -p $O
for r in 8 16 32 48 64 96; do
  timeout -k 10 240 python -u -m kgs.serve bench --requests 256 --input-len 512 --output-len 256 --max-batch 256 --max-model-len 2048 --request-rate $r --chunked-prefill 2048 > $O/rate$r.log 2>&1 || exit $?
  tail -1 $O/rate$r.log | cut -c1-400
done
