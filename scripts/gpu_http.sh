# One GPU call: kgs.serve over real HTTP (uvicorn server child process, 64
# concurrent streaming clients), default server settings and with prefix caching.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/http
mkdir -p $O
timeout -k 10 500 python -u bench/http_load.py --clients 64 --requests 256 --input-len 512 --output-len 128 --port 8011 --server-log $O/server_default.log --server-args "--max-batch 256 --max-model-len 2048" > $O/default.log 2>&1 && tail -1 $O/default.log | cut -c1-800 && \
timeout -k 10 500 python -u bench/http_load.py --clients 256 --requests 256 --input-len 512 --output-len 128 --port 8012 --server-log $O/server_c256.log --server-args "--max-batch 256 --max-model-len 2048" > $O/c256.log 2>&1 && tail -1 $O/c256.log | cut -c1-800
