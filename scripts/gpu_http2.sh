# One GPU call: HTTP load with the engine in its own process (--engine-process).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/http2
mkdir -p $O
timeout -k 10 500 python -u bench/http_load.py --clients 64 --requests 256 --input-len 512 --output-len 128 --port 8013 --server-log $O/server_c64.log --server-args "--max-batch 256 --max-model-len 2048 --engine-process" > $O/c64.log 2>&1 && tail -1 $O/c64.log | cut -c1-800 && \
timeout -k 10 500 python -u bench/http_load.py --clients 256 --requests 256 --input-len 512 --output-len 128 --port 8014 --server-log $O/server_c256.log --server-args "--max-batch 256 --max-model-len 2048 --engine-process" > $O/c256.log 2>&1 && tail -1 $O/c256.log | cut -c1-800
