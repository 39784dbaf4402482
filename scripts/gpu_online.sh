# One GPU call: workspace/split-K GPU tests, serving GPU tests, then online
# serving (Poisson arrivals) at four request rates.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/online
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-900; echo "== $name rc=$rc"; return $rc; }
run tests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_serve_gpu.py tests/test_decode_gpu.py -x -v -k "splitk or serve or engine or paged" --timeout 120 --timeout-method thread || exit $?
for r in 64 4 16 32; do
  run rate$r 300 python -u -m kgs.serve bench --requests 256 --input-len 512 --output-len 256 --max-batch 256 --max-model-len 2048 --request-rate $r || exit $?
done
