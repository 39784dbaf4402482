set -o pipefail
mkdir -p gpurun_out
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -25 gpurun_out/$name.log; echo "== $name rc=$rc"; return $rc; }
run smoke 400 python __graft_entry__.py smoke && \
run tests 500 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu && \
run bench 300 python bench.py --steps 10 --warmup 3 --verify --compare-torch && \
run sweep 300 python bench/gemm_sweep.py --shapes 4096,8192
