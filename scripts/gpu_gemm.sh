set -o pipefail
mkdir -p gpurun_out/g
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/g/$name.log 2>&1; local rc=$?; tail -15 gpurun_out/g/$name.log; echo "== $name rc=$rc"; return $rc; }
run tests 600 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu && \
run sweep 600 python bench/gemm_sweep.py --shapes 4096,8192,8192x8192x16384,16384x16384x8192 --variants fast,pp2,w4 --rounds 7 --out gpurun_out/g/sweep.json
