set -o pipefail
mkdir -p gpurun_out/p32
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/p32/$name.log 2>&1; local rc=$?; tail -8 gpurun_out/p32/$name.log; echo "== $name rc=$rc"; return $rc; }
run tests 600 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "p32 or fast" && \
run sweep 600 python bench/gemm_sweep.py --shapes 8192,4096,16384x16384x8192,8192x8192x2048 --variants fast,p32 --rounds 7 --out gpurun_out/p32/sweep.json
