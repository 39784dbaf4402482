set -o pipefail
# fp8 GEMM: numerics (all kernel tests, bf16 included: the kernel signature changed) + speed
O=gpurun_out/fp8
mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -x > $O/tests.log 2>&1; rc=$?; tail -25 $O/tests.log; [ $rc -eq 0 ] && \
timeout -k 10 600 python bench/gemm_sweep.py --dtype fp8 --shapes 4096,8192,16384x16384x8192,4000x4000x4000 --variants auto --rounds 5 --out $O/sweep.json > $O/sweep.log 2>&1; rc=$?
tail -8 $O/sweep.log; exit $rc
