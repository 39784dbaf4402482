set -o pipefail
# bounded (ragged-shape) GEMM: numerics + speed vs the generic kernel and hipBLASLt
O=gpurun_out/bounded
mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -x > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] && \
timeout -k 10 600 python bench/gemm_sweep.py --shapes 8192,8000x8000x8000,4000x4000x4000,8192x8192x8200,12345x6784x4096 --variants bounded,generic --rounds 5 --out $O/sweep.json > $O/sweep.log 2>&1; rc=$?
grep shape $O/sweep.log; exit $rc
