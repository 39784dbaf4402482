# four-wave persistent fp8 GEMM: numerics, sweep vs the 8-wave kernel and hipBLASLt fp8, bench --dtype fp8
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s10; mkdir -p $O
KT="fp8 or persistent" bash scripts/gpu.sh r3s10 kt || exit 1
timeout -k 10 600 python bench/gemm_sweep.py --dtype fp8 --data normal \
  --shapes 8192,16384x16384x8192,8192x28672x4096,8192x6144x4096,4096x8192x14336,8192x4096x14336 \
  --variants fast,w4p --rounds 7 --out $O/fp8_sweep.json > $O/fp8_sweep.log 2>&1 || exit 1
grep shape $O/fp8_sweep.log | cut -c1-400
timeout -k 10 300 python bench.py --dtype fp8 > $O/bench_fp8.log 2>&1 || exit 1
tail -1 $O/bench_fp8.log | cut -c1-300
