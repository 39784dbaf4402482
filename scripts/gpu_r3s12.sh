# fp8 four-wave persistent kernel after the knob change (12 / 12 / 2): more knobs, bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s12; mkdir -p $O
KT="fp8" bash scripts/gpu.sh r3s12 kt || exit 1
timeout -k 10 600 python bench/gemm_sweep.py --dtype fp8 --data normal \
  --shapes 8192,16384x16384x8192,8192x6144x4096,8192x28672x4096 \
  --variants w4p,fast,w4f8_0_14_12_2,w4f8_0_12_8_3,w4f8_0_10_8_3,w4f8_0_12_6_4 --rounds 7 \
  --out $O/fp8_knobs2.json > $O/fp8_knobs2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --dtype fp8 > $O/bench_fp8.log 2>&1 || exit 1
tail -1 $O/bench_fp8.log | cut -c1-200
