# fp8 four-wave persistent kernel: maps (tall mirror / long-K G8) and schedule knobs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s11; mkdir -p $O
KT="fp8" bash scripts/gpu.sh r3s11 kt || exit 1
timeout -k 10 600 python bench/gemm_sweep.py --dtype fp8 --data normal --shapes 8192,16384x16384x8192,8192x6144x4096 \
  --variants w4p,w4f8_0_12_12_2,w4f8_0_10_12_2,w4f8_0_16_24_1,w4f8_0_10_24_1,w4f8_0_12_20_2 --rounds 7 \
  --out $O/fp8_knobs.json > $O/fp8_knobs.log 2>&1 || exit 1
timeout -k 10 600 python bench/gemm_sweep.py --dtype fp8 --data normal \
  --shapes 4096x8192x14336,8192x4096x14336,8192x28672x4096,16384x4096x14336 \
  --variants w4p,fast,w4f8_8_12_24_1,w4f8_140000000_12_24_1,w4f8_0_12_24_1 --rounds 7 \
  --out $O/fp8_maps.json > $O/fp8_maps.log 2>&1 || exit 1
