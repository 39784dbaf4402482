set -o pipefail
mkdir -p gpurun_out/g2
timeout -k 10 600 python bench/gemm_sweep.py --shapes 8192,4096,16384x16384x8192 --variants fast,pp2,pp2_noprio,pp2_gm4,pp2_gm16,pp2_gm2 --rounds 7 --out gpurun_out/g2/sweep.json > gpurun_out/g2/sweep.log 2>&1; rc=$?
cat gpurun_out/g2/sweep.log | grep shape
exit $rc
