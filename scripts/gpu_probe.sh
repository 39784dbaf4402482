set -o pipefail
mkdir -p gpurun_out/probe
timeout -k 10 300 python bench/gemm_sweep.py --shapes 8192,16384x16384x8192 --variants fast,probe_l2,probe_2xmfma --rounds 7 --out gpurun_out/probe/sweep.json > gpurun_out/probe/sweep.log 2>&1; rc=$?
grep shape gpurun_out/probe/sweep.log; exit $rc
