set -o pipefail
mkdir -p gpurun_out/probe2
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "repeatable" > gpurun_out/probe2/t.log 2>&1 && \
timeout -k 10 300 python - > gpurun_out/probe2/check.log 2>&1 <<'PY'
import torch
from kgs.ops import gemm_nt
for v in ("lockstep", "lockstep_1bar"):
    for (M, N, K) in ((2048, 2048, 2048), (1024, 3072, 4096)):
        a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16(); b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
        ref = gemm_nt(a, b, variant="fast")
        outs = [gemm_nt(a, b, variant=v) for _ in range(10)]
        print(v, M, N, K, all(torch.equal(o, ref) for o in outs))
PY
cat gpurun_out/probe2/check.log && \
timeout -k 10 300 python bench/gemm_sweep.py --shapes 8192,16384x16384x8192 --variants fast,lockstep,lockstep_1bar --rounds 7 --out gpurun_out/probe2/sweep.json > gpurun_out/probe2/sweep.log 2>&1; rc=$?
grep shape gpurun_out/probe2/sweep.log; exit $rc
