set -o pipefail
# A/B probe of experimental GEMM variants against production. Usage: bash scripts/gpu_probe.sh VARIANT[,VARIANT...]
VARS=${1:-pl}
mkdir -p gpurun_out/probe3
true && \
timeout -k 10 300 python - "$VARS" > gpurun_out/probe3/check.log 2>&1 <<'PY'
import sys, torch
from kgs.ops import gemm_nt
ok = True
for v in sys.argv[1].split(","):
    for (M, N, K) in ((512, 512, 128), (2048, 2048, 2048), (1024, 3072, 4096)):
        a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16(); b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
        ref = gemm_nt(a, b, variant="fast")
        outs = [gemm_nt(a, b, variant=v) for _ in range(10)]
        good = all(torch.equal(o, ref) for o in outs)
        err = (outs[0].float() - ref.float()).abs().max().item()
        print(v, M, N, K, good, err, flush=True)
        ok &= good
sys.exit(0 if ok else 1)
PY
rc=$?; cat gpurun_out/probe3/check.log; [ $rc -eq 0 ] && \
timeout -k 10 300 python bench/gemm_sweep.py --shapes 4096,8192,16384x16384x8192,6144x12288x8192 --variants fast,$VARS --rounds 7 --out gpurun_out/probe3/sweep.json > gpurun_out/probe3/sweep.log 2>&1; rc=$?
grep shape gpurun_out/probe3/sweep.log; exit $rc
