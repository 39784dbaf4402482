set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3s5; mkdir -p $O
KT="gemm or standin or overlap" bash scripts/gpu.sh r3s5 kt || exit 1
for v in auto w4_oneshot; do for l in 0 64; do
  timeout -k 10 200 python bench/overlap.py --variant $v --standin-lds-kb $l --out $O/overlap_${v}_lds$l.json > $O/overlap_${v}_lds$l.log 2>&1 || exit 1
  tail -1 $O/overlap_${v}_lds$l.log | cut -c1-600
done; done
SHAPES=8192,16384x16384x8192,8192x4096x14336,4096x8192x14336,8192x28672x4096,4096 VARIANTS=fast,w4_oneshot bash scripts/gpu.sh r3s5 gemm_llm bench
