# persistent GEMM: dynamic ticket queue vs static walk vs one-shot, same process
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
KT="gemm" bash scripts/gpu.sh r3s6 kt || exit 1
SHAPES=8192,16384x16384x8192,8192x28672x4096,8192x6144x4096 VARIANTS=fast,w4p_0,w4ps_0,w4_oneshot \
  bash scripts/gpu.sh r3s6 gemm_llm || exit 1
mv gpurun_out/r3s6/gemm_llm.json gpurun_out/r3s6/ab_square.json
SHAPES=4096x8192x14336,8192x4096x14336,16384x4096x14336 VARIANTS=fast,w4p_8,w4ps_8,w4p_140000008,w4ps_140000008,w4_oneshot \
  bash scripts/gpu.sh r3s6 gemm_llm || exit 1
mv gpurun_out/r3s6/gemm_llm.json gpurun_out/r3s6/ab_longk.json
