# persistent GEMM A/B (hybrid queue vs static walk); the same box ran the b256 decode trace in profiles/r3/decode/decode_step_breakdown_b256_r3.md
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
KT="gemm or standin" bash scripts/gpu.sh r3s8 kt || exit 1
SHAPES=8192,16384x16384x8192,8192x28672x4096,8192x6144x4096,4096x8192x14336 VARIANTS=fast,w4ps_0,w4_oneshot \
  bash scripts/gpu.sh r3s8 gemm_llm bench || exit 1
