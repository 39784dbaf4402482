# One GPU call: tests, smoke, bench, GEMM sweep, rocprofv3 trace + counters.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/round
mkdir -p $O
run() { local name=$1; shift; local t=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; tail -6 $O/$name.log; echo "== $name rc=$rc"; return $rc; }
run tests 900 python -m pytest tests -x -q -m gpu && \
run smoke 300 python __graft_entry__.py smoke && \
run bench 300 python bench.py && \
run sweep 600 python bench/gemm_sweep.py --shapes 4096,8192,16384x16384x8192 --variants fast,narrow_store --rounds 7 --out $O/sweep.json && \
run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o gemm -- python3 bench/gemm_profile.py --iters 20 --torch && \
run pmc1 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $O/pmc1 -o gemm -- python3 bench/gemm_profile.py --iters 5 --torch && \
run pmc2 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/pmc2 -o gemm -- python3 bench/gemm_profile.py --iters 5 --torch && \
run pmc3 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $O/pmc3 -o gemm -- python3 bench/gemm_profile.py --iters 5 --torch
