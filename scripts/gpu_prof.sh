set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o gemm -- python3 bench/gemm_profile.py --iters 20 --torch > gpurun_out/prof/trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof/pmc1 -o gemm -- python3 bench/gemm_profile.py --iters 5 --torch > gpurun_out/prof/pmc1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof/pmc2 -o gemm -- python3 bench/gemm_profile.py --iters 5 --torch > gpurun_out/prof/pmc2.log 2>&1
rc=$?
find gpurun_out/prof -name "*.csv" | head -20
tail -5 gpurun_out/prof/*.log
exit $rc
