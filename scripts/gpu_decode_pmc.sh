# One GPU call: decode kernels, kernel trace + two counter passes (each pass
# its own run; counters never combined with tracing).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/decode_pmc
rm -rf $O && mkdir -p $O
P="python3 bench/decode_profile.py"
timeout -k 10 -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o t -- $P > $O/trace.log 2>&1 && \
timeout -k 10 -s KILL 180 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_fetch -o f -- $P > $O/fetch.log 2>&1 && \
timeout -k 10 -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_mfma -o m -- $P > $O/mfma.log 2>&1 && \
python3 bench/decode_profile.py --summarize $O > $O/summary.md && cat $O/summary.md
