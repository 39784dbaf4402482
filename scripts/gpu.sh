# One GPU-box call, assembled from named steps:
#
#   gpurun --timeout 1200 -- 'bash scripts/gpu.sh OUT step [step ...]'
#
# Parameters go in as environment variables (KT, SHAPES, VARIANTS, MNK, BATCHES, B, ...), e.g.
#   gpurun -- 'SHAPES=8192,4096 VARIANTS=fast,w4_oneshot bash scripts/gpu.sh r4x gemm_llm bench'
# -- one command line per experiment, no per-run wrapper scripts.
#
# Every step runs under its own `timeout -k 10`, logs to gpurun_out/OUT/<step>.log
# and the chain stops at the first failure (no retries, nothing after a fault).
# Counter passes (pmc_*) are separate rocprofv3 runs with --pmc only; they are
# never combined with tracing.
#
# Steps:
#   tests        full GPU pytest tier (per-test thread timeout)
#   smoke        __graft_entry__.smoke()
#   bench        python bench.py (driver defaults)
#   bench_long   sustained >=10 s run of the bench config (steps=400)
#   gemm_sweep   kgs vs hipBLASLt interleaved sweep of the headline shapes
#   gemm_trace   rocprofv3 kernel trace + stats of the GEMM profile driver
#   gemm_pmc     two counter passes over the GEMM (stall / MFMA busy)
#   overlap      GEMM vs comm-kernel overlap measurement (bench/overlap.py)
#   overlap_trace  kernel trace of the overlap run
#   counters_list  rocprofv3 -L (the counter names this box offers)
#   step_ab      the bench step under the persistent / one-shot / hipBLASLt paths, interleaved ($MNK);
#                step_ab_long: 3-second blocks (sustained clocks)
#   gateup_pmc   counter passes (SQ waits, FETCH_SIZE, TCC hit/miss, TA/TCP/TD stalls) + trace of the batch-256
#                gate|up kernel, default vs nt weight loads
#   serve_nt_ab  batch-$B serving with nt weight loads off / on / on + SwiGLU-packed gate|up, twice
#   serve_overlap_ab  batch-$B serving, sequential vs overlapped engine steps, twice
#   mall_probe   batch-256 decode projections with weights cold (HBM) vs hot (MALL)
#   serve_nt_rep the round-4 faulting serving configuration (nt on, output 256) x2, nt off, nt on traced
#   uninit_probe serving under allocator fill patterns 0 / 0x400 (uninitialised reads show as a difference)
#   serve_rep    batch-256 serving $N times back to back with step breadcrumbs (KGS_STEP_TRACE)
#   serve_tq     batch-256 serving, ticket pool checked after every step, with and without hipGraphs
#   prefix_regress  the graph-replay regression test against gpurun_ab/prefix (the pre-fix library)
#   overlap_rccl_ab persistent (static first ticket) vs one-shot grid against the RCCL-shaped CU hold
#   lib_ab       this tree's kernel library vs another build ($LIB_B), interleaved, five sweep shapes
#   fp8_sweep    kgs fp8 vs hipBLASLt fp8, N(0,1) operands ($SHAPES, $VARIANTS: e.g. w4f8_<X>_<B1>_<R>_<P> knobs)
#   overlap_variants  bench/overlap.py for the persistent and one-shot grids, stand-in LDS 0 / 64 KiB
#   gemm_waits   the persistent GEMM's wait-stamp build: lgkm / barrier / vm wait cycles per K-step category
#   p2p_staging  P2P all-reduce with cached vs uncached staging buffers, local ranks on one GPU
#   wait_split   SQ_WAIT_ANY vs K at 8192 x 8192 x K (persistent nt / deferred / one-shot / hipBLASLt): per-K-step
#                and fixed (tile change + launch) parts (bench/wait_split.py)
#   gemm_pmc2    kgs vs hipBLASLt at $MNK: SQ waits / MFMA busy, L2 hit-miss-DRAM, L1 latency / pending stalls
#   bench_trace  kernel trace of bench.py (GEMM durations and the gaps between them)
#   overlap_rccl GEMM first-ticket / grid policies vs an RCCL-shaped CU hold (normal and high-priority side stream)
#   serve        kgs.serve batch-256 serving bench (serve_nofuse: split-K reduces unfused)
#   decode_trace kernel trace of batch-256 decode (decode_trace_b1: batch 1; serve_b1: batch-1 serving)
#   e2e          kgs bench --no-kind chained tail (plugin -> pod -> first GEMM)
#   e2e_sweep    the same through `kgs bench --no-kind --sweep 1` (one point on a 1-GPU box)
#   gemm_l2      TCC hit/miss, FETCH_SIZE and kernel trace of kgs vs hipBLASLt at $MNK ($VAR: kgs variant)
#   stride_probe per-K-step time vs K and row stride, GROUP_M variants ($CASES, $VARIANTS)
#   gateup_probe decode gate|up + SwiGLU routing candidates vs hipBLASLt, HBM-streamed weights
#   gemm_llm     kgs vs hipBLASLt on the Llama-shaped GEMMs ($SHAPES overrides)
#   prefill      Llama-3-8B prefill, batch 4 x 2048 (kgs / torch / fp8); prefill_trace: its kernel trace
#   gpuinfo      kgs-gpuinfo --json (amd-smi + KFD views)
#   gemm_tail    per-workgroup start / per-tile end stamps of the persistent GEMM (head, tail, XCD spread)
#   w4x_sweep    decode-batch GEMM sweep (four-wave tiles, slices, stages vs hipBLASLt)
#   kt           GPU tests matching $KT (pytest -k)
#   memset_repro pure-HIP hipGraph memset-node check ($G graphs, $R replays, $P extra nodes; no torch);
#                memset_repro_torch: the same binary on torch's bundled HIP runtime
#   attn_bench   flash-attention forward vs SDPA
#   serve_b16    batch-16 serving; skinny_tune: skinny GEMM variant x split-K tune at batches $MS
#   online_sweep online serving (Poisson arrivals, 2048-row chunked steps) at 8-96 req/s
#   serve_sweep  offline serving at batch 1 / 64 / 128 / 256 / 512, fp8 KV, fp8 prefill + fp8 KV (256 and 512)
#   bench_fp8    bench.py --dtype fp8 (e4m3 operands, extra)
#   stages_probe LDS stages x tiles on the four decode projections
#   route_ab     128-row decode tiles probe, then serve_ab; serve_ab: batch-256 serving A/B/A with
#                $AENV / $BENV (one VAR=value each) and $ROUTES (KGS_W4X_ROUTES), trace of B
#   rope_attn_probe  rope_cache + attention vs the fused launch vs attention alone, with counters
#   attn_pmc     two counter passes over production attention and the w4 experiment (VALU / MFMA
#                busy and co-issue, waits; instruction mix, LDS)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${1:?usage: gpu.sh OUT step...}
shift
O=gpurun_out/$OUT
mkdir -p "$O"

run() {
    local name=$1 t=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    tail -3 "$O/$name.log" | cut -c1-900
    echo "== $name rc=$rc"
    return $rc
}

PMC_GEMM="python3 bench/gemm_profile.py --iters 5 --torch --mnk ${MNK:-8192} --variant ${VAR:-auto}"

step() {
    case "$1" in
        tests) KGS_EVIDENCE_DIR="$O" run tests 1100 python -u -m pytest tests -x -v -m gpu --timeout 120 \
            --timeout-method thread ;;
        smoke) run smoke 300 python __graft_entry__.py smoke ;;
        bench) run bench 300 python bench.py ;;
        bench_long) run bench_long 300 python bench.py --steps 4000 --warmup 20 ;;
        bench_fp8) run bench_fp8 300 python bench.py --dtype fp8 ;;
        gemm_sweep) run gemm_sweep 600 python bench/gemm_sweep.py --shapes 4096,8192,16384x16384x8192 \
            --variants fast --rounds 7 --out "$O/gemm_sweep.json" ;;
        gemm_trace) run gemm_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o gemm \
            -- python3 bench/gemm_profile.py --iters 20 --torch ;;
        attn_pmc) run attn_pmc1 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES \
            SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE \
            --output-format csv -d "$O/apmc1" -o attn -- python3 bench/attn_pmc_driver.py &&
            run attn_pmc2 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F SQ_INSTS_LDS \
            SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
            --output-format csv -d "$O/apmc2" -o attn -- python3 bench/attn_pmc_driver.py ;;
        gemm_pmc) run pmc_stall 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
            SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d "$O/pmc1" -o gemm -- $PMC_GEMM &&
            run pmc_mfma 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU \
            GRBM_GUI_ACTIVE --output-format csv -d "$O/pmc2" -o gemm -- $PMC_GEMM ;;
        overlap) run overlap 300 python bench/overlap.py --out "$O/overlap.json" ;;
        counters_list) run counters_list 120 rocprofv3 -L ;;
        step_ab) run step_ab 400 python bench/step_ab.py --mnk ${MNK:-8192} --paths ${PATHS:-fast,w4_oneshot,hipblaslt} \
            --out "$O/step_ab_${MNK:-8192}.json" ;;
        step_ab_long) run step_ab_long 600 python bench/step_ab.py --mnk ${MNK:-8192} --seconds 3 --rounds 5 \
            --paths ${PATHS:-fast,w4_oneshot,hipblaslt} \
            --out "$O/step_ab_long_${MNK:-8192}.json" ;;
        gateup_pmc)  # counter passes over the batch-256 gate|up + SwiGLU kernel (default vs nt weight loads)
            local GU="python3 bench/decode_gateup_probe.py --batches 256 --iters 30"
            GU="$GU --variants ${VARIANTS:-swiglu_bm256_bn128,swiglu_bm256_bn128_nt}"
            run gu_pmc_sq 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
                SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_MFMA GRBM_GUI_ACTIVE \
                GRBM_COUNT --output-format csv -d "$O/gu_pmc_sq" -o gu -- $GU &&
            run gu_pmc_fetch 120 timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE \
                --output-format csv -d "$O/gu_pmc_fetch" -o gu -- $GU &&
            run gu_pmc_tcc 120 timeout -s KILL 100 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum \
                TCC_EA0_RDREQ_DRAM_sum GRBM_GUI_ACTIVE --output-format csv -d "$O/gu_pmc_tcc" -o gu -- $GU &&
            run gu_pmc_ta 120 timeout -s KILL 100 rocprofv3 --pmc TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum \
                TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum \
                TCP_TCR_TCP_STALL_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE \
                --output-format csv -d "$O/gu_pmc_ta" -o gu -- $GU &&
            run gu_trace 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/gu_trace" -o gu -- $GU ;;
        serve_nt_ab)  # batch-$B serving: nt weight loads off / on / on + gate|up panels, A B C A B C
            local SB="python -u -m kgs.serve bench --requests ${B:-256} --input-len 512 --output-len 256"
            SB="$SB --max-batch ${B:-256} --max-model-len 2048"
            for r in 1 2; do
                (export KGS_NT_WEIGHTS=0 KGS_GATEUP_PANELS=0; run serve_nt0_$r 300 $SB) &&
                (export KGS_NT_WEIGHTS=1 KGS_GATEUP_PANELS=0; run serve_nt1_$r 300 $SB) &&
                (export KGS_NT_WEIGHTS=1 KGS_GATEUP_PANELS=1; run serve_nt1gp_$r 300 $SB) || return 1
            done ;;
        serve_overlap_ab)  # batch-$B serving: one step at a time vs overlapped steps (EngineConfig.overlap), A B A B
            local SB="python -u -m kgs.serve bench --requests ${B:-256} --input-len 512 --output-len 256"
            SB="$SB --max-batch ${B:-256} --max-model-len 2048"
            for r in 1 2; do
                run serve_seq_b${B:-256}_$r 300 $SB --overlap off &&
                run serve_ovl_b${B:-256}_$r 300 $SB || return 1
            done ;;
        mall_probe)  # each batch-256 decode projection (production route) with its weights cold (1.5 GB ring,
            # streamed from HBM) vs hot (two copies: MALL-resident where they fit)
            local P
            for P in qkv:pw4x_bm256_bn128_s4_nt o:pw4x_bm128_bn128_s4_nt down:pw4x_bm256_bn128_s8_nt \
                     gateup:pswiglu_bm256_bn128_nt; do
                run mall_${P%%:*}_cold 120 python bench/decode_gateup_probe.py --proj ${P%%:*} --batches 256 \
                    --variants ${P#*:} --iters 60 --ring-gb 1.5 &&
                run mall_${P%%:*}_hot 120 python bench/decode_gateup_probe.py --proj ${P%%:*} --batches 256 \
                    --variants ${P#*:} --iters 60 --ring-gb 0.001 || return 1
            done ;;
        host_phases)  # batch-256 serving, overlapped, per-step host phase times (KGS_HOST_PHASES); then with gc.freeze
            local SB="python -u -m kgs.serve bench --requests 256 --input-len 512 --output-len 256"
            SB="$SB --max-batch 256 --max-model-len 2048"
            (export KGS_HOST_PHASES=1 KGS_HOST_PHASES_OUT="$O/phases.json"; run host_phases 300 $SB) &&
            (export KGS_HOST_PHASES=1 KGS_HOST_PHASES_OUT="$O/phases_gcf.json"; run host_phases_gcf 300 $SB --gc-freeze) ;;
        lib_serve_ab)  # batch-256 serving and the Llama prefill bench: this tree's kernels vs $LIB_B, A B A B
            local SB="python -u -m kgs.serve bench --requests 256 --input-len 512 --output-len 256"
            SB="$SB --max-batch 256 --max-model-len 2048"
            for r in 1 2; do
                run serve_head_$r 300 $SB &&
                (export KGS_KERNELS_LIB=$LIB_B; run serve_libb_$r 300 $SB) || return 1
            done
            run prefill_head 300 python -u -m kgs.models.llama --backends kgs &&
            (export KGS_KERNELS_LIB=$LIB_B; run prefill_libb 300 python -u -m kgs.models.llama --backends kgs) ;;
        mall_prefetch) run mall_prefetch 300 python bench/mall_prefetch_probe.py --out "$O/mall_prefetch.json" ;;
        addc_ab)  # prompt-pass residual add in the GEMM store (KGS_PREFILL_ADDC) on / off: serving b256 + prefill bench
            local SB="python -u -m kgs.serve bench --requests 256 --input-len 512 --output-len 256"
            SB="$SB --max-batch 256 --max-model-len 2048"
            for r in 1 2; do
                (export KGS_PREFILL_ADDC=1; run serve_addc1_$r 300 $SB) &&
                (export KGS_PREFILL_ADDC=0; run serve_addc0_$r 300 $SB) &&
                (export KGS_PREFILL_ADDC=1; run prefill_addc1_$r 300 python -u -m kgs.models.llama --backends kgs) &&
                (export KGS_PREFILL_ADDC=0; run prefill_addc0_$r 300 python -u -m kgs.models.llama --backends kgs) ||
                    return 1
            done ;;
        rope_probe) run rope_probe 200 python bench/rope_cache_probe.py &&
            (export KGS_KERNELS_LIB=$LIB_B; run rope_probe_libb 200 python bench/rope_cache_probe.py) ;;
        serve_nt_rep)  # the round-4 faulting configuration (batch $B, output 256, nt on) twice, nt off,
            # then nt on under a kernel trace (the last dispatches name a faulting kernel)
            local SB="python -u -m kgs.serve bench --requests ${B:-256} --input-len 512 --output-len 256"
            SB="$SB --max-batch ${B:-256} --max-model-len 2048"
            (export KGS_NT_WEIGHTS=1; run serve_nt1_a 300 $SB) &&
            (export KGS_NT_WEIGHTS=1; run serve_nt1_b 300 $SB) &&
            (export KGS_NT_WEIGHTS=0; run serve_nt0_a 300 $SB) &&
            (export KGS_NT_WEIGHTS=1; run serve_nt1_trace 300 rocprofv3 --kernel-trace --stats --output-format csv \
                -d "$O/nt1_trace" -o d -- python3 -m kgs.serve bench --requests ${B:-256} --input-len 512 \
                --output-len 256 --max-batch ${B:-256} --max-model-len 2048) ;;
        uninit_probe)  # serving under two allocator fill patterns (bench/uninit_probe.py): must agree bitwise
            (export KGS_STEP_TRACE="$O/steps_u0.log"; run uninit_0 300 python bench/uninit_probe.py --pattern 0 \
                --out "$O/uninit_0.json") &&
            (export KGS_STEP_TRACE="$O/steps_u400.log"; run uninit_400 300 python bench/uninit_probe.py \
                --pattern 0x400 --out "$O/uninit_400.json") ;;
        serve_rep)  # the batch-256 serving bench $N times back to back (default policy), step breadcrumbs on
            local SB="python -u -m kgs.serve bench --requests 256 --input-len 512 --output-len 256"
            SB="$SB --max-batch 256 --max-model-len 2048"
            for r in $(seq 1 ${N:-3}); do
                (export KGS_STEP_TRACE="$O/steps_serve_$r.log" KGS_TQ_CHECK=1; run serve_rep_$r 300 $SB) || return 1
            done ;;
        serve_tq)  # batch-256 serving with the ticket pool checked after every step: graphs on, then off
            local SB="python -u -m kgs.serve bench --requests 256 --input-len 512 --output-len 32"
            SB="$SB --max-batch 256 --max-model-len 2048"
            # a Python error (rc 1: the pool check raised) still runs the eager leg; a fault or kill does not
            (export KGS_STEP_TRACE="$O/steps_tq_graphs.log" KGS_TQ_CHECK=1; run serve_tq_graphs 300 $SB)
            [ $? -le 1 ] &&
            (export KGS_STEP_TRACE="$O/steps_tq_eager.log" KGS_TQ_CHECK=1; run serve_tq_eager 300 $SB --no-graphs) ;;
        prefix_regress)  # the replay regression test against the pre-fix library (memset node): expected to fail
            (export KGS_KERNELS_LIB=gpurun_ab/prefix/libkgs_kernels.so
             run prefix_regress 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -k captured_persistent \
                --timeout 120 --timeout-method thread)
            [ $? -le 1 ] ;;  # 1 = the test failed (the point); a fault / kill still stops the chain
        overlap_rccl_ab) run overlap_rccl_ab 400 python bench/overlap_rccl.py --policies static,oneshot \
            --out "$O/overlap_rccl_ab.json" ;;
        lib_ab)  # two builds of libkgs_kernels.so interleaved in one process ($LIB_B, default the pre-pack build)
            run lib_ab 600 python bench/lib_ab.py --lib-b ${LIB_B:-gpurun_ab/prepack/libkgs_kernels.so} \
                --out "$O/lib_ab.json" ;;
        fp8_sweep) run fp8_sweep 600 python bench/gemm_sweep.py --dtype fp8 --data normal \
            --shapes ${SHAPES:-8192,16384x16384x8192,8192x28672x4096,8192x6144x4096,4096x8192x14336,8192x4096x14336} \
            --variants ${VARIANTS:-fast,w4p} --rounds 7 --out "$O/fp8_sweep.json" ;;
        overlap_variants)  # persistent vs one-shot GEMM against the comm stand-in, without / with 64 KiB LDS
            for v in auto w4_oneshot; do for l in 0 64; do
                run overlap_${v}_lds$l 200 python bench/overlap.py --variant $v --standin-lds-kb $l \
                    --out "$O/overlap_${v}_lds$l.json" || return 1
            done; done ;;
        gemm_pmc2)  # kgs vs hipBLASLt at $MNK: SQ waits + MFMA, L2 hit/miss + DRAM requests, L1 latency / stalls
            local G="python3 bench/gemm_profile.py --iters 10 --torch --mnk ${MNK:-8192} --variant ${VAR:-auto}"
            run g2_sq 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
                SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE \
                GRBM_COUNT --output-format csv -d "$O/g2_sq_${MNK:-8192}" -o g -- $G &&
            run g2_tcc 120 timeout -s KILL 100 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum \
                TCC_EA0_RDREQ_DRAM_sum GRBM_GUI_ACTIVE --output-format csv -d "$O/g2_tcc_${MNK:-8192}" -o g -- $G &&
            run g2_tcp 120 timeout -s KILL 100 rocprofv3 --pmc TA_BUSY_avr TCP_TCC_READ_REQ_sum \
                TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE \
                --output-format csv -d "$O/g2_tcp_${MNK:-8192}" -o g -- $G ;;
        gemm_waits) run gemm_waits 300 python bench/gemm_waits.py --shapes ${SHAPES:-8192,8192x4096x14336,16384x16384x8192} \
            --out "$O/gemm_waits.json" ;;
        p2p_staging) run p2p_staging 300 python bench/p2p_staging_ab.py --out "$O/p2p_staging_ab.json" ;;
        wait_split)  # SQ waits of the persistent GEMM vs K at a fixed tile grid: steady K-loop vs tile change
            local W="python3 bench/wait_split.py --plan $O/ws_plan.json"
            run ws_sq 240 timeout -s KILL 230 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
                SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE \
                GRBM_COUNT --output-format csv -d "$O/ws_sq" -o w -- $W &&
            run ws_sum 60 python3 bench/wait_split.py --summary "$O/ws_sq" --plan $O/ws_plan.json \
                --json "$O/wait_split.json" ;;
        bench_trace) run bench_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/btrace" -o b \
            -- python3 bench.py --steps 20 --warmup 5 ;;
        overlap_rccl) run overlap_rccl 300 python bench/overlap_rccl.py --out "$O/overlap_rccl_shape.json" &&
            run overlap_rccl_hi 300 python bench/overlap_rccl.py --side-priority high \
                --out "$O/overlap_rccl_shape_hiprio.json" ;;
        overlap_trace) run overlap_trace 300 rocprofv3 --kernel-trace --output-format csv -d "$O/otrace" -o ov \
            -- python3 bench/overlap.py --iters 3 ;;
        serve) run serve 400 python -u -m kgs.serve bench --requests 256 --input-len 512 --output-len 256 \
            --max-batch 256 --max-model-len 2048 ;;
        serve_nofuse) run serve_nofuse 400 python -u -m kgs.serve bench --requests 256 --input-len 512 \
            --output-len 256 --max-batch 256 --max-model-len 2048 --no-fuse-splitk ;;
        decode_trace) run decode_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/dtrace" -o d \
            -- python3 -m kgs.serve bench --requests 256 --input-len 512 --output-len ${OL:-32} --max-batch 256 \
            --max-model-len 2048 ${DT_FLAGS:-} ;;
        decode_trace_b1) run decode_trace_b1 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/dtrace1" \
            -o d -- python3 -m kgs.serve bench --requests 2 --input-len 512 --output-len 64 --max-batch 1 \
            --max-model-len 2048 ;;
        decode_trace_b64) run decode_trace_b64 300 rocprofv3 --kernel-trace --stats --output-format csv \
            -d "$O/dtrace64" -o d -- python3 -m kgs.serve bench --requests 64 --input-len 512 --output-len 32 \
            --max-batch 64 --max-model-len 2048 ;;
        decode_trace_b128) run decode_trace_b128 300 rocprofv3 --kernel-trace --stats --output-format csv \
            -d "$O/dtrace128" -o d -- python3 -m kgs.serve bench --requests 128 --input-len 512 --output-len 32 \
            --max-batch 128 --max-model-len 2048 ;;
        gateup_probe) run gateup_probe 400 python bench/decode_gateup_probe.py --batches ${BATCHES:-128,256,512} \
            --proj ${PROJ:-gateup} ${VARIANTS:+--variants $VARIANTS} --out "$O/gateup_probe_${PROJ:-gateup}.json" ;;
        paged_sweep) run paged_sweep 300 python bench/paged_split_sweep.py --batches ${BATCHES:-64,128,256} \
            --ctx ${CTX:-528} --splits ${SPLITS:-1,2,4} --pipe ${PIPE:-both} ;;
        serve_b1) run serve_b1 300 python -u -m kgs.serve bench --requests 2 --input-len 512 --output-len 256 \
            --max-batch 1 --max-model-len 2048 ;;
        serve_b1_f8) run serve_b1_f8 300 python -u -m kgs.serve bench --requests 2 --input-len 512 --output-len 256 \
            --max-batch 1 --max-model-len 2048 --decode-weights fp8 ;;
        serve_b16) run serve_b16 300 python -u -m kgs.serve bench --requests 16 --input-len 512 --output-len 256 \
            --max-batch 16 --max-model-len 2048 ;;
        skinny_tune) run skinny_tune 400 python bench/decode_bench.py --tune --ms "${MS:-1,16}" --iters 20 ;;
        attn_bench) run attn_bench 300 python bench/attention_bench.py ;;
        attn_pmc) run attn_pmc1 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
            SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d "$O/apmc1" -o attn \
            -- python3 bench/attention_bench.py --only attn --iters 5 &&
            run attn_pmc2 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU \
            SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d "$O/apmc2" -o attn \
            -- python3 bench/attention_bench.py --only attn --iters 5 ;;
        skinny_tune_70b) run skinny_tune_70b 500 python bench/decode_bench.py --tune --model llama3-70b --ms "${MS:-1,16}" --iters 10 ;;
        skinny_tune_fp8) run skinny_tune_fp8 400 python bench/decode_bench.py --tune --fp8 --ms "${MS:-1,16}" --iters 20 ;;
        prefill) run prefill 300 python -u -m kgs.models.llama --backends kgs,torch,fp8 ;;
        prefill_trace) run prefill_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ptrace" \
            -o p -- python3 -m kgs.models.llama --backends kgs --iters 2 ;;
        serve_prefill_trace)  # kernel trace of the serving bench's prompt pass (256 x 512 tokens, 2 output tokens)
            run serve_prefill_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/sptrace" -o p \
                -- python3 -m kgs.serve bench --requests 256 --input-len 512 --output-len 2 --max-batch 256 \
                --max-model-len 2048 &&
            python bench/prof_summary.py "$O/sptrace" > "$O/serve_prefill_summary.md" ;;
        e2e) run e2e 300 python -m kgs bench --no-kind --gpus 1 --timings-json "$O/e2e.json" ;;
        gemm_l2) # L2 hit/miss + HBM bytes of kgs vs hipBLASLt at $MNK (two counter passes) + a kernel trace
            local G="python3 bench/gemm_profile.py --mnk ${MNK:-8192x4096x14336} --iters 10 --torch --variant ${VAR:-auto}"
            run l2_hit 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv \
                -d "$O/l2_hit_${MNK:-8192x4096x14336}" -o g -- $G &&
            run l2_fetch 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv \
                -d "$O/l2_fetch_${MNK:-8192x4096x14336}" -o g -- $G &&
            run l2_trace 120 rocprofv3 --kernel-trace --stats --output-format csv \
                -d "$O/l2_trace_${MNK:-8192x4096x14336}" -o g -- $G ;;
        stride_probe) run stride_probe 600 python bench/gemm_stride_probe.py \
            --cases ${CASES:-8192x4096x14336,8192x4096x14336@16384,8192x4096x16384,8192x4096x8192,8192x8192x8192,4096x4096x4096} \
            --variants ${VARIANTS:-fast,w4h_1_24_20_1_2,w4h_1_24_20_1_8,w4h_1_24_20_1_16,w4h_1_24_20_1_32} \
            --out "$O/stride_probe.json" ;;
        e2e_sweep) run e2e_sweep 300 python -m kgs bench --no-kind --sweep 1 --sweep-json "$O/e2e_sweep.json" ;;
        gemm_power) run gemm_power 200 python bench/gemm_power.py --mnk ${MNK:-8192} --seconds 2 --rounds 2 \
            --out "$O/gemm_power.json" ;;
        fp8_tall) run fp8_tall 400 python bench/gemm_sweep.py --dtype fp8 --data normal \
            --shapes ${SHAPES:-8192x4096x14336,16384x4096x14336,4096x8192x14336,8192x28672x4096,8192} \
            --variants ${VARIANTS:-fast,gn4,gn8,gn2} --rounds 7 --out "$O/fp8_tall.json" ;;
        gemm_llm) run gemm_llm 600 python bench/gemm_sweep.py \
            --shapes ${SHAPES:-8192x4096x14336,4096,8192x28672x4096,8192x6144x4096,8192} \
            --variants ${VARIANTS:-fast} --rounds 7 --out "$O/gemm_llm.json" ;;
        gemm_tail) run gemm_tail 300 python bench/gemm_tail.py --shapes ${SHAPES:-8192,8192x4096x14336,16384x16384x8192} \
            --launches ${L:-20} --out "$O/gemm_tail.json" ;;
        gpuinfo) run gpuinfo 60 kgs/_native/kgs-gpuinfo --json ;;
        route_ab)  # 128-row tiles for the split-K decode projections at 192-384 rows, then serving A/B/A
            # with $ROUTES (KGS_W4X_ROUTES syntax) and a kernel trace of the B routes
            for P in o qkv down; do
                run rt_$P 300 python bench/decode_gateup_probe.py --proj $P --batches ${BATCHES:-192,256,384} \
                    --variants pw4x_bm256_bn128_s8,pw4x_bm256_bn128_s4,pw4x_bm128_bn128_s8,pw4x_bm128_bn128_s4,pw4x_bm128_bn128_s4_t4,pw4x_bm128_bn128_s2,pw4x_bm128_bn128_s2_t4 \
                    --out "$O/rt_$P.json" || return 1
            done && step serve_ab ;;
        serve_ab)  # batch-256 serving A/B/A: $AENV (e.g. KGS_ROPE_ATTN=0) vs $BENV / $ROUTES (KGS_W4X_ROUTES);
            # kernel trace of B. AENV / BENV: one VAR=value each (optional)
            local SA="python -u -m kgs.serve bench --requests 256 --input-len 512 --output-len 256 --max-batch 256 --max-model-len 2048"
            (export ${AENV:-KGS_AB=a}; run serve_a1 300 $SA) &&
            (export ${BENV:-KGS_AB=b}; [ -n "$ROUTES" ] && export KGS_W4X_ROUTES="$ROUTES"; run serve_b 300 $SA) &&
            (export ${AENV:-KGS_AB=a}; run serve_a2 300 $SA) &&
            (export ${BENV:-KGS_AB=b}; [ -n "$ROUTES" ] && export KGS_W4X_ROUTES="$ROUTES"
             run dtrace_b 300 rocprofv3 --kernel-trace --stats --output-format csv \
                -d "$O/dtrace_b" -o d -- python3 -m kgs.serve bench --requests 256 --input-len 512 --output-len 32 \
                --max-batch 256 --max-model-len 2048) ;;
        rope_attn_probe)  # two launches vs the fused rope+attention launch vs attention alone, then counters
            run rap 200 python bench/rope_attn_probe.py &&
            run rap_pmc_two 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES \
                SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --output-format csv -d "$O/pmc_two" -o rap \
                -- python3 bench/rope_attn_probe.py --variants two --iters 10 &&
            run rap_pmc_fused 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES \
                SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --output-format csv -d "$O/pmc_fused" -o rap \
                -- python3 bench/rope_attn_probe.py --variants fused --iters 10 ;;
        stages_probe)  # LDS stages (t2/t3/t4) x tiles on all four decode projections, HBM-streamed weights
            run st_gateup 300 python bench/decode_gateup_probe.py --batches ${BATCHES:-128,256} \
                --variants swiglu_bm256_bn128,swiglu_bm256_bn128_t3,pswiglu_bm256_bn128,pswiglu_bm256_bn128_t3,swiglu_bm128_bn128,swiglu_bm128_bn128_t3,swiglu_bm128_bn128_t4,swiglu_bm128_bn256_t3 \
                --out "$O/st_gateup.json" &&
            for P in down qkv o; do
                run st_$P 300 python bench/decode_gateup_probe.py --proj $P --batches ${BATCHES:-128,256} \
                    --variants pw4x_bm256_bn128_s8,pw4x_bm256_bn128_s8_t3,pw4x_bm256_bn128_s4,pw4x_bm256_bn128_s4_t3,pw4x_bm128_bn128_s8,pw4x_bm128_bn128_s8_t3,pw4x_bm128_bn128_s8_t4,pw4x_bm128_bn128_s4_t4,pw4x_bm128_bn128_s2_t4,hipblaslt \
                    --out "$O/st_$P.json" || return 1
            done ;;
        w4x_sweep) run w4x_sweep 600 python bench/decode_w4x_sweep.py --batches ${BATCHES:-128,256,512} \
            --shapes ${SHAPES:-qkv,o,gate_up,down} --out "$O/w4x_sweep.jsonl" ;;
        serve_sweep)
            local SB="python -u -m kgs.serve bench --input-len 512 --output-len 256 --max-model-len 2048"
            run serve_b1 300 $SB --requests 2 --max-batch 1 &&
                run serve_b16 300 $SB --requests 16 --max-batch 16 &&
                run serve_b64 300 $SB --requests 64 --max-batch 64 &&
                run serve_b128 300 $SB --requests 128 --max-batch 128 &&
                run serve_b256 300 $SB --requests 256 --max-batch 256 &&
                run serve_b512 300 $SB --requests 512 --max-batch 512 &&
                run serve_b256_kv8 300 $SB --requests 256 --max-batch 256 --kv-cache-dtype fp8 &&
                run serve_b256_f8 300 $SB --requests 256 --max-batch 256 --kv-cache-dtype fp8 --prefill-weights fp8 &&
                run serve_b512_f8 300 $SB --requests 512 --max-batch 512 --kv-cache-dtype fp8 --prefill-weights fp8 ;;
        panels_ab)  # tile-panel decode weights on / off, batch 128 and 256
            local SB="python -u -m kgs.serve bench --input-len 512 --output-len 256 --max-model-len 2048"
            run serve_b128_panels 300 $SB --requests 128 --max-batch 128 &&
                run serve_b128_rowmajor 300 $SB --requests 128 --max-batch 128 --no-w4x-panels &&
                run serve_b256_panels 300 $SB --requests 256 --max-batch 256 &&
                run serve_b256_rowmajor 300 $SB --requests 256 --max-batch 256 --no-w4x-panels ;;
        online_sweep)
            local OB="python -u -m kgs.serve bench --requests 256 --input-len 512 --output-len 256 --max-batch 256"
            OB="$OB --max-model-len 2048 --chunked-prefill 2048"
            run online_r8 300 $OB --request-rate 8 && run online_r16 300 $OB --request-rate 16 &&
                run online_r32 300 $OB --request-rate 32 && run online_r64 300 $OB --request-rate 64 &&
                run online_r96 300 $OB --request-rate 96 ;;
        online_overlap_ab)  # online serving (Poisson 32 req/s, chunked prefill): sequential vs overlapped steps, A B A B
            local OB="python -u -m kgs.serve bench --requests 256 --input-len 512 --output-len 256 --max-batch 256"
            OB="$OB --max-model-len 2048 --chunked-prefill 2048 --request-rate ${RATE:-32}"
            for r in 1 2; do
                run online_seq_$r 300 $OB --overlap off && run online_ovl_$r 300 $OB --overlap on || return 1
            done ;;
        memset_repro) run memset_repro 300 kgs/_native/kgs-graph-memset-repro ${G:-4} ${R:-200} ${P:-8} ;;
        memset_repro_torch)  # the same binary on torch's bundled HIP runtime (the one the serving engine used)
            local th=/tmp/kgs_torchhip
            mkdir -p $th && ln -sf "$(python3 -c 'import os, torch; print(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))')" $th/libamdhip64.so.7 &&
            LD_LIBRARY_PATH=$th${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} run memset_repro_torch 300 \
                kgs/_native/kgs-graph-memset-repro ${G:-4} ${R:-200} ${P:-8} ;;
        kt) run kt 600 python -u -m pytest tests -x -v -m gpu -k "$KT" --timeout 120 --timeout-method thread ;;
        *) echo "unknown step $1" >&2; return 2 ;;
    esac
}

for s in "$@"; do
    step "$s" || exit $?
done
