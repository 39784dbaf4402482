"""rocprofv3 helpers (kgs.utils.profile): command shapes the GPU pool accepts and
the CSV -> markdown summary used for profiles/*.md."""
import csv
import os

from kgs.utils.profile import COUNTER_SETS, pmc_command, short, summarize, trace_command


def test_commands_put_the_program_right_after_dashdash():
    prog = ["python3", "-m", "kgs.workload.worker"]
    for cmd in (pmc_command(prog, "/tmp/o", COUNTER_SETS["pipe"]), trace_command(prog, "/tmp/o")):
        assert cmd[0] == "rocprofv3"
        assert cmd[cmd.index("--") + 1:] == prog  # no env/bash hop before the program
    pmc = pmc_command(prog, "/tmp/o", COUNTER_SETS["mfma"])
    # counters are never combined with tracing in one pass
    assert not any(f in pmc for f in ("--kernel-trace", "--sys-trace", "-s", "--runtime-trace", "-r"))
    assert "--pmc" not in trace_command(prog, "/tmp/o")


def test_counter_sets_fit_the_pmc_slots():
    for name, cs in COUNTER_SETS.items():
        sq = [c for c in cs if c.startswith("SQ_")]
        tcc = [c for c in cs if c.startswith("TCC_")]
        assert len(sq) <= 8 and len(tcc) <= 4, name  # gfx950 per-pass slots (MI355X_MICROARCH.md)


def test_short_names():
    assert short("void kgs::g256::gemm_nt_256<0, 7>(unsigned short const*)").startswith("kgs gemm_nt_256")
    assert short("Custom_Cijk_Alik_Bljk_BBS_BH_MT256x256x64").startswith("hipBLASLt")


def _write(path, header, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows)


def test_summarize_trace_and_counters(tmp_path):
    k = "void kgs::g256::gemm_nt_256<0, 7>(unsigned short const*)"
    _write(str(tmp_path / "trace" / "g_kernel_trace.csv"),
           ["Kernel_Name", "Start_Timestamp", "End_Timestamp", "VGPR_Count", "Accum_VGPR_Count", "LDS_Block_Size",
            "Workgroup_Size", "Grid_Size"],
           [[k, 0, 700000, 216, 0, 131072, 512, 524288], [k, 0, 710000, 216, 0, 131072, 512, 524288]])
    _write(str(tmp_path / "pmc1" / "g_counter_collection.csv"), ["Kernel_Name", "Counter_Name", "Counter_Value"],
           [[k, "SQ_VALU_MFMA_BUSY_CYCLES", 1.0e9], [k, "GRBM_GUI_ACTIVE", 1.0e7],
            [k, "SQ_LDS_BANK_CONFLICT", 0], [k, "SQ_LDS_IDX_ACTIVE", 1.0e8],
            [k, "TCC_HIT_sum", 80], [k, "TCC_MISS_sum", 20]])
    md = summarize(str(tmp_path))
    assert "| 2 | 0.7050 | 0.7000 |" in md           # dispatches, median ms, min ms
    assert "1560 |" in md                              # 2*8192^3 / 0.705 ms
    assert "MFMA busy/SIMD vs GPU cycles 78.1%" in md  # 1e9 / 1024 / (1e7 / 8)
    assert "LDS conflict cycles 0.0% of LDS active" in md and "L2 hit 80.0%" in md


def _trace(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for name, s, e in rows:
            w.writerow({"Kernel_Name": name, "Start_Timestamp": s, "End_Timestamp": e})


def test_step_idle_counts_only_gaps_no_kernel_covers(tmp_path):
    """bench/step_idle.py: a step's idle time is its period minus the UNION
    of kernel and copy intervals (overlapping kernels on two streams are not
    counted twice, a gap between them is)."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("step_idle", os.path.join(os.path.dirname(__file__), "..", "bench",
                                                                            "step_idle.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    p = tmp_path / "t.csv"
    # step 1 ends at 1000 ns; step 2: kernels [1500, 3000] and [2000, 4000] overlap, then a 1000 ns gap,
    # then [5000, 6000], then its argmax [6000, 7000]
    _trace(p, [("kgs::tfm::argmax_rows", 0, 1000), ("a", 1500, 3000), ("b", 2000, 4000), ("c", 5000, 6000),
               ("kgs::tfm::argmax_rows", 6000, 7000)])
    period, idle = mod.step_idle(str(p), 10)
    assert period == [6.0] and idle == [1.5]  # 500 ns before "a" + 1000 ns between "b" and "c", in us


def test_isa_diff_normalises_block_labels():
    """bench/isa_diff.py: two assemblies that differ only in basic-block
    label numbers (a kernel added before them renumbers the labels) compare
    equal; a changed instruction does not."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("isa_diff", os.path.join(os.path.dirname(__file__), "..", "bench",
                                                                           "isa_diff.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    a = "_Z1kv:  ; @k\n\ts_mov_b32 s0, 1\n.LBB0_2:\n\ts_cbranch_scc1 .LBB0_2 ; loop\n.Lfunc_end0:\n"
    b = "_Z1kv:  ; @k\n\ts_mov_b32 s0, 1\n.LBB7_2:\n\ts_cbranch_scc1 .LBB7_2\n.Lfunc_end7:\n"
    c = "_Z1kv:  ; @k\n\ts_mov_b32 s0, 2\n.LBB0_2:\n\ts_cbranch_scc1 .LBB0_2\n.Lfunc_end0:\n"
    ka, kb, kc = mod.kernels(a), mod.kernels(b), mod.kernels(c)
    assert list(ka) == ["_Z1kv"] and ka == kb and ka != kc
