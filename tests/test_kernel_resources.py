"""Compile-time resource guard for the production kernels (CPU: hipcc
cross-compiles gfx950 here). A VGPR spill in a hot kernel is a silent
performance regression -- the fp8 GEMM once lost 25 % to six spilled VGPRs
introduced by an unrelated scheduling fence -- so spills fail the suite."""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HIPCC = "/opt/rocm/bin/hipcc"

# The experiments translation unit alone takes about 10 minutes of hipcc; a test that waits on it
# gets its own budget instead of the suite's 600-s default.
pytestmark = [pytest.mark.skipif(not Path(HIPCC).exists() and shutil.which("hipcc") is None,
                                 reason="hipcc not available"),
              pytest.mark.timeout(1800)]


def _compile(src: str, odir: Path, save_temps: bool = False, subdir: str = "kernels") -> tuple[dict, str]:
    """Resource remarks per kernel (and, with save_temps, the device assembly)."""
    cmd = [HIPCC if Path(HIPCC).exists() else "hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c",
           "-I", str(ROOT / "native" / "kernels"),
           str(ROOT / "native" / subdir / src), "-o", str(odir / (src + ".o")),
           "-Rpass-analysis=kernel-resource-usage"]
    if save_temps:
        cmd.append("-save-temps=obj")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=1500, cwd=odir)
    assert out.returncode == 0, out.stderr[-2000:]
    res, name = {}, None
    for line in out.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
            res[name] = {}
            continue
        m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[bytes/\w+\])?: (\d+)", line)
        if m and name:
            res[name][m.group(1).strip()] = int(m.group(2))
    asm = ""
    if save_temps:
        (s_file,) = list(odir.glob(f"{Path(src).stem}-hip-amdgcn-amd-amdhsa-gfx950.s"))
        asm = s_file.read_text()
    return res, asm


def _resources(src: str, tmp_path) -> dict:
    return _compile(src, tmp_path)[0]


# The big translation units compile concurrently (one hipcc each, started together
# by the first fixture that needs any of them): the module's wall time is the
# slowest compile, not the sum.
_BUILDS = {"gemm_bf16.hip": ("kernels", True), "gemm_persistent.hip": ("kernels", True),
           "attention.hip": ("kernels", False), "gemm_w4h.hip": ("experiments", True)}


@pytest.fixture(scope="module")
def builds(tmp_path_factory):
    from concurrent.futures import ThreadPoolExecutor

    pool = ThreadPoolExecutor(len(_BUILDS))
    futs = {src: pool.submit(_compile, src, tmp_path_factory.mktemp(Path(src).stem), temps, sub)
            for src, (sub, temps) in _BUILDS.items()}
    yield futs
    pool.shutdown(wait=True)


@pytest.fixture(scope="module")
def gemm_build(builds):
    """gemm_bf16.hip (one-shot kernels) + gemm_persistent.hip (the persistent
    launcher), resources and assembly merged."""
    res, asm = {}, ""
    for src in ("gemm_bf16.hip", "gemm_persistent.hip"):
        r, a = builds[src].result()
        res.update(r)
        asm += a
    return res, asm


def test_gemm_production_kernels_do_not_spill(gemm_build):
    res, _ = gemm_build
    prod = [n for n in res if re.search(r"gemm_nt_256ILi[0-4]ELi(7|519|263)E", n)]
    prod += [n for n in res if re.search(r"gemm_nt_256ILi[0-2]ELi(1031|1543)E", n)]
    prod += [n for n in res if re.search(r"gemm_nt_256ILi[01]ELi(525319|525831)E", n)]
    prod += [n for n in res if "gemm_nt_w4" in n]
    assert len(prod) >= 19 + 10, list(res)[:20]
    bad = {n: r.get("VGPRs Spill") for n, r in res.items() if n in prod and r.get("VGPRs Spill", 0)}
    assert not bad, bad


def _functions(asm: str, pattern: str) -> dict:
    out = {}
    for m in re.finditer(r"\n(_Z\S+):", asm):
        if re.search(pattern, m.group(1)):
            out[m.group(1)] = asm[m.end():asm.find(".Lfunc_end", m.end())]
    return out


def test_four_wave_gemms_touch_agprs_only_through_named_asm(gemm_build):
    """The four-wave GEMMs keep their accumulators in NAMED AGPRs (acc_regs.h).
    Guard the two ways that went wrong before (gemm_w4.h header): the register
    allocator moving accumulators (any v_accvgpr_mov, or a v_accvgpr_write that
    is not the zero reset), and an AGPR read before the s_nop padding that
    follows the last MFMA (a stale fragment: the MFMA -> VALU hazard is not
    checked by hipcc for asm MFMAs)."""
    _, asm = gemm_build
    funcs = _functions(asm, r"gemm_nt_w4p?I|gemm_fp8_w4pI")
    assert len(funcs) >= 10 + 2 * 5 + 5, sorted(funcs)[:5]
    for name, body in funcs.items():
        lines = body.splitlines()
        assert not any("v_accvgpr_mov" in ln for ln in lines), name
        writes = [ln for ln in lines if "v_accvgpr_write" in ln]
        assert all(re.search(r"v_accvgpr_write_b32 a\d+, 0\b", ln) for ln in writes), (name, writes[:3])
        pads = [i for i, ln in enumerate(lines) if "s_nop 7" in ln]
        assert pads, name
        for i, ln in enumerate(lines):
            if "v_accvgpr_read" in ln:
                # every read follows a padding that follows every MFMA before it
                last_mfma = max((j for j in range(i) if "v_mfma" in lines[j]), default=-1)
                assert any(last_mfma < p < i for p in pads), (name, i, ln)


def test_attention_fits_two_workgroups_per_cu(builds):
    res = builds["attention.hip"].result()[0]
    (name, r), = [(n, r) for n, r in res.items() if "attn3fwd" in n]
    assert r.get("VGPRs Spill", 0) == 0
    assert r["VGPRs"] + r.get("AGPRs", 0) <= 256  # 2 waves / SIMD
    assert r["LDS Size"] <= 80 * 1024            # 2 workgroups / CU (160 KiB)


def test_persistent_gemm_k_loop_has_no_full_vmcnt_drain(gemm_build):
    """The persistent kernel's K-steps keep one K-tile of LDS-DMA in flight; a
    compiler-inserted ``s_waitcnt vmcnt(0)`` in the loop would drain it every
    K-step. Two ways it crept in while gemm_w4p.h was written: a second
    __shared__ object (LDS-DMA alias tracking then waits before every fragment
    read) and a uniform-address ticket atomic (the atomic optimizer's broadcast
    waits right after it). Only the prologue's and the exit's may remain."""
    _, asm = gemm_build
    funcs = _functions(asm, r"gemm_nt_w4pILi0E|gemm_fp8_w4pILi0E")
    assert len(funcs) >= 2
    for name, body in funcs.items():
        lines = body.splitlines()
        full = [i for i, ln in enumerate(lines)
                if re.search(r"s_waitcnt vmcnt\(0\)", ln) and "ASMSTART" not in lines[i - 1]]
        assert len(full) <= 3, (name, full)


def _stray_agpr_lines(body: str) -> tuple[int, list]:
    inside, stray, seen = False, [], 0
    for ln in body.splitlines():
        if "ASMSTART" in ln:
            inside = True
            continue
        if "ASMEND" in ln:
            inside = False
            continue
        code = ln.split(";")[0].strip()
        if not code or code.startswith("."):
            continue
        if re.search(r"(?<![\w.])a\[?\d+", code):
            if inside:
                seen += 1
            else:
                stray.append(code)
    return seen, stray


def test_experiment_persistent_gemms_never_touch_agprs_outside_asm(builds):
    """Round 6: a deferred-store build (gemm_w4p.h DD 6, SPS 4: 24 units of C
    held in VGPRs) reached 256 VGPRs and the allocator copied VGPRs into
    accumulator AGPRs (v_accvgpr_write a5, v3 ...): the MFMAs then overwrote
    them and the kernel faulted on the GPU (illegal address). Every persistent
    instance of the experiments library is held to the production rule, so an
    instance at the register limit fails here, on the CPU, not on a GPU box."""
    _, asm = builds["gemm_w4h.hip"].result()
    funcs = _functions(asm, r"gemm_nt_w4pI|gemm_fp8_w4pI")
    assert len(funcs) >= 40, len(funcs)
    for name, body in funcs.items():
        seen, stray = _stray_agpr_lines(body)
        assert seen >= 256, (name, seen)
        assert not stray, (name, stray[:5])


def test_named_agpr_kernels_never_touch_agprs_outside_asm(gemm_build):
    """KGS_ACC_RESERVE clobbers a0..a255 only at kernel entry, so
    after it the allocator could legally put an AV-class value, a spill or a
    direct AGPR load/store in an accumulator register and corrupt it. In the
    named-accumulator kernels (the persistent bf16 / fp8 GEMMs) no instruction
    outside an inline-asm block may name an a-register at all -- stricter than
    the mov/write check above, which misses compiler-emitted global_load /
    ds_read / VALU forms with AGPR operands."""
    _, asm = gemm_build
    funcs = _functions(asm, r"gemm_nt_w4pI|gemm_fp8_w4pI")
    assert len(funcs) >= 2 * 5 * 4, len(funcs)
    for name, body in funcs.items():
        inside, stray, seen = False, [], 0
        for ln in body.splitlines():
            if "ASMSTART" in ln:
                inside = True
                continue
            if "ASMEND" in ln:
                inside = False
                continue
            code = ln.split(";")[0].strip()
            if not code or code.startswith("."):
                continue
            if re.search(r"(?<![\w.])a\[?\d+", code):
                if inside:
                    seen += 1
                else:
                    stray.append(code)
        assert seen >= 256, (name, seen)  # the accumulators are there, through asm
        assert not stray, (name, stray[:5])


def _vregs(text: str) -> set:
    out = set()
    for a, b in re.findall(r"(?<![\w.])v\[(\d+):(\d+)\]", text):
        out |= set(range(int(a), int(b) + 1))
    out |= {int(a) for a in re.findall(r"(?<![\w.\[])v(\d+)\b", text)}
    return out


def _tr_read_hazards(body: str) -> list:
    """Instructions that name a VGPR an inline-asm ``ds_read_b64_tr_b16`` is
    still filling, i.e. before the next ``s_waitcnt`` with ``lgkmcnt(0)``
    (textual order; only lgkmcnt(0) retires the reads)."""
    pending, bad = set(), []
    for ln in body.splitlines():
        code = ln.split(";")[0].strip()
        if not code or code.startswith(".") or code.endswith(":"):
            continue
        if code.startswith("s_waitcnt") and "lgkmcnt(0)" in code:
            pending = set()
        elif code.startswith("ds_read_b64_tr_b16"):
            dst, addr = code.split(None, 1)[1].split(",", 1)
            if _vregs(addr) & pending:
                bad.append(code)
            pending |= _vregs(dst)
        elif _vregs(code) & pending:
            bad.append(code)
    return bad


def test_tr_read_hazard_check_catches_an_early_use():
    body = ("\tds_read_b64_tr_b16 v[10:11], v5\n\ts_waitcnt lgkmcnt(0)\n\tv_mov_b32 v20, v10\n"
            "\tds_read_b64_tr_b16 v[12:13], v5 offset:1024\n\tv_mov_b32 v21, v13\n\ts_waitcnt lgkmcnt(0)\n")
    assert _tr_read_hazards(body) == ["v_mov_b32 v21, v13"]


def test_transposed_layout_tr_reads_are_waited_before_use(gemm_build):
    """the transposed-layout GEMMs issue ds_read_b64_tr_b16 as inline
    asm (gemm_pipeline.h tr_frag), so hipcc's waitcnt pass does not know those
    VGPRs arrive asynchronously. Results are right only while no instruction
    touches a destination before phase()'s s_waitcnt lgkmcnt(0): a register
    copy of the shufflevector result, or an MFMA scheduled above the wait,
    would read a stale fragment. Checked on every build, every such kernel."""
    _, asm = gemm_build
    funcs = {n: b for n, b in _functions(asm, r".").items() if "ds_read_b64_tr_b16" in b}
    assert len(funcs) >= 8, len(funcs)  # A-, B- and AB-transposed layouts x epilogues
    for name, body in funcs.items():
        assert _tr_read_hazards(body) == [], name


def test_counted_store_wait_allows_only_the_epilogue_stores_and_k_tile_2(tmp_path):
    """gemm_w4p.h CST 3 (experiments `w4pw_0`): K-step 0 after an epilogue waits
    vmcnt(ND + stores) = vmcnt(48) for the next tile's K-tile-1 DMAs. That is right
    only if the 48 vector-memory ops issued just before the wait are this K-step's
    16 DMAs and the epilogue's 32 stores, with the K-tile-1 DMAs before them, and
    if the prologue drains both K-tiles (the first tile has no epilogue)."""
    src = tmp_path / "w4pw.hip"
    src.write_text('#include "gemm_w4p.h"\n'
                   "void launch(hipStream_t s, const unsigned short* a, const unsigned short* b, unsigned short* c,"
                   " int* q) {\n"
                   "  hipLaunchKernelGGL((kgs::w4p::gemm_nt_w4p<kgs::EPI_NONE, 0, 1, false, false, 300>), dim3(256),"
                   " dim3(256), 0, s, a, b, c, nullptr, 8192, 8192, 8192, 8192, 8192, 8192, q);\n}\n")
    out = subprocess.run([HIPCC if Path(HIPCC).exists() else "hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                          "-I", str(ROOT / "native" / "kernels"), "-c", str(src), "-o", str(tmp_path / "w.o"),
                          "-save-temps=obj"], capture_output=True, text=True, timeout=900, cwd=tmp_path)
    assert out.returncode == 0, out.stderr[-2000:]
    (s_file,) = list(tmp_path.glob("w4pw-hip-amdgcn-amd-amdhsa-gfx950.s"))
    lines = [ln.split(";")[0].strip() for ln in s_file.read_text().splitlines()]
    lines = [ln for ln in lines if ln]
    vmem = re.compile(r"^(buffer_|global_|flat_)")
    waits = [i for i, ln in enumerate(lines) if ln == "s_waitcnt vmcnt(48)"]
    assert len(waits) == 1, waits
    before = [ln for ln in lines[:waits[0]] if vmem.match(ln)]
    youngest = before[-48:]
    assert sum(ln.startswith("buffer_load_dwordx4") and ln.endswith(" lds") for ln in youngest) == 16
    assert sum(ln.startswith("global_store_dwordx4") for ln in youngest) == 32
    assert all(ln.startswith("buffer_load_dwordx4") and ln.endswith(" lds") for ln in before[-64:-48])  # K-tile 1
    # prologue: the first full drain comes after the first 32 DMAs (K-tiles 0 and 1) and before any store
    first_drain = lines.index("s_waitcnt vmcnt(0)", next(i for i, ln in enumerate(lines) if ln.endswith(" lds")))
    pro = [ln for ln in lines[:first_drain] if vmem.match(ln)]
    assert sum(ln.endswith(" lds") for ln in pro) == 32 and not any("store" in ln for ln in pro)


def _code_lines(body: str) -> list:
    out = []
    for ln in body.splitlines():
        code = ln.split(";")[0].strip()
        if code and not code.startswith(".") and not code.startswith("#"):
            out.append(code)
    return out


def _ar_protocol_violations(body: str, n_barriers: int) -> list:
    """Where the P2P all-reduce's cross-GPU ordering (allreduce_p2p.hip
    block_barrier) is missing from one kernel's ISA:
      * every flag store (system scope: ``global_store_dword ... sc0 sc1``) has
        a ``buffer_wbl2 sc0 sc1`` before it, since the last s_barrier, and an
        ``s_waitcnt vmcnt(0)`` between the two (the write-back finished), with
        no other store in between;
      * every flag poll (``global_load_dword ... sc0 sc1``) is followed by
        ``s_waitcnt vmcnt(0)``, then ``buffer_inv sc0 sc1``, then another
        ``s_waitcnt vmcnt(0)`` before the next s_barrier (no peer load first);
      * before every s_barrier, the last vector store / atomic since the
        previous one is retired by an ``s_waitcnt vmcnt(0)``."""
    lines = _code_lines(body)
    errs = []
    is_flag_store = [bool(re.match(r"global_store_dword\s.*\bsc0 sc1\b", ln)) for ln in lines]
    is_poll = [bool(re.match(r"global_load_dword\s.*\bsc0 sc1\b", ln)) for ln in lines]
    vm0 = [bool(re.match(r"s_waitcnt\s.*vmcnt\(0\)", ln)) for ln in lines]
    bar = [ln.startswith("s_barrier") for ln in lines]
    if sum(is_flag_store) < n_barriers:
        errs.append(f"{sum(is_flag_store)} system-scope flag stores < {n_barriers} barriers")
    if sum(is_poll) < n_barriers:
        errs.append(f"{sum(is_poll)} system-scope flag polls < {n_barriers} barriers")
    for i in (i for i, f in enumerate(is_flag_store) if f):
        j = i - 1
        while j >= 0 and not bar[j] and not lines[j].startswith("buffer_wbl2"):
            j -= 1
        if j < 0 or bar[j] or not re.match(r"buffer_wbl2\s+sc0 sc1\b", lines[j]):
            errs.append(f"flag store {i} ({lines[i]}): no buffer_wbl2 sc0 sc1 before it")
            continue
        mid = lines[j + 1:i]
        if not any(vm0[j + 1:i]):
            errs.append(f"flag store {i}: no s_waitcnt vmcnt(0) between buffer_wbl2 and the store")
        if any(re.match(r"(global|buffer|flat)_(store|atomic)", ln) for ln in mid):
            errs.append(f"flag store {i}: another store between buffer_wbl2 and the flag")
    for i in (i for i, f in enumerate(is_poll) if f):
        nb = next((k for k in range(i + 1, len(lines)) if bar[k]), len(lines))
        seq = [k for k in range(i + 1, nb)]
        w1 = next((k for k in seq if vm0[k]), None)
        inv = next((k for k in seq if re.match(r"buffer_inv\s+sc0 sc1\b", lines[k])), None)
        if w1 is None or inv is None or not w1 < inv:
            errs.append(f"poll {i}: no s_waitcnt vmcnt(0) then buffer_inv sc0 sc1 before the next barrier")
            continue
        if not any(vm0[k] for k in range(inv + 1, nb)):
            errs.append(f"poll {i}: buffer_inv not waited for before the barrier")
        if any(re.match(r"global_load_dwordx", lines[k]) for k in range(i + 1, inv)):
            errs.append(f"poll {i}: a data load before the invalidate")
    prev = 0
    for b in (k for k, f in enumerate(bar) if f):
        last_vm = max((k for k in range(prev, b) if re.match(r"(global|buffer|flat)_(store|atomic)", lines[k])),
                      default=None)
        if last_vm is not None and not any(vm0[last_vm + 1:b]):
            errs.append(f"barrier {b}: store {last_vm} ({lines[last_vm]}) not retired before it")
        prev = b
    return errs


def _ar_build(tmp_path, source: str):
    src = tmp_path / "allreduce_p2p.hip"
    src.write_text(source)
    cmd = [HIPCC if Path(HIPCC).exists() else "hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c",
           "-I", str(ROOT / "native" / "kernels"), str(src), "-o", str(tmp_path / "ar.o"), "-save-temps=obj"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd=tmp_path)
    assert out.returncode == 0, out.stderr[-2000:]
    (s_file,) = list(tmp_path.glob("allreduce_p2p-hip-amdgcn-amd-amdhsa-gfx950.s"))
    funcs = _functions(s_file.read_text(), r"allreduce_(one|two)shotILb[01]ELi[2-8]E")
    assert len(funcs) == 2 * 2 * 7, sorted(funcs)
    return {n: _ar_protocol_violations(b, 2 if "oneshot" in n else 3) for n, b in funcs.items()}


AR_SRC = ROOT / "native" / "kernels" / "allreduce_p2p.hip"


def test_p2p_allreduce_orders_its_flags_for_xgmi_peers(tmp_path):
    """cross-GPU correctness of the P2P all-reduce rests on
    the flag protocol's system-scope release / acquire. Pinned in the compiled
    ISA of every one- / two-shot instance with 2-8 ranks (both dtypes): L2
    written back and the write-back waited for before each flag store, the
    poll's invalidate waited for before any wave reads peer data, every wave's
    stores retired before each barrier."""
    bad = {n: e for n, e in _ar_build(tmp_path, AR_SRC.read_text()).items() if e}
    assert not bad, {n: e[:3] for n, e in list(bad.items())[:3]}


@pytest.mark.parametrize("mutation", ["agent_scope", "round5_release_store"])
def test_p2p_allreduce_order_check_catches_weakened_builds(tmp_path, mutation):
    """The checker above fails on builds whose ordering is too weak for xGMI
    peers: the release / acquire at agent scope (no system write-back /
    invalidate), and round 5's form -- the release store as one atomic, whose
    expansion lost the wait between buffer_wbl2 and the flag store."""
    src = AR_SRC.read_text()
    if mutation == "agent_scope":
        mutated = src.replace('__builtin_amdgcn_fence(__ATOMIC_RELEASE, "")', '__builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent")')
        mutated = mutated.replace("__HIP_MEMORY_SCOPE_SYSTEM", "__HIP_MEMORY_SCOPE_AGENT")
    else:
        old = ('    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: buffer_wbl2 sc0 sc1\n'
               '    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");\n'
               '    __hip_atomic_store(&P.sig[p]->flag[phase][b][rank], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);\n')
        new = '    __hip_atomic_store(&P.sig[p]->flag[phase][b][rank], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);\n'
        assert old in src
        mutated = src.replace(old, new)
    assert mutated != src
    bad = {n: e for n, e in _ar_build(tmp_path, mutated).items() if e}
    assert bad, "the weakened build passed the ordering check"
