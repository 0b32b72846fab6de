"""Static check of the persistent conv kernels' untracked loads (CPU; needs hipcc).

The loader waves of conv3x3_fwd_x6r_kernel / conv3x3_wgrad_x6w_kernel keep global
loads in flight across barriers with inline-asm loads and counted waits; the compiler
does not know those registers are still being written.  tools/asm_audit.py walks the
compiled gfx950 assembly and fails on any instruction that touches a register of a
load that may still be in flight (the failure mode that turns into a memory fault).
"""
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "ug-pg-unet_amd" / "csrc"
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
X6R = "_ZN4ugpg22conv3x3_fwd_x6r_kernelIL{}EEEvNS_11ConvFwdArgsE"  # (last: PAIR)
KERNELS = [
    X6R.format("i3ELb1ELi32ELi8ELb0ELi1ELb0ELi0"),
    X6R.format("i3ELb1ELi16ELi8ELb0ELi1ELb0ELi0"),
    X6R.format("i1ELb0ELi32ELi8ELb0ELi1ELb0ELi0"),
    X6R.format("i1ELb0ELi32ELi8ELb1ELi1ELb0ELi0"),
    X6R.format("i1ELb0ELi32ELi8ELb0ELi2ELb0ELi0"),    # single-piece 256 x 128 items
    X6R.format("i1ELb0ELi32ELi8ELb1ELi2ELb0ELi0"),
    X6R.format("i1ELb0ELi32ELi16ELb0ELi1ELb0ELi0"),   # single-piece 512 x 64 items
    X6R.format("i1ELb0ELi32ELi16ELb1ELi1ELb0ELi0"),
    X6R.format("i1ELb0ELi32ELi8ELb0ELi1ELb1ELi0"),    # 256 x 64, K = 64: resident weights
    X6R.format("i1ELb0ELi32ELi8ELb1ELi1ELb1ELi0"),
    X6R.format("i1ELb0ELi16ELi8ELb0ELi1ELb0ELi0"),    # single-piece 8 x 16 items (16-wide images)
    X6R.format("i1ELb0ELi32ELi8ELb0ELi2ELb0ELi1"),    # 4 x 2-tile forms, whole-line bf16 epilogue
    X6R.format("i1ELb0ELi32ELi8ELb1ELi2ELb0ELi1"),
    X6R.format("i1ELb0ELi32ELi16ELb0ELi1ELb0ELi1"),
    X6R.format("i1ELb0ELi32ELi16ELb1ELi1ELb0ELi1"),
    X6R.format("i1ELb0ELi32ELi8ELb1ELi2ELb0ELi2"),    # the same forms' data gradient with partials
    X6R.format("i1ELb0ELi32ELi16ELb1ELi1ELb0ELi2"),
    "_ZN4ugpg24conv3x3_wgrad_x6w_kernelILi4ELi16ELi3ELi0ELb0EEEvNS_9WgradArgsE",
    "_ZN4ugpg24conv3x3_wgrad_x6w_kernelILi4ELi16ELi3ELi0ELb1EEEvNS_9WgradArgsE",  # lazy BN dy
    "_ZN4ugpg24conv3x3_wgrad_x6w_kernelILi4ELi16ELi1ELi0ELb0EEEvNS_9WgradArgsE",
    "_ZN4ugpg24conv3x3_wgrad_x6w_kernelILi4ELi16ELi1ELi1ELb0EEEvNS_9WgradArgsE",
    "_ZN4ugpg24conv3x3_wgrad_x6w_kernelILi4ELi16ELi1ELi2ELb0EEEvNS_9WgradArgsE",
    "_ZN4ugpg24conv3x3_wgrad_x6w_kernelILi4ELi16ELi1ELi3ELb0EEEvNS_9WgradArgsE",
]


def _build_flags():
    import importlib.util
    spec = importlib.util.spec_from_file_location("ugpg_build", ROOT / "ug-pg-unet_amd" / "build.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return [*mod.FLAGS, *mod.PER_FILE.get("conv_x6.hip", [])]


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    if not Path(HIPCC).exists():
        pytest.skip("hipcc not available")
    d = tmp_path_factory.mktemp("asm")
    r = subprocess.run([HIPCC, *_build_flags(),
                        f"-I{CSRC}", f"-I{ROOT / 'include'}", "-c", str(CSRC / "conv_x6.hip"),
                        "-o", str(d / "x.o"), "--save-temps",
                        "-Rpass-analysis=kernel-resource-usage"], cwd=d, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return next(d.glob("*gfx950.s")), r.stderr


@pytest.mark.parametrize("kernel", KERNELS)
def test_no_register_touched_while_its_load_is_in_flight(asm, kernel):
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "asm_audit.py"), str(asm[0]), kernel],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:]


# The single-piece 4 x 2-tile forms hold 128 accumulator registers per lane: the
# allocator spills a few loop-invariant addresses, reloaded only in the per-item epilogue
# (bounded here, and never inside the MFMA loop -- test below; the loader pipeline's
# counted waits model scratch operations in tools/asm_audit.py)
SPILL_ALLOWANCE = {k: 128 for k in KERNELS[4:8]}


@pytest.mark.parametrize("kernel", KERNELS)
def test_no_register_spills(asm, kernel):
    """A spill in these one-wave-per-SIMD kernels costs 20-30 % when it lands in the MFMA
    loop (scratch traffic); the register budget is 256 per lane at 8 waves per CU."""
    import re
    remarks = asm[1].split("Function Name: ")
    mine = [r for r in remarks if r.startswith(kernel)]
    assert mine, f"no resource-usage remark for {kernel}"
    scratch = int(re.search(r"ScratchSize \[bytes/lane\]: (\d+)", mine[0]).group(1))
    assert scratch <= SPILL_ALLOWANCE.get(kernel, 0), mine[0][:800]
    text = asm[0].read_text()
    start = text.index(kernel + ":")
    body = text[start:text.index(".Lfunc_end", start)].splitlines()
    mf = [i for i, l in enumerate(body) if "v_mfma" in l]
    inside = [l.strip() for l in body[mf[0]:mf[-1] + 1] if "scratch_" in l]
    assert not inside, f"scratch operations inside the MFMA loop: {inside[:5]}"


@pytest.mark.parametrize("kernel", KERNELS)
def test_no_packed_f32_valu(asm, kernel):
    """v_pk_add/mul/fma_f32 beside MFMAs cost more than they save
    (MI355X_MICROARCH.md); build.py compiles conv_x6.hip without SLP vectorization and
    the kernels spell out their f32x4 arithmetic per component."""
    import re
    text = asm[0].read_text()
    start = text.index(kernel + ":")
    body = text[start:text.index(".Lfunc_end", start)]
    assert not re.findall(r"\bv_pk_(add|mul|fma)_f32", body)


@pytest.fixture(scope="module")
def all_asm(tmp_path_factory):
    """Device assembly of every libugpg source, built with the library's flags."""
    if not Path(HIPCC).exists():
        pytest.skip("hipcc not available")
    import importlib.util
    spec = importlib.util.spec_from_file_location("ugpg_build", ROOT / "ug-pg-unet_amd" / "build.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    d = tmp_path_factory.mktemp("all_asm")
    out = {}
    for src in sorted(CSRC.glob("*.hip")):
        s = d / (src.stem + ".s")
        r = subprocess.run([HIPCC, *mod.FLAGS, *mod.PER_FILE.get(src.name, []), f"-I{CSRC}",
                            f"-I{ROOT / 'include'}", "-S", "--offload-device-only", str(src), "-o",
                            str(s)], capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-2000:]
        out[src.name] = s
    return out


def test_no_packed_fp32_valu_anywhere(all_asm):
    """No v_pk_{add,mul,fma}_f32 in any kernel of the library: a packed-FP32 write to a VGPR
    that a just-issued global load reads as its address corrupted the last 16 lanes of the
    load under concurrent GPU load (build.py NO_PK)."""
    import re
    bad = {}
    for name, s in all_asm.items():
        n = len(re.findall(r"\bv_pk_(?:add|mul|fma)_f32\b", s.read_text()))
        if n:
            bad[name] = n
    assert not bad, bad


def test_no_vmem_operand_overwritten_by_packed_valu(all_asm):
    """The hazard pattern itself (tools/vmem_war_scan.py): no packed-FP32 VALU writes a VGPR
    that one of the preceding vector-memory instructions reads."""
    sys.path.insert(0, str(ROOT / "tools"))
    from vmem_war_scan import scan
    hits = {name: len(scan(s)) for name, s in all_asm.items()}
    assert not any(hits.values()), hits


def test_vmem_war_scan_finds_the_pattern(tmp_path):
    """tools/vmem_war_scan.py itself: a packed-FP32 write to a VGPR a just-issued global
    load reads as its address is flagged (the corrupting sequence of DESIGN.md §6a);
    the same write after the load retired (s_waitcnt vmcnt(0)), to a different
    register, or by a plain VALU, is not."""
    sys.path.insert(0, str(ROOT / "tools"))
    from vmem_war_scan import scan
    asm = tmp_path / "k.s"
    asm.write_text("""k_bad:
\tglobal_load_dword v24, v[28:29], off
\tv_mov_b32_e32 v1, 0
\tv_pk_mul_f32 v[28:29], v[6:7], v[32:33]
\ts_endpgm
k_ok:
\tglobal_load_dword v24, v[28:29], off
\ts_waitcnt vmcnt(0)
\tv_pk_mul_f32 v[28:29], v[6:7], v[32:33]
\tglobal_load_dword v25, v[30:31], off
\tv_pk_mul_f32 v[40:41], v[6:7], v[32:33]
\tv_mov_b32_e32 v30, 0
\ts_endpgm
""")
    hits = scan(asm)
    assert [h[0] for h in hits] == ["k_bad"], hits


def test_polygon_scan_has_no_fused_multiply_add(all_asm):
    """Pillow's scan converter rounds x = (y - y0) * dx and + x0 separately (x86 SSE float);
    a fused v_fma_f32 moved one boundary pixel in 4 of the 361 golden canvases (GPU run
    s2 of round 4).  csrc/augment.hip turns contraction off in poly_x_at."""
    import re
    text = all_asm["augment.hip"].read_text()
    start = text.index("_ZN4ugpg16poly_scan_kernel")
    start = text.index("_ZN4ugpg16poly_scan_kernel", text.index(":", start))  # the label
    body = text[start:text.index(".Lfunc_end", start)]
    assert not re.findall(r"\bv_(?:fma|fmac|mad|mac)_f32", body)
