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
KERNELS = [
    "_ZN4ugpg22conv3x3_fwd_x6r_kernelILi3ELb1EEEvNS_11ConvFwdArgsE",
    "_ZN4ugpg22conv3x3_fwd_x6r_kernelILi3ELb0EEEvNS_11ConvFwdArgsE",
    "_ZN4ugpg22conv3x3_fwd_x6r_kernelILi1ELb0EEEvNS_11ConvFwdArgsE",
    "_ZN4ugpg24conv3x3_wgrad_x6w_kernelILi4ELi16ELi3EEEvNS_9WgradArgsE",
    "_ZN4ugpg24conv3x3_wgrad_x6w_kernelILi4ELi16ELi1EEEvNS_9WgradArgsE",
]


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    if not Path(HIPCC).exists():
        pytest.skip("hipcc not available")
    d = tmp_path_factory.mktemp("asm")
    r = subprocess.run([HIPCC, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                        f"-I{CSRC}", f"-I{ROOT / 'include'}", "-c", str(CSRC / "conv_x6.hip"),
                        "-o", str(d / "x.o"), "--save-temps"], cwd=d, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return next(d.glob("*gfx950.s"))


@pytest.mark.parametrize("kernel", KERNELS)
def test_no_register_touched_while_its_load_is_in_flight(asm, kernel):
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "asm_audit.py"), str(asm), kernel],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:]
