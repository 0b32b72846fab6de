"""Build libugpg.so (HIP, gfx950) in-tree: ug-pg-unet_amd/ugpg/libugpg.so.

    python ug-pg-unet_amd/build.py [--force]

Plain hipcc, one object per translation unit (compiled in parallel), no torch
dependency in the library.  Incremental: a TU is rebuilt only when it or a header
is newer than its object.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
INCLUDE = HERE.parent / "include"
BUILD = HERE / "build"
LIB = HERE / "ugpg" / "libugpg.so"
ARCH = os.environ.get("UGPG_ARCH", "gfx950")
# Device code without packed-FP32 VALU (v_pk_add/mul/fma_f32): a packed-FP32 write to a
# VGPR that a just-issued global load still reads as its address corrupted the last 16
# lanes of that load under concurrent GPU load (another stream or process) -- measured on
# the logits combine, 10-717 of 3000 launches wrong with them, 0 of 6000 without
# (tools/xproc_bisect.py --micro).  The host compile ignores the feature
# (ignored there, with a warning).
NO_PK = ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
         "-Wno-unused-variable", "-Wno-unused-but-set-variable", *NO_PK]


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and Path(c).exists():
            return c
    raise RuntimeError("hipcc not found: libugpg.so cannot be built")


def _sources():
    return sorted(CSRC.glob("*.hip"))


def _newest_header() -> float:
    hs = list(CSRC.glob("*.h")) + list(INCLUDE.glob("*.h"))
    return max((h.stat().st_mtime for h in hs), default=0.0)


# memory-bound kernels: no FMA contraction, so interpolation weights round exactly
# like ATen's CPU kernels (align_corners source index = rounded(scale*o))
# conv_x6.hip: no SLP vectorization -- packed f32 VALU (v_pk_add_f32 ...) issued beside the
# MFMA waves slows them (MI355X_MICROARCH.md, 'price of one filler beside MFMAs')
PER_FILE = {"ops.hip": ["-ffp-contract=off"], "conv_x6.hip": ["-fno-slp-vectorize"]}


ID_MARK = b"UGPG_BUILD_ID="


def content_id() -> str:
    """Content hash of the sources alone: csrc/*.hip, csrc/*.h, include/*.h."""
    h = hashlib.sha256()
    for f in sorted(list(CSRC.glob("*.hip")) + list(CSRC.glob("*.h")) + list(INCLUDE.glob("*.h")),
                    key=lambda f: (f.parent.name, f.name)):
        h.update(f"{f.parent.name}/{f.name}".encode() + b"\0" + f.read_bytes() + b"\0")
    return h.hexdigest()[:32]


def source_id(defines=()) -> str:
    """Build id: the sources' content hash, then a hash of the compile configuration (flags,
    target arch, experimental defines) -- 65 characters.  Embedded in the library
    (ugpg_build_id()); build() relinks on any difference, and ugpg._C refuses a libugpg.so
    whose CONTENT part differs from the sources next to it, so a stale prebuilt library
    cannot be loaded silently while a library built for another
    UGPG_ARCH or with defines is not mistaken for a stale one."""
    cfg = hashlib.sha256(repr((FLAGS, PER_FILE, tuple(defines))).encode()).hexdigest()[:32]
    return f"{content_id()}-{cfg}"


ID_LEN = 65


def lib_id(lib: Path) -> str | None:
    """The build id embedded in a built library (read from its bytes; nothing is loaded)."""
    try:
        data = Path(lib).read_bytes()
    except OSError:
        return None
    i = data.find(ID_MARK)
    return data[i + len(ID_MARK):i + len(ID_MARK) + ID_LEN].decode("ascii", "replace") if i >= 0 else None


def _id_object(bdir: Path, sid: str) -> Path:
    """A host-only object exporting ugpg_build_id() (gcc; rebuilt when the id changes)."""
    src, obj = bdir / "build_id.c", bdir / "build_id.o"
    text = (f'static const char id[] = "{ID_MARK.decode()}{sid}";\n'
            f'const char* ugpg_build_id(void) {{ return id + {len(ID_MARK)}; }}\n')
    if not src.exists() or src.read_text() != text or not obj.exists():
        src.write_text(text)
        r = subprocess.run(["gcc", "-O2", "-fPIC", "-c", str(src), "-o", str(obj)],
                           capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"build id object failed:\n{r.stderr}")
    return obj


def _compile(src: Path, force: bool, bdir: Path = BUILD, defines=()) -> Path:
    obj = bdir / (src.stem + ".o")
    if not force and obj.exists() and obj.stat().st_mtime >= max(src.stat().st_mtime, _newest_header()):
        return obj
    cmd = [_hipcc(), *FLAGS, *PER_FILE.get(src.name, []), *[f"-D{d}" for d in defines], "-c",
           str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr}")
    return obj


def build(force: bool = False, verbose: bool = True, defines=(), out: Path | None = None) -> Path:
    """Build libugpg.so; `defines`/`out` build an experimental variant (its own object
    directory) for A/B timing via UGPG_LIB."""
    lib = Path(out) if out else LIB
    bdir = BUILD if not defines else BUILD / ("v_" + "_".join(d.replace("=", "") for d in defines))
    bdir.mkdir(parents=True, exist_ok=True)
    # objects built with other flags are stale
    stamp, flags = bdir / "flags.txt", repr((FLAGS, PER_FILE))
    if not stamp.exists() or stamp.read_text() != flags:
        force = True
    srcs = _sources()
    jobs = min(len(srcs), int(os.environ.get("MAX_JOBS", "8")))
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: _compile(s, force, bdir, defines), srcs))
    sid = source_id(defines)
    objs.append(_id_object(bdir, sid))
    newest = max(o.stat().st_mtime for o in objs)
    LIB_ = lib
    if force or not LIB_.exists() or LIB_.stat().st_mtime < newest or lib_id(LIB_) != sid:
        tmp = LIB_.with_suffix(".so.tmp")
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(tmp),
               "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
        os.replace(tmp, LIB_)
    stamp.write_text(flags)
    if verbose:
        print(f"built {LIB_} ({LIB_.stat().st_size / 1e6:.1f} MB)")
    return LIB_


SAN_FLAGS = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined"]


def build_sanitized(out: Path | None = None, verbose: bool = False) -> Path:
    """ASan + UBSan on the HOST side of the C-ABI (argument validation, error plumbing,
    plan/workspace arithmetic, the communicator's host code): the usual gfx950 build with
    each -fsanitize= behind -Xarch_host, device code untouched.  For CPU tests of the host
    paths (tests/test_abi.py, loaded with the ASan runtime preloaded); never used on a GPU."""
    bdir = BUILD / "asan"
    bdir.mkdir(parents=True, exist_ok=True)
    lib = Path(out) if out else bdir / "libugpg_asan.so"

    def one(src):
        obj = bdir / (src.stem + ".o")
        if not obj.exists() or obj.stat().st_mtime < max(src.stat().st_mtime, _newest_header()):
            cmd = [_hipcc(), "-O1", "-g", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
                   "-fno-omit-frame-pointer", *PER_FILE.get(src.name, []), *SAN_FLAGS, "-c",
                   str(src), "-o", str(obj)]
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"sanitized hipcc failed for {src.name}:\n{r.stderr}")
        return obj

    srcs = _sources()
    with cf.ThreadPoolExecutor(max_workers=max(1, min(len(srcs), int(os.environ.get("MAX_JOBS", "8"))))) as ex:
        objs = list(ex.map(one, srcs))
    objs.append(_id_object(bdir, source_id()))
    if not lib.exists() or lib.stat().st_mtime < max(o.stat().st_mtime for o in objs):
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-shared-libsan", *SAN_FLAGS,
               *map(str, objs), "-o", str(lib), "-L/opt/rocm/lib", "-lrccl",
               "-Wl,-rpath,/opt/rocm/lib"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"sanitized link failed:\n{r.stderr}")
    if verbose:
        print(f"built {lib}")
    return lib


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="experimental define")
    ap.add_argument("--out", default=None, help="output .so (experimental variants)")
    a = ap.parse_args()
    try:
        build(force=a.force, defines=tuple(a.defines), out=a.out)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
