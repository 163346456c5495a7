"""In-tree native build for the gfx950 HIP kernels (no hipify, no JIT cache).

Every ``csrc/*.hip`` file is compiled by ``hipcc --offload-arch=gfx950`` into an object; the
host-only torch binding (``csrc/bindings.cpp``) is compiled by ``g++`` against the torch
headers; both are linked into ``deconv_api_amd/_C<EXT_SUFFIX>`` next to this file, so the
shared object travels with the source tree to the GPU box. The HIP runtime is resolved to the
one torch already loaded (same soname ``libamdhip64.so.7``).

Provenance: the build embeds ``source_hash()`` (sha256 over every ``csrc`` file's bytes plus the
compile flags) into the binding as the string ``DV_SOURCE_HASH:<hex>`` (``_C.source_hash()``).
``ops/native.py`` recomputes it from the tree before importing and refuses a binary built from
other sources (``DV_AUTOBUILD=1``: rebuilds instead), so a GPU run can not silently use a stale
``_C`` pushed with a newer tree.

Usage: ``python -m deconv_api_amd._build [--force] [-j N] [--debug]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import re
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
BUILD = PKG.parent / "build" / "native"
ARCH = os.environ.get("DV_OFFLOAD_ARCH", "gfx950")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
TARGET = PKG / f"_C{EXT}"


def _flags(debug: bool) -> list:
    return (["-O1", "-g"] if debug else ["-O3"]), (["-DDV_DEBUG=1"] if debug else [])


def source_hash(debug: bool = False) -> str:
    """sha256 of the native sources (file names + bytes, sorted) and the flags they compile with."""
    h = hashlib.sha256()
    opt, defs = _flags(debug)
    h.update(" ".join([ARCH, *opt, *defs]).encode())
    for p in sorted(CSRC.iterdir()):
        if p.suffix in (".hip", ".h", ".cpp"):
            h.update(p.name.encode() + b"\0")
            h.update(p.read_bytes())
    return h.hexdigest()


_HASH_RE = re.compile(rb"DV_SOURCE_HASH:([0-9a-f]{64})")


def embedded_hash(so: Path = TARGET):
    """The hash a built ``_C`` carries (read from the file, without loading it); None if absent."""
    try:
        m = _HASH_RE.search(Path(so).read_bytes())
    except OSError:
        return None
    return m.group(1).decode() if m else None


def _torch_paths():
    import torch.utils.cpp_extension as ce

    inc = ce.include_paths(device_type="cuda")
    lib = ce.library_paths(device_type="cuda")
    return inc, lib


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm install expected under /opt/rocm)")


def _newer(src_paths, out: Path) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(p.stat().st_mtime > t for p in src_paths)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build step failed ({r.returncode}):\n{' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def build(force: bool = False, jobs: int | None = None, debug: bool = False, verbose: bool = False) -> Path:
    # debug objects live apart so switching modes never mixes -DDV_DEBUG and release objects;
    # -O1 (not -O0): the kernels' inline-asm immediates need constant folding
    bdir = BUILD.parent / "native-debug" if debug else BUILD
    bdir.mkdir(parents=True, exist_ok=True)
    inc, libdirs = _torch_paths()
    headers = sorted(CSRC.glob("*.h"))
    hip_srcs = sorted(CSRC.glob("*.hip"))
    opt, defs = _flags(debug)
    shash = source_hash(debug)
    stamp = bdir / "source_hash.txt"
    stale_hash = not stamp.exists() or stamp.read_text().strip() != shash
    hipcc = _hipcc()
    objs = []
    tasks = []
    for src in hip_srcs:
        obj = bdir / (src.stem + ".o")
        objs.append(obj)
        if force or _newer([src, *headers], obj):
            tasks.append([hipcc, *opt, *defs, f"--offload-arch={ARCH}", "-fPIC", "-std=c++17",
                          "-Wno-unused-result", f"-I{CSRC}", "-c", str(src), "-o", str(obj)])
    for src in sorted(CSRC.glob("*.cpp")):  # host-only C++ (no torch / HIP): the JPEG encoder
        if src.name == "bindings.cpp":
            continue
        obj = bdir / (src.stem + ".o")
        objs.append(obj)
        if force or _newer([src, *headers], obj):
            tasks.append(["g++", *opt, *defs, "-fPIC", "-std=c++17", "-pthread", "-D_GLIBCXX_USE_CXX11_ABI=1",
                          f"-I{CSRC}", "-c", str(src), "-o", str(obj)])
    bsrc = CSRC / "bindings.cpp"
    bobj = bdir / "bindings.o"
    objs.append(bobj)
    if force or stale_hash or _newer([bsrc, *headers], bobj):
        py_inc = sysconfig.get_paths()["include"]
        tasks.append(["g++", *opt, *defs, f"-DDV_SOURCE_HASH=\"{shash}\"", "-fPIC", "-std=c++17",
                      "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                      "-DTORCH_API_INCLUDE_EXTENSION_H", "-DTORCH_EXTENSION_NAME=_C", "-D_GLIBCXX_USE_CXX11_ABI=1",
                      *[f"-I{p}" for p in inc], f"-I{py_inc}", f"-I{CSRC}", "-c", str(bsrc), "-o", str(bobj)])
    if tasks:
        jobs = jobs or min(8, os.cpu_count() or 4)
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            for out in ex.map(_run, tasks):
                if verbose and out.strip():
                    print(out)
    if force or tasks or debug or _newer(objs, TARGET):
        link = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *[str(o) for o in objs], "-o", str(TARGET)]
        for d in libdirs:
            link += [f"-L{d}"]
        torch_lib = libdirs[0]
        link += [f"-Wl,-rpath,{torch_lib}", "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip",
                 "-ltorch_hip", "-lamdhip64", "-pthread"]
        _run(link)
    stamp.write_text(shash + "\n")
    return TARGET


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    out = build(force=a.force, jobs=a.jobs, debug=a.debug, verbose=a.verbose)
    print(f"built {out}")


if __name__ == "__main__":
    sys.exit(main())
