"""Build the native runtime extension in-tree for gfx950.

Explicit hipcc / g++ invocations (no hipify, no JIT cache): the .hip kernel sources are
compiled by hipcc for ``--offload-arch=gfx950`` only; the torch-facing C++ (bindings,
reducer, RCCL communicator) is host code compiled against torch's headers; everything is
linked into ``distributed_pytorch_training_amd/_C<ext-suffix>`` next to the package so the
built object travels with the repository snapshot to the GPU box.

Linking uses torch's bundled ``libamdhip64.so.7`` / ``librccl.so.1`` (same sonames as
/opt/rocm's), so one HIP runtime and one RCCL live in the process.

Usage: ``python csrc/build.py [--jobs N] [--force] [--debug] [--asan]``

``--asan``: the HOST C++ (reducer, communicators, watchdog, bindings) is
compiled with AddressSanitizer into ``build/asan/_C*.so`` - never over the in-tree extension;
the GPU kernels are not instrumented (no GPU sanitizer on this pool).  Run with
``LD_PRELOAD=$(gcc -print-file-name=libasan.so) ASAN_OPTIONS=detect_leaks=0
DPT_NATIVE_LIB=build/asan/_C*.so python -m pytest tests/test_ddp_gloo.py`` (tests/test_asan.py).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
PKG = ROOT / "distributed_pytorch_training_amd"
BUILD = ROOT / "build" / "native"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("DPT_OFFLOAD_ARCH", "gfx950")

HIP_SOURCES = sorted((CSRC / "kernels").glob("*.hip"))
CPP_SOURCES = [CSRC / "watchdog.cpp", CSRC / "rccl_comm.cpp", CSRC / "host_comm.cpp", CSRC / "pg_comm.cpp",
               CSRC / "reducer.cpp", CSRC / "bindings.cpp"]


def _torch_paths():
    import torch
    import torch.utils.cpp_extension as ce

    tdir = Path(torch.__file__).resolve().parent
    incs = [tdir / "include", tdir / "include" / "torch" / "csrc" / "api" / "include"]
    return tdir, incs, bool(torch._C._GLIBCXX_USE_CXX11_ABI)


def output_path(asan: bool = False, variant: str = "") -> Path:
    name = "_C" + sysconfig.get_config_var("EXT_SUFFIX")
    if variant:  # outside build/ (gpurun-ignored): the A/B library travels to the GPU box
        return ROOT / "variants" / variant / name
    return (ROOT / "build" / "asan" / name) if asan else (PKG / name)


def _variant_tag(defines) -> str:
    return "_".join(d.replace("=", "-") for d in sorted(defines)) if defines else ""


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("build step failed:\n" + " ".join(map(str, cmd)) + "\n" + r.stdout + r.stderr)
    return r


def _stamp(src: Path, flags) -> str:
    h = hashlib.sha1()
    h.update(" ".join(map(str, flags)).encode())
    h.update(src.read_bytes())
    for hdr in sorted(CSRC.rglob("*.h")):
        h.update(hdr.read_bytes())
    return h.hexdigest()[:16]


def build(jobs: int = 4, force: bool = False, debug: bool = False, verbose: bool = False,
          asan: bool = False, defines=()) -> Path:
    """``defines`` (``NAME=VALUE`` strings): an A/B build of the kernel library with those
    compile-time switches, written to variants/<tag>/ (never over the in-tree extension);
    load it with ``DPT_NATIVE_LIB=<path>``."""
    tdir, tincs, cxx11 = _torch_paths()
    variant = _variant_tag(defines)
    kbuild = (ROOT / "build" / f"variant-{variant}" / "obj") if variant else BUILD
    kbuild.mkdir(parents=True, exist_ok=True)
    BUILD.mkdir(parents=True, exist_ok=True)
    host_build = BUILD.parent / "native-asan" if asan else BUILD
    host_build.mkdir(parents=True, exist_ok=True)
    py_inc = sysconfig.get_paths()["include"]
    opt = ["-O0", "-g"] if debug else ["-O3"]
    host_opt = ["-O1", "-g", "-fsanitize=address", "-fno-omit-frame-pointer"] if asan else opt
    common_defs = ["-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DHIPBLAS_V2",
                   f"-D_GLIBCXX_USE_CXX11_ABI={int(cxx11)}"]
    hip_flags = [str(ROCM / "bin" / "hipcc"), f"--offload-arch={ARCH}", "-std=c++17", "-fPIC",
                 *opt, "-Wall", "-Wno-unused-result", *common_defs, *[f"-D{d}" for d in defines],
                 f"-I{CSRC}", f"-I{CSRC / 'kernels'}"]
    cpp_flags = ["g++", "-std=c++17", "-fPIC", "-fvisibility=hidden", *host_opt, "-Wall", "-Wno-unused-variable", "-Wno-sign-compare",
                 *common_defs, "-DTORCH_API_INCLUDE_EXTENSION_H", "-DTORCH_EXTENSION_NAME=_C",
                 f"-I{CSRC}", *[f"-I{p}" for p in tincs], f"-I{ROCM / 'include'}", f"-I{py_inc}"]

    jobs_list = []
    for src in HIP_SOURCES:
        jobs_list.append((src, hip_flags))
    for src in CPP_SOURCES:
        jobs_list.append((src, cpp_flags))

    def compile_one(item):
        src, flags = item
        obj = (kbuild if src.suffix == ".hip" else host_build) / (src.stem + (".hip.o" if src.suffix == ".hip" else ".o"))
        stamp = obj.parent / (obj.name + ".stamp")
        key = _stamp(src, flags)
        if not force and obj.exists() and stamp.exists() and stamp.read_text() == key:
            return obj, False
        cmd = [*flags, "-c", str(src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd), flush=True)
        _run(cmd)
        stamp.write_text(key)
        return obj, True

    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        results = list(ex.map(compile_one, jobs_list))
    objs = [o for o, _ in results]
    out = output_path(asan, variant)
    out.parent.mkdir(parents=True, exist_ok=True)
    rebuilt = any(changed for _, changed in results)
    if rebuilt or force or not out.exists():
        tlib = tdir / "lib"
        link = [str(ROCM / "bin" / "hipcc"), f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs),
                "-o", str(out), f"-L{tlib}", f"-Wl,-rpath,{tlib}",
                "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
                "-l:librccl.so.1", "-l:libamdhip64.so.7"]
        if verbose:
            print(" ".join(link), flush=True)
        _run(link)
        _check_undefined(out)
    return out


def _check_undefined(so: Path) -> None:
    """A shared library links with unresolved symbols; catch our own (a declaration whose
    definition changed signature) here instead of at import time on the GPU box."""
    nm = ROCM / "lib" / "llvm" / "bin" / "llvm-nm"
    if not nm.exists():
        return
    r = subprocess.run([str(nm), "-u", "-C", str(so)], capture_output=True, text=True)
    bad = [l.strip() for l in r.stdout.splitlines() if "dpt::" in l]
    if bad:
        so.unlink()
        raise RuntimeError("unresolved framework symbols in the extension:\n  " + "\n  ".join(bad))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--jobs", type=int, default=int(os.environ.get("MAX_JOBS", "4")))
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--asan", action="store_true", help="host code with AddressSanitizer -> build/asan/")
    ap.add_argument("-D", "--define", action="append", default=[],
                    help="NAME=VALUE kernel compile switch: an A/B build under variants/<tag>/")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    out = build(jobs=min(a.jobs, 16), force=a.force, debug=a.debug, verbose=a.verbose, asan=a.asan,
                defines=tuple(a.define))
    print(f"built {out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
