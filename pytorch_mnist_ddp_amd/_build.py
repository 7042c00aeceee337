"""In-tree native build: hipcc (gfx950) -> ``pytorch_mnist_ddp_amd/_C<ext>.so``.

No hipify, no torch cpp_extension JIT cache: every ``.hip`` kernel file is compiled for
``--offload-arch=gfx950`` only, host-only runtime files (engine, RCCL communicator, pybind11
bindings) are compiled as plain C++ with the HIP headers, and the objects are linked into one
Python extension placed next to this file (so the built ``.so`` travels with the source tree
to the GPU box).  Rebuilds are incremental (object newer than its source and every header).

Usage: ``python -m pytorch_mnist_ddp_amd._build [--force] [--jobs N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
CSRC = os.path.join(ROOT, "csrc")
OBJ_DIR = os.path.join(ROOT, "build", "obj")
ARCH = "gfx950"
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
OUTPUT = os.path.join(PKG_DIR, "_C" + EXT_SUFFIX)
# debug variant with the in-kernel timeline (csrc/include/timeline.h): same module name, own file
OBJ_DIR_TL = os.path.join(ROOT, "build", "obj_tl")
OUTPUT_TL = os.path.join(PKG_DIR, "_C_tl" + EXT_SUFFIX)


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.isabs(c) and os.path.exists(c) or not os.path.isabs(c)):
            return c
    return "hipcc"


def _torch_lib_dir() -> str | None:
    try:
        import importlib.util
        spec = importlib.util.find_spec("torch")
        if spec and spec.origin:
            d = os.path.join(os.path.dirname(spec.origin), "lib")
            return d if os.path.isdir(d) else None
    except Exception:
        pass
    return None


def _includes() -> list[str]:
    inc = ["-I" + CSRC, "-I" + sysconfig.get_paths()["include"]]
    try:
        import pybind11
        inc.append("-I" + pybind11.get_include())
    except ImportError:
        pass
    return inc


def sources() -> tuple[list[str], list[str]]:
    kernels = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    host = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp"))) + [os.path.join(CSRC, "bindings.cpp")]
    return kernels, host


def _headers() -> list[str]:
    return sorted(glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True))


def _obj_path(src: str, timeline: bool = False) -> str:
    rel = os.path.relpath(src, CSRC).replace(os.sep, "__")
    return os.path.join(OBJ_DIR_TL if timeline else OBJ_DIR, rel + ".o")


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _compile(src: str, kernel: bool, verbose: bool, timeline: bool = False) -> str:
    obj = _obj_path(src, timeline)
    cmd = [_hipcc(), "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", *_includes()]
    if timeline:
        cmd.append("-DMNIST_TIMELINE")
    if kernel:
        cmd += ["-x", "hip", f"--offload-arch={ARCH}", "-munsafe-fp-atomics", "-fno-slp-vectorize"]
    else:
        rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
        cmd += ["-x", "c++", "-D__HIP_PLATFORM_AMD__", "-I" + os.path.join(rocm, "include")]
    cmd += ["-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int | None = None, verbose: bool = False, timeline: bool = False) -> str:
    """Compile + link the extension if anything changed; return the .so path.  ``timeline``: the
    debug variant with in-kernel wave timestamps (``_C_tl``, loaded when MNIST_AMD_TIMELINE=1)."""
    obj_dir, output = (OBJ_DIR_TL, OUTPUT_TL) if timeline else (OBJ_DIR, OUTPUT)
    os.makedirs(obj_dir, exist_ok=True)
    kernels, host = sources()
    headers = _headers()
    todo = [(s, True) for s in kernels] + [(s, False) for s in host]
    stale = [(s, k) for s, k in todo if force or _stale(_obj_path(s, timeline), [s, *headers])]
    jobs = jobs or min(8, max(1, len(stale)))
    if stale:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            list(ex.map(lambda sk: _compile(sk[0], sk[1], verbose, timeline), stale))
    objs = [_obj_path(s, timeline) for s, _ in todo]
    if force or stale or _stale(output, objs):
        cmd = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", output + ".tmp", "-ldl"]
        tl = _torch_lib_dir()
        if tl:  # resolve libamdhip64/librccl to the copies torch ships (one HIP runtime per process)
            cmd += ["-Wl,-rpath," + tl]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{r.stdout}\n{r.stderr}")
        os.replace(output + ".tmp", output)
    return output


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--timeline", action="store_true", help="debug variant with in-kernel timestamps (_C_tl)")
    a = ap.parse_args(argv)
    out = build(force=a.force, jobs=a.jobs, verbose=a.verbose, timeline=a.timeline)
    print(out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
