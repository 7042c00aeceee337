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
# debug variants, same module name (PyInit__C), own file and object directory:
#   "tl": in-kernel wave timeline (csrc/include/timeline.h; MNIST_AMD_TIMELINE=1 loads it)
#   "rw": race-window widening, 0..RACE_WIDEN_US us random sleeps before every kernel's first global
#         read and every stream hand-off signal (device_utils.h; MNIST_AMD_RACE_WIDEN=1 loads it)
RACE_WIDEN_US = 20
VARIANTS = {
    "": (os.path.join(ROOT, "build", "obj"), OUTPUT, []),
    "tl": (os.path.join(ROOT, "build", "obj_tl"), os.path.join(PKG_DIR, "_C_tl" + EXT_SUFFIX), ["-DMNIST_TIMELINE"]),
    "rw": (os.path.join(ROOT, "build", "obj_rw"), os.path.join(PKG_DIR, "_C_rw" + EXT_SUFFIX),
           [f"-DMNIST_RACE_WIDEN={RACE_WIDEN_US}"]),
}
OBJ_DIR_TL, OUTPUT_TL = VARIANTS["tl"][0], VARIANTS["tl"][1]


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


def _obj_path(src: str, variant: str = "") -> str:
    rel = os.path.relpath(src, CSRC).replace(os.sep, "__")
    return os.path.join(VARIANTS[variant][0], rel + ".o")


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _compile(src: str, kernel: bool, verbose: bool, variant: str = "") -> str:
    obj = _obj_path(src, variant)
    cmd = [_hipcc(), "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", *_includes(),
           *VARIANTS[variant][2]]
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


def build(force: bool = False, jobs: int | None = None, verbose: bool = False, timeline: bool = False,
          variant: str = "") -> str:
    """Compile + link the extension if anything changed; return the .so path.  ``variant`` (or
    ``timeline`` = "tl"): a debug build (``VARIANTS``)."""
    build_datagen(force=force, verbose=verbose)
    if timeline:
        variant = "tl"
    obj_dir, output = VARIANTS[variant][0], VARIANTS[variant][1]
    os.makedirs(obj_dir, exist_ok=True)
    kernels, host = sources()
    headers = _headers()
    todo = [(s, True) for s in kernels] + [(s, False) for s in host]
    stale = [(s, k) for s, k in todo if force or _stale(_obj_path(s, variant), [s, *headers])]
    jobs = jobs or min(8, max(1, len(stale)))
    if stale:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            list(ex.map(lambda sk: _compile(sk[0], sk[1], verbose, variant), stale))
    objs = [_obj_path(s, variant) for s, _ in todo]
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


DATAGEN_SRC = os.path.join(CSRC, "data", "synthetic_gen.cpp")
DATAGEN_OUT = os.path.join(PKG_DIR, "_datagen" + EXT_SUFFIX)


def build_datagen(force: bool = False, verbose: bool = False) -> str:
    """The synthetic-data generator (``_datagen``: pure C++17 + pybind11, no HIP) - host compiler,
    strict IEEE float evaluation (no contraction) so every build emits the same bytes."""
    if not force and not _stale(DATAGEN_OUT, [DATAGEN_SRC, os.path.join(CSRC, "data", "synth_render.h")]):
        return DATAGEN_OUT
    cxx = os.environ.get("CXX", "g++")
    cmd = [cxx, "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-ffp-contract=off", "-fno-fast-math",
           *_includes(), DATAGEN_SRC, "-o", DATAGEN_OUT + ".tmp", "-pthread"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"datagen build failed\n{r.stdout}\n{r.stderr}")
    os.replace(DATAGEN_OUT + ".tmp", DATAGEN_OUT)
    return DATAGEN_OUT


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--timeline", action="store_true", help="debug variant with in-kernel timestamps (_C_tl)")
    ap.add_argument("--race-widen", action="store_true", help="debug variant with race-window widening (_C_rw)")
    ap.add_argument("-D", dest="defines", action="append", default=[], metavar="NAME[=VALUE]",
                    help="A/B build: extra preprocessor define (with --out; loaded via MNIST_AMD_EXT_PATH)")
    ap.add_argument("--out", default=None, help="A/B build: output .so path (own object directory)")
    a = ap.parse_args(argv)
    if a.out:
        flags = ["-D" + d for d in a.defines] + (["-DMNIST_TIMELINE"] if a.timeline else [])
        name = "ab_" + "_".join(d.replace("=", "-") for d in a.defines + (["tl"] if a.timeline else []))
        VARIANTS[name] = (os.path.join(ROOT, "build", "obj_" + name), os.path.abspath(a.out), flags)
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        out = build(force=a.force, jobs=a.jobs, verbose=a.verbose, variant=name)
    else:
        out = build(force=a.force, jobs=a.jobs, verbose=a.verbose,
                    variant="tl" if a.timeline else "rw" if a.race_widen else "")
    print(out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
