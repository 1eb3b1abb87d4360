"""Build the native extension ``apmbackend_amd/_apm_native.so`` with hipcc for gfx950.

Every HIP kernel (``csrc/kernels/*.hip``) and every host runtime file (``csrc/runtime/*.cpp``,
``csrc/bindings.cpp``) is compiled by hipcc directly -- no hipify, no torch cpp_extension --
and linked into one in-tree shared object (it travels to the GPU box with the repo snapshot).
Incremental: an object is rebuilt when its source or any header is newer.

    python -m apmbackend_amd.build_native [--force] [-j N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(os.path.dirname(PKG), "build", "native")
TARGET = os.path.join(PKG, "_apm_native" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def hipcc() -> str:
    p = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
    if not os.path.exists(p):
        raise RuntimeError("hipcc not found (ROCm required to build the native runtime)")
    return p


def _includes():
    import pybind11
    return ["-I" + CSRC, "-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"]]


COMMON = ["-O3", "-fPIC", "-std=c++17", "-ffp-contract=off", "-Wno-unused-result"]


def _sources():
    hips = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    cpps = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp"))) + [os.path.join(CSRC, "bindings.cpp")]
    return hips, cpps


def _headers_mtime() -> float:
    hs = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def csrc_hash() -> str:
    """sha256 over every native source (path + bytes), embedded in the .so at link time so
    ``_native.load()`` can refuse an extension built from a different tree."""
    import hashlib
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(CSRC, "**", "*"), recursive=True))
    for f in files:
        if os.path.isfile(f) and f.endswith((".hip", ".cpp", ".h")):
            h.update(os.path.relpath(f, CSRC).encode() + b"\0")
            with open(f, "rb") as fh:
                h.update(fh.read())
            h.update(b"\0")
    return h.hexdigest()[:32]


def _provenance_src(digest: str) -> str:
    """A generated translation unit holding the source hash (rewritten only when it changes)."""
    path = os.path.join(BUILD, "provenance.cpp")
    text = f'extern "C" const char* apm_csrc_hash() {{ return "{digest}"; }}\n'
    old = None
    if os.path.exists(path):
        with open(path) as fh:
            old = fh.read()
    if old != text:
        with open(path, "w") as fh:
            fh.write(text)
    return path


def _obj(src: str) -> str:
    if not os.path.abspath(src).startswith(CSRC + os.sep):
        return os.path.join(BUILD, os.path.basename(src) + ".o")
    rel = os.path.relpath(src, CSRC).replace(os.sep, "_")
    return os.path.join(BUILD, rel + ".o")


def _compile(src: str, is_hip: bool, force: bool, hmt: float) -> str:
    obj = _obj(src)
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), hmt):
        return obj
    cmd = [hipcc()] + COMMON + _includes() + [f"--offload-arch={ARCH}"]
    if is_hip:
        cmd += ["-munsafe-fp-atomics"]
    cmd += ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


LAST_BUILD = {"relinked": False, "compiled": 0, "hash": None}


def build(force: bool = False, jobs: int = 0, verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    hips, cpps = _sources()
    digest = csrc_hash()
    cpps = cpps + [_provenance_src(digest)]
    hmt = _headers_mtime()
    before = {s: (os.path.getmtime(_obj(s)) if os.path.exists(_obj(s)) else 0.0) for s in hips + cpps}
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(jobs) as ex:
        futs = [ex.submit(_compile, s, True, force, hmt) for s in hips]
        futs += [ex.submit(_compile, s, False, force, hmt) for s in cpps]
        objs = [f.result() for f in futs]
    newest = max(os.path.getmtime(o) for o in objs)
    LAST_BUILD.update(relinked=False, hash=digest,
                      compiled=sum(1 for s_ in hips + cpps if os.path.getmtime(_obj(s_)) != before[s_]))
    if force or not os.path.exists(TARGET) or os.path.getmtime(TARGET) < newest:
        LAST_BUILD["relinked"] = True
        cmd = [hipcc(), "-shared", f"--offload-arch={ARCH}", "-o", TARGET + ".tmp"] + objs + [
            "-L" + os.path.join(ROCM, "lib"), "-lamdhip64", "-lrccl", "-lrocprofiler-sdk-roctx", "-Wl,-rpath," + os.path.join(ROCM, "lib"),
            "-lpthread"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(TARGET + ".tmp", TARGET)
        if verbose:
            print(f"[build_native] linked {TARGET}")
    elif verbose:
        print(f"[build_native] up to date: {TARGET}")
    return TARGET


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=0)
    a = ap.parse_args(argv)
    build(a.force, a.jobs)


if __name__ == "__main__":
    main()
