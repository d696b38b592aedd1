"""Native (HIP / C++) library build + loader.

Every hot op of the framework lives in a hand-written HIP source under
``h2o3_amd/ops/csrc/*.hip`` compiled for gfx950 into an in-tree shared
library (``h2o3_amd/ops/lib/lib<name>.so``) that is loaded with ``ctypes``.
Host-side C++ runtime pieces (CSV tokenizer, ...) live in
``h2o3_amd/native/*.cpp`` and are compiled with g++ the same way.

There is deliberately no torch-extension JIT: the libraries are plain C ABI,
take raw device pointers plus a ``hipStream_t`` (torch's current stream), and
are built once by ``build_all()`` (called from ``__graft_entry__.build``).

On a machine with a GPU, ``get_lib`` raises if a HIP library is missing so a
silent PyTorch fallback can never masquerade as the native path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(_HERE, "csrc")
LIBDIR = os.path.join(_HERE, "lib")
NATIVE_SRC = os.path.join(os.path.dirname(_HERE), "native")

ARCH = os.environ.get("H2O3_AMD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

_lock = threading.Lock()
_libs: dict[str, ctypes.CDLL] = {}


def _hip_sources():
    return sorted(f for f in os.listdir(CSRC) if f.endswith(".hip"))


def _cpp_sources():
    if not os.path.isdir(NATIVE_SRC):
        return []
    return sorted(f for f in os.listdir(NATIVE_SRC) if f.endswith(".cpp"))


def lib_path(name: str) -> str:
    return os.path.join(LIBDIR, f"lib{name}.so")


def _needs_build(src: str, out: str, deps=()) -> bool:
    if not os.path.exists(out):
        return True
    mt = os.path.getmtime(out)
    for d in (src,) + tuple(deps):
        if os.path.getmtime(d) > mt:
            return True
    return False


def _source_flags(src: str) -> list[str]:
    """Extra compiler flags a source asks for on a `// hipcc-flags: ...` line
    among its first 40 lines."""
    with open(src) as f:
        for i, line in enumerate(f):
            if i >= 40:
                break
            if line.startswith("// hipcc-flags:"):
                return line.split(":", 1)[1].split()
    return []


def build_one_hip(fname: str, force: bool = False, verbose: bool = False) -> str:
    src = os.path.join(CSRC, fname)
    name = os.path.splitext(fname)[0]
    out = lib_path(name)
    headers = [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    if force or _needs_build(src, out, headers):
        os.makedirs(LIBDIR, exist_ok=True)
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC",
               "-ffp-contract=fast", *_source_flags(src), *os.environ.get("H2O3_HIPCC_EXTRA", "").split(),
               "-I", CSRC, "-o", out + ".tmp", src]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        os.replace(out + ".tmp", out)
    return out


def build_one_cpp(fname: str, force: bool = False, verbose: bool = False) -> str:
    src = os.path.join(NATIVE_SRC, fname)
    name = os.path.splitext(fname)[0]
    out = lib_path(name)
    if force or _needs_build(src, out):
        os.makedirs(LIBDIR, exist_ok=True)
        cmd = ["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-pthread", "-o", out + ".tmp", src]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        os.replace(out + ".tmp", out)
    return out


def build_all(force: bool = False, verbose: bool = False, jobs: int = 8) -> list[str]:
    """Compile every HIP source for gfx950 and every host C++ source."""
    from concurrent.futures import ThreadPoolExecutor
    outs = []
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(build_one_hip, f, force, verbose) for f in _hip_sources()]
        futs += [ex.submit(build_one_cpp, f, force, verbose) for f in _cpp_sources()]
        for fu in futs:
            outs.append(fu.result())
    return outs


def gpu_present() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


def get_lib(name: str, required: bool | None = None):
    """Load lib<name>.so. ``required`` defaults to True when a GPU is present."""
    with _lock:
        if name in _libs:
            return _libs[name]
        p = lib_path(name)
        if not os.path.exists(p):
            # try building on the fly (hipcc is available in the image)
            try:
                src_hip = os.path.join(CSRC, name + ".hip")
                src_cpp = os.path.join(NATIVE_SRC, name + ".cpp")
                if os.path.exists(src_hip):
                    build_one_hip(name + ".hip")
                elif os.path.exists(src_cpp):
                    build_one_cpp(name + ".cpp")
            except Exception:
                pass
        if not os.path.exists(p):
            req = gpu_present() if required is None else required
            if req:
                raise RuntimeError(f"native library {p} missing: run __graft_entry__.build()")
            return None
        lib = ctypes.CDLL(p)
        _libs[name] = lib
        return lib


def loaded_libs() -> list[str]:
    return [lib_path(n) for n in _libs]
