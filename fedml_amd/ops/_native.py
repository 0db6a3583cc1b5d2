"""Build + load the hand-written HIP kernel library (``libfedml_kernels.so``).

The kernels are plain HIP C++ with a C ABI (``FA_EXPORT`` launchers taking raw
device pointers and a ``hipStream_t``), compiled by ``hipcc --offload-arch=gfx950``
into one shared object that lives IN-TREE under ``fedml_amd/_native/`` so it
travels with the repo snapshot to the GPU box. It is loaded with ctypes *after*
``import torch``: both link ``libamdhip64.so.7`` by soname, so the library binds to
the HIP runtime torch already loaded and shares its streams/allocator.

On a GPU process every op dispatches to this library; if the library is missing
there, ops raise instead of silently falling back to PyTorch.
"""
import ctypes
import glob
import os
import subprocess
import threading

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_CSRC = os.path.join(_PKG, "ops", "csrc")
_OUT_DIR = os.path.join(_PKG, "_native")
LIB_PATH = os.path.join(_OUT_DIR, "libfedml_kernels.so")
ARCH = os.environ.get("FEDML_AMD_ARCH", "gfx950")

_lock = threading.Lock()
_lib = None
_load_error = None


def sources():
    return sorted(glob.glob(os.path.join(_CSRC, "*.hip")))


def _stale() -> bool:
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    deps = sources() + glob.glob(os.path.join(_CSRC, "*.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile every ``csrc/*.hip`` for gfx950 into one shared library (parallel objects)."""
    os.makedirs(_OUT_DIR, exist_ok=True)
    if not force and not _stale():
        return LIB_PATH
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    objs = []
    procs = []
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-I", _CSRC,
             "-Wno-unused-result"]
    for src in sources():
        obj = os.path.join(_OUT_DIR, os.path.basename(src).replace(".hip", ".o"))
        objs.append(obj)
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < max(
                [os.path.getmtime(src)] + [os.path.getmtime(h) for h in glob.glob(os.path.join(_CSRC, "*.h"))]):
            cmd = [hipcc, *flags, "-c", src, "-o", obj]
            if verbose:
                print(" ".join(cmd))
            procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    for src, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{out.decode(errors='replace')}")
    tmp = LIB_PATH + ".tmp"
    subprocess.check_call([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp])
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


def lib(required: bool = False):
    """Return the loaded ctypes library. ``required`` → raise if it is unavailable."""
    global _lib, _load_error
    with _lock:
        if _lib is None and _load_error is None:
            try:
                import torch  # noqa: F401  (bind to torch's HIP runtime first)
                alt = os.environ.get("FEDML_AMD_LIB")   # A/B measurements: another build of the same library
                if alt:
                    _lib = ctypes.CDLL(alt, mode=ctypes.RTLD_GLOBAL)
                else:
                    if _stale():
                        build()
                    _lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            except Exception as e:  # pragma: no cover - depends on toolchain
                _load_error = e
        if _lib is None and required:
            raise RuntimeError(f"fedml_amd HIP kernel library unavailable ({LIB_PATH}): {_load_error}")
        return _lib


def available() -> bool:
    return lib() is not None
