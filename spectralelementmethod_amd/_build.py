"""Build libsem_hip.so in-tree with hipcc for gfx950 (no JIT cache, no torch
extension machinery: the library exposes a plain C ABI, include/sem_hip.h)."""
import os
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_NAME = "libsem_hip.so"
LIB_PATH = os.environ.get("SEM_LIB_PATH", os.path.join(PKG_DIR, LIB_NAME))
SOURCES = ["sem_device.hip", "sem_dd.hip", "sem_sc.hip", "sem_basis.cpp"]
DEPS = SOURCES + ["sem_internal.h", "sem_kernels.h", "gll_table.h"]
ARCH = os.environ.get("SEM_OFFLOAD_ARCH", "gfx950")


def rocm_path():
    return os.environ.get("ROCM_PATH", "/opt/rocm")


def hipcc():
    cand = os.path.join(rocm_path(), "bin", "hipcc")
    return cand if os.path.exists(cand) else "hipcc"


def needs_rebuild():
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    deps = [os.path.join(CSRC, d) for d in DEPS]
    deps.append(os.path.join(os.path.dirname(PKG_DIR), "include", "sem_hip.h"))
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force=False, verbose=True, out=None, defines=()):
    """Compile the library (``out`` and ``defines`` build diagnostic
    variants, e.g. for A/B timing in one process)."""
    out = out or LIB_PATH
    if not force and out == LIB_PATH and not needs_rebuild():
        return LIB_PATH
    cmd = [hipcc(), "--offload-arch=" + ARCH, "-O3", "-fPIC", "-shared", "-std=c++17",
           "-munsafe-fp-atomics", "-Wall", "-Wno-unused-result",
           *["-D" + d for d in defines],
           *[os.path.join(CSRC, s) for s in SOURCES],
           # RCCL for the multi-GPU interface sum (resolves to the librccl.so.1
           # torch already loaded when imported through _lib)
           "-L" + os.path.join(rocm_path(), "lib"), "-lrccl", "-o", out + ".tmp"]
    if verbose:
        print("[sem build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    build(force=True)
