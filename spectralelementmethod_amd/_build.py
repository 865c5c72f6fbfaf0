"""Build libsem_hip.so in-tree with hipcc for gfx950 (no JIT cache, no torch
extension machinery: the library exposes a plain C ABI, include/sem_hip.h).

The operator kernels are instantiated per order in csrc/sem_launch.hip, which
is compiled once per range of orders; all objects compile in parallel and are
linked into one shared library."""
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_NAME = "libsem_hip.so"
LIB_PATH = os.environ.get("SEM_LIB_PATH", os.path.join(PKG_DIR, LIB_NAME))
SOURCES = ["sem_device.hip", "sem_dd.hip", "sem_sc.hip", "sem_basis.cpp", "sem_hex.hip",
           "sem_order.cpp"]
# (lo, hi) order ranges of sem_launch.hip, balanced by compile time (the
# unrolled column kernels grow with n)
LAUNCH_RANGES = [(2, 5), (6, 8), (9, 9), (10, 11), (12, 13), (14, 15), (16, 16), (17, 17)]
# the constant-D Poisson launches (sem_launch_cd.hip), per range with extra
# compiler flags: machine LICM off where hoisting the materialised
# coefficients out of the round loop costs registers / occupancy
# (profiles/r04/const_d/)
NO_LICM = ("-mllvm", "-disable-machine-licm")
LAUNCH_CD_RANGES = [((2, 6), ()), ((7, 7), NO_LICM), ((8, 10), ()), ((11, 13), ()),
                    ((14, 15), ()), ((16, 16), ()), ((17, 17), NO_LICM)]
DEPS = SOURCES + ["sem_launch.hip", "sem_launch_cd.hip", "sem_internal.h", "sem_kernels.h", "sem_ctx.h", "sem_hex.h", "gll_table.h",
                  "deo_const.h"]
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


def _jobs():
    n = os.environ.get("MAX_JOBS") or str(os.cpu_count() or 4)
    return max(1, min(16, int(n)))


def build(force=False, verbose=True, out=None, defines=(), orders=None):
    """Compile the library (``out`` and ``defines`` build diagnostic
    variants, e.g. for A/B timing in one process; a ``defines`` entry that
    starts with "-" is passed to hipcc as is; ``orders`` = (lo, hi)
    restricts the kernel instantiations to those orders)."""
    out = out or LIB_PATH
    if not force and out == LIB_PATH and not needs_rebuild():
        return LIB_PATH
    objdir = out + ".objs"
    os.makedirs(objdir, exist_ok=True)
    common = [hipcc(), "--offload-arch=" + ARCH, "-O3", "-fPIC", "-std=c++17",
              "-munsafe-fp-atomics", "-Wall", "-Wno-unused-result",
              "-Wno-pass-failed",  # occupancy requests the allocator meets lower (PoissonMinWaves)
              *[d if d.startswith("-") else "-D" + d for d in defines]]
    units = [(s, [], os.path.join(objdir, s + ".o")) for s in SOURCES]
    ranges = [orders] if orders else LAUNCH_RANGES
    for lo, hi in ranges:
        units.append(("sem_launch.hip", ["-DSEM_N_LO=%d" % lo, "-DSEM_N_HI=%d" % hi],
                      os.path.join(objdir, "sem_launch_%d_%d.o" % (lo, hi))))
    for (lo, hi), flags in LAUNCH_CD_RANGES:
        if orders and (hi < orders[0] or lo > orders[1]):
            continue
        lo, hi = (max(lo, orders[0]), min(hi, orders[1])) if orders else (lo, hi)
        units.append(("sem_launch_cd.hip", ["-DSEM_N_LO=%d" % lo, "-DSEM_N_HI=%d" % hi,
                                            *flags],
                      os.path.join(objdir, "sem_launch_cd_%d_%d.o" % (lo, hi))))

    headers = [os.path.join(CSRC, d) for d in DEPS if d.endswith(".h")]
    headers.append(os.path.join(os.path.dirname(PKG_DIR), "include", "sem_hip.h"))
    t_headers = max(os.path.getmtime(h) for h in headers if os.path.exists(h))

    def compile_one(u):
        src, extra, obj = u
        cmd = common + extra + ["-c", os.path.join(CSRC, src), "-o", obj]
        stamp = obj + ".cmd"  # incremental: same command, object newer than its inputs
        if (not force and os.path.exists(obj) and os.path.exists(stamp)
                and open(stamp).read() == " ".join(cmd)
                and os.path.getmtime(obj) > max(t_headers, os.path.getmtime(cmd[-3]))):
            return obj
        if verbose:
            print("[sem build]", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        with open(stamp, "w") as f:
            f.write(" ".join(cmd))
        return obj

    with ThreadPoolExecutor(_jobs()) as ex:
        objs = list(ex.map(compile_one, units))
    # RCCL for the multi-GPU interface sum (resolves to the librccl.so.1 torch
    # already loaded when imported through _lib)
    link = [hipcc(), "--offload-arch=" + ARCH, "-shared", "-fPIC", *objs,
            "-L" + os.path.join(rocm_path(), "lib"), "-lrccl", "-o", out + ".tmp"]
    if verbose:
        print("[sem build]", " ".join(link), flush=True)
    subprocess.run(link, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    build(force=True)
