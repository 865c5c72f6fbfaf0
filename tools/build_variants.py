"""Build diagnostic variants of libsem_hip.so (build_variants/lib_<name>.so)
with extra -D defines, in parallel; optionally print each variant's register
use for one kernel (-Rpass-analysis=kernel-resource-usage).

  python tools/build_variants.py name=DEF1,DEF2 name2=DEF3 ... [--only-n 9] [--kres PATTERN]
"""
import concurrent.futures as cf
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from spectralelementmethod_amd import _build  # noqa: E402


def main():
    args = sys.argv[1:]
    only_n, kres = None, None
    if "--only-n" in args:
        i = args.index("--only-n")
        only_n = args[i + 1]
        del args[i:i + 2]
    if "--kres" in args:
        i = args.index("--kres")
        kres = args[i + 1]
        del args[i:i + 2]
    os.makedirs(os.path.join(ROOT, "build_variants"), exist_ok=True)
    jobs = {}
    for spec in args:
        name, _, defs = spec.partition("=")
        defines = [d for d in defs.split(",") if d]
        if only_n:
            defines.append("SEM_ONLY_N=%s" % only_n)
        jobs[name] = defines

    def one(name):
        out = os.path.join(ROOT, "build_variants", "lib_%s.so" % name)
        cmd = [_build.hipcc(), "--offload-arch=" + _build.ARCH, "-O3", "-fPIC", "-shared",
               "-std=c++17", "-munsafe-fp-atomics", "-Wno-unused-result",
               *["-D" + d for d in jobs[name]],
               *[os.path.join(_build.CSRC, s) for s in _build.SOURCES],
               "-L" + os.path.join(_build.rocm_path(), "lib"), "-lrccl", "-o", out]
        if kres:
            cmd.append("-Rpass-analysis=kernel-resource-usage")
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            return name, "FAILED\n" + r.stderr[-2000:]
        txt = ""
        if kres:
            log = os.path.join(ROOT, "build_variants", "kres_%s.txt" % name)
            with open(log, "w") as f:
                f.write(r.stderr)
            txt = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "kres_summary.py"),
                                  log, kres], capture_output=True, text=True).stdout
        return name, "ok " + " ".join(jobs[name]) + "\n" + txt

    with cf.ThreadPoolExecutor(max_workers=min(6, len(jobs))) as ex:
        for name, msg in ex.map(one, jobs):
            print("[%s] %s" % (name, msg), flush=True)


if __name__ == "__main__":
    main()
