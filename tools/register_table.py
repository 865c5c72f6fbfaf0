#!/usr/bin/env python
"""Register table of the Poisson column kernel instantiations
(k_poisson_apply<n, NODAL, M16 = true, SEAM, DOT = false, CD>, csrc/sem_kernels.h;
CD: D as compile-time constants, compiled with the flags _build.py gives the
constant-D unit of that order)
from the compiler's own resource report, one small translation unit per
instantiation compiled for gfx950 (no GPU needed):

  python tools/register_table.py [n ...] > profiles/r04/register_table.txt

Columns: VGPRs (arch + acc), SGPRs, SGPRs spilled to VGPR lanes (v_writelane
count), scratch bytes per lane and scratch instructions in the code,
occupancy (waves per SIMD), and the number of scalar loads / waits on them
(the high-order D coefficient reads)."""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "spectralelementmethod_amd", "csrc")
TU = """#include "sem_kernels.h"
namespace semk {
template __global__ void k_poisson_apply<%(n)d, %(nodal)s, true, %(seam)s, false, %(cd)s>(
    const MapRef, const double* __restrict__, const double2* __restrict__,
    const double* __restrict__, double* __restrict__, int64_t, int64_t, int, int,
    const DEO<%(n)d>, const WVec<%(n)d>, const SeamPlan);
}
"""


def one(n, nodal, seam, extra=(), cd=False):
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "k.hip")
        asm = os.path.join(d, "k.s")
        with open(src, "w") as f:
            f.write(TU % dict(n=n, nodal="true" if nodal else "false",
                              seam="true" if seam else "false", cd="true" if cd else "false"))
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
               "-munsafe-fp-atomics", "-Wno-unused-result", "-Wno-pass-failed", "-I", CSRC,
               "--cuda-device-only", "-S", src, "-o", asm] + list(extra)
        subprocess.run(cmd, check=True, capture_output=True)
        s = open(asm).read()
    # the kernel's own block (the file also holds nothing else)
    def last(key):
        m = re.findall(r"; %s: (\d+)" % key, s)
        return int(m[-1]) if m else -1
    return dict(vgpr=last("TotalNumVgprs"), sgpr=last("TotalNumSgprs"),
                scratch=last("ScratchSize"), occ=last("Occupancy"),
                sgpr_spill=len(re.findall(r"v_writelane_b32", s)),
                scratch_ops=len(re.findall(r"\bscratch_(load|store)", s)),
                sloads=len(re.findall(r"^\s+s_load_dword", s, re.M)),
                lgkm0=len(re.findall(r"s_waitcnt lgkmcnt\(0\)", s)))


def main():
    orders = [int(a) for a in sys.argv[1:]] or list(range(2, 18))
    print("%-4s %-6s %-5s %-5s %5s %5s %9s %8s %8s %4s %7s %7s" % (
        "n", "geom", "plan", "D", "VGPR", "SGPR", "sgpr2lane", "scratch", "scr_ops", "occ",
        "s_load", "waits"))
    sys.path.insert(0, ROOT)
    from spectralelementmethod_amd import _build
    cd_flags = {n: list(fl) for (lo, hi), fl in _build.LAUNCH_CD_RANGES for n in range(lo, hi + 1)}
    for n in orders:
        for cd in (False, True):
            for nodal in (True, False):
                for seam in (True, False):
                    r = one(n, nodal, seam, extra=cd_flags.get(n, []) if cd else (), cd=cd)
                    print("%-4d %-6s %-5s %-5s %5d %5d %9d %8d %8d %4d %7d %7d" % (
                        n, "nodal" if nodal else "stored", "seam" if seam else "col",
                        "const" if cd else "arg", r["vgpr"],
                        r["sgpr"], r["sgpr_spill"], r["scratch"], r["scratch_ops"], r["occ"],
                        r["sloads"], r["lgkm0"]), flush=True)


if __name__ == "__main__":
    main()
