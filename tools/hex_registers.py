#!/usr/bin/env python
"""Resource table of the hexahedral kernels (csrc/sem_hex.h) from the
compiler's own report (-Rpass-analysis=kernel-resource-usage) of sem_hex.hip
built for gfx950 -- no GPU needed:

  python tools/hex_registers.py [extra hipcc flags ...]

One row per kernel instantiation: VGPRs, AGPRs, VGPR spills, occupancy
(waves per SIMD), LDS bytes per workgroup."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "spectralelementmethod_amd", "csrc", "sem_hex.hip")


def main(extra):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17",
           "-munsafe-fp-atomics", "-Wno-pass-failed", "-Rpass-analysis=kernel-resource-usage",
           "-c", SRC, "-o", os.devnull] + list(extra)
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: (.*?): (.*?) \[-Rpass", line)
        if not m:
            continue
        key, val = m.group(1).strip(), m.group(2).strip()
        if key == "Function Name":
            cur = {"name": subprocess.run(["c++filt", val],
                                          capture_output=True, text=True).stdout.strip()}
            rows.append(cur)
        elif cur is not None:
            cur[key] = val
    print("%-52s %6s %6s %6s %5s %7s" % ("kernel", "VGPRs", "AGPRs", "spill", "occ", "LDS"))
    for r in rows:
        name = re.sub(r"\(.*", "", r["name"]).replace("void semh::", "")
        print("%-52s %6s %6s %6s %5s %7s" % (name, r.get("VGPRs", "?"), r.get("AGPRs", "?"),
                                           r.get("VGPRs Spill", "?"),
                                           r.get("Occupancy [waves/SIMD]", "?"),
                                           r.get("LDS Size [bytes/block]", "?")))


if __name__ == "__main__":
    main(sys.argv[1:])
