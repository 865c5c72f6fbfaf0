"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks: one line per
kernel with VGPRs, SGPRs, spills, scratch, occupancy, LDS."""
import re
import sys

cur = None
rows = []
for line in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(.+?): (\S+) \[-Rpass", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = m.group(2)
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for r in rows:
    if pat not in r["name"]:
        continue
    nm = re.sub(r"_ZN4semk\d+", "", r["name"])[:34]
    print("%-34s vgpr %4s agpr %3s sgpr %4s vspill %3s sspill %4s scratch %4s occ %2s lds %6s" % (
        nm, r.get("VGPRs"), r.get("AGPRs"), r.get("TotalSGPRs"), r.get("VGPRs Spill"),
        r.get("SGPRs Spill"), r.get("ScratchSize [bytes/lane]"), r.get("Occupancy [waves/SIMD]"),
        r.get("LDS Size [bytes/block]")))
