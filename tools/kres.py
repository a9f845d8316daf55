"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks: one line per kernel.
usage: hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python tools/kres.py [name-regex]"""
import re
import sys

pat = re.compile(sys.argv[1]) if len(sys.argv) > 1 else None
cur, rows = None, []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"(VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1)] = int(m.group(2))
for r in rows:
    if pat and not pat.search(r["name"]):
        continue
    print(f"{r.get('VGPRs', '?'):>4} v {r.get('AGPRs', '?'):>3} a spill {r.get('VGPRs Spill', '?'):>4} "
          f"occ {r.get('Occupancy [waves/SIMD]', '?')}  {r['name']}")
