"""Per-kernel VGPR / spill summary from hipcc -Rpass-analysis=kernel-resource-usage output (stdin)."""
import re
import sys

name = None
rows = {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = m.group(1)
        rows[name] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|VGPRs Spill|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", line)
    if m and name:
        rows[name][m.group(1)] = int(m.group(2))
for n, r in rows.items():
    if len(sys.argv) > 1 and sys.argv[1] not in n:
        continue
    print(f"{r.get('VGPRs', '?'):>4} vgpr {r.get('AGPRs', '?'):>4} agpr spill {r.get('VGPRs Spill', '?'):>4} "
          f"occ {r.get('Occupancy [waves/SIMD]', '?')}  {n[-60:]}")
