"""Print per-kernel VGPR / spill / occupancy from hipcc -Rpass-analysis=kernel-resource-usage output (stdin)."""
import re
import subprocess
import sys

cur, rows = None, {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip().split("(")[0]
        rows[cur] = {}
        continue
    m = re.search(r"(VGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1)] = m.group(2)
for k, v in rows.items():
    print(f"{k:45s} vgpr {v.get('VGPRs','?'):>4} spill {v.get('VGPRs Spill','?'):>3} sspill {v.get('SGPRs Spill','?'):>3} occ {v.get('Occupancy [waves/SIMD]','?')}")
