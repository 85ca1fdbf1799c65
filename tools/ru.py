"""Print VGPR / spill / occupancy remarks of selected kernels from a hipcc -Rpass-analysis=kernel-resource-usage log:
python tools/ru.py LOG PATTERN..."""
import re
import sys

lines = open(sys.argv[1]).read().splitlines()
pats = sys.argv[2:]
cur = None
for l in lines:
    m = re.search(r"Function Name: (\S+)", l)
    if m:
        cur = m.group(1)
        continue
    if cur and any(p in cur for p in pats) and any(k in l for k in ("VGPRs:", "Spill", "Occupancy", "ScratchSize", "AGPRs:")):
        print(cur[:60], l.split("remark: ")[-1].split(" [")[0])
