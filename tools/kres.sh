#!/bin/bash
# Register / scratch / occupancy of every k_render instantiation (compile-time, no GPU):
#   bash tools/kres.sh [extra hipcc flags]
cd "$(dirname "$0")/../montecarlopathtracing_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=on \
  -fno-hip-fp32-correctly-rounded-divide-sqrt -Wno-unused-function "$@" -c mcpt_device.hip -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re, sys
cur, res = None, {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1); res[cur] = {}; continue
    for key, short in (("VGPRs:", "vgpr"), ("ScratchSize [bytes/lane]:", "scratch"), ("Occupancy [waves/SIMD]:", "waves")):
        if cur and key in line and "AGPR" not in line:
            res[cur][short] = line.split(key)[1].split()[0]
for k, v in res.items():
    if "k_render" in k:
        print(k, v)
'
