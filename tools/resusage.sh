#!/bin/bash
# Per-kernel VGPR / SGPR / scratch / occupancy of the HIP sources (gfx950).
cd "$(dirname "$0")/.." || exit 1
for f in parmmg_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -I include \
    -I parmmg_amd/csrc -c "$f" -o /tmp/resusage.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk '/Function Name:/ {n=$(NF-1)} /VGPRs:/ && !/AGPR/ {v=$(NF-1)} /TotalSGPRs:/ {s=$(NF-1)}
       /ScratchSize/ {sc=$(NF-1)} /Occupancy/ {o=$(NF-1)} /SGPRs Spill:/ {sp=$(NF-1);
       printf "%-60s vgpr=%-4s sgpr=%-4s spill=%-4s scratch=%-5s occ=%s\n", substr(n,1,60), v, s, sp, sc, o}'
done
