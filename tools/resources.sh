#!/bin/bash
# Per-kernel register / LDS / scratch / occupancy report for every .hip source (gfx950).
cd "$(dirname "$0")/.." || exit 1
for f in csrc/kernels/*.hip; do
  hipcc -x hip --offload-arch=gfx950 -O3 -munsafe-fp-atomics -fno-slp-vectorize -Icsrc -c "$f" -o /dev/null \
    -Rpass-analysis=kernel-resource-usage 2>&1 | awk '
    /Function Name/ {n=$(NF-1)} /VGPRs:/ {v=$(NF-1)} /AGPRs:/ {ag=$(NF-1)} /ScratchSize/ {sc=$(NF-1)}
    /Occupancy/ {o=$(NF-1)} /LDS Size/ {printf "%-60s vgpr=%-4s agpr=%-4s scratch=%-4s occ=%-2s lds=%s\n", substr(n,1,60), v, ag, sc, o, $(NF-1)}'
done
