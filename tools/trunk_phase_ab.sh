#!/bin/bash
# Build phase-timing binaries for the working-tree trunk_fwd and a git revision (default HEAD),
# to be run side by side on the GPU box:  tools/trunk_phase_ab.sh [rev]  (run here, on the CPU)
cd "$(dirname "$0")/.." || exit 1
rev=${1:-HEAD}
git show "$rev:csrc/kernels/trunk_fwd.hip" > tools/_trunk_base.hip || exit 1
F="-x hip --offload-arch=gfx950 -O3 -fno-slp-vectorize -Icsrc/kernels"
hipcc $F tools/phase_timing.hip -o tools/phase_timing.bin &&
hipcc $F -DTRUNK_SRC='"_trunk_base.hip"' tools/phase_timing.hip -o tools/phase_timing_base.bin &&
echo "built tools/phase_timing.bin (working tree) and tools/phase_timing_base.bin ($rev)"
