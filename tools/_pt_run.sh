# scratch driver for tools/trunk_phase_ab.sh binaries (base = strip kernel at the base revision)
for r in 1 2; do
for B in 200 1200; do
  echo "### base strip B=$B"; MNIST_TRUNK_STRIP=1 timeout -k 10 60 ./tools/phase_timing_base.bin $B 1 || exit 1
  echo "### cur strip B=$B"; MNIST_TRUNK_STRIP=1 timeout -k 10 60 ./tools/phase_timing.bin $B 1 || exit 1
  echo "### cur img B=$B"; timeout -k 10 60 ./tools/phase_timing.bin $B 1 || exit 1
done; done
