set -o pipefail
mkdir -p gpurun_out/c1pairs
timeout -k 10 120 python tools/trunk_bits.py > gpurun_out/c1pairs/bits_head.txt 2>&1 || { cat gpurun_out/c1pairs/bits_head.txt; exit 1; }
MNIST_AMD_EXT_PATH=$PWD/tools/so/c1pairs.so timeout -k 10 120 python tools/trunk_bits.py > gpurun_out/c1pairs/bits_pairs.txt 2>&1 || { cat gpurun_out/c1pairs/bits_pairs.txt; exit 1; }
paste gpurun_out/c1pairs/bits_head.txt gpurun_out/c1pairs/bits_pairs.txt
cmp -s gpurun_out/c1pairs/bits_head.txt gpurun_out/c1pairs/bits_pairs.txt && echo BITWISE_SAME || { echo BITS_DIFFER; exit 3; }
bash tools/ab_ext.sh c1pairs "c1pairs" && bash tools/ab_ext.sh c1pairs8k "c1pairs" --batch-size 8192 --steps 200 --warmup 20
