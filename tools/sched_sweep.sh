# Step-time sweep over DDP schedule variants (1 GPU, comms attached at world_size 1).
R=$PWD
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29533"
for sc in 1 2 3; do
  MNIST_AMD_DIST_SCHED=$sc timeout -k 10 200 $TR bench.py --gpus 1 --force-comm --steps 300 --warmup 30 --no-full-run > gpurun_out/sw_fc_s$sc.log 2>&1 || exit 1
  echo "comm sched=$sc $(tail -1 gpurun_out/sw_fc_s$sc.log | grep -o '"ms_per_step": [0-9.]*')"
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_fc2 -o run --output-format csv -- python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29534 $R/bench.py --gpus 1 --force-comm --steps 200 --warmup 20 --no-full-run > $R/gpurun_out/prof_fc2.log 2>&1; echo PROF_EXIT $?
