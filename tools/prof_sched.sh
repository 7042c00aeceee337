# kernel-trace timeline of the DDP schedule $1 at world_size 1 (comms attached)
R=$PWD; SC=${1:-3}
cd /tmp && export TMPDIR=/tmp && MNIST_AMD_DIST_SCHED=$SC timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_s$SC -o run --output-format csv -- python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29535 $R/bench.py --gpus 1 --force-comm --steps 200 --warmup 20 --no-full-run > $R/gpurun_out/prof_s$SC.log 2>&1; echo PROF_EXIT $?
