set -o pipefail
# window A/B: the driver's exact command (20 timed steps after 5 warmup), several launch settings
for rep in 1 2; do
  for c in "X=0" "MNIST_AMD_GRAPH_RAMP=1" "MNIST_AMD_GRAPH_RAMP=2" "MNIST_AMD_GRAPH_RAMP=4" "DEBUG_HIP_GRAPH_BATCH_SIZE=1" "DEBUG_HIP_GRAPH_BATCH_SIZE=8" "DEBUG_HIP_GRAPH_BATCH_SIZE=64" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1"; do
    env $c timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-full-run > gpurun_out/win.log 2>&1 || { tail -20 gpurun_out/win.log; exit 1; }
    echo "$c $(grep '^{' gpurun_out/win.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["timed_enqueue_ms"], d["last_train_loss"])')"
  done
done
for c in "X=0" "MNIST_AMD_GRAPH_RAMP=2" "DEBUG_HIP_GRAPH_BATCH_SIZE=8"; do
  env $c timeout -k 10 120 python bench.py --steps 600 --warmup 50 --no-full-run > gpurun_out/win.log 2>&1 || { tail -20 gpurun_out/win.log; exit 1; }
  echo "s600 $c $(grep '^{' gpurun_out/win.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["timed_enqueue_ms"], d["last_train_loss"])')"
done
bash tools/gpu_job.sh "torchrun w8 8 --steps 20 --warmup 5 --epochs 2 --no-script-run"
