# 20-epoch README config on 1 GPU: fused bf16 engine vs module path (fused kernels via autograd) vs stock torch fp32.
for mode in "fused:--engine fused" "module:--engine module" "fp32:--dtype fp32"; do
  tag=${mode%%:*}; flags=${mode#*:}
  timeout -k 10 600 python mnist_ddp.py --batch-size 200 --epochs 20 --synthetic --log-interval 1000 $flags \
    --json-log gpurun_out/acc_$tag.jsonl > gpurun_out/acc_$tag.log 2>&1 || exit 1
  echo "$tag: $(grep 'Test set' gpurun_out/acc_$tag.log | tail -1) $(grep 'Total cost' gpurun_out/acc_$tag.log)"
done
