# 20-epoch README config on 1 GPU: fused bf16 engine vs module path (fused kernels via autograd) vs the
# fused fp32 step vs stock torch fp32 ops (module engine, --dtype fp32), on the synthetic split
O=${1:-gpurun_out/accuracy}; mkdir -p $O
for mode in "fused:--engine fused" "module:--engine module" "fp32:--dtype fp32" "torch_fp32:--engine module --dtype fp32"; do
  tag=${mode%%:*}; flags=${mode#*:}
  timeout -k 10 600 python mnist_ddp.py --batch-size 200 --epochs 20 --synthetic --log-interval 1000 $flags \
    --json-log $O/acc_$tag.jsonl > $O/acc_$tag.log 2>&1 || exit 1
  echo "$tag: $(grep 'Test set' $O/acc_$tag.log | tail -1) $(grep 'Total cost' $O/acc_$tag.log)"
done
