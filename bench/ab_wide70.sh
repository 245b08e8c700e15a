S="python bench.py --model llama3-70b --sessions 50 --steps 2 --warmup 1"
bash gpurun_step.sh "w70A:400:FT_WIDE_DECODE_PLAN=0 $S" "w70B:400:$S" && FT_BENCH_SHARED_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/dp2_torchrun.log 2>&1
