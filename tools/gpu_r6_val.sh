# Round-6 validation: GPU tests + smoke + the four benches (tools/gpu_full.sh), then the PS bench on one GPU and the
# forced-collective (torchrun, 1 rank, native RCCL communicator + capture) ResNet-50 bench.
set -o pipefail
tag=${1:-r6}
bash tools/gpu_full.sh $tag || exit 1
timeout -k 10 600 python -u bench.py --model resnet50_ps --steps 10 --warmup 3 > gpurun_out/${tag}_bench_ps.log 2>&1 || { tail -20 gpurun_out/${tag}_bench_ps.log; exit 1; }
tail -n 1 gpurun_out/${tag}_bench_ps.log | cut -c1-300
DTF_FORCE_COLLECTIVE=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench_fc.log 2>&1 || { tail -20 gpurun_out/${tag}_bench_fc.log; exit 1; }
tail -n 1 gpurun_out/${tag}_bench_fc.log | cut -c1-400
