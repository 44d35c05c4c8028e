# forced-collective (1 rank, RCCL) vs single-replica ResNet-50 step: which part of the collective path slows the step
FC="RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 DTF_FORCE_COLLECTIVE=1"
S="--steps 20 --warmup 5"
AB="|$S;$FC MASTER_PORT=29571|$S;$FC MASTER_PORT=29572 DTF_COMM=torch|$S;$FC MASTER_PORT=29573|$S --hiprio 0;|$S --hiprio 0;$FC MASTER_PORT=29574 DTF_WGRAD_STREAM=0|$S;DTF_WGRAD_STREAM=0|$S;$FC MASTER_PORT=29575|$S --graph 0;|$S --graph 0" bash tools/gpu_ab.sh
