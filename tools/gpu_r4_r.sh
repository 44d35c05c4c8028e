# round 4 session R2: finalize rounding sensitivity of the ResNet test's input gradient
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for e in "DTF_BN_FIN_G=4 DTF_BN_GROUP_TARGET=1" "DTF_BN_GROUP_TARGET=1" "DTF_BN_GROUP_TARGET=2" "DTF_BN_GROUP_TARGET=8" "DTF_BN_FIN_G=4 DTF_BN_GROUP_TARGET=8" "DTF_BN_GROUP_TARGET=64" "DTF_BN_FIN_G=4 DTF_BN_GROUP_TARGET=64"; do
  echo -n "$e: "; env $e timeout -k 10 120 python -u tools/diag_resnet_link.py 2>&1 | grep "^x " || { echo "diag failed"; break; }
done
