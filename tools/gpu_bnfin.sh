cd $GRAFT_REPO_ROOT
for g in 0 8 16 32 64; do echo "== DTF_BN_GROUPS=$g"; DTF_BN_GROUPS=$g timeout -k 10 120 python tools/bench_bn_finalize.py || exit 1; done
timeout -k 10 300 python tools/bench_bn.py
