# round 4 session Q2: per-step HBM traffic of the ResNet-50 step (FETCH_SIZE / WRITE_SIZE, one counter pass each)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r4q2_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/r4q2_fetch.log 2>&1; rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit 1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/r4q2_write -o run -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/r4q2_write.log 2>&1; rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit 1
cd $R
f=$(find gpurun_out/r4q2_fetch -name "*counter_collection.csv" | head -1); w=$(find gpurun_out/r4q2_write -name "*counter_collection.csv" | head -1)
python tools/hbm_bytes.py $f $w 40 > gpurun_out/r4q2_hbm.txt 2>&1; echo "hbm rc=$?"
head -50 gpurun_out/r4q2_hbm.txt
rm -f $f $w
