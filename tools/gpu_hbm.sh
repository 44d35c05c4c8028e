# Per-step HBM traffic of one bench step by kernel (FETCH_SIZE / WRITE_SIZE, one counter pass each):
#   bash tools/gpu_hbm.sh <tag> [bench args]      -> gpurun_out/<tag>_hbm.txt
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
tag=${1:-hbm}; shift
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/${tag}_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 3 "$@" > $R/gpurun_out/${tag}_fetch.log 2>&1; rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit 1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/${tag}_write -o run -- python3 $R/bench.py --steps 3 --warmup 3 "$@" > $R/gpurun_out/${tag}_write.log 2>&1; rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit 1
cd $R
f=$(find gpurun_out/${tag}_fetch -name "*counter_collection.csv" | head -1); w=$(find gpurun_out/${tag}_write -name "*counter_collection.csv" | head -1)
python tools/hbm_bytes.py $f $w 40 > gpurun_out/${tag}_hbm.txt 2>&1; echo "hbm rc=$?"
head -50 gpurun_out/${tag}_hbm.txt
rm -f $f $w
