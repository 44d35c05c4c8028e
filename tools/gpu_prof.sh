# rocprofv3 kernel trace of one model's bench step (steady-state stats): bash tools/gpu_prof.sh <model> <tag> [bench args]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
m=${1:-resnet50}; tag=${2:-r6}; shift 2
mkdir -p gpurun_out/prof_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_$tag -o kt -- python3 -u bench.py --model $m --steps 6 --warmup 3 "$@" > gpurun_out/prof_$tag/bench.log 2>&1 || exit 1
f=$(find gpurun_out/prof_$tag -name "*kernel_trace.csv" | head -1)
python3 tools/steady_stats.py "$f" --top 40 --marker ${MARKER:-optim_kernel} > gpurun_out/prof_$tag/steady.txt 2>&1
python3 tools/timeline.py "$f" 4 12 > gpurun_out/prof_$tag/timeline.txt 2>&1 || true
python3 tools/step_list.py "$f" --marker ${MARKER:-optim_kernel} > gpurun_out/prof_$tag/step_list.txt 2>&1 || true
rm -f "$f"
head -8 gpurun_out/prof_$tag/steady.txt
head -40 gpurun_out/prof_$tag/timeline.txt
