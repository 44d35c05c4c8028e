# steady-state kernel stats of the three transformer benches: bash tools/gpu_r5_prof2.sh <tag>
set -o pipefail
tag=${1:-r5p}
MARKER=embed_fwd_kernel bash tools/gpu_r5_prof.sh gpt2_medium ${tag}_gpt2 && \
MARKER=embed_fwd_kernel bash tools/gpu_r5_prof.sh gpt2_medium_fp8 ${tag}_fp8 && \
MARKER=embed_fwd_kernel bash tools/gpu_r5_prof.sh bert_base ${tag}_bert
